// rt_math.h — the reference's value types restated for host (packer) and device
// (kernels): Vector3 (Raytracer.h:39-149), Pixel (Raytracer.h:373-418) and the
// EPSILON comparisons (Raytracer.h:12, Raytracer.cpp:16-18, :382, :427, :558-560).
//
// Every operation keeps the reference's operation order and rounding; this file
// (and everything that includes it) must be compiled with -ffp-contract=off.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RTM_HD __host__ __device__ __forceinline__
#define RTM_HDM __host__ __device__ __forceinline__  // member functions
#else
#define RTM_HD static inline
#define RTM_HDM inline
#endif

struct rv3 {
    float x, y, z;
};

// The float with these bits.
RTM_HD float rt_bits_f32(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __uint_as_float(u);
#else
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
#endif
}

// The bits of this float.
RTM_HD uint32_t rt_f32_bits(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __float_as_uint(f);
#else
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    return u;
#endif
}

RTM_HD rv3 v3(float x, float y, float z) { rv3 r; r.x = x; r.y = y; r.z = z; return r; }
RTM_HD rv3 v3_add(rv3 a, rv3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
RTM_HD rv3 v3_sub(rv3 a, rv3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
RTM_HD rv3 v3_mul(rv3 a, rv3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }   // component-wise
RTM_HD rv3 v3_scale(rv3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
RTM_HD rv3 v3_neg(rv3 a) { return v3(-a.x, -a.y, -a.z); }
RTM_HD float v3_dot(rv3 a, rv3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
RTM_HD rv3 v3_cross(rv3 a, rv3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
// Vector3::normalize: three divisions by the length, only if length > 0 (Raytracer.h:109-116)
RTM_HD rv3 v3_normalize(rv3 a) {
    float len = sqrtf(a.x * a.x + a.y * a.y + a.z * a.z);
    if (len > 0) { a.x /= len; a.y /= len; a.z /= len; }
    return a;
}
// v3_normalize for |a| in [0.5, 2] with components 0 or in [2^-60, 4] (the AO
// sampler's unit vectors), on the device: the instruction sequences hipcc emits
// for correctly rounded sqrtf and fp32 division, minus their range scaling and
// fixup (identities in this range), the three divisions sharing one refined
// reciprocal. Same bits as v3_normalize (GPU self-test rt580_selftest_math).
// The host build is v3_normalize.
#if defined(__HIP_DEVICE_COMPILE__)
// rt_sqrt_nr: s = +0, NaN or s in [2^-96, +inf] (sqrt(+0) = +0 and sqrt(+inf) =
// +inf fall out of the sequence; no residual fma overflows)
__device__ __forceinline__ float rt_sqrt_nr(float s) {
    const float y = __builtin_amdgcn_sqrtf(s);
    const float ym = __uint_as_float(__float_as_uint(y) - 1u);
    const float yp = __uint_as_float(__float_as_uint(y) + 1u);
    float r = y;
    if (__builtin_fmaf(-ym, y, s) <= 0.0f) r = ym;
    if (__builtin_fmaf(-yp, y, s) > 0.0f) r = yp;
    return r;
}
__device__ __forceinline__ float rt_div_nr(float n, float d, float y) {  // y = refined 1/d
    float q = n * y;
    const float e1 = __builtin_fmaf(-d, q, n);
    q = __builtin_fmaf(e1, y, q);
    const float e2 = __builtin_fmaf(-d, q, n);
    q = __builtin_fmaf(e2, y, q);
    return n == 0.0f ? n : q;
}
__device__ __forceinline__ bool rt_div_nr_ok(float n) {
    const float a = fabsf(n);
    return n == 0.0f || (a >= 0x1p-60f && a <= 4.0f);
}
// Callers guarantee the range: the AO sampler's vectors (rt_kernels.hip ao_body).
__device__ __forceinline__ rv3 v3_normalize_unit(rv3 a) {
    const float s = a.x * a.x + a.y * a.y + a.z * a.z;
    const float len = rt_sqrt_nr(s);
    const float y0 = __builtin_amdgcn_rcpf(len);
    const float y = __builtin_fmaf(__builtin_fmaf(-len, y0, 1.0f), y0, y0);
    return v3(rt_div_nr(a.x, len, y), rt_div_nr(a.y, len, y), rt_div_nr(a.z, len, y));
}
#else
RTM_HD rv3 v3_normalize_unit(rv3 a) { return v3_normalize(a); }
RTM_HD float rt_sqrt_nr(float s) { return sqrtf(s); }
RTM_HD float rt_div_nr(float n, float d, float) { return n / d; }
#endif
RTM_HD float v3_length(rv3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
// Vector3::reflect (Raytracer.h:143-148)
RTM_HD rv3 v3_reflect(rv3 I, rv3 N) {
    float d = v3_dot(I, N);
    d *= 2;
    return v3_sub(I, v3_scale(N, d));
}

// (double)x < 1e-6 for a float x  <=>  x <= RT_EPS_FLOOR (largest float below 1e-6).
// Exhaustively checked over all 2^32 floats in tests/native/eps_check.cpp.
#define RT_EPS_FLOOR 0x1.0c6f7ap-20f
RTM_HD bool rt_lt_eps(float x) { return x <= RT_EPS_FLOOR; }   // x < EPSILON, x <= EPSILON
RTM_HD bool rt_gt_eps(float x) { return x > RT_EPS_FLOOR; }    // x > EPSILON (GreaterThanZero)

// static_cast<short>(float) as the reference's x86-64 build executes it:
// cvttss2si to int32 (NaN and out-of-range -> INT32_MIN), keep the low 16 bits.
RTM_HD int32_t rt_f2s(float f) {
    int32_t i = (f > -2147483904.0f && f < 2147483648.0f) ? (int32_t)f : (int32_t)0x80000000u;
    return (int32_t)(int16_t)(uint16_t)(uint32_t)i;
}

// Pixel: int16 r,g,b kept in int32 lanes (values always equal their int16 wrap).
struct rpix {
    int32_t r, g, b;
};
RTM_HD rpix px(int32_t r, int32_t g, int32_t b) { rpix p; p.r = r; p.g = g; p.b = b; return p; }
RTM_HD int32_t rt_wrap16(int32_t v) { return (int32_t)(int16_t)(uint16_t)(uint32_t)v; }
RTM_HD int32_t rt_clamp255(int32_t v) { return v > 255 ? 255 : (v < 0 ? 0 : v); }
RTM_HD rpix px_clamp(rpix p) { return px(rt_clamp255(p.r), rt_clamp255(p.g), rt_clamp255(p.b)); }
// Pixel(const Vector3&): truncate x*255, NO clamp (the clamp() result is discarded, Raytracer.h:380)
RTM_HD rpix px_from(rv3 v) { return px(rt_f2s(v.x * 255), rt_f2s(v.y * 255), rt_f2s(v.z * 255)); }
// Pixel::operator*(float): truncate then clamp (Raytracer.h:394-400)
RTM_HD rpix px_mul(rpix p, float s) {
    return px_clamp(px(rt_f2s((float)p.r * s), rt_f2s((float)p.g * s), rt_f2s((float)p.b * s)));
}
// Pixel::operator+: int16 wrap, no clamp (Raytracer.h:403-409)
RTM_HD rpix px_add(rpix a, rpix b) { return px(rt_wrap16(a.r + b.r), rt_wrap16(a.g + b.g), rt_wrap16(a.b + b.b)); }

// fmax(x, 0) of Raytracer.cpp:242,252 (NaN -> 0)
RTM_HD float rt_fmax0(float x) { return x > 0.0f ? x : 0.0f; }
// Clipf (Raytracer.cpp:206-210); NaN passes through
RTM_HD float rt_clipf(float x, float lo, float hi) {
    if (x < lo) return lo;
    if (x > hi) return hi;
    return x;
}

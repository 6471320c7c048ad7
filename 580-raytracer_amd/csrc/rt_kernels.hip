// rt_kernels.hip — MI355X (gfx950) kernels for the reference's per-pixel path:
//   Render loop (Raytracer.cpp:916-935) -> GenerateRay (:832-858) -> Raycast
//   (:28-129) -> IntersectScene (:473-526) / IntersectTriangle (:348-409) /
//   IntersectSphere (:419-464) / CalculateLocalColor (:213-267) /
//   CalculateAmbientOcclusion (:269-330) / ComputeFresnel (:131-166) /
//   CalculateRefraction (:168-203).
//
// Pipeline for one frame (or one rank's interleaved rows):
//   1. count_kernel   one thread per pixel walks the reflect/refract tree with
//                     closest-hit queries only and counts the AO calls (hit nodes x
//                     ambient lights) and rays; per-row totals by wave-reduced atomics.
//   2. row_base_kernel exclusive scan of per-row AO calls (raster order) -> the
//                     absolute index of each row's first AO call in the reference's
//                     single serial RNG stream (skipped when the caller supplies it,
//                     e.g. after an all-gather of per-row counts across ranks).
//   3. render_kernel  one thread per pixel: in-row prefix of AO calls (wave scan +
//                     LDS), RNG skip-ahead, iterative fixed-depth reflect/refract
//                     stack, shading, AO, int16 Pixel blend; writes Pixel[w] rows.
//
// Bit-exactness rules: compiled with -ffp-contract=off; fp32
// division/sqrt correctly rounded (hipcc default); denormals preserved; glibc
// powf/sincos restated in rt_libm.h; double only where the reference is double.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt580.h"
#include "rt_libm.h"
#include "rt_math.h"
#include "rt_kernels.h"

namespace rt580 {

// ---------------------------------------------------------------- RNG
// minstd_rand0: x' = 16807 x mod (2^31-1), seed 1 (libstdc++ default_random_engine).
__device__ __forceinline__ uint32_t mersenne31_mul(uint32_t a, uint32_t b) {
    uint64_t p = (uint64_t)a * (uint64_t)b;              // < 2^62
    uint64_t r = (p & 0x7fffffffull) + (p >> 31);         // < 2^32
    r = (r & 0x7fffffffull) + (r >> 31);                  // <= 2^31
    uint32_t v = (uint32_t)r;
    return v >= 0x7fffffffu ? v - 0x7fffffffu : v;
}

// a^(2^i) mod m, i = 0..30, for O(31) skip-ahead (filled by the host).
__constant__ uint32_t c_minstd_pow2[32];

__device__ __forceinline__ uint32_t minstd_jump(uint32_t state, uint64_t k) {
    k %= 2147483646ull;  // period of a primitive root mod 2^31-1
    uint32_t s = state;
    for (int i = 0; i < 31; i++)
        if ((k >> i) & 1ull) s = mersenne31_mul(s, c_minstd_pow2[i]);
    return s;
}

struct Rng {
    uint64_t index;       // draws consumed (absolute position in the global stream)
    uint32_t state;       // minstd state after `index` draws
    int engine;
    const uint32_t* mt;   // mt19937 outputs (engine 1)

    __device__ __forceinline__ float canonical() {
        float ret;
        if (engine == RT_RNG_MINSTD_RAND0) {
            state = mersenne31_mul(state, 16807u);
            ret = (float)(state - 1u) / 2147483648.0f;   // generate_canonical<float,24>, r = 2^31-2
        } else {
            ret = (float)mt[index] / 4294967296.0f;      // r = 2^32
        }
        index++;
        if (ret >= 1.0f) ret = 0x1.fffffep-1f;           // nextafter(1, 0)
        return ret;
    }
    // uniform_real_distribution<float>::operator(): canonical * (b - a) + a
    __device__ __forceinline__ float uniform(float a, float b) { return canonical() * (b - a) + a; }
};

// ---------------------------------------------------------------- scene queries
struct Hit {
    float t, a, b, g;
    int prim;
};

__device__ __forceinline__ rv3 ld3(const float* p) { return v3(p[0], p[1], p[2]); }

// IntersectTriangle (Raytracer.cpp:348-409) with the ray-invariant part precomputed.
__device__ __forceinline__ bool tri_test(const rt_prim& P, rv3 o, rv3 d, float& t, float& a, float& b,
                                         float& g) {
    rv3 N = ld3(P.nrm);
    float nd = v3_dot(N, d);
    if (rt_lt_eps(fabsf(nd))) return false;            // NearlyEquals(nd, 0)
    t = -(v3_dot(N, o) + P.d) / nd;
    if (rt_lt_eps(t)) return false;                     // t <= EPSILON
    rv3 Pp = v3_add(o, v3_scale(d, t));
    rv3 v0 = ld3(P.p0), v1 = ld3(P.p1), v2 = ld3(P.p2);
    // CalcTriangleAreaSigned (Raytracer.cpp:937-942): 0.5 * dot(cross(B-A, C-A), N)
    float aa = 0.5f * v3_dot(v3_cross(v3_sub(v1, Pp), v3_sub(v2, Pp)), N);
    a = aa / P.area;
    float bb = 0.5f * v3_dot(v3_cross(v3_sub(Pp, v0), v3_sub(v2, v0)), N);
    b = bb / P.area;
    float gg = 0.5f * v3_dot(v3_cross(v3_sub(v1, v0), v3_sub(Pp, v0)), N);
    g = gg / P.area;
    return !(a < 0 || b < 0 || g < 0);
}

// IntersectSphere (Raytracer.cpp:419-464)
__device__ __forceinline__ bool sph_test(const rt_prim& P, rv3 o, rv3 d, float& t) {
    rv3 oc = v3_sub(o, ld3(P.p0));
    float b = 2.0f * v3_dot(d, oc);
    float c = v3_dot(oc, oc) - P.d;
    float disc = (b * b) - (4.0f * c);
    if (rt_lt_eps(disc)) return false;
    float sq = sqrtf(disc);
    float t0 = (-b + sq) / 2.0f;
    float t1 = (-b - sq) / 2.0f;
    bool g0 = rt_gt_eps(t0), g1 = rt_gt_eps(t1);
    if (!g0 && !g1) return false;
    if (!g0) t = t1;
    else if (!g1) t = t0;
    else t = fminf(t0, t1);
    return true;
}

// IntersectScene, closest hit: primitives in the reference's order, the first
// hit is taken unconditionally and later ones only if strictly closer (:487-498).
__device__ bool closest_hit(const DevScene& S, rv3 o, rv3 d, Hit& h) {
    bool found = false;
    for (int i = 0; i < S.n_prims; i++) {
        const rt_prim P = S.prims[i];
        float t, a = 0, b = 0, g = 0;
        bool hit = P.kind == RT_PRIM_TRIANGLE ? tri_test(P, o, d, t, a, b, g) : sph_test(P, o, d, t);
        if (hit && (!found || t < h.t)) {
            found = true;
            h.t = t; h.a = a; h.b = b; h.g = g; h.prim = i;
        }
    }
    return found;
}

// IntersectScene when only the boolean is used (directional shadows, AO rays).
__device__ bool any_hit(const DevScene& S, rv3 o, rv3 d) {
    for (int i = 0; i < S.n_prims; i++) {
        const rt_prim P = S.prims[i];
        float t, a, b, g;
        bool hit = P.kind == RT_PRIM_TRIANGLE ? tri_test(P, o, d, t, a, b, g) : sph_test(P, o, d, t);
        if (hit) return true;
    }
    return false;
}

// ---------------------------------------------------------------- camera
// GenerateRay (Raytracer.cpp:832-858): double NDC, no +0.5 pixel centre.
__device__ __forceinline__ void generate_ray(const DevFrame& F, int x, int y, rv3& o, rv3& d) {
    double ndcx = (2.0 * x) / F.width - 1;
    double ndcy = 1 - (2.0 * y) / F.height;
    ndcx *= F.ndc_kx;
    ndcy *= F.ndc_ky;
    o = v3(F.cam_from[0], F.cam_from[1], F.cam_from[2]);
    rv3 dir = v3((float)ndcx, (float)ndcy, -1.0f);
    if (F.view_inverse_ok) {
        const float* m = F.view_inv;
        d = v3_normalize(v3(m[0] * dir.x + m[1] * dir.y + m[2] * dir.z,
                            m[3] * dir.x + m[4] * dir.y + m[5] * dir.z,
                            m[6] * dir.x + m[7] * dir.y + m[8] * dir.z));
    } else {
        d = v3(0, 0, 0);
    }
}

// ---------------------------------------------------------------- shading
struct HitInfo {
    rv3 p, n;  // world hit point, geometric normal (hitInfo.normal)
    int prim;
    int kind;
    float a, b, g;
};

__device__ __forceinline__ void resolve_hit(const DevScene& S, rv3 o, rv3 d, const Hit& h, HitInfo& hi) {
    const rt_prim P = S.prims[h.prim];
    hi.p = v3_add(o, v3_scale(d, h.t));
    hi.prim = h.prim;
    hi.kind = P.kind;
    hi.a = h.a; hi.b = h.b; hi.g = h.g;
    if (P.kind == RT_PRIM_TRIANGLE) hi.n = ld3(S.shade[h.prim].hit_nrm);
    else hi.n = v3_normalize(v3_sub(hi.p, ld3(P.p0)));
}

// CalculateLocalColor (Raytracer.cpp:213-267); L is the normalized to-light vector.
__device__ rpix local_color(const DevScene& S, const DevFrame& F, const HitInfo& h, const rt_light& l,
                            const rt_material& m, rv3 L) {
    rv3 n;
    if (h.kind == RT_PRIM_TRIANGLE) {
        const rt_prim_shade& sh = S.shade[h.prim];
        rv3 in = v3_add(v3_add(v3_scale(ld3(sh.vn0), h.a), v3_scale(ld3(sh.vn1), h.b)), v3_scale(ld3(sh.vn2), h.g));
        n = v3_normalize(v3_normalize(in));  // InterpolateVector3 (:333-338) + :237
    } else {
        n = v3_normalize(h.n);
    }
    rv3 lc = ld3(l.color);
    float ds = rt_fmax0(v3_dot(L, n));
    rv3 diffuse = v3_scale(v3_scale(lc, ds), l.intensity);
    rv3 R = v3_normalize(v3_reflect(L, n));
    rv3 V = v3_normalize(v3_sub(v3(F.cam_from[0], F.cam_from[1], F.cam_from[2]), h.p));
    float ss = rt_fmax0(v3_dot(V, R));
    ss = rt_glibc_powf(ss, m.spec_exp);
    rv3 spec = v3_scale(v3_scale(lc, ss), l.intensity);
    rv3 lighting = v3_add(v3_scale(diffuse, m.kd), v3_scale(spec, m.ks));
    rv3 col = v3_mul(ld3(m.cs), lighting);
    col.x = rt_clipf(col.x, 0.0f, 1.0f);
    col.y = rt_clipf(col.y, 0.0f, 1.0f);
    col.z = rt_clipf(col.z, 0.0f, 1.0f);
    return px_from(col);
}

// CalculateAmbientOcclusion (Raytracer.cpp:315-330) with RandomInHemisphere (:283-292)
// and RandomUnitVector (:269-281).
__device__ float ambient_occlusion(const DevScene& S, const DevFrame& F, rv3 hp, rv3 n, Rng& rng) {
    float occ = 0.0f;
    for (int i = 0; i < F.ao_samples; i++) {
        float z = rng.uniform(-1.0f, 1.0f);
        float ang = rng.uniform(0.0f, F.ao_angle_max);
        float r = sqrtf(1 - z * z);
        double sa, ca;
        rt_glibc_sincos((double)ang, &sa, &ca);
        rv3 v = v3_normalize(v3((float)((double)r * ca), (float)((double)r * sa), z));
        if (!(v3_dot(v, n) > 0.0f)) v = v3_neg(v);
        rv3 o = v3_add(hp, v3_scale(v, 0.2f));
        rv3 d = v3_normalize(v);  // Ray constructor
        if (any_hit(S, o, d)) occ += 1.0f;
    }
    return 1.0f - ((float)occ / (float)F.ao_samples);
}

// Raycast's light loop (Raytracer.cpp:39-82). Returns the (unclamped) local color.
__device__ rpix shade_lights(const DevScene& S, const DevFrame& F, const HitInfo& h, const rt_material& m,
                             Rng& rng) {
    rpix local = px(0, 0, 0);
    for (int li = 0; li < S.n_lights; li++) {
        const rt_light l = S.lights[li];
        if (l.kind == RT_LIGHT_AMBIENT) {
            rv3 amb = v3_scale(v3_mul(v3_scale(ld3(m.cs), m.ka), ld3(l.color)), l.intensity);
            float ao = F.ao_enabled ? ambient_occlusion(S, F, h.p, h.n, rng) : 1.0f;
            amb = v3_scale(amb, ao);
            local = px_add(local, px_from(amb));
            continue;
        }
        rv3 L, L2;
        bool occluded;
        if (l.kind == RT_LIGHT_DIRECTIONAL) {
            L = ld3(l.L);
            L2 = ld3(l.L2);
            occluded = any_hit(S, v3_add(h.p, v3_scale(L, 0.2f)), L2);
        } else {
            rv3 tl = v3_sub(ld3(l.position), h.p);
            L = v3_normalize(tl);
            L2 = v3_normalize(L);
            float dist = v3_length(tl);
            Hit sh;
            bool hit = closest_hit(S, v3_add(h.p, v3_scale(L, 0.2f)), L2, sh);
            occluded = hit && !(sh.t > dist);
        }
        if (!occluded) local = px_add(local, local_color(S, F, h, l, m, L));
    }
    return local;
}

// CalculateRefraction (Raytracer.cpp:168-203)
__device__ __forceinline__ rv3 refraction_dir(rv3 I, rv3 N, float ior) {
    float cosi = v3_dot(I, N);
    if (cosi < -1) cosi = -1;
    else if (cosi > 1) cosi = 1;
    float n1 = 1, n2 = ior;
    rv3 n = N;
    if (cosi < 0) {
        cosi = -1 * cosi;
    } else {
        float t = n1; n1 = n2; n2 = t;
        n = v3_neg(N);
    }
    float eta = n1 / n2;
    float k = 1 - eta * eta * (1 - cosi * cosi);
    if (k < 0) return v3(0, 0, 0);
    return v3_add(v3_scale(I, eta), v3_scale(n, (eta * cosi - sqrtf(k))));
}

// ComputeFresnel (Raytracer.cpp:131-166)
__device__ __forceinline__ void fresnel(float ior, rv3 N, rv3 I, float& kr, float& kt) {
    float cosi = rt_clipf(v3_dot(I, N), -1.0f, 1.0f);
    bool inside = cosi > 0;
    float ei = 1, et = ior;
    if (inside) { float t = ei; ei = et; et = t; cosi = -cosi; }
    float s = 1 - cosi * cosi;
    float sint = ei / et * sqrtf(0.f < s ? s : 0.f);
    if (sint >= 1) {
        kr = 1; kt = 0;
    } else {
        float s2 = 1 - sint * sint;
        float cost = sqrtf(0.f < s2 ? s2 : 0.f);
        cosi = fabsf(cosi);
        float Rs = ((et * cosi) - (ei * cost)) / ((et * cosi) + (ei * cost));
        float Rp = ((ei * cosi) - (et * cost)) / ((ei * cosi) + (et * cost));
        kr = (Rs * Rs + Rp * Rp) / 2;
        kt = 1 - kr;
    }
}

// One pending node of the reflect/refract recursion (Raycast is a binary tree,
// evaluated bottom-up because the int16 blend is non-linear).
struct Frame {
    rpix local, refl;
    float kr, kt, ks, ktm;
    rv3 ro, rd;      // refraction child ray (if ktm > 0)
    int stage;       // 1: reflection child pending, 2: refraction child pending
};

// Raycast's blend (Raytracer.cpp:114-128)
__device__ __forceinline__ rpix combine(const Frame& f, rpix refr) {
    rpix fR = px_mul(px_mul(f.refl, f.kr), f.ks);
    rpix fT = px_mul(px_mul(refr, f.kt), f.ktm);
    float alb = 1 - f.ks - f.ktm;
    alb = alb > 0.0f ? alb : 0.0f;   // std::max(alb, 0.0f)
    rpix out = px_add(px_add(px_mul(f.local, alb), px_mul(fR, f.ks)), px_mul(fT, f.ktm));
    return px_clamp(out);
}

struct Tally {
    uint32_t hits, tree_rays;
};

// Iterative Raycast over the recursion tree. COUNT: structure only (closest hits),
// no lights, no AO, no RNG draws.
template <bool COUNT>
__device__ rpix trace_pixel(const DevScene& S, const DevFrame& F, rv3 o, rv3 d, Rng& rng, Tally& tally) {
    Frame st[RT_MAX_DEPTH + 1];
    int lvl = 0;
    rpix ret;
    for (;;) {
        // ---- evaluate the node (o, d) at level lvl with bounces = depth - lvl
        const int bounces = F.depth - lvl;
        Hit h;
        tally.tree_rays++;
        bool descended = false;
        if (!closest_hit(S, o, d, h)) {
            ret = px(254, 64, 205);  // BG_COLOR (Raytracer.h:597)
        } else {
            tally.hits++;
            HitInfo hi;
            resolve_hit(S, o, d, h, hi);
            const rt_material m = S.mats[S.prims[h.prim].shape];
            rpix local = px(0, 0, 0);
            if (!COUNT) local = shade_lights(S, F, hi, m, rng);
            if (bounces == 0) {
                ret = px_clamp(local);
            } else {
                Frame& f = st[lvl];
                f.local = local;
                f.refl = px(0, 0, 0);
                f.ks = m.ks;
                f.ktm = m.kt;
                fresnel(m.ior, hi.n, d, f.kr, f.kt);
                if (m.kt > 0) {
                    rv3 td = refraction_dir(d, hi.n, m.ior);
                    f.ro = v3_add(hi.p, v3_scale(td, 0.2f));
                    f.rd = v3_normalize(td);
                }
                if (m.ks > 0) {
                    rv3 rd = v3_normalize(v3_reflect(d, hi.n));
                    o = v3_add(hi.p, v3_scale(rd, 0.2f));
                    d = v3_normalize(rd);
                    f.stage = 1;
                    lvl++;
                    descended = true;
                } else if (m.kt > 0) {
                    o = f.ro;
                    d = f.rd;
                    f.stage = 2;
                    lvl++;
                    descended = true;
                } else {
                    ret = combine(f, px(0, 0, 0));
                }
            }
        }
        if (descended) continue;
        // ---- return `ret` to the parents
        bool resumed = false;
        while (lvl > 0) {
            Frame& p = st[lvl - 1];
            if (p.stage == 1) {
                p.refl = ret;
                if (p.ktm > 0) {
                    p.stage = 2;
                    o = p.ro;
                    d = p.rd;
                    resumed = true;  // same level: sibling subtree
                    break;
                }
                ret = combine(p, px(0, 0, 0));
            } else {
                ret = combine(p, ret);
            }
            lvl--;
        }
        if (!resumed) return ret;
    }
}

// ---------------------------------------------------------------- kernels
__device__ __forceinline__ int frame_row(const DevFrame& F, int local_row) {
    return F.row_begin + local_row * F.row_step;
}

__global__ void __launch_bounds__(256) count_kernel(DevScene S, DevFrame F, uint32_t* __restrict__ pix_calls,
                                                    uint32_t* __restrict__ row_calls,
                                                    uint32_t* __restrict__ row_tree,
                                                    uint32_t* __restrict__ row_hits) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t npix = (int64_t)F.n_rows * F.width;
    if (idx >= npix) return;
    const int lr = (int)(idx / F.width);
    const int x = (int)(idx - (int64_t)lr * F.width);
    rv3 o, d;
    generate_ray(F, x, frame_row(F, lr), o, d);
    Rng rng;
    Tally t = {0, 0};
    trace_pixel<true>(S, F, o, d, rng, t);
    uint32_t calls = t.hits * (uint32_t)F.n_ambient;
    pix_calls[idx] = calls;
    atomicAdd(&row_calls[lr], calls);
    atomicAdd(&row_tree[lr], t.tree_rays);
    atomicAdd(&row_hits[lr], t.hits);
}

// Exclusive scan of per-row AO calls in raster order (one workgroup).
__global__ void __launch_bounds__(1024) row_base_kernel(const uint32_t* __restrict__ row_calls, int n_rows,
                                                        uint64_t* __restrict__ row_base) {
    __shared__ uint64_t partial[1024];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n_rows; base += 1024) {
        int i = base + threadIdx.x;
        uint64_t v = i < n_rows ? row_calls[i] : 0;
        partial[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            uint64_t add = threadIdx.x >= off ? partial[threadIdx.x - off] : 0;
            __syncthreads();
            partial[threadIdx.x] += add;
            __syncthreads();
        }
        if (i < n_rows) row_base[i] = carry + partial[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += partial[1023];
        __syncthreads();
    }
}

// One workgroup per local row: exclusive in-row prefix of AO calls + the row's
// base -> absolute AO-call index of each pixel.
__global__ void __launch_bounds__(1024) pixel_base_kernel(const uint32_t* __restrict__ pix_calls, int width,
                                                          const uint64_t* __restrict__ row_base,
                                                          uint64_t* __restrict__ pix_base) {
    __shared__ uint32_t partial[1024];
    __shared__ uint64_t carry;
    const int lr = blockIdx.x;
    const uint32_t* calls = pix_calls + (int64_t)lr * width;
    uint64_t* out = pix_base + (int64_t)lr * width;
    if (threadIdx.x == 0) carry = row_base[lr];
    __syncthreads();
    for (int base = 0; base < width; base += 1024) {
        int i = base + threadIdx.x;
        uint32_t v = i < width ? calls[i] : 0;
        partial[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 1024; off <<= 1) {
            uint32_t add = threadIdx.x >= off ? partial[threadIdx.x - off] : 0;
            __syncthreads();
            partial[threadIdx.x] += add;
            __syncthreads();
        }
        if (i < width) out[i] = carry + partial[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += partial[1023];
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) render_kernel(DevScene S, DevFrame F, const uint64_t* __restrict__ pix_base,
                                                     int16_t* __restrict__ fb) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t npix = (int64_t)F.n_rows * F.width;
    if (idx >= npix) return;
    const int lr = (int)(idx / F.width);
    const int x = (int)(idx - (int64_t)lr * F.width);
    rv3 o, d;
    generate_ray(F, x, frame_row(F, lr), o, d);
    Rng rng;
    rng.engine = F.rng_engine;
    rng.mt = F.mt_stream;
    rng.index = F.ao_enabled ? pix_base[idx] * (uint64_t)(2 * F.ao_samples) : 0;
    rng.state = F.rng_engine == RT_RNG_MINSTD_RAND0 ? minstd_jump(F.rng_seed, rng.index) : 0;
    Tally t = {0, 0};
    rpix p = trace_pixel<false>(S, F, o, d, rng, t);
    fb[idx * 3 + 0] = (int16_t)p.r;
    fb[idx * 3 + 1] = (int16_t)p.g;
    fb[idx * 3 + 2] = (int16_t)p.b;
}

__global__ void select_rows_kernel(const uint64_t* __restrict__ all_base, int row_begin, int row_step,
                                   int n_rows, uint64_t* __restrict__ sel_base) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n_rows) sel_base[k] = all_base[row_begin + k * row_step];
}

// ---------------------------------------------------------------- launchers
hipError_t launch_select_rows(const uint64_t* all_base, int row_begin, int row_step, int n_rows,
                              uint64_t* sel_base, hipStream_t s) {
    if (n_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(select_rows_kernel, dim3((n_rows + 255) / 256), dim3(256), 0, s, all_base, row_begin,
                       row_step, n_rows, sel_base);
    return hipGetLastError();
}

void upload_minstd_table(hipStream_t s) {
    uint32_t t[32];
    uint64_t a = 16807;
    for (int i = 0; i < 32; i++) {
        t[i] = (uint32_t)a;
        a = (a * a) % 2147483647ull;
    }
    (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(c_minstd_pow2), t, sizeof t, 0, hipMemcpyHostToDevice, s);
}

hipError_t launch_count(const DevScene& S, const DevFrame& F, uint32_t* pix_calls, uint32_t* row_calls,
                        uint32_t* row_tree, uint32_t* row_hits, hipStream_t s) {
    int64_t npix = (int64_t)F.n_rows * F.width;
    if (npix == 0) return hipSuccess;
    dim3 grid((unsigned)((npix + 255) / 256));
    hipLaunchKernelGGL(count_kernel, grid, dim3(256), 0, s, S, F, pix_calls, row_calls, row_tree, row_hits);
    return hipGetLastError();
}

hipError_t launch_row_base(const uint32_t* row_calls, int n_rows, uint64_t* row_base, hipStream_t s) {
    hipLaunchKernelGGL(row_base_kernel, dim3(1), dim3(1024), 0, s, row_calls, n_rows, row_base);
    return hipGetLastError();
}

hipError_t launch_pixel_base(const uint32_t* pix_calls, int width, int n_rows, const uint64_t* row_base,
                             uint64_t* pix_base, hipStream_t s) {
    if (n_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(pixel_base_kernel, dim3(n_rows), dim3(1024), 0, s, pix_calls, width, row_base, pix_base);
    return hipGetLastError();
}

hipError_t launch_render(const DevScene& S, const DevFrame& F, const uint64_t* pix_base, int16_t* fb,
                         hipStream_t s) {
    int64_t npix = (int64_t)F.n_rows * F.width;
    if (npix == 0) return hipSuccess;
    dim3 grid((unsigned)((npix + 255) / 256));
    hipLaunchKernelGGL(render_kernel, grid, dim3(256), 0, s, S, F, pix_base, fb);
    return hipGetLastError();
}

}  // namespace rt580

// rt_libm.h — bit-exact restatements of the two glibc 2.35 libm routines that
// sit on the reference's per-pixel path, usable on host (g++) and device (hipcc).
//
//   rt_glibc_powf   == glibc powf, x86_64 ifunc variant __powf_fma
//                      (sysdeps/ieee754/flt-32/e_powf.c, ARM optimized-routines
//                      algorithm: log2 via 16-entry table + degree-5 poly, exp2 via
//                      32-entry table + degree-3 poly, all in double; the FMA build
//                      contracts every a*b+c, reproduced here with explicit fma()).
//                      Called by CalculateLocalColor, Raytracer.cpp:253.
//   rt_glibc_sincos == glibc sincos (sysdeps/ieee754/dbl-64/s_sincos.c with the
//                      do_sin / do_cos / reduce_sincos / TAYLOR_SIN helpers of
//                      s_sin.c; plain SSE2 build, no FMA). The reference's
//                      `x = r*cos(a); y = r*sin(a)` (Raytracer.cpp:277-278) is
//                      compiled by g++ into one sincos call (checked in the oracle
//                      binary's disassembly).
//
// glibc is NOT correctly rounded, so a correctly rounded (or vendor) pow/sin/cos
// would not reproduce the reference's bits. Tables come from this image's libm
// (tools/gen_glibc_tables.py -> glibc_tables.inc). Equality with the host glibc
// is checked EXHAUSTIVELY over the input domains the path uses
// (tests/native/libm_check.cpp driven by tests/test_native_checks.py; the device
// leg, the device powf against the host's glibc, in tests/test_gpu_libm.py).
//
// Licence: the algorithms and tables restated here are glibc's (GNU LGPL 2.1
// or later; the powf tables come from ARM's optimized-routines, MIT/Apache-2.0
// in that project). INTEGRATION.md records this.
//
// Every floating-point expression below must be compiled WITHOUT contraction
// (-ffp-contract=off): the FMA points of __powf_fma are the explicit fma() calls.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#define RT_TABLE_QUAL static __device__ __constant__ const
#define RT_TABLE(name) name
#else
#define RT_HD static inline
#define RT_TABLE_QUAL static const
#define RT_TABLE(name) name
#endif

#if defined(__HIPCC__)
// Device copies live in __constant__ memory; the host build (tests) uses the
// same generated initialisers through a second, host-only definition.
namespace rt_dev {
#include "glibc_tables.inc"
#include "sct128_table.inc"
}
namespace rt_host {
#undef RT_TABLE_QUAL
#define RT_TABLE_QUAL static const
#include "glibc_tables.inc"
#include "sct128_table.inc"
}
#if defined(__HIP_DEVICE_COMPILE__)
#define RT_T(name) rt_dev::name
#else
#define RT_T(name) rt_host::name
#endif
#else
namespace rt_host {
#include "glibc_tables.inc"
#include "sct128_table.inc"
}
#define RT_T(name) rt_host::name
#endif

RT_HD uint32_t rt_f2u(float f) { union { float f; uint32_t u; } v; v.f = f; return v.u; }
RT_HD float rt_u2f(uint32_t u) { union { float f; uint32_t u; } v; v.u = u; return v.f; }
RT_HD uint64_t rt_d2u(double d) { union { double d; uint64_t u; } v; v.d = d; return v.u; }
RT_HD double rt_u2d(uint64_t u) { union { double d; uint64_t u; } v; v.u = u; return v.d; }

// ---------------------------------------------------------------------------
// powf (e_powf.c)
// ---------------------------------------------------------------------------
RT_HD int rt_powf_zeroinfnan(uint32_t ix) { return 2u * ix - 1u >= 2u * 0x7f800000u - 1u; }

// 0: not integer, 1: odd integer, 2: even integer (e_powf.c checkint)
RT_HD int rt_powf_checkint(uint32_t iy) {
    int e = (int)(iy >> 23 & 0xff);
    if (e < 0x7f) return 0;
    if (e > 0x7f + 23) return 2;
    if (iy & ((1u << (0x7f + 23 - e)) - 1u)) return 0;
    if (iy & (1u << (0x7f + 23 - e))) return 1;
    return 2;
}

RT_HD int rt_issignalingf(float x) {
    uint32_t ix = rt_f2u(x);
    return 2u * (ix ^ 0x00400000u) > 2u * 0x7fc00000u;
}

// log2_inline: x = 2^k z, z in [OFF, 2*OFF]; log2(x) = log1p(z/c-1)/ln2 + log2(c) + k
RT_HD double rt_powf_log2_inline(uint32_t ix) {
    const uint32_t OFF = 0x3f330000u;
    uint32_t tmp = ix - OFF;
    int i = (int)((tmp >> (23 - 4)) % 16u);
    uint32_t top = tmp & 0xff800000u;
    uint32_t iz = ix - top;
    int k = (int32_t)top >> 23;
    double invc = RT_T(rt_powf_log2_tab)[2 * i];
    double logc = RT_T(rt_powf_log2_tab)[2 * i + 1];
    double z = (double)rt_u2f(iz);
    const double* A = RT_T(rt_powf_log2_poly);
    double r = fma(z, invc, -1.0);           // z * invc - 1
    double y0 = logc + (double)k;
    double r2 = r * r;
    double y = fma(A[0], r, A[1]);           // A[0] * r + A[1]
    double p = fma(A[2], r, A[3]);           // A[2] * r + A[3]
    double r4 = r2 * r2;
    double q = fma(A[4], r, y0);             // A[4] * r + y0
    q = fma(p, r2, q);                       // p * r2 + q
    y = fma(y, r4, q);                       // y * r4 + q
    return y;
}

RT_HD float rt_powf_exp2_inline(double xd, uint32_t sign_bias) {
    double kd = xd + RT_EXP2F_SHIFT_SCALED;
    uint64_t ki = rt_d2u(kd);
    kd -= RT_EXP2F_SHIFT_SCALED;            // k/N
    double r = xd - kd;
    uint64_t t = RT_T(rt_exp2f_tab)[ki % 32];
    uint64_t ski = ki + sign_bias;
    t += ski << (52 - 5);
    double s = rt_u2d(t);
    const double* C = RT_T(rt_exp2f_poly);
    double z = fma(C[0], r, C[1]);           // C[0] * r + C[1]
    double r2 = r * r;
    double y = fma(C[2], r, 1.0);            // C[2] * r + 1
    y = fma(z, r2, y);                       // z * r2 + y
    y = y * s;
    return (float)y;
}

RT_HD float rt_glibc_powf(float x, float y) {
    uint32_t sign_bias = 0;
    uint32_t ix = rt_f2u(x), iy = rt_f2u(y);
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u || rt_powf_zeroinfnan(iy)) {
        if (rt_powf_zeroinfnan(iy)) {
            if (2u * iy == 0) return rt_issignalingf(x) ? x + y : 1.0f;
            if (ix == 0x3f800000u) return rt_issignalingf(y) ? x + y : 1.0f;
            if (2u * ix > 2u * 0x7f800000u || 2u * iy > 2u * 0x7f800000u) return x + y;
            if (2u * ix == 2u * 0x3f800000u) return 1.0f;
            if ((2u * ix < 2u * 0x3f800000u) == !(iy & 0x80000000u)) return 0.0f;
            return y * y;
        }
        if (rt_powf_zeroinfnan(ix)) {
            float x2 = x * x;
            if ((ix & 0x80000000u) && rt_powf_checkint(iy) == 1) { x2 = -x2; sign_bias = 1; }
            if (2u * ix == 0 && (iy & 0x80000000u)) return (sign_bias ? -1.0f : 1.0f) / 0.0f;
            return (iy & 0x80000000u) ? 1.0f / x2 : x2;
        }
        // x and y are non-zero finite
        if (ix & 0x80000000u) {
            int yint = rt_powf_checkint(iy);
            if (yint == 0) { float d = x - x; return d / d; }
            if (yint == 1) sign_bias = 1u << (5 + 11);
            ix &= 0x7fffffffu;
        }
        if (ix < 0x00800000u) {
            ix = rt_f2u(x * 0x1p23f);
            ix &= 0x7fffffffu;
            ix -= 23u << 23;
        }
    }
    double logx = rt_powf_log2_inline(ix);
    double ylogx = (double)y * logx;
    if ((rt_d2u(ylogx) >> 47 & 0xffff) >= rt_d2u(126.0) >> 47) {
        // |y*log(x)| >= 126
        if (ylogx > 0x1.fffffffd1d571p+6) {   // __math_oflowf
            float v = sign_bias ? -0x1p97f : 0x1p97f;
            return v * 0x1p97f;
        }
        // (0x1.fffffffa3aae2p+6 check: only differs in directed rounding modes)
        if (ylogx <= -150.0) {                 // __math_uflowf
            float v = sign_bias ? -0x1p-95f : 0x1p-95f;
            return v * 0x1p-95f;
        }
        if (ylogx < -149.0) {                  // __math_may_uflowf
            float v = sign_bias ? -0x1.4p-75f : 0x1.4p-75f;
            return v * 0x1.4p-75f;
        }
    }
    return rt_powf_exp2_inline(ylogx, sign_bias);
}

// ---------------------------------------------------------------------------
// sincos (s_sincos.c + s_sin.c helpers), no FMA
// ---------------------------------------------------------------------------
#define RT_SC_SN3 (-RT_SC_SN3_NEG)
#define RT_SC_CS4 (-RT_SC_CS4_NEG)
#define RT_SC_S1 (-RT_SC_S1_NEG)
#define RT_SC_S3 (-RT_SC_S3_NEG)
#define RT_SC_S5 (RT_SC_S5_NEG)   // stored value already negative

RT_HD double rt_sc_taylor_sin(double xx, double a, double da) {
    double poly = (((RT_SC_S5 * xx + RT_SC_S4) * xx + RT_SC_S3) * xx + RT_SC_S2) * xx + RT_SC_S1;
    double t = ((poly * a - 0.5 * da) * xx + da);
    return a + t;
}

// do_cos / do_sin read the 440-entry __sincostab through `tab` (constant memory
// by default; the AO kernel passes a copy staged in LDS).
RT_HD double rt_sc_do_cos_t(const double* tab, double x, double dx) {
    if (x < 0) dx = -dx;
    double ax = fabs(x);
    double ux = RT_SC_BIG + ax;
    uint32_t lo = (uint32_t)rt_d2u(ux);
    x = ax - (ux - RT_SC_BIG) + dx;
    double xx = x * x;
    double s = x + x * xx * (RT_SC_SN3 + xx * RT_SC_SN5);
    double c = xx * (RT_SC_CS2 + xx * (RT_SC_CS4 + xx * RT_SC_CS6));
    int k = (int)(lo << 2);
    double sn = tab[k], ssn = tab[k + 1];
    double cs = tab[k + 2], ccs = tab[k + 3];
    double cor = (ccs - s * ssn - cs * c) - sn * s;
    return cs + cor;
}

RT_HD double rt_sc_do_sin_t(const double* tab, double x, double dx) {
    double xold = x;
    if (fabs(x) < RT_SC_TAYLOR_CUT) return rt_sc_taylor_sin(x * x, x, dx);
    if (x <= 0) dx = -dx;
    double ax = fabs(x);
    double ux = RT_SC_BIG + ax;
    uint32_t lo = (uint32_t)rt_d2u(ux);
    x = ax - (ux - RT_SC_BIG);
    double xx = x * x;
    double s = x + (dx + x * xx * (RT_SC_SN3 + xx * RT_SC_SN5));
    double c = x * dx + xx * (RT_SC_CS2 + xx * (RT_SC_CS4 + xx * RT_SC_CS6));
    int k = (int)(lo << 2);
    double sn = tab[k], ssn = tab[k + 1];
    double cs = tab[k + 2], ccs = tab[k + 3];
    double cor = (ssn + s * ccs - sn * c) + cs * s;
    return copysign(sn + cor, xold);
}

RT_HD double rt_sc_do_cos(double x, double dx) { return rt_sc_do_cos_t(RT_T(rt_sincostab), x, dx); }
RT_HD double rt_sc_do_sin(double x, double dx) { return rt_sc_do_sin_t(RT_T(rt_sincostab), x, dx); }

RT_HD int rt_sc_reduce(double x, double* a, double* da) {
    double t = (x * RT_SC_HPINV + RT_SC_TOINT);
    double xn = t - RT_SC_TOINT;
    uint32_t lo = (uint32_t)rt_d2u(t);
    double y = (x - xn * RT_SC_MP1) - xn * RT_SC_MP2;
    int n = (int)(lo & 3u);
    double t1 = xn * RT_SC_PP3;
    double t2 = y - t1;
    double db = (y - t2) - t1;
    t1 = xn * RT_SC_PP4;
    double b = t2 - t1;
    db += (t2 - b) - t1;
    *a = b;
    *da = db;
    return n;
}

// Branch-light form of rt_glibc_sincos for SIMD execution: every range of
// s_sincos.c ends in do_sin(a, da) and do_cos(a, da) on a range-specific (a, da),
// followed by a swap / negation / copysign. Computing (a, da) per lane and then
// ONE do_sin and ONE do_cos keeps a wavefront of random angles on a single path
// (the divergent form runs up to three). Same operations on the same operands,
// so the same bits (checked exhaustively against glibc, tests/native/libm_check.cpp).
RT_HD void rt_glibc_sincos_simd_t(const double* tab, double x, double* sinx, double* cosx) {
    const uint32_t k = (uint32_t)(rt_d2u(x) >> 32) & 0x7fffffffu;
    double a = x, da = 0.0;
    int mode;  // 0: small, 1: 0.855..2.426, 2: reduced
    int n = 0;
    if (k < 0x3feb6000u) {
        mode = 0;
    } else if (k < 0x400368fdu) {
        mode = 1;
        const double y = RT_SC_HP0 - fabs(x);
        a = y + RT_SC_HP1;
        da = (y - a) + RT_SC_HP1;
    } else {
        mode = 2;
        n = rt_sc_reduce(x, &a, &da) & 3;
        if (n == 1 || n == 2) { a = -a; da = -da; }
    }
    const double S = rt_sc_do_sin_t(tab, a, da);
    const double C = rt_sc_do_cos_t(tab, a, da);
    double sv, cv;
    if (mode == 0) { sv = S; cv = C; }
    else if (mode == 1) { sv = copysign(C, x); cv = S; }
    else {
        const double Cn = (n & 2) ? -C : C;
        if (n & 1) { cv = S; sv = Cn; } else { sv = S; cv = Cn; }
    }
    if (k < 0x3e400000u) { sv = x; cv = 1.0; }              // |x| < 2^-27
    if (k >= 0x419921fbu) { sv = cv = (x - x) / (x - x); }  // outside the path's domain
    *sinx = sv;
    *cosx = cv;
}

RT_HD void rt_glibc_sincos_simd(double x, double* sinx, double* cosx) {
    rt_glibc_sincos_simd_t(RT_T(rt_sincostab), x, sinx, cosx);
}

// Valid for |x| < 105414350 (the reference only passes angles in [0, 2*pi)).
// Larger finite |x| would need __branred; it returns NaN there so a misuse is loud.
RT_HD void rt_glibc_sincos(double x, double* sinx, double* cosx) {
    uint32_t k = (uint32_t)(rt_d2u(x) >> 32) & 0x7fffffffu;
    if (k < 0x400368fdu) {
        if (k < 0x3e400000u) { *sinx = x; *cosx = 1.0; return; }
        if (k < 0x3feb6000u) { *sinx = rt_sc_do_sin(x, 0); *cosx = rt_sc_do_cos(x, 0); return; }
        double y = RT_SC_HP0 - fabs(x);
        double a = y + RT_SC_HP1;
        double da = (y - a) + RT_SC_HP1;
        *sinx = copysign(rt_sc_do_cos(a, da), x);
        *cosx = rt_sc_do_sin(a, da);
        return;
    }
    if (k < 0x419921fbu) {
        double a, da;
        int n = rt_sc_reduce(x, &a, &da) & 3;
        if (n == 1 || n == 2) { a = -a; da = -da; }
        double* ps = sinx; double* pc = cosx;
        if (n & 1) { double* tmp = pc; pc = ps; ps = tmp; }
        *ps = rt_sc_do_sin(a, da);
        double xx = rt_sc_do_cos(a, da);
        *pc = (n & 2) ? -xx : xx;
        return;
    }
    // inf/nan -> x/x (NaN); huge finite arguments are outside the path's domain
    *sinx = *cosx = (x - x) / (x - x);
}

// ---------------------------------------------------------------------------
// AO hemisphere direction, x = (float)((double)r * cos(a)), y = (float)((double)r * sin(a))
// (RandomUnitVector, Raytracer.cpp:277-278), fast path with an exact fallback.
//
// rt_fast_sincos: Cody-Waite reduction by pi/128 (k <= 256), a table of
// sin/cos(k pi/128) (sct128_table.inc, correctly rounded, tools/gen_sct128.py)
// and short Taylor polynomials of the remainder (|x| <= pi/256: sin to x^5,
// truncation < 1e-17; cos to x^6, < 1e-19), combined by the angle-addition
// formulas. Its distance from glibc's sincos is at most RT_AO_SC_ERR for every
// float angle in [0, 2*pi) (exhaustive: tests/native/libm_check.cpp "aodir").
//
// Only the float rounding of r*cos(a) reaches the output. With r <= 1 and
// E = RT_AO_SC_ERR, the reference's double product X_g and ours X_f differ by at
// most B = E + 2^-53 (one half-ulp of each product). If X_f lies farther than B
// from every float rounding boundary around f = (float)X_f, the reference rounds
// to the same f. Otherwise (rare: |r cos a| tiny) the lane takes glibc's exact
// sincos (rt_glibc_sincos_simd_t).
// ---------------------------------------------------------------------------
#define RT_AO_SC_ERR 0x1p-50

RT_HD void rt_fast_sincos(double a, double* sinx, double* cosx) {
    const double kd = rint(a * 0x1.45f306dc9c883p+5);           // round(a * 128/pi): 0..256 on [0, 2pi]
    double x = fma(-kd, 0x1.921fb54442d18p-6, a);               // a - k*pi/128 (head, one rounding)
    x = fma(-kd, 0x1.1a62633145c07p-60, x);                     // - k*(pi/128 tail); |x| <= pi/256
    const double x2 = x * x;
    const double sx = fma(x * x2, fma(x2, 0x1.1111111111111p-7, -0x1.5555555555555p-3), x);  // sin x to x^5
    const double cm = x2 * fma(fma(x2, -0x1.6c16c16c16c17p-10, 0x1.5555555555555p-5), x2, -0.5);  // cos x - 1 to x^6
    const int k = (int)kd;
    const double S = RT_T(rt_sct128)[2 * k], C = RT_T(rt_sct128)[2 * k + 1];  // sin, cos (k pi/128)
    *sinx = S + fma(C, sx, S * cm);                             // S cos x + C sin x
    *cosx = C + fma(-S, sx, C * cm);                            // C cos x - S sin x
}

// Would RN_float(X_g) equal f = RN_float(X) for every X_g within RT_AO_SC_ERR + 2^-53
// of X? For a normal f = m 2^e (m in [0.5, 1)) the rounding boundaries are
// 2^(e-25) away from f, or 2^(e-26) below a power of two (m = 0.5).
RT_HD bool rt_f32_round_safe(double X, float f) {
    int e;
    (void)frexpf(f, &e);
    const double h = ldexp(1.0, (rt_f2u(f) & 0x7fffffu) ? e - 25 : e - 26);
    return fabs(X - (double)f) + (RT_AO_SC_ERR + 0x1p-53) < h;
}

// r in [0, 1], a in [0, 2*pi); tab = __sincostab for the fallback.
RT_HD void rt_ao_dir_xy(const double* tab, float r, float a, float* xo, float* yo) {
    double sa, ca;
    rt_fast_sincos((double)a, &sa, &ca);
    double X = (double)r * ca, Y = (double)r * sa;
    float fx = (float)X, fy = (float)Y;
    if (!(rt_f32_round_safe(X, fx) && rt_f32_round_safe(Y, fy))) {
        rt_glibc_sincos_simd_t(tab, (double)a, &sa, &ca);
        fx = (float)((double)r * ca);
        fy = (float)((double)r * sa);
    }
    *xo = fx;
    *yo = fy;
}

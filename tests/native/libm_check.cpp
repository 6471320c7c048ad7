// Exhaustive host check: rt_libm.h restatements vs this machine's glibc.
//   libm_check sincos            all float a in [0, 2*pi)   (AO angle domain, Raytracer.cpp:270-278)
//   libm_check powf  y1 y2 ...   all float x in [0, 1.0001] for each exponent y (Raytracer.cpp:253)
//   libm_check powf_random N     N random (x, y) pairs over the whole float range
//   libm_check aodir N           rt_fast_sincos within RT_AO_SC_ERR of glibc for all float a
//                                in [0, 2*pi), then N random AO samples (z, a) through
//                                rt_ao_dir_xy vs the reference's (float)((double)r*cos(a))
// Prints "mismatches=<n> checked=<m>" and the first few mismatches; exit 1 if any.
#include "../../580-raytracer_amd/csrc/rt_libm.h"
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <thread>
#include <vector>
#include <random>

static std::atomic<long> g_bad{0}, g_checked{0};

// RT_STRIDE=k: only the inputs u with u % k == 0 (the quick default of the CPU
// suite; k = 1, the exhaustive run, with RT580_EXHAUSTIVE=1)
static uint64_t stride() {
    const char* e = std::getenv("RT_STRIDE");
    const long k = e ? std::atol(e) : 1;
    return k > 1 ? (uint64_t)k : 1;
}
static std::atomic<int> g_printed{0};

static void report(const char* what, double in1, double in2, double got, double want) {
    if (g_printed.fetch_add(1) < 10)
        std::printf("MISMATCH %s in=(%a, %a) port=%a glibc=%a\n", what, in1, in2, got, want);
}

template <class F>
static void parallel(uint64_t n, F f) {
    unsigned nt = std::thread::hardware_concurrency();
    if (const char* e = std::getenv("RT_THREADS")) nt = (unsigned)std::atoi(e);
    if (nt < 1) nt = 1;
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; t++)
        th.emplace_back([=] {
            uint64_t lo = n * t / nt, hi = n * (t + 1) / nt;
            f(lo, hi);
        });
    for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    if (!std::strcmp(argv[1], "sincos")) {
        uint32_t hi = rt_f2u(6.2831855f);   // first float >= 2*pi (float)
        parallel(hi, [](uint64_t lo, uint64_t hi) {
            long bad = 0;
            for (uint64_t u = lo; u < hi; u++) {
                double a = (double)rt_u2f((uint32_t)u);
                double s0, c0, s1, c1, s2, c2;
                sincos(a, &s0, &c0);
                rt_glibc_sincos(a, &s1, &c1);
                rt_glibc_sincos_simd(a, &s2, &c2);
                if (rt_d2u(s0) != rt_d2u(s1)) { bad++; report("sin", a, 0, s1, s0); }
                if (rt_d2u(c0) != rt_d2u(c1)) { bad++; report("cos", a, 0, c1, c0); }
                if (rt_d2u(s0) != rt_d2u(s2)) { bad++; report("sin_simd", a, 0, s2, s0); }
                if (rt_d2u(c0) != rt_d2u(c2)) { bad++; report("cos_simd", a, 0, c2, c0); }
            }
            g_bad += bad; g_checked += (long)(hi - lo);
        });
    } else if (!std::strcmp(argv[1], "powf")) {
        for (int i = 2; i < argc; i++) {
            float y = std::strtof(argv[i], nullptr);
            uint32_t hi = rt_f2u(1.0001f) + 1;
            parallel(hi, [y](uint64_t lo, uint64_t hi) {
                long bad = 0, n = 0;
                const uint64_t st = stride();
                for (uint64_t u = (lo + st - 1) / st * st; u < hi; u += st, n++) {
                    float x = rt_u2f((uint32_t)u);
                    float r0 = powf(x, y), r1 = rt_glibc_powf(x, y);
                    if (rt_f2u(r0) != rt_f2u(r1)) { bad++; report("powf", x, y, r1, r0); }
                }
                g_bad += bad; g_checked += n;
            });
        }
    } else if (!std::strcmp(argv[1], "powf_random")) {
        uint64_t n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 100000000ull;
        parallel(n, [](uint64_t lo, uint64_t hi) {
            std::mt19937_64 g(lo * 2654435761ull + 580);
            long bad = 0;
            for (uint64_t i = lo; i < hi; i++) {
                uint64_t r = g();
                float x = rt_u2f((uint32_t)r), y = rt_u2f((uint32_t)(r >> 32));
                if (i & 1) y = (float)((int)(r >> 40) % 2000) * 0.5f;   // integer-ish exponents
                if (i & 2) x = rt_u2f((uint32_t)r & 0x3fffffffu);        // x in [0, 2)
                float r0 = powf(x, y), r1 = rt_glibc_powf(x, y);
                bool same = rt_f2u(r0) == rt_f2u(r1) || (r0 != r0 && r1 != r1);
                if (!same) { bad++; report("powf_random", x, y, r1, r0); }
            }
            g_bad += bad; g_checked += (long)(hi - lo);
        });
    } else if (!std::strcmp(argv[1], "aodir")) {
        uint32_t hi = rt_f2u(6.2831855f);
        std::atomic<uint64_t> max_err_bits{0};
        parallel(hi, [&](uint64_t lo, uint64_t hi) {
            long bad = 0;
            double mx = 0;
            for (uint64_t u = lo; u < hi; u++) {
                double a = (double)rt_u2f((uint32_t)u);
                double s0, c0, s1, c1;
                sincos(a, &s0, &c0);
                rt_fast_sincos(a, &s1, &c1);
                double e = fmax(fabs(s0 - s1), fabs(c0 - c1));
                if (!(e <= RT_AO_SC_ERR)) { bad++; report("fast_sincos_err", a, e, s1, s0); }
                if (e > mx) mx = e;
            }
            uint64_t b = rt_d2u(mx), cur = max_err_bits.load();
            while (b > cur && !max_err_bits.compare_exchange_weak(cur, b)) {}
            g_bad += bad; g_checked += (long)(hi - lo);
        });
        std::printf("max_abs_err=%a bound=%a\n", rt_u2d(max_err_bits.load()), RT_AO_SC_ERR);
        uint64_t n = argc > 2 ? std::strtoull(argv[2], nullptr, 10) : 100000000ull;
        std::atomic<long> fallback{0};
        parallel(n, [&](uint64_t lo, uint64_t hi) {
            std::mt19937_64 g(lo * 2654435761ull + 581);
            long bad = 0, fb = 0;
            for (uint64_t i = lo; i < hi; i++) {
                uint64_t w = g();
                // the sampler's values: canonical floats k / 2^31 (Raytracer.cpp:270-276)
                float u0 = (float)(uint32_t)(w & 0x7fffffffu) / 2147483648.0f;
                float u1 = (float)(uint32_t)((w >> 32) & 0x7fffffffu) / 2147483648.0f;
                if (i % 7 == 0) u0 = rt_u2f(rt_f2u(0.5f) + (uint32_t)(w >> 40) % 64) ;  // z near 0
                if (i % 11 == 0) u1 = rt_u2f(rt_f2u(0.25f) + (uint32_t)((w >> 20) % 4096) - 2048);  // a near pi/2
                if (u0 >= 1.0f) u0 = 0.99999994f;
                if (u1 >= 1.0f) u1 = 0.99999994f;
                const float z = u0 * (1.0f - (-1.0f)) + (-1.0f);
                const float ang = u1 * ((float)(2 * 3.14159265) - 0.0f) + 0.0f;
                const float r = sqrtf(1 - z * z);
                double sg, cg;
                sincos((double)ang, &sg, &cg);
                const float x0 = (float)((double)r * cg), y0 = (float)((double)r * sg);
                float x1, y1;
                rt_ao_dir_xy(RT_T(rt_sincostab), r, ang, &x1, &y1);
                double sa, ca;
                rt_fast_sincos((double)ang, &sa, &ca);
                if (!(rt_f32_round_safe((double)r * ca, (float)((double)r * ca)) &&
                      rt_f32_round_safe((double)r * sa, (float)((double)r * sa)))) fb++;
                if (rt_f2u(x0) != rt_f2u(x1) || rt_f2u(y0) != rt_f2u(y1)) { bad++; report("aodir", r, ang, x1, x0); }
            }
            g_bad += bad; g_checked += (long)(hi - lo); fallback += fb;
        });
        std::printf("fallback=%ld of %llu samples\n", fallback.load(), (unsigned long long)n);
    } else {
        return 2;
    }
    std::printf("mismatches=%ld checked=%ld\n", g_bad.load(), g_checked.load());
    return g_bad.load() ? 1 : 0;
}

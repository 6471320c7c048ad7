// Host glibc powf over an array (test helper for tests/test_gpu_libm.py):
// out[i] = powf(x[i], y) with this machine's libm, on `threads` threads.
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

extern "C" void glibc_powf_array(const float* x, float y, float* out, uint64_t n, int threads) {
    float (*volatile pf)(float, float) = ::powf;  // the library call, never folded
    if (threads < 1) threads = 1;
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++)
        th.emplace_back([=] {
            const uint64_t lo = n * t / threads, hi = n * (t + 1) / threads;
            for (uint64_t i = lo; i < hi; i++) out[i] = pf(x[i], y);
        });
    for (auto& x : th) x.join();
}

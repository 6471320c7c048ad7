// rt_oracle CLI (TEST INFRASTRUCTURE ONLY): renders with the CPU restatement.
// usage: rt_oracle <dir containing Assets/> <scene.json> <w> <h> <depth> <out.ppm|->
//                  [--ao N] [--ao-off] [--mt] [--threads T] [--rows a b] [--faithful]
// Prints one JSON line with timing and ray counters on stdout.
#include "rt_oracle.h"
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s <root> <scene> <w> <h> <depth> <out.ppm|-> [--ao N] [--ao-off] [--mt] [--threads T] [--rows a b] [--faithful]\n", argv[0]);
        return 2;
    }
    int w = std::atoi(argv[3]), h = std::atoi(argv[4]), depth = std::atoi(argv[5]);
    int ao = 128, ao_on = 1, engine = 0, threads = 1, r0 = 0, r1 = h;
    for (int i = 7; i < argc; i++) {
        if (!std::strcmp(argv[i], "--ao") && i + 1 < argc) ao = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--ao-off")) ao_on = 0;
        else if (!std::strcmp(argv[i], "--mt")) engine = 1;
        else if (!std::strcmp(argv[i], "--faithful")) oracle_set_mode(1);
        else if (!std::strcmp(argv[i], "--threads") && i + 1 < argc) threads = std::atoi(argv[++i]);
        else if (!std::strcmp(argv[i], "--rows") && i + 2 < argc) { r0 = std::atoi(argv[++i]); r1 = std::atoi(argv[++i]); }
        else { std::fprintf(stderr, "bad arg %s\n", argv[i]); return 2; }
    }
    std::vector<int16_t> fb((size_t)w * (r1 - r0) * 3);
    uint64_t c[6] = {0};
    auto t0 = std::chrono::steady_clock::now();
    int st = oracle_render(argv[1], argv[2], w, h, depth, ao, ao_on, engine, threads, r0, r1, fb.data(), c, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    if (st) return st;
    if (std::strcmp(argv[6], "-") != 0 && oracle_write_ppm(argv[6], w, r1 - r0, fb.data())) return 1;
    double s = std::chrono::duration<double>(t1 - t0).count();
    std::printf("{\"seconds\": %.6f, \"threads\": %d, \"rays_total\": %llu, \"rays_primary\": %llu, "
                "\"rays_secondary\": %llu, \"rays_shadow\": %llu, \"rays_ao\": %llu, \"ao_calls\": %llu, "
                "\"mrays_per_s\": %.4f}\n",
                s, threads, (unsigned long long)c[0], (unsigned long long)c[1], (unsigned long long)c[2],
                (unsigned long long)c[3], (unsigned long long)c[4], (unsigned long long)c[5], c[0] / s / 1e6);
    return 0;
}

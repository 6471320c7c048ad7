// mt19937 block jump-ahead (580-raytracer_amd/csrc/rt_mt.h) against the engine
// itself: the draws from W_J (mt_jump of the seeded window by J) equal
// std::mt19937's draws J, J+1, ... after discard(J), for J around the twist
// boundaries and far out; the block checkpoints equal the direct jumps; a jump
// split in two equals the whole jump (up to 2^33 + 5 draws, where discard
// would take a minute).
//
// usage: mt_check [max_discard]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "../../580-raytracer_amd/csrc/rt_mt.h"

using namespace rt580;

static int check_at(uint64_t J, int n = 1500) {
    std::mt19937 g(5489u);
    g.discard(J);
    const MtWindow w = mt_jump(mt_seed_window(5489u), J);
    std::vector<uint32_t> d((size_t)n);
    mt_draws(w, (uint64_t)n, d.data());
    for (int k = 0; k < n; k++) {
        const uint32_t want = (uint32_t)g();
        if (d[(size_t)k] != want) {
            std::printf("J=%llu draw %d: %08x want %08x\n", (unsigned long long)J, k, d[(size_t)k], want);
            return 1;
        }
    }
    return 0;
}

int main(int argc, char** argv) {
    const uint64_t max_discard = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 200000000ull;
    int bad = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (uint64_t J : {0ull, 1ull, 2ull, 396ull, 397ull, 623ull, 624ull, 625ull, 1247ull, 1248ull, 99991ull,
                       (unsigned long long)kMtBlock, (unsigned long long)kMtBlock + 7, 1000003ull, 123456789ull})
        if (J <= max_discard) bad += check_at(J);
    if (max_discard >= 200000000ull) bad += check_at(max_discard - 3);
    const double t_check = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // checkpoints k kMtBlock against direct jumps, and split jumps far out
    t0 = std::chrono::steady_clock::now();
    std::vector<MtWindow> cpv;
    if (!mt_checkpoints(5489u, 0, 40, cpv)) return 1;
    const MtWindow* cp = cpv.data();
    // a run started far out (one jump to k0), then extended, then a request
    // before it (a new run): the same windows as direct jumps
    std::vector<MtWindow> far_run, ext, back;
    if (!mt_checkpoints(5489u, 5000, 5003, far_run) || !mt_checkpoints(5489u, 5002, 5006, ext) ||
        !mt_checkpoints(5489u, 3, 5, back))
        return 1;
    for (auto [k, w] : {std::pair<uint64_t, const MtWindow*>{5000, &far_run[0]}, {5002, &far_run[2]},
                        {5005, &ext[3]}, {3, &back[0]}, {4, &back[1]}}) {
        const MtWindow d = mt_jump(mt_seed_window(5489u), k * kMtBlock);
        if (std::memcmp(&d, w, sizeof d) != 0) {
            std::printf("checkpoint %llu (cached run) differs from the direct jump\n", (unsigned long long)k);
            bad++;
        }
    }
    const double t_cp = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const MtWindow w0 = mt_seed_window(5489u);
    for (uint64_t k : {0ull, 1ull, 17ull, 39ull}) {
        const MtWindow d = mt_jump(w0, k * kMtBlock);
        if (std::memcmp(&d, &cp[k], sizeof d) != 0) {
            std::printf("checkpoint %llu differs from the direct jump\n", (unsigned long long)k);
            bad++;
        }
    }
    const uint64_t far = (1ull << 33) + 5, part = 987654321ull;
    const MtWindow a = mt_jump(w0, far), b = mt_jump(mt_jump(w0, part), far - part);
    std::vector<uint32_t> da(700), db(700);
    mt_draws(a, 700, da.data());
    mt_draws(b, 700, db.data());
    if (da != db) {
        std::printf("split jump to %llu differs\n", (unsigned long long)far);
        bad++;
    }
    std::printf("mismatches=%d (jumps against discard %.1f s, 40 checkpoints %.2f s)\n", bad, t_check, t_cp);
    return bad != 0;
}

// far_candidate_filter (rt_isect.h, the cell kernels' division-free pair test)
// passes every pair far_candidate passes: random planes, origins and directions
// at the scales of the test scenes, and pairs placed so that num / nd lands at
// T_j within a few ulps.
//
// usage: farcand_check <pairs> [seed]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "../../580-raytracer_amd/csrc/rt_bvh.h"
#include "../../580-raytracer_amd/csrc/rt_isect.h"

using namespace rt580;

int main(int argc, char** argv) {
    const long n = argc > 1 ? std::atol(argv[1]) : 1000000;
    std::mt19937_64 rng(argc > 2 ? std::atoll(argv[2]) : 580);
    std::uniform_real_distribution<float> U(-1.0f, 1.0f);
    long bad = 0, exact = 0, filtered = 0;
    for (long r = 0; r < n; r++) {
        const float sc = std::ldexp(1.0f, (int)(rng() % 24) - 4);
        FarTri ft{};
        rv3 N = v3_normalize(v3(U(rng), U(rng), U(rng)));
        ft.n[0] = N.x; ft.n[1] = N.y; ft.n[2] = N.z;
        const rv3 o = v3(U(rng) * sc, U(rng) * sc, U(rng) * sc);
        const rv3 d = v3_normalize(v3(U(rng), U(rng), U(rng)));
        FarRay fr;
        fr.R = std::fabs(U(rng)) * sc;
        ft.d = U(rng) * 4.0f * sc;
        ft.dhi = fr.R + std::fabs(U(rng)) * 4.0f * sc;
        if (r % 2) {  // put the crossing at T_j (within a few ulps)
            const float T = far_T(fr, ft.dhi), nd = v3_dot(N, d);
            const float t = T * (1.0f + (float)((int)(rng() % 9) - 4) * 0x1p-23f);
            ft.d = -(v3_dot(N, o) + t * nd);
        }
        const bool c = far_candidate(ft, fr, o, d), f = far_candidate_filter(ft, fr, o, d);
        exact += c;
        filtered += f;
        if (c && !f) {
            if (bad < 5) std::printf("pair %ld passes far_candidate only\n", r);
            bad++;
        }
    }
    std::printf("pairs=%ld far_candidate=%ld filter=%ld mismatches=%ld\n", n, exact, filtered, bad);
    return bad ? 1 : 0;
}

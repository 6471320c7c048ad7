// The direction grid's geometry (rt_bvh.cpp build_dir_grid): every direction
// whose device-side cell (rt_isect.h grid_cell, float) lies in a quadtree node
// must be within that node's assumed chord radius of its decoded centre, at
// every level -- else the build prunes a node that holds the direction and the
// grid misses a far hit. Random directions, directions near cell edges and
// the fold (d.z ~ 0), and near the octahedron's vertices.
//
// usage: octgrid_check <directions> [seed]
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
    std::uniform_real_distribution<double> U(-1.0, 1.0);
    const int L = 11;
    long bad = 0;
    double worst = 0;  // largest chord / (half diagonal + 1e-6) seen
    for (long r = 0; r < n; r++) {
        double v[3] = {U(rng), U(rng), U(rng)};
        if (r % 4 == 1) v[2] = std::ldexp(U(rng), -20);            // near the fold
        if (r % 4 == 2) { v[0] = std::ldexp(U(rng), -18); }         // near a map axis
        if (r % 4 == 3) { v[0] = std::ldexp(U(rng), -12); v[1] = std::ldexp(U(rng), -12); }  // near a vertex
        const double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        if (!(l > 0)) continue;
        const rv3 d = v3((float)(v[0] / l), (float)(v[1] / l), (float)(v[2] / l));
        const double dl = std::sqrt((double)d.x * d.x + (double)d.y * d.y + (double)d.z * d.z);
        const double u[3] = {d.x / dl, d.y / dl, d.z / dl};
        const uint32_t cell = grid_cell(d, L);
        const int ci = (int)(cell >> L), cj = (int)(cell & ((1u << L) - 1));
        for (int lev = 1; lev <= L; lev++) {
            double c[3];
            oct_node_centre(lev, ci >> (L - lev), cj >> (L - lev), c);
            const double ch = std::sqrt((c[0] - u[0]) * (c[0] - u[0]) + (c[1] - u[1]) * (c[1] - u[1]) +
                                        (c[2] - u[2]) * (c[2] - u[2]));
            const double rho = oct_node_radius(lev);
            const double hd = std::sqrt(0.5) * 2.0 / (double)(1 << lev) + 1e-6;
            if (ch / hd > worst) worst = ch / hd;
            if (ch > rho && bad++ < 10)
                std::printf("MISMATCH direction (%.9g %.9g %.9g) level %d chord %g radius %g\n", d.x, d.y, d.z, lev, ch,
                            rho);
        }
    }
    std::printf("directions=%ld worst_chord_per_half_diagonal=%.4f radius_factor=%.4f mismatches=%ld\n", n, worst,
                oct_node_radius(1) / (std::sqrt(0.5) + 1e-6), bad);
    return bad ? 1 : 0;
}

// BVH exactness check (CPU): for random rays of every kind the path casts
// (camera, AO-style hemisphere rays from surface points, reflection-style rays,
// and grazing rays nearly parallel to a triangle's plane that provoke the
// reference's far "hits"), the BVH queries of rt_isect.h must return exactly
// what the reference's brute-force IntersectScene loop returns
// (Raytracer.cpp:473-526: every primitive in order, first hit taken, later hits
// only if strictly closer): the same primitive, t and barycentrics bit for bit,
// and the same any-hit boolean.
//
// usage: bvh_check <assets root> <scene.json> <rays> [seed]
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../580-raytracer_amd/csrc/rt_isect.h"
#include "../../580-raytracer_amd/csrc/rt_scene.h"

using namespace rt580;

// The reference's loop with the plain (dividing) tests: tri_test<..., false>.
static bool ref_test(const rt_prim& p, rv3 o, rv3 d, float& t, float& a, float& b, float& g) {
    a = b = g = 0.0f;
    return p.kind == RT_PRIM_TRIANGLE ? tri_test<true, false>(p, o, d, t, a, b, g) : sph_test(p, o, d, t);
}

static bool brute_closest(const std::vector<rt_prim>& P, rv3 o, rv3 d, Hit& h) {
    bool found = false;
    for (int j = 0; j < (int)P.size(); j++) {
        float t, a, b, g;
        if (ref_test(P[j], o, d, t, a, b, g) && (!found || t < h.t)) {
            found = true;
            h.t = t; h.a = a; h.b = b; h.g = g; h.prim = j;
        }
    }
    return found;
}

static bool brute_any(const std::vector<rt_prim>& P, rv3 o, rv3 d) {
    float t, a, b, g;
    for (const rt_prim& p : P)
        if (ref_test(p, o, d, t, a, b, g)) return true;
    return false;
}

static uint32_t fbits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s <root> <scene> <rays> [seed]\n", argv[0]);
        return 2;
    }
    Scene s;
    std::string err;
    if (load_scene_json(argv[1], argv[2], s, err) != RT_SUCCESS) {
        std::fprintf(stderr, "load failed: %s\n", err.c_str());
        return 1;
    }
    PackedScene ps;
    pack_scene(s, ps);
    const std::vector<rt_prim>& P = ps.prims;
    BvhBuild B;
    const bool ok = build_bvh(P.data(), (int)P.size(), B);
    std::printf("prims=%zu tris=%d bvh_ok=%d nodes=%zu depth=%d far_nodes=%zu far_depth=%d brute=%zu S=%g "
                "build_ms=%.1f\n", P.size(), B.n_tri, ok, B.nodes.size(), B.depth, B.far_nodes.size(), B.far_depth,
                B.brute.size(), B.scale, B.build_ms);
    if (!ok) {
        std::printf("mismatches=0 (no BVH for this scene)\n");
        return 0;
    }
    collapse_bvh4(B);
    std::printf("bvh4 nodes=%zu\n", B.nodes4.size());
    BvhView V;
    V.all = P.data();
    V.nodes = B.nodes.data();
    V.nodes4 = B.nodes4q.empty() ? nullptr : B.nodes4q.data();
    V.prims = B.prims.data();
    V.ids = B.ids.data();
    V.far_nodes = B.far_nodes.empty() ? nullptr : B.far_nodes.data();
    V.far_tris = B.far_tris.empty() ? nullptr : B.far_tris.data();
    V.brute = B.brute.data();
    V.n_brute = (int)B.brute.size();
    V.n_far = (int)B.far_tris.size();
    V.has_tree = !B.nodes.empty();
    V.has_far = !B.far_nodes.empty();
    V.scale = B.scale;
    // far search: the direction grid (default) or, with RT_FAR_TREE=1, the plane tree only
    const bool use_grid = !(std::getenv("RT_FAR_TREE") && std::atoi(std::getenv("RT_FAR_TREE")) == 1);
    // the product's rule (rt_shim.cpp rt_gpu_upload_scene): 2048^2 cells
    const int glog2 = std::getenv("RT_GRID_LOG2") ? std::atoi(std::getenv("RT_GRID_LOG2")) : 11;
    if (use_grid) build_dir_grid(P.data(), B, glog2);
    V.grid_start = B.grid_start.empty() ? nullptr : B.grid_start.data();
    V.grid_items = B.grid_items.data();
    V.grid_always = B.grid_always.data();
    if (!B.grid_start.empty()) {  // cell-list lengths (the far passes' per-ray candidate counts)
        std::vector<uint32_t> len(B.grid_start.size() - 1);
        for (size_t c = 0; c + 1 < B.grid_start.size(); c++) len[c] = B.grid_start[c + 1] - B.grid_start[c];
        std::sort(len.begin(), len.end());
        const size_t m = len.size();
        std::printf("grid lists: cells=%zu median=%u p99=%u p99.99=%u max=%u\n", m, len[m / 2], len[m * 99 / 100],
                    len[std::min(m - 1, m * 9999 / 10000)], len[m - 1]);
    }
    V.n_always = (int)B.grid_always.size();
    V.grid_log2 = B.grid_start.empty() ? 0 : B.grid_log2;
    V.grid_r = B.grid_r;
    std::printf("grid log2=%d r=%g items=%zu always=%zu build_ms=%.1f\n", V.grid_log2, V.grid_r, B.grid_items.size(),
                B.grid_always.size(), B.grid_ms);

    const long nrays = std::atol(argv[3]);
    const unsigned seed = argc > 4 ? (unsigned)std::atoi(argv[4]) : 580u;
    const rv3 cam = s.camera.from;
    std::vector<int> tris;
    for (int j = 0; j < (int)P.size(); j++)
        if (P[j].kind == RT_PRIM_TRIANGLE) tris.push_back(j);
    BvhView Vnear = V;  // control: without the far search some results must differ
    Vnear.has_far = 0;
    // the half-resolution grid of row-share frames (coarsen_dir_grid): same answers
    BvhView Vc = V;
    if (use_grid && V.grid_log2 > 1) {
        coarsen_dir_grid(B);
        Vc.grid_start = B.grid2_start.data();
        Vc.grid_items = B.grid2_items.data();
        Vc.grid_log2 = V.grid_log2 - 1;
        std::printf("coarse grid log2=%d items=%zu\n", Vc.grid_log2, B.grid2_items.size());
    }
    std::atomic<long> bad{0}, hits{0}, anyhits{0}, far_closest{0}, near_only_bad{0}, point_checks{0}, bad4{0};
#ifdef RT_BVH_COUNT
    std::atomic<long> cnt[3][6] = {};  // [closest, any, any 4-wide near][counter]
#endif
    const int NT = 8;
    std::vector<std::thread> th;
    for (int tid = 0; tid < NT; tid++)
        th.emplace_back([&, tid] {
            std::mt19937 rng(seed * 7919u + tid);
            std::uniform_real_distribution<float> U(0.0f, 1.0f);
            for (long r = tid; r < nrays; r += NT) {
                const int kind = (int)(r % 4);
                rv3 o, d;
                const rt_prim& T = P[tris[rng() % tris.size()]];
                float u = U(rng), v = U(rng);
                if (u + v > 1) { u = 1 - u; v = 1 - v; }
                const rv3 p0 = ld3(T.p0), p1 = ld3(T.p1), p2 = ld3(T.p2), N = ld3(T.nrm);
                const rv3 sp = v3_add(p0, v3_add(v3_scale(v3_sub(p1, p0), u), v3_scale(v3_sub(p2, p0), v)));
                if (kind == 0) {  // camera ray towards a surface point (jittered)
                    o = cam;
                    d = v3_normalize(v3_sub(v3_add(sp, v3((U(rng) - 0.5f), (U(rng) - 0.5f), (U(rng) - 0.5f))), cam));
                } else if (kind == 1 || kind == 2) {  // AO / reflection style: hemisphere from a surface point
                    const float z = U(rng) * 2 - 1, a = U(rng) * 6.2831853f, rr = std::sqrt(1 - z * z);
                    d = v3_normalize(v3(rr * std::cos(a), rr * std::sin(a), z));
                    if (!(v3_dot(d, N) > 0.0f)) d = v3_neg(d);
                    o = v3_add(sp, v3_scale(d, 0.2f));
                    d = v3_normalize(d);
                } else {  // grazing: nearly parallel to some triangle's plane (provokes far hits)
                    const rt_prim& G = P[tris[rng() % tris.size()]];
                    const rv3 n = ld3(G.nrm);
                    rv3 w = v3_normalize(v3_cross(n, v3(U(rng) - 0.5f, U(rng) - 0.5f, U(rng) - 0.5f)));
                    const float eps = std::ldexp(1.0f, -(int)(rng() % 22)) * (U(rng) - 0.5f);
                    d = v3_normalize(v3_add(w, v3_scale(n, eps)));
                    o = v3_add(sp, v3_scale(ld3(T.nrm), 0.2f));
                }
                Hit hb, hv;
                const bool cb = brute_closest(P, o, d, hb);
#ifdef RT_BVH_COUNT
                g_bvh_cnt = BvhCounters{};
#endif
                const bool cv = bvh_closest(V, o, d, hv);
#ifdef RT_BVH_COUNT
                {
                    const long* c = &g_bvh_cnt.nodes;
                    for (int q = 0; q < 6; q++) cnt[0][q] += c[q];
                    g_bvh_cnt = BvhCounters{};
                }
#endif
                const bool ab = brute_any(P, o, d);
                const bool av = bvh_any(V, o, d);
#ifdef RT_BVH_COUNT
                if (kind == 1 || kind == 2) {
                    const long* c = &g_bvh_cnt.nodes;
                    for (int q = 0; q < 6; q++) cnt[1][q] += c[q];
                }
#endif
                // point-light shadow form (Raytracer.cpp:75): occluded iff the
                // closest hit has !(t > dist); near query with the t bound, valid
                // when dist is below every far threshold (rt_kernels.hip PHASE 3)
                bool point_ok = true;
                if (V.has_far) {
                    const float dist = std::ldexp(U(rng), (int)(rng() % 6)) ;  // (0, 32)
                    const float Troot = far_T(far_ray(V, o), B.far_nodes[0].min_dhi);
                    if (dist < Troot) {
                        const bool want = cb && !(hb.t > dist);
                        point_ok = bvh_any(V, o, d, /*with_far=*/false, dist) == want;
                        point_checks++;
                    }
                }
                // the 4-wide near query answers exactly as the binary one (with and without a t bound)
                if (V.nodes4) {
#ifdef RT_BVH_COUNT
                    g_bvh_cnt = BvhCounters{};
#endif
                    const bool a2 = bvh_any(V, o, d, false), a4 = bvh4_any_near(V, o, d);
#ifdef RT_BVH_COUNT
                    if (kind == 1 || kind == 2) {
                        const long* c = &g_bvh_cnt.nodes;
                        for (int q = 0; q < 6; q++) cnt[2][q] += c[q];
                    }
#endif
                    const float tb = std::ldexp(U(rng), (int)(rng() % 6));
                    if (a2 != a4 || bvh_any(V, o, d, false, tb) != bvh4_any_near(V, o, d, tb)) {
                        if (bad4.fetch_add(1) < 10) std::printf("MISMATCH4 ray %ld kind %d: binary %d 4-wide %d\n", r, kind, a2, a4);
                    }
                    // ao_trace_kernel's step budget: a decided answer equals the full query's
                    for (int budget : {1, 2, 4, 8}) {
                        uint32_t sa[RT_BVH_STACK + 4];
                        const int q = bvh4_any_near_budget(V, o, d, ArrStack{sa}, budget);
                        if (q >= 0 && (q == 1) != a4 && bad4.fetch_add(1) < 10)
                            std::printf("MISMATCH4 budget %d ray %ld kind %d: %d vs %d\n", budget, r, kind, q, a4);
                    }
                    // ... and an undecided walk resumed from its saved state (ao_late_kernel)
                    for (int budget : {1, 2, 4, 8}) {
                        uint32_t sa[RT_BVH_STACK + 4];
                        int sp;
                        int32_t c, n;
                        const int q = bvh4_any_near_budget_state(V, o, d, ArrStack{sa}, budget, sp, c, n);
                        int q2 = q;
                        if (q < 0) q2 = bvh4_any_near_resume_budget(V, o, d, ArrStack{sa}, 2 * budget, sp, c, n);
                        const bool res = q2 < 0 ? bvh4_any_near_resume(V, o, d, ArrStack{sa}, sp, c, n) : q2 == 1;
                        if (res != a4 && bad4.fetch_add(1) < 10)
                            std::printf("MISMATCH4 resume budget %d ray %ld kind %d: %d vs %d\n", budget, r, kind, res, a4);
                    }
                    Hit h2, h4;
                    const bool c2 = bvh_closest(V, o, d, h2, false), c4 = bvh4_closest_near(V, o, d, h4);
                    if (c2 != c4 || (c2 && (h2.prim != h4.prim || fbits(h2.t) != fbits(h4.t) || fbits(h2.a) != fbits(h4.a) ||
                                            fbits(h2.b) != fbits(h4.b) || fbits(h2.g) != fbits(h4.g)))) {
                        if (bad4.fetch_add(1) < 10)
                            std::printf("MISMATCH4 closest ray %ld kind %d: binary (%d, %d) 4-wide (%d, %d)\n", r, kind, c2,
                                        c2 ? h2.prim : -1, c4, c4 ? h4.prim : -1);
                    }
                }
                bool same = cb == cv && ab == av && point_ok;
                if (same && cb)
                    same = hb.prim == hv.prim && fbits(hb.t) == fbits(hv.t) && fbits(hb.a) == fbits(hv.a) &&
                           fbits(hb.b) == fbits(hv.b) && fbits(hb.g) == fbits(hv.g);
                if (Vc.grid_log2 != V.grid_log2) {
                    Hit hc;
                    const bool cc = bvh_closest(Vc, o, d, hc), ac = bvh_any(Vc, o, d);
                    if (cc != cv || ac != av ||
                        (cc && (hc.prim != hv.prim || fbits(hc.t) != fbits(hv.t) || fbits(hc.a) != fbits(hv.a) ||
                                fbits(hc.b) != fbits(hv.b) || fbits(hc.g) != fbits(hv.g))))
                        same = false;
                }
                {
                    Hit hn;
                    const bool cn = bvh_closest(Vnear, o, d, hn);
                    const bool an = bvh_any(Vnear, o, d);
                    if (cn != cb || an != ab || (cb && (hn.prim != hb.prim || fbits(hn.t) != fbits(hb.t))))
                        near_only_bad++;
                }
                if (cb) hits++;
                if (ab) anyhits++;
                if (cb && hb.t > 1e5f) far_closest++;
                if (!same) {
                    if (bad.fetch_add(1) < 10)
                        std::printf("MISMATCH ray %ld kind %d: brute (%d, prim %d, t %.9g) bvh (%d, prim %d, t %.9g) "
                                    "any %d/%d\n", r, kind, cb, cb ? hb.prim : -1, cb ? hb.t : 0.0f, cv,
                                    cv ? hv.prim : -1, cv ? hv.t : 0.0f, ab, av);
                }
            }
        });
    for (auto& t : th) t.join();
#ifdef RT_BVH_COUNT
    const char* names[6] = {"nodes", "leaf_tris", "far_nodes", "far_cands", "far_tests", "brute_tests"};
    for (int w = 0; w < 3; w++) {
        std::printf("%s per ray:", w == 2 ? "any-hit near 4-wide (AO-style rays)"
                                          : (w ? "any-hit (AO-style rays)" : "closest (all rays)"));
        const double div = w ? nrays / 2.0 : (double)nrays;
        for (int q = 0; q < 6; q++) std::printf(" %s=%.1f", names[q], cnt[w][q] / div);
        std::printf("\n");
    }
#endif
    std::printf("rays=%ld closest_hits=%ld any_hits=%ld far_closest_hits=%ld differ_without_far_search=%ld "
                "point_shadow_checks=%ld mismatches=%ld bvh4_mismatches=%ld\n", nrays, (long)hits, (long)anyhits, (long)far_closest,
                (long)near_only_bad, (long)point_checks, (long)bad, (long)bad4);
    return (bad || bad4) ? 1 : 0;
}

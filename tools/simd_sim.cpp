// SIMD-efficiency model of the AO any-hit traversal (development tool).
//
// Casts AO-style rays in waves of 64 as the GPU forms them (one hit point per
// wave, 64 cosine-free hemisphere directions, like ao_body's items of one
// call) through the 4-wide traversal of rt_isect.h, records each lane's steps
// (a step = inner-node iterations down to a leaf, then the leaf's triangle
// tests), and prices a wave as lock-step execution of the while-while loop:
// per outer iteration, max node iterations + max leaf tests over the lanes
// still running. Prints the lane-average work and the wave cost, so
// efficiency = average / cost.
//
// usage: simd_sim <assets root> <scene.json> <waves> [seed]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../580-raytracer_amd/csrc/rt_isect.h"
#include "../580-raytracer_amd/csrc/rt_scene.h"

using namespace rt580;

struct Step {
    int nodes, tris;
};

// bvh4_any_near with the steps recorded
static bool trace(const BvhView& V, rv3 o, rv3 d, std::vector<Step>& steps) {
    steps.clear();
    if (dir_zero(d)) return false;
    const SlabRay sr = slab_ray(V, o, d);
    uint32_t stk[RT_BVH_STACK + 4];
    int sp = 0;
    int32_t c = 0, n = 0;
    for (;;) {
        Step s{0, 0};
        // descend, counting iterations
        bool leaf = true;
        while (n == 0) {
            s.nodes++;
            int sp0 = sp;
            int32_t c0 = c, n0 = n;
            // one node iteration of bvh4_descend
            Node4 nd;
            load_node4(V.nodes4 + c0, nd);
            float t[4];
            bool ok[4];
            for (int j = 0; j < 4; j++) {
                const float lo[3] = {nd.lo[0][j], nd.lo[1][j], nd.lo[2][j]};
                const float hi[3] = {nd.hi[0][j], nd.hi[1][j], nd.hi[2][j]};
                const bool in = slab(lo, hi, sr, t[j]);
                ok[j] = (nd.link[j] != 0xffffffffu) & in;
            }
            int best = -1;
            float bt = INFINITY;
            for (int j = 0; j < 4; j++)
                if (ok[j] && (best < 0 || t[j] < bt)) { best = j; bt = t[j]; }
            for (int j = 0; j < 4; j++) {
                stk[sp] = nd.link[j];
                sp += (ok[j] && j != best) ? 1 : 0;
            }
            (void)sp0; (void)n0;
            if (best >= 0) { c = (int32_t)(nd.link[best] & 0x7ffffffu); n = (int32_t)(nd.link[best] >> 27); }
            else if (!bvh4_pop(ArrStack{stk}, sp, c, n)) { leaf = false; break; }
        }
        if (!leaf) { steps.push_back(s); return false; }
        bool hit = false;
        for (int k = c; k < c + n && !hit; k++) {
            s.tris++;
            float tt, a, b, g;
            hit = tri_test<false, true>(V.prims[k], o, d, tt, a, b, g);
        }
        steps.push_back(s);
        if (hit) return true;
        if (!bvh4_pop(ArrStack{stk}, sp, c, n)) return false;
    }
}

int main(int argc, char** argv) {
    if (argc < 4) { std::fprintf(stderr, "usage: %s <root> <scene> <waves> [seed]\n", argv[0]); return 2; }
    Scene s;
    std::string err;
    if (load_scene_json(argv[1], argv[2], s, err) != RT_SUCCESS) { std::fprintf(stderr, "%s\n", err.c_str()); return 1; }
    PackedScene ps;
    pack_scene(s, ps);
    const std::vector<rt_prim>& P = ps.prims;
    BvhBuild B;
    if (!build_bvh(P.data(), (int)P.size(), B)) { std::printf("no bvh\n"); return 0; }
    collapse_bvh4(B);
    BvhView V{};
    V.all = P.data(); V.nodes = B.nodes.data(); V.nodes4 = B.nodes4q.data(); V.prims = B.prims.data();
    V.ids = B.ids.data(); V.has_tree = 1; V.scale = B.scale;
    const long waves = std::atol(argv[3]);
    std::mt19937 rng(argc > 4 ? std::atoi(argv[4]) : 580);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    std::vector<int> tris;
    for (int j = 0; j < (int)P.size(); j++) if (P[j].kind == RT_PRIM_TRIANGLE) tris.push_back(j);
    double lane_nodes = 0, lane_tris = 0, wave_nodes = 0, wave_tris = 0, lane_steps = 0, wave_steps = 0, hits = 0;
    std::vector<std::vector<Step>> lanes(64);
    for (long w = 0; w < waves; w++) {
        const rt_prim& T = P[tris[rng() % tris.size()]];
        float u = U(rng), v = U(rng);
        if (u + v > 1) { u = 1 - u; v = 1 - v; }
        const rv3 p0 = ld3(T.p0), p1 = ld3(T.p1), p2 = ld3(T.p2), N = v3_normalize(ld3(T.nrm));
        const rv3 hp = v3_add(p0, v3_add(v3_scale(v3_sub(p1, p0), u), v3_scale(v3_sub(p2, p0), v)));
        size_t maxs = 0;
        for (int l = 0; l < 64; l++) {
            const float z = U(rng) * 2 - 1, a = U(rng) * 6.2831853f, r = std::sqrt(1 - z * z);
            rv3 d = v3_normalize(v3(r * std::cos(a), r * std::sin(a), z));
            if (!(v3_dot(d, N) > 0.0f)) d = v3_neg(d);
            const rv3 o = v3_add(hp, v3_scale(d, 0.2f));
            hits += trace(V, o, d, lanes[l]);
            for (const Step& st : lanes[l]) { lane_nodes += st.nodes; lane_tris += st.tris; }
            lane_steps += lanes[l].size();
            maxs = std::max(maxs, lanes[l].size());
        }
        for (size_t i = 0; i < maxs; i++) {
            int mn = 0, mt = 0;
            for (int l = 0; l < 64; l++)
                if (i < lanes[l].size()) { mn = std::max(mn, lanes[l][i].nodes); mt = std::max(mt, lanes[l][i].tris); }
            wave_nodes += mn;
            wave_tris += mt;
        }
        wave_steps += maxs;
    }
    // persistent waves with refill (ao_trace_persist_kernel): a stream of the
    // same rays (wave-major order), lanes refilled once >= refill are idle
    for (int refill : {1, 8, 16, 32, 64}) {
        std::mt19937 r2(argc > 4 ? std::atoi(argv[4]) : 580);
        // regenerate the same rays' step lists, in order
        std::vector<std::vector<Step>> all;
        all.reserve(waves * 64);
        for (long w = 0; w < waves; w++) {
            const rt_prim& T = P[tris[r2() % tris.size()]];
            float u = U(r2), v = U(r2);
            if (u + v > 1) { u = 1 - u; v = 1 - v; }
            const rv3 p0 = ld3(T.p0), p1 = ld3(T.p1), p2 = ld3(T.p2), N = v3_normalize(ld3(T.nrm));
            const rv3 hp = v3_add(p0, v3_add(v3_scale(v3_sub(p1, p0), u), v3_scale(v3_sub(p2, p0), v)));
            for (int l = 0; l < 64; l++) {
                const float z = U(r2) * 2 - 1, a = U(r2) * 6.2831853f, r = std::sqrt(1 - z * z);
                rv3 d = v3_normalize(v3(r * std::cos(a), r * std::sin(a), z));
                if (!(v3_dot(d, N) > 0.0f)) d = v3_neg(d);
                const rv3 o = v3_add(hp, v3_scale(d, 0.2f));
                std::vector<Step> st;
                trace(V, o, d, st);
                all.push_back(st);
            }
        }
        // one wave consumes the stream
        size_t next = 0;
        std::vector<int> ray(64, -1);
        std::vector<size_t> pos(64, 0);
        double cn = 0, ct = 0, iters = 0, refills = 0;
        for (;;) {
            int idle = 0;
            for (int l = 0; l < 64; l++) idle += ray[l] < 0;
            if (next < all.size() && (idle == 64 || idle >= refill)) {
                refills++;
                for (int l = 0; l < 64; l++)
                    if (ray[l] < 0 && next < all.size()) { ray[l] = (int)next++; pos[l] = 0; }
            }
            int mn = 0, mt = 0, act = 0;
            for (int l = 0; l < 64; l++) {
                if (ray[l] < 0) continue;
                act++;
                const Step& st = all[ray[l]][pos[l]];
                mn = std::max(mn, st.nodes);
                mt = std::max(mt, st.tris);
                if (++pos[l] == all[ray[l]].size()) ray[l] = -1;
            }
            if (!act) break;
            cn += mn; ct += mt; iters++;
        }
        std::printf("persistent refill=%d: node eff=%.3f tri eff=%.3f iterations=%.0f refills=%.0f\n", refill,
                    lane_nodes / 64.0 / cn, lane_tris / 64.0 / ct, iters, refills);
    }
    // block-local direction sort: B calls of nearby hit points (one triangle,
    // jittered points), their B*64 rays ordered by octahedral direction cell
    // (2^L x 2^L), then cut into waves of 64 (lock-step cost as above)
    for (int Bc : {4, 16}) {
        for (int L : {1, 2, 3}) {
            std::mt19937 r3(7);
            double cn = 0, ct = 0, ln = 0, lt = 0;
            long nw = 0;
            for (long blk = 0; blk < waves / Bc; blk++) {
                const rt_prim& T = P[tris[r3() % tris.size()]];
                const rv3 p0 = ld3(T.p0), p1 = ld3(T.p1), p2 = ld3(T.p2), N = v3_normalize(ld3(T.nrm));
                std::vector<std::pair<uint32_t, std::vector<Step>>> rays;
                for (int cidx = 0; cidx < Bc; cidx++) {
                    float u = U(r3), v = U(r3);
                    if (u + v > 1) { u = 1 - u; v = 1 - v; }
                    const rv3 hp = v3_add(p0, v3_add(v3_scale(v3_sub(p1, p0), u), v3_scale(v3_sub(p2, p0), v)));
                    for (int l = 0; l < 64; l++) {
                        const float z = U(r3) * 2 - 1, a = U(r3) * 6.2831853f, r = std::sqrt(1 - z * z);
                        rv3 d = v3_normalize(v3(r * std::cos(a), r * std::sin(a), z));
                        if (!(v3_dot(d, N) > 0.0f)) d = v3_neg(d);
                        const rv3 o = v3_add(hp, v3_scale(d, 0.2f));
                        std::vector<Step> st;
                        trace(V, o, d, st);
                        for (const Step& x : st) { ln += x.nodes; lt += x.tris; }
                        rays.push_back({grid_cell(d, L), st});
                    }
                }
                std::stable_sort(rays.begin(), rays.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
                for (size_t w0 = 0; w0 < rays.size(); w0 += 64) {
                    size_t maxs = 0;
                    for (size_t l = w0; l < w0 + 64; l++) maxs = std::max(maxs, rays[l].second.size());
                    for (size_t i = 0; i < maxs; i++) {
                        int mn = 0, mt = 0;
                        for (size_t l = w0; l < w0 + 64; l++)
                            if (i < rays[l].second.size()) {
                                mn = std::max(mn, rays[l].second[i].nodes);
                                mt = std::max(mt, rays[l].second[i].tris);
                            }
                        cn += mn; ct += mt;
                    }
                    nw++;
                }
            }
            std::printf("block sort B=%d L=%d: node eff=%.3f tri eff=%.3f (wave nodes %.1f tris %.1f)\n", Bc, L,
                        ln / 64.0 / cn, lt / 64.0 / ct, cn / nw, ct / nw);
        }
    }
    // step budget K, then compaction: lanes run at most K steps in the first
    // pass; the unfinished rays (queued in order) run in a second pass, either
    // resumed (stack saved) or restarted from the root (redo their K steps)
    for (int K : {4, 8, 16, 32}) {
        std::mt19937 r4(argc > 4 ? std::atoi(argv[4]) : 580);
        std::vector<std::vector<Step>> all;
        all.reserve(waves * 64);
        for (long w = 0; w < waves; w++) {
            const rt_prim& T = P[tris[r4() % tris.size()]];
            float u = U(r4), v = U(r4);
            if (u + v > 1) { u = 1 - u; v = 1 - v; }
            const rv3 p0 = ld3(T.p0), p1 = ld3(T.p1), p2 = ld3(T.p2), N = v3_normalize(ld3(T.nrm));
            const rv3 hp = v3_add(p0, v3_add(v3_scale(v3_sub(p1, p0), u), v3_scale(v3_sub(p2, p0), v)));
            for (int l = 0; l < 64; l++) {
                const float z = U(r4) * 2 - 1, a = U(r4) * 6.2831853f, r = std::sqrt(1 - z * z);
                rv3 d = v3_normalize(v3(r * std::cos(a), r * std::sin(a), z));
                if (!(v3_dot(d, N) > 0.0f)) d = v3_neg(d);
                const rv3 o = v3_add(hp, v3_scale(d, 0.2f));
                std::vector<Step> st;
                trace(V, o, d, st);
                all.push_back(st);
            }
        }
        auto wave_cost = [&](const std::vector<const std::vector<Step>*>& ws, size_t from, size_t lim, double& cn,
                             double& ct) {
            size_t maxs = 0;
            for (auto* x : ws) maxs = std::max(maxs, std::min(x->size(), lim));
            for (size_t i = from; i < maxs; i++) {
                int mn = 0, mt = 0;
                for (auto* x : ws)
                    if (i < x->size() && i < lim) { mn = std::max(mn, (*x)[i].nodes); mt = std::max(mt, (*x)[i].tris); }
                cn += mn; ct += mt;
            }
        };
        double c1n = 0, c1t = 0, cRn = 0, cRt = 0, cSn = 0, cSt = 0, base_n = 0, base_t = 0;
        std::vector<const std::vector<Step>*> late;
        for (size_t w0 = 0; w0 < all.size(); w0 += 64) {
            std::vector<const std::vector<Step>*> ws;
            for (size_t l = w0; l < w0 + 64; l++) ws.push_back(&all[l]);
            wave_cost(ws, 0, (size_t)-1, base_n, base_t);
            wave_cost(ws, 0, (size_t)K, c1n, c1t);
            for (auto* x : ws) if (x->size() > (size_t)K) late.push_back(x);
        }
        for (size_t w0 = 0; w0 < late.size(); w0 += 64) {
            std::vector<const std::vector<Step>*> ws(late.begin() + w0, late.begin() + std::min(late.size(), w0 + 64));
            wave_cost(ws, 0, (size_t)-1, cRn, cRt);        // restart: all steps again
            wave_cost(ws, (size_t)K, (size_t)-1, cSn, cSt); // resume: steps K..
        }
        std::printf("budget K=%d: late rays %.3f | lock-step nodes+tris: base %.0f, resume %.0f (%.3f), restart %.0f (%.3f)\n",
                    K, late.size() / (double)all.size(), base_n + base_t, c1n + c1t + cSn + cSt,
                    (c1n + c1t + cSn + cSt) / (base_n + base_t), c1n + c1t + cRn + cRt,
                    (c1n + c1t + cRn + cRt) / (base_n + base_t));
    }
    // Speculative while-while (postponed leaves): a lane that reaches a leaf
    // while others still descend keeps it and goes on descending from its stack,
    // so the wave's idle node iterations advance its next leaf; the leaf phase
    // then tests the postponed leaf (and the current entry, if it is a leaf too).
    // Lane op sequences: 0 = a node iteration, k > 0 = a leaf of k tests (the
    // last op when it hits). Lock-step cost = node iterations + test iterations
    // (per iteration, the slowest lane), with and without a leaf budget K.
    {
        std::mt19937 r5(argc > 4 ? std::atoi(argv[4]) : 580);
        std::vector<std::vector<int>> ops;
        ops.reserve(waves * 64);
        for (long w = 0; w < waves; w++) {
            const rt_prim& T = P[tris[r5() % tris.size()]];
            float u = U(r5), v = U(r5);
            if (u + v > 1) { u = 1 - u; v = 1 - v; }
            const rv3 p0 = ld3(T.p0), p1 = ld3(T.p1), p2 = ld3(T.p2), N = v3_normalize(ld3(T.nrm));
            const rv3 hp = v3_add(p0, v3_add(v3_scale(v3_sub(p1, p0), u), v3_scale(v3_sub(p2, p0), v)));
            for (int l = 0; l < 64; l++) {
                const float z = U(r5) * 2 - 1, a = U(r5) * 6.2831853f, r = std::sqrt(1 - z * z);
                rv3 d = v3_normalize(v3(r * std::cos(a), r * std::sin(a), z));
                if (!(v3_dot(d, N) > 0.0f)) d = v3_neg(d);
                const rv3 o = v3_add(hp, v3_scale(d, 0.2f));
                std::vector<Step> st;
                trace(V, o, d, st);
                std::vector<int> q;
                for (const Step& x : st) {
                    for (int k = 0; k < x.nodes; k++) q.push_back(0);
                    if (x.tris) q.push_back(x.tris);
                }
                ops.push_back(q);
            }
        }
        for (int K : {1 << 30, 4}) {
            double an = 0, at = 0, bn = 0, bt = 0, spec_nodes = 0;
            for (size_t w0 = 0; w0 < ops.size(); w0 += 64) {
                // (A) while-while
                {
                    std::vector<size_t> pos(64, 0);
                    std::vector<int> leaves(64, 0);
                    for (;;) {
                        bool any = false;
                        for (int l = 0; l < 64; l++) any |= pos[l] < ops[w0 + l].size() && leaves[l] < K;
                        if (!any) break;
                        int mn = 0, mt = 0;
                        for (int l = 0; l < 64; l++) {
                            const std::vector<int>& q = ops[w0 + l];
                            if (leaves[l] >= K) continue;
                            int c = 0;
                            while (pos[l] < q.size() && q[pos[l]] == 0) { pos[l]++; c++; }
                            mn = std::max(mn, c);
                        }
                        for (int l = 0; l < 64; l++) {
                            const std::vector<int>& q = ops[w0 + l];
                            if (leaves[l] >= K || pos[l] >= q.size()) continue;
                            mt = std::max(mt, q[pos[l]]);
                            pos[l]++;
                            leaves[l]++;
                        }
                        an += mn;
                        at += mt;
                    }
                }
                // (B) speculative
                {
                    std::vector<size_t> pos(64, 0);
                    std::vector<int> post(64, 0), leaves(64, 0);
                    auto live = [&](int l) { return leaves[l] < K && (post[l] > 0 || pos[l] < ops[w0 + l].size()); };
                    for (;;) {
                        bool any = false;
                        for (int l = 0; l < 64; l++) any |= live(l);
                        if (!any) break;
                        // postpone leading leaves
                        for (int l = 0; l < 64; l++) {
                            const std::vector<int>& q = ops[w0 + l];
                            if (live(l) && !post[l] && pos[l] < q.size() && q[pos[l]] > 0) post[l] = q[pos[l]++];
                        }
                        for (;;) {  // node iterations until every live lane holds a leaf
                            bool need = false;
                            for (int l = 0; l < 64; l++) need |= live(l) && !post[l];
                            if (!need) break;
                            for (int l = 0; l < 64; l++) {
                                const std::vector<int>& q = ops[w0 + l];
                                if (!live(l) || pos[l] >= q.size() || q[pos[l]] > 0) continue;
                                pos[l]++;
                                if (post[l]) spec_nodes++;
                                if (!post[l] && pos[l] < q.size() && q[pos[l]] > 0) post[l] = q[pos[l]++];
                            }
                            bn++;
                        }
                        int mt = 0;
                        for (int l = 0; l < 64; l++) {
                            if (!live(l) || !post[l]) continue;
                            const std::vector<int>& q = ops[w0 + l];
                            int t = post[l];
                            post[l] = 0;
                            leaves[l]++;
                            if (leaves[l] < K && pos[l] < q.size() && q[pos[l]] > 0) {  // the current entry is a leaf too
                                t += q[pos[l]++];
                                leaves[l]++;
                            }
                            mt = std::max(mt, t);
                        }
                        bt += mt;
                    }
                }
            }
            // (C) speculative with up to two held leaves: the node phase ends
            // when every live lane holds at least one; the leaf phase tests the
            // held ones in order (stopping at a hit) and the current entry if a leaf
            double cn2 = 0, ct2 = 0;
            for (size_t w0 = 0; w0 < ops.size(); w0 += 64) {
                std::vector<size_t> pos(64, 0);
                std::vector<std::vector<int>> held(64);
                std::vector<int> leaves(64, 0);
                std::vector<bool> done(64, false);
                auto live = [&](int l) { return !done[l] && leaves[l] < K && (!held[l].empty() || pos[l] < ops[w0 + l].size()); };
                for (;;) {
                    bool any = false;
                    for (int l = 0; l < 64; l++) any |= live(l);
                    if (!any) break;
                    for (int l = 0; l < 64; l++) {
                        const std::vector<int>& q = ops[w0 + l];
                        while (live(l) && held[l].size() < 2 && pos[l] < q.size() && q[pos[l]] > 0) held[l].push_back(q[pos[l]++]);
                    }
                    for (;;) {
                        bool need = false;
                        for (int l = 0; l < 64; l++) need |= live(l) && held[l].empty();
                        if (!need) break;
                        for (int l = 0; l < 64; l++) {
                            const std::vector<int>& q = ops[w0 + l];
                            if (!live(l) || pos[l] >= q.size() || q[pos[l]] > 0) continue;
                            pos[l]++;
                            while (held[l].size() < 2 && pos[l] < q.size() && q[pos[l]] > 0) held[l].push_back(q[pos[l]++]);
                        }
                        cn2++;
                    }
                    int mt = 0;
                    for (int l = 0; l < 64; l++) {
                        if (!live(l)) continue;
                        const std::vector<int>& q = ops[w0 + l];
                        int t = 0;
                        for (size_t h = 0; h < held[l].size() && leaves[l] < K; h++) {
                            t += held[l][h];
                            leaves[l]++;
                        }
                        held[l].clear();
                        // a hit ends the lane's sequence: its ops are exhausted once the held leaves were the last
                        if (pos[l] >= q.size()) done[l] = true;
                        mt = std::max(mt, t);
                    }
                    ct2 += mt;
                }
            }
            const double nw = ops.size() / 64.0;
            std::printf("while-while%s: nodes %.1f tests %.1f per wave | speculative: nodes %.1f tests %.1f "
                        "(speculative node steps per lane %.2f) | two held: nodes %.1f tests %.1f\n",
                        K < (1 << 30) ? " budget 4" : "", an / nw, at / nw, bn / nw, bt / nw, spec_nodes / ops.size(),
                        cn2 / nw, ct2 / nw);
        }
    }
    const double R = waves * 64.0;
    std::printf("rays=%.0f hit=%.3f per ray: nodes=%.2f tris=%.2f steps=%.2f | per wave (lock-step): nodes=%.1f tris=%.1f "
                "steps=%.1f | node eff=%.3f tri eff=%.3f\n", R, hits / R, lane_nodes / R, lane_tris / R, lane_steps / R,
                wave_nodes / waves, wave_tris / waves, wave_steps / waves, lane_nodes / 64.0 / wave_nodes,
                lane_tris / 64.0 / wave_tris);
    return 0;
}

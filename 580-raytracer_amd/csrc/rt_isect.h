// rt_isect.h — per-primitive tests and the exact-semantics BVH queries,
// compiled for the device (rt_kernels.hip) and the host (tests/native BVH
// checker). Requires -ffp-contract=off like everything else.
//
//   tri_test      IntersectTriangle (Raytracer.cpp:348-409), ray-invariant part
//                 precomputed on the host (rt_scene.cpp)
//   sph_test      IntersectSphere (Raytracer.cpp:419-464)
//   bvh_closest   IntersectScene closest hit (Raytracer.cpp:473-526)
//   bvh_any       IntersectScene where only the boolean is read
// See rt_bvh.h for why the culling below never changes a result.
#pragma once
#include <stdint.h>

#include "../../include/rt580.h"
#include "rt_bvh.h"
#include "rt_math.h"

namespace rt580 {

struct Hit {
    float t, a, b, g;
    int prim;
};

RTM_HD rv3 ld3(const float* p) { return v3(p[0], p[1], p[2]); }

// (num / den) < 0 exactly as the division would decide it, without dividing.
// With opposite signs the quotient is negative unless |num/den| rounds to -0,
// i.e. |num| / |den| <= 2^-150 (half the least denormal; the tie rounds to 0):
// so test |num| * 2^150 > |den|, the scaling exact (or +inf when the quotient is
// far from that bound). den = +-0 gives +-inf (< 0 when signs differ) as here.
RTM_HD bool quot_lt0(float num, float den) {
    if (num != num || den != den || num == 0.0f) return false;  // NaN, or +-0 / den
    if (signbit(num) == signbit(den)) return false;             // > 0, +0 or +inf
    return (fabsf(num) * 0x1p100f) * 0x1p50f > fabsf(den);
}

// IntersectTriangle. WANT_BARY: also return alpha/beta/gamma (closest hit); the
// any-hit form only needs the accept/reject decision. Both decide exactly as
// the reference's divisions would.
// tcut: a hit with t > tcut is reported as a miss before the sub-areas are
// computed (closest-hit callers pass their best t -- such a hit cannot win;
// bounded any-hit callers their bound): the same decision for every hit that
// matters, less work for the ones that do not.
template <bool WANT_BARY, bool SIGN = false>
RTM_HD bool tri_test(const rt_prim& P, rv3 o, rv3 d, float& t, float& a, float& b, float& g, float tcut = INFINITY) {
    const rv3 N = ld3(P.nrm);
    const float nd = v3_dot(N, d);
    if (rt_lt_eps(fabsf(nd))) return false;  // NearlyEquals(nd, 0)
    const float num = -(v3_dot(N, o) + P.d);
    // t = num / nd <= EPSILON: decided by signs when t <= 0 (|nd| > EPSILON here)
    if (SIGN && num == num && (num == 0.0f || signbit(num) != signbit(nd))) return false;
    t = num / nd;
    if (rt_lt_eps(t)) return false;           // t <= EPSILON
    if (t > tcut) return false;
    const rv3 Pp = v3_add(o, v3_scale(d, t));
    const rv3 v0 = ld3(P.p0), v1 = ld3(P.p1), v2 = ld3(P.p2);
    // CalcTriangleAreaSigned (Raytracer.cpp:937-942): 0.5 * dot(cross(B-A, C-A), N)
    const float aa = 0.5f * v3_dot(v3_cross(v3_sub(v1, Pp), v3_sub(v2, Pp)), N);
    const float bb = 0.5f * v3_dot(v3_cross(v3_sub(Pp, v0), v3_sub(v2, v0)), N);
    const float gg = 0.5f * v3_dot(v3_cross(v3_sub(v1, v0), v3_sub(Pp, v0)), N);
    if (SIGN) {
        if (quot_lt0(aa, P.area) || quot_lt0(bb, P.area) || quot_lt0(gg, P.area)) return false;
        if (WANT_BARY) {
            a = aa / P.area;
            b = bb / P.area;
            g = gg / P.area;
        }
        return true;
    }
    a = aa / P.area;
    b = bb / P.area;
    g = gg / P.area;
    return !(a < 0 || b < 0 || g < 0);
}

RTM_HD bool sph_test(const rt_prim& P, rv3 o, rv3 d, float& t) {
    rv3 oc = v3_sub(o, ld3(P.p0));
    float b = 2.0f * v3_dot(d, oc);
    float c = v3_dot(oc, oc) - P.d;
    // Origin outside (c >= 0) and moving away (b > 0): disc <= RN(b*b), so
    // sqrtf(disc) <= b (tests/native/eps_check.cpp) and t0, t1 <= 0 -- the
    // reference rejects, decided here without the square root.
    if (b > 0.0f && c >= 0.0f && b < 0x1p60f) return false;
    float disc = (b * b) - (4.0f * c);
    if (rt_lt_eps(disc)) return false;
    float sq = rt_sqrt_nr(disc);  // == sqrtf: disc > EPSILON or NaN here (rt_math.h)
    float t0 = (-b + sq) / 2.0f;
    float t1 = (-b - sq) / 2.0f;
    bool g0 = rt_gt_eps(t0), g1 = rt_gt_eps(t1);
    if (!g0 && !g1) return false;
    if (!g0) t = t1;
    else if (!g1) t = t0;
    else t = fminf(t0, t1);
    return true;
}

RTM_HD bool prim_test_closest(const rt_prim& P, rv3 o, rv3 d, float& t, float& a, float& b, float& g,
                              float tcut = INFINITY) {
    a = b = g = 0.0f;
    return P.kind == RT_PRIM_TRIANGLE ? tri_test<true, true>(P, o, d, t, a, b, g, tcut) : sph_test(P, o, d, t);
}

RTM_HD bool prim_test_any(const rt_prim& P, rv3 o, rv3 d) {
    float t, a, b, g;
    return P.kind == RT_PRIM_TRIANGLE ? tri_test<false, true>(P, o, d, t, a, b, g) : sph_test(P, o, d, t);
}

// ---------------------------------------------------------------- BVH queries
struct BvhView {
    const rt_prim* all;         // scene primitives by index
    const BvhNode* nodes;
    const Bvh4QNode* nodes4;    // the same tree 4-wide, quantized boxes (rt_bvh.h); null: binary only
    const rt_prim* prims;       // spatial leaf order
    const uint32_t* ids;
    const FarNode* far_nodes;
    const FarTri* far_tris;
    const uint32_t* brute;      // spheres + unanalysable triangles, ascending
    int n_brute;
    int n_far;                  // far_tris entries
    float dhi_median;           // typical D_hi (routing of far-origin rays)
    int has_tree, has_far;
    float scale;                // S
    // far-search direction grid (rt_bvh.h build_dir_grid); grid_log2 == 0: none
    const uint32_t* grid_start;
    const uint32_t* grid_items;
    const uint32_t* grid_always;
    const uint32_t* grid_live;  // bit c: cell c's list is not empty (the far queues' filter, far_live)
    int n_always;
    int grid_log2;
    float grid_r;
};

// Octahedral cell of direction d, 2^L cells per axis: map coordinate
// x = d.x / (|d.x| + |d.y| + |d.z|) (folded for d.z < 0), cell floor((x/2 + 1/2) 2^L).
// build_dir_grid's cell radii allow 1e-6 map units for these float roundings.
RTM_HD uint32_t grid_cell(rv3 d, int L) {
    const float s = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    float x = d.x / s, y = d.y / s;
    if (d.z < 0.0f) {
        const float ax = fabsf(x), ay = fabsf(y);
        x = (1.0f - ay) * (x < 0.0f ? -1.0f : 1.0f);
        y = (1.0f - ax) * (y < 0.0f ? -1.0f : 1.0f);
    }
    const float m = (float)(1 << L);
    const uint32_t i = (uint32_t)fminf(fmaxf((x * 0.5f + 0.5f) * m, 0.0f), m - 1.0f);
    const uint32_t j = (uint32_t)fminf(fmaxf((y * 0.5f + 0.5f) * m, 0.0f), m - 1.0f);
    return (i << L) | j;
}

// Does this origin use the direction grid (|o| <= grid_r, with the float norm's rounding)?
RTM_HD bool grid_origin(const BvhView& V, rv3 o) {
    return V.grid_log2 > 0 && sqrtf(o.x * o.x + o.y * o.y + o.z * o.z) * 1.0001f <= V.grid_r;
}

#define RT_U 5.9604644775390625e-08f  // 2^-24

// Host-only traversal counters (tests/native/bvh_check.cpp -DRT_BVH_COUNT).
#if defined(RT_BVH_COUNT) && !defined(__HIP_DEVICE_COMPILE__)
struct BvhCounters {
    long nodes, leaf_tris, far_nodes, far_cands, far_tests, brute_tests;
};
inline thread_local BvhCounters g_bvh_cnt;
#define RT_CNT(f, n) (g_bvh_cnt.f += (n))
#else
#define RT_CNT(f, n) ((void)0)
#endif

// A zero direction (CalculateRefraction's total internal reflection result,
// Raytracer.cpp:197-199, is still traced) makes nd = dot(N, d) = 0 for every
// triangle, which tri_test rejects (NearlyEquals): only spheres can be hit.
RTM_HD bool dir_zero(rv3 d) { return d.x == 0.0f && d.y == 0.0f && d.z == 0.0f; }

// Closest hit keeps the lexicographic minimum of (t, primitive index).
RTM_HD bool lex_better(float t, int id, bool found, const Hit& h) {
    return !found || t < h.t || (t == h.t && id < h.prim);
}

// "Fat ray" slab test. An accepted near hit at t has its float hit point Pp
// within D_lo + h of the triangle (rt_bvh.h), and the exact ray point o + d t
// within u (2t + |o|) of Pp per component. So the exact ray meets the triangle's
// box (inflated by delta_j >= D_lo) grown by alpha + beta t with
// alpha >= u |o| + h + rounding, beta = 16u >= 2u + slack for the rounding of
// the slab arithmetic itself. Per axis, for t >= 0:
//   c_lo t >= lo - alpha - o   and   c_hi t <= hi + alpha - o
// with c_lo = d + beta, c_hi = d - beta. Raising c_lo or lowering c_hi only
// weakens a constraint at t >= 0, so for |d| <= beta (where c_lo, c_hi may be
// 0) c_lo = max(d + beta, beta), c_hi = min(d - beta, -beta): every reciprocal
// is finite. (Axis-parallel rays are common -- the shadow rays of an
// axis-aligned directional light -- so such an axis keeps its one-sided
// bounds rather than going untested.) Each bound is one FMA,
// lo * (1/c_lo) - (o + alpha) / c_lo; the rounding of the hoisted product
// (o + alpha) / c_lo and of o + alpha moves the plane by at most
// 2u (|o| + alpha), which 40u (|o| + S) covers on top of the 32u the bound
// itself needs; alpha = 48u (|o| + S) also covers node4_slab's folded decode.
// The culling is then conservative for every t >= 0, with no bound on the ray
// length.
//   Per axis the two plane distances t1 (lo), t2 (hi) give, for d > beta, the
// interval [t1, t2]; for d < -beta [t2, t1]; for |d| <= beta [max(t1, t2),
// inf). With k = -inf (|d| > beta) or +inf (|d| <= beta): low =
// med3(t1, t2, k), high = max(t1, t2, k) -- for |d| > beta the min/max form
// can only widen an interval whose planes are both behind the origin, which
// the high >= 0 test rejects anyway.
struct SlabRay {
    float ip[3], im[3];    // 1 / c_lo, 1 / c_hi
    float nol[3], noh[3];  // -(o + alpha) / c_lo, -(o - alpha) / c_hi
    float k[3];            // -inf, or +inf for |d| <= beta
};

RTM_HD float rt_med3(float a, float b, float c) {
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_fmed3f(a, b, c);
#else
    return fmaxf(fminf(a, b), fminf(fmaxf(a, b), c));
#endif
}

RTM_HD SlabRay slab_ray(const BvhView& V, rv3 o, rv3 d) {
    SlabRay r;
    const float beta = 16.0f * RT_U;
    const float ov[3] = {o.x, o.y, o.z}, dv[3] = {d.x, d.y, d.z};
    const float oi = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    const float alpha = 48.0f * RT_U * (oi + V.scale);  // 40u for slab(), 8u more for node4_slab
    for (int k = 0; k < 3; k++) {
        const bool par = !(dv[k] > beta) && !(dv[k] < -beta);
        const float clo = par ? fmaxf(dv[k] + beta, beta) : dv[k] + beta;
        const float chi = par ? fminf(dv[k] - beta, -beta) : dv[k] - beta;
        r.ip[k] = 1.0f / clo;
        r.im[k] = 1.0f / chi;
        r.nol[k] = -((ov[k] + alpha) * r.ip[k]);
        r.noh[k] = -((ov[k] - alpha) * r.im[k]);
        r.k[k] = par ? INFINITY : -INFINITY;
    }
    return r;
}

// Entry distance tn = max(0, low) of the fat box; accepted iff tn <= high.
RTM_HD bool slab(const float* lo, const float* hi, const SlabRay& r, float& tn) {
    float tmin = 0.0f, tmax = INFINITY;
    for (int k = 0; k < 3; k++) {
        const float t1 = fmaf(lo[k], r.ip[k], r.nol[k]);
        const float t2 = fmaf(hi[k], r.im[k], r.noh[k]);
        tmin = fmaxf(tmin, rt_med3(t1, t2, r.k[k]));
        tmax = fminf(tmax, fmaxf(fmaxf(t1, t2), r.k[k]));
    }
    tn = tmin;
    return tmin <= tmax;
}

// Far-search threshold for a ray: a hit with t < T_j = (D_hi(j) - R)(1 - 1e-4),
// R = |o|_2 + sqrt(3) S, has its hit point within D_lo of the triangle, so the
// spatial BVH finds it. Monotone in D_hi, so a node's bound from its minimum
// is <= every member's.
struct FarRay {
    float R;
};
RTM_HD FarRay far_ray(const BvhView& V, rv3 o) {
    FarRay f;
    f.R = sqrtf(o.x * o.x + o.y * o.y + o.z * o.z) * 1.0001f + 1.7321f * V.scale;
    return f;
}
RTM_HD float far_T(const FarRay& r, float dhi) { return (dhi - r.R) * 0.9999f; }

// Could any plane of this node be crossed beyond T_node (and so need the far
// test)? Interval arithmetic with padding that covers every rounding of both
// this bound and the reference's num / nd (see rt_bvh.h).
RTM_HD bool far_node_may(const FarNode& n, const FarRay& r, rv3 o, rv3 d, float& T) {
    T = far_T(r, n.min_dhi);
    if (!(T > 0.0f)) return true;
    const float T2 = T * (1.0f - 0x1p-20f);
    const rv3 q = v3_add(o, v3_scale(d, T2));
    float gl = 0, gh = 0, fl = n.dlo, fh = n.dhi;
    const float dv[3] = {d.x, d.y, d.z}, qv[3] = {q.x, q.y, q.z};
    for (int k = 0; k < 3; k++) {
        const float a0 = n.nlo[k] * dv[k], a1 = n.nhi[k] * dv[k];
        gl += fminf(a0, a1);
        gh += fmaxf(a0, a1);
        const float b0 = n.nlo[k] * qv[k], b1 = n.nhi[k] * qv[k];
        fl += fminf(b0, b1);
        fh += fmaxf(b0, b1);
    }
    const float oi = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    const float P = 32.0f * RT_U * (3.0f * oi + 3.0f * T2 + fmaxf(fabsf(n.dlo), fabsf(n.dhi))) + 1e-30f;
    const float Pg = 16.0f * RT_U;
    const bool prune = (fl > P && gl > Pg) || (fh < -P && gh < -Pg);
    return !prune;
}

// Is this plane crossed at t >= T_j (computed exactly as tri_test computes t)?
// The division is only done when |num| >= 0.999 T |nd| with matching signs
// (num / nd >= T needs that, with room for the roundings).
RTM_HD bool far_candidate(const FarTri& ft, const FarRay& r, rv3 o, rv3 d) {
    const rv3 N = ld3(ft.n);
    const float nd = v3_dot(N, d);
    if (rt_lt_eps(fabsf(nd))) return false;
    const float num = -(v3_dot(N, o) + ft.d);
    const float T = far_T(r, ft.dhi);
    if (T > 0.0f && !(num * nd > 0.0f && fabsf(num) >= 0.999f * T * fabsf(nd))) return false;
    const float t = num / nd;
    return t >= T;
}

// far_candidate without the division: a superset of it (every pair with
// t >= T_j passes, and the few with 0.999 T_j <= t < T_j, or T_j <= 0, too).
// For the cell kernels, which queue the passing pairs for the reference's full
// test: a pair that then hits is a hit of the reference's own loop whatever its
// t, and one with t < T_j was already found by the near walk (the same key), so
// the any-hit flag and the closest key are unchanged. Saves the division that a
// wave executes whenever any of its 64 pairs passes (about half its steps).
RTM_HD bool far_candidate_filter(const FarTri& ft, const FarRay& r, rv3 o, rv3 d) {
    const rv3 N = ld3(ft.n);
    const float nd = v3_dot(N, d);
    if (rt_lt_eps(fabsf(nd))) return false;
    const float num = -(v3_dot(N, o) + ft.d);
    const float T = far_T(r, ft.dhi);
    return !(T > 0.0f) || (num * nd > 0.0f && fabsf(num) >= 0.999f * T * fabsf(nd));
}

// The far search of bvh_closest on its own (per ray): merges into h.
RTM_HD bool far_closest(const BvhView& V, rv3 o, rv3 d, Hit& h, bool found) {
    if (dir_zero(d)) return found;
    const FarRay fr = far_ray(V, o);
    if (grid_origin(V, o)) {
        const uint32_t cell = grid_cell(d, V.grid_log2);
        const uint32_t b = V.grid_start[cell], e = V.grid_start[cell + 1];
        const int n_list = (int)(e - b);
        for (int q = -V.n_always; q < n_list; q++) {
            const FarTri& ft = V.far_tris[q < 0 ? V.grid_always[q + V.n_always] : V.grid_items[b + (uint32_t)q]];
            RT_CNT(far_cands, 1);
            if (!far_candidate(ft, fr, o, d)) continue;
            RT_CNT(far_tests, 1);
            const int j = (int)ft.id;
            float t, a, bb, g;
            if (tri_test<true, true>(V.all[j], o, d, t, a, bb, g, found ? h.t : INFINITY) && lex_better(t, j, found, h)) {
                found = true;
                h.t = t; h.a = a; h.b = bb; h.g = g; h.prim = j;
            }
        }
        return found;
    }
    int32_t fstk[RT_BVH_STACK];
    int fsp = 0;
    fstk[fsp++] = 0;
    while (fsp > 0) {
        const FarNode& fnode = V.far_nodes[fstk[--fsp]];
        RT_CNT(far_nodes, 1);
        float T;
        if (!far_node_may(fnode, fr, o, d, T)) continue;
        if (found && h.t < T) continue;  // every far hit below has t >= T
        if (fnode.count == 0) {
            fstk[fsp++] = fnode.first + 1;
            fstk[fsp++] = fnode.first;
            continue;
        }
        RT_CNT(far_cands, fnode.count);
        for (int k = fnode.first; k < fnode.first + fnode.count; k++) {
            const FarTri& ft = V.far_tris[k];
            if (!far_candidate(ft, fr, o, d)) continue;
            RT_CNT(far_tests, 1);
            const int j = (int)ft.id;
            float t, a, b, g;
            if (tri_test<true, true>(V.all[j], o, d, t, a, b, g, found ? h.t : INFINITY) && lex_better(t, j, found, h)) {
                found = true;
                h.t = t; h.a = a; h.b = b; h.g = g; h.prim = j;
            }
        }
    }
    return found;
}

// with_far = false: brute list + spatial BVH only; the caller then runs the far
// search itself unless found && h.t < far_T_root (see trace_kernel's phases).
RTM_HD bool bvh_closest(const BvhView& V, rv3 o, rv3 d, Hit& h, bool with_far = true) {
    bool found = false;
    h.t = 0; h.a = h.b = h.g = 0; h.prim = -1;
    RT_CNT(brute_tests, V.n_brute);
    for (int k = 0; k < V.n_brute; k++) {
        const int j = (int)V.brute[k];
        float t, a, b, g;
        if (prim_test_closest(V.all[j], o, d, t, a, b, g, found ? h.t : INFINITY) && lex_better(t, j, found, h)) {
            found = true;
            h.t = t; h.a = a; h.b = b; h.g = g; h.prim = j;
        }
    }
    if (!V.has_tree || dir_zero(d)) return found;
    const SlabRay sr = slab_ray(V, o, d);
    uint32_t stk[RT_BVH_STACK];
    float tstk[RT_BVH_STACK];
    int sp = 0;
    int32_t c = 0, n = 0;  // root (internal)
    for (;;) {
        if (n == 0) {
            RT_CNT(nodes, 1);
            const BvhNode& nd = V.nodes[c];
            float t0, t1;
            bool h0 = nd.n0 >= 0 && slab(nd.lo0, nd.hi0, sr, t0) && (!found || t0 <= h.t);
            bool h1 = nd.n1 >= 0 && slab(nd.lo1, nd.hi1, sr, t1) && (!found || t1 <= h.t);
            if (h0 && h1) {
                const bool first0 = t0 <= t1;
                const int32_t fc = first0 ? nd.c1 : nd.c0, fn = first0 ? nd.n1 : nd.n0;
                stk[sp] = ((uint32_t)fn << 27) | (uint32_t)fc;
                tstk[sp] = first0 ? t1 : t0;
                sp++;
                c = first0 ? nd.c0 : nd.c1;
                n = first0 ? nd.n0 : nd.n1;
                continue;
            }
            if (h0 || h1) {
                c = h0 ? nd.c0 : nd.c1;
                n = h0 ? nd.n0 : nd.n1;
                continue;
            }
        } else {
            RT_CNT(leaf_tris, n);
            for (int k = c; k < c + n; k++) {
                float t, a, b, g;
                if (tri_test<true, true>(V.prims[k], o, d, t, a, b, g, found ? h.t : INFINITY)) {
                    const int id = (int)V.ids[k];
                    if (lex_better(t, id, found, h)) {
                        found = true;
                        h.t = t; h.a = a; h.b = b; h.g = g; h.prim = id;
                    }
                }
            }
        }
        bool popped = false;
        while (sp > 0) {
            sp--;
            if (found && tstk[sp] > h.t) continue;
            c = (int32_t)(stk[sp] & 0x7ffffffu);
            n = (int32_t)(stk[sp] >> 27);
            popped = true;
            break;
        }
        if (!popped) break;
    }
    if (!V.has_far || !with_far) return found;
    return far_closest(V, o, d, h, found);
}

// The far search of bvh_any on its own (per ray).
RTM_HD bool far_any(const BvhView& V, rv3 o, rv3 d) {
    if (dir_zero(d)) return false;
    const FarRay fr = far_ray(V, o);
    if (grid_origin(V, o)) {
        const uint32_t cell = grid_cell(d, V.grid_log2);
        const uint32_t b = V.grid_start[cell], e = V.grid_start[cell + 1];
        const int n_list = (int)(e - b);
        for (int q = -V.n_always; q < n_list; q++) {
            const FarTri& ft = V.far_tris[q < 0 ? V.grid_always[q + V.n_always] : V.grid_items[b + (uint32_t)q]];
            RT_CNT(far_cands, 1);
            if (far_candidate(ft, fr, o, d) && prim_test_any(V.all[ft.id], o, d)) return true;
        }
        return false;
    }
    int32_t fstk[RT_BVH_STACK];
    int fsp = 0;
    fstk[fsp++] = 0;
    while (fsp > 0) {
        const FarNode& fnode = V.far_nodes[fstk[--fsp]];
        RT_CNT(far_nodes, 1);
        float T;
        if (!far_node_may(fnode, fr, o, d, T)) continue;
        if (fnode.count == 0) {
            fstk[fsp++] = fnode.first + 1;
            fstk[fsp++] = fnode.first;
            continue;
        }
        RT_CNT(far_cands, fnode.count);
        for (int k = fnode.first; k < fnode.first + fnode.count; k++) {
            const FarTri& ft = V.far_tris[k];
            if (far_candidate(ft, fr, o, d) && prim_test_any(V.all[ft.id], o, d)) return true;
        }
    }
    return false;
}

// with_far = false: brute list + spatial BVH only (the caller runs the far
// search itself, e.g. the sorted wave-cooperative pass of rt_kernels.hip).
// tmax (near part only, with_far = false): count a hit only if !(t > tmax) --
// the reference's point-light shadow test, occluded iff the closest hit has
// !(t > |light - hit|) (Raytracer.cpp:75), is "some hit with !(t > dist)" for
// finite t; boxes entered beyond tmax are skipped (the fat box of a hit at t
// is entered at or before t).
RTM_HD bool prim_hit_within(const rt_prim& P, rv3 o, rv3 d, float tmax) {
    float t, a, b, g;
    const bool h = P.kind == RT_PRIM_TRIANGLE ? tri_test<false, true>(P, o, d, t, a, b, g, tmax) : sph_test(P, o, d, t);
    return h && !(t > tmax);
}

RTM_HD bool bvh_any(const BvhView& V, rv3 o, rv3 d, bool with_far = true, float tmax = INFINITY) {
    RT_CNT(brute_tests, V.n_brute);
    for (int k = 0; k < V.n_brute; k++)
        if (prim_hit_within(V.all[V.brute[k]], o, d, tmax)) return true;
    if (!V.has_tree || dir_zero(d)) return false;
    const SlabRay sr = slab_ray(V, o, d);
    uint32_t stk[RT_BVH_STACK];
    int sp = 0;
    int32_t c = 0, n = 0;
    for (;;) {
        if (n == 0) {
            RT_CNT(nodes, 1);
            const BvhNode& nd = V.nodes[c];
            float t0, t1;
            const bool h0 = nd.n0 >= 0 && slab(nd.lo0, nd.hi0, sr, t0) && !(t0 > tmax);
            const bool h1 = nd.n1 >= 0 && slab(nd.lo1, nd.hi1, sr, t1) && !(t1 > tmax);
            if (h0 && h1) {
                const bool first0 = t0 <= t1;
                stk[sp++] = first0 ? (((uint32_t)nd.n1 << 27) | (uint32_t)nd.c1)
                                   : (((uint32_t)nd.n0 << 27) | (uint32_t)nd.c0);
                c = first0 ? nd.c0 : nd.c1;
                n = first0 ? nd.n0 : nd.n1;
                continue;
            }
            if (h0 || h1) {
                c = h0 ? nd.c0 : nd.c1;
                n = h0 ? nd.n0 : nd.n1;
                continue;
            }
        } else {
            RT_CNT(leaf_tris, n);
            for (int k = c; k < c + n; k++) {
                float t, a, b, g;
                if (tri_test<false, true>(V.prims[k], o, d, t, a, b, g, tmax) && !(t > tmax)) return true;
            }
        }
        if (sp == 0) break;
        sp--;
        c = (int32_t)(stk[sp] & 0x7ffffffu);
        n = (int32_t)(stk[sp] >> 27);
    }
    if (!V.has_far || !with_far) return false;
    return far_any(V, o, d);
}

// Whole-record loads (one batch of 16-byte loads per node / primitive on the
// device, so a traversal step waits for memory once, not once per field).
// A quantized 4-wide node (rt_bvh.h Bvh4QNode) decoded: child boxes
// lo/hi[axis][child] = fmaf(q, scale, origin) (exact product, one rounding, as
// the host's quantizer assumed) and the child links.
struct Node4 {
    float lo[3][4], hi[3][4];
    uint32_t link[4];
};
RTM_HD void load_node4(const Bvh4QNode* p, Node4& out) {
    Bvh4QNode q;
#ifdef __HIP_DEVICE_COMPILE__
    const float4* s = reinterpret_cast<const float4*>(p);
    float4* d = reinterpret_cast<float4*>(&q);
#pragma unroll
    for (int i = 0; i < 4; i++) d[i] = s[i];
#else
    q = *p;
#endif
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float scale = rt_bits_f32(((q.exps >> (8 * a)) & 255u) << 23);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            out.lo[a][j] = fmaf((float)q.qlo[a][j], scale, q.origin[a]);
            out.hi[a][j] = fmaf((float)q.qhi[a][j], scale, q.origin[a]);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) out.link[j] = q.link[j];
}

// The fat slab test (slab) of the four children of a quantized node, with the
// decode folded into the plane arithmetic: a child plane fmaf(q, scale,
// origin) gives t = q (scale / c) + (origin - o -+ alpha) / c, evaluated as
// fmaf(q, A, B) with A = scale * (1 / c) (exact: scale is a power of two,
// 2^-100 <= scale <= 2^90, rt_bvh.cpp quantize4) and B = fmaf(origin, 1 / c,
// -(o -+ alpha) / c) once per axis -- 12 operations per node instead of the
// 24 decoding ones. Against slab() on the decoded box this adds the rounding
// of B and evaluates the plane at the exact q scale + origin instead of its
// rounding (which the quantizer placed outside the float box): together below
// u (2.04 S + |o| + alpha), which slab_ray's alpha = 48u (|o| + S) covers on top
// of what slab() needs (40u). in[j]: the fat box is entered at tn[j] <= its exit.
RTM_HD void node4_slab(const Bvh4QNode* p, const SlabRay& r, float tn[4], bool in[4], uint32_t link[4]) {
    Bvh4QNode q;
#ifdef __HIP_DEVICE_COMPILE__
    const float4* s = reinterpret_cast<const float4*>(p);
    float4* d = reinterpret_cast<float4*>(&q);
#pragma unroll
    for (int i = 0; i < 4; i++) d[i] = s[i];
#else
    q = *p;
#endif
    float tmin[4] = {0.0f, 0.0f, 0.0f, 0.0f}, tmax[4] = {INFINITY, INFINITY, INFINITY, INFINITY};
#pragma unroll
    for (int a = 0; a < 3; a++) {
        const float scale = rt_bits_f32(((q.exps >> (8 * a)) & 255u) << 23);
        const float alo = scale * r.ip[a], blo = fmaf(q.origin[a], r.ip[a], r.nol[a]);
        const float ahi = scale * r.im[a], bhi = fmaf(q.origin[a], r.im[a], r.noh[a]);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const float t1 = fmaf((float)q.qlo[a][j], alo, blo);
            const float t2 = fmaf((float)q.qhi[a][j], ahi, bhi);
            tmin[j] = fmaxf(tmin[j], rt_med3(t1, t2, r.k[a]));
            tmax[j] = fminf(tmax[j], fmaxf(fmaxf(t1, t2), r.k[a]));
        }
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
        tn[j] = tmin[j];
        in[j] = tmin[j] <= tmax[j];
        link[j] = q.link[j];
    }
}

RTM_HD void load_prim(const rt_prim* p, rt_prim& out) {
#ifdef __HIP_DEVICE_COMPILE__
    const float4* s = reinterpret_cast<const float4*>(p);
    float4* d = reinterpret_cast<float4*>(&out);
#pragma unroll
    for (int i = 0; i < 4; i++) d[i] = s[i];
#else
    out = *p;
#endif
}

// bvh_any's near part over the 4-wide tree (same boxes, same leaves, same
// tests; only the grouping differs, so the same boolean). Per node: the fat
// slab test of its up to four children (branch-free), the nearest accepted
// child entered, the other accepted ones stacked. While-while loop: a lane
// descends inner nodes until it holds a leaf (bvh4_descend), then tests the
// leaf (bvh4_leaf_hit), then resumes from the stack (bvh4_pop).
// Stack entries: n << 27 | c (BvhNode's child link); RT_BVH_STACK + 4 slots
// (collapse_bvh4 bounds the depth; the branch-free push writes one past).
// The stack as a plain per-lane array ...
struct ArrStack {
    uint32_t* a;
    RTM_HDM void put(int i, uint32_t v) const { a[i] = v; }
    RTM_HDM uint32_t get(int i) const { return a[i]; }
    RTM_HDM uint32_t get_lds_first(int i) const { return a[i]; }
    RTM_HDM void push4(int& sp, const uint32_t v[4], const bool take[4]) const {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            a[sp] = v[j];
            sp += take[j] ? 1 : 0;
        }
    }
};
// ... or (device) its first D entries in LDS, one column per lane (stride
// TB: lanes hit consecutive banks), the rest in a per-lane array.
template <int D, int STRIDE>
struct LdsStack {
    uint32_t* l;  // &lds[0][lane]
    uint32_t* a;  // entries D..
    RTM_HDM void put(int i, uint32_t v) const {
        if (i < D) l[i * STRIDE] = v;
        else a[i - D] = v;
    }
    RTM_HDM uint32_t get(int i) const { return i < D ? l[i * STRIDE] : a[i - D]; }
    // get() as an LDS read that always issues plus a private-memory read only
    // for entries past D (the compiler otherwise selects the address space per
    // lane and emits a flat load, which waits on both memory counters)
    RTM_HDM uint32_t get_lds_first(int i) const {
        uint32_t e = l[(i < D ? i : D - 1) * STRIDE];
#ifdef __HIP_DEVICE_COMPILE__
        asm volatile("" : "+v"(e));  // keeps the two loads apart (no address select)
#endif
        if (i >= D) e = a[i - D];
        return e;
    }
    // the node step's four pushes (v[j] written at the top, the top raised when
    // take[j]): one test of the depth instead of one per entry
    RTM_HDM void push4(int& sp, const uint32_t v[4], const bool take[4]) const {
        if (sp + 4 <= D) {
            uint32_t* p = l + sp * STRIDE;
            int k = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                p[k * STRIDE] = v[j];
                k += take[j] ? 1 : 0;
            }
            sp += k;
        } else {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                put(sp, v[j]);
                sp += take[j] ? 1 : 0;
            }
        }
    }
};

template <class STK>
RTM_HD bool bvh4_pop(const STK& stk, int& sp, int32_t& c, int32_t& n) {
    if (sp == 0) return false;
    sp--;
    const uint32_t e = stk.get_lds_first(sp);
    c = (int32_t)(e & 0x7ffffffu);
    n = (int32_t)(e >> 27);
    return true;
}

// From (c, n) down to a leaf (n > 0): false when the subtree and the stack hold none.
template <class STK>
RTM_HD bool bvh4_descend(const BvhView& V, const SlabRay& sr, float tmax, const STK& stk, int& sp, int32_t& c,
                         int32_t& n) {
    while (n == 0) {
        RT_CNT(nodes, 1);
        Node4 nd;
        float t[4];
        bool ok[4];
        node4_slab(V.nodes4 + c, sr, t, ok, nd.link);
#pragma unroll
        for (int j = 0; j < 4; j++) ok[j] = (nd.link[j] != 0xffffffffu) & ok[j] & !(t[j] > tmax);
        int best = -1;
        float bt = INFINITY;
#pragma unroll
        for (int j = 0; j < 4; j++)
            if (ok[j] & ((best < 0) | (t[j] < bt))) {
                best = j;
                bt = t[j];
            }
        bool take[4];
#pragma unroll
        for (int j = 0; j < 4; j++) take[j] = ok[j] & (j != best);
        stk.push4(sp, nd.link, take);
        if (best >= 0) {
            const uint32_t e = best == 0 ? nd.link[0] : best == 1 ? nd.link[1] : best == 2 ? nd.link[2] : nd.link[3];
            c = (int32_t)(e & 0x7ffffffu);
            n = (int32_t)(e >> 27);
        } else if (!bvh4_pop(stk, sp, c, n)) {
            return false;
        }
    }
    return true;
}

// Any primitive of leaf slots [c, c + n) hit with !(t > tmax)?
RTM_HD bool bvh4_leaf_hit(const BvhView& V, rv3 o, rv3 d, float tmax, int32_t c, int32_t n) {
    RT_CNT(leaf_tris, n);
    for (int k = c; k < c + n; k++) {
        rt_prim P;
        load_prim(V.prims + k, P);
        float tt, a, b, g;
        if (tri_test<false, true>(P, o, d, tt, a, b, g, tmax) && !(tt > tmax)) return true;
    }
    return false;
}

// bvh4_any_near with a caller-provided stack
template <class STK>
RTM_HD bool bvh4_any_near_s(const BvhView& V, rv3 o, rv3 d, const STK& stk, float tmax = INFINITY) {
    RT_CNT(brute_tests, V.n_brute);
    for (int k = 0; k < V.n_brute; k++)
        if (prim_hit_within(V.all[V.brute[k]], o, d, tmax)) return true;
    if (!V.has_tree || dir_zero(d)) return false;
    const SlabRay sr = slab_ray(V, o, d);
    int sp = 0;
    int32_t c = 0, n = 0;  // root (internal)
    for (;;) {
        if (!bvh4_descend(V, sr, tmax, stk, sp, c, n)) return false;
        if (bvh4_leaf_hit(V, o, d, tmax, c, n)) return true;
        if (!bvh4_pop(stk, sp, c, n)) return false;
    }
}

// bvh4_any_near_s with at most `budget` leaf visits (descent to a leaf + its
// tests): 1 hit, 0 no hit, -1 undecided (the caller runs the full query later;
// the boolean does not depend on the order or the split of the visits).
template <class STK>
RTM_HD int bvh4_any_near_budget(const BvhView& V, rv3 o, rv3 d, const STK& stk, int budget) {
    for (int k = 0; k < V.n_brute; k++)
        if (prim_hit_within(V.all[V.brute[k]], o, d, INFINITY)) return 1;
    if (!V.has_tree || dir_zero(d)) return 0;
    const SlabRay sr = slab_ray(V, o, d);
    int sp = 0;
    int32_t c = 0, n = 0;  // root (internal)
    for (int visits = 0;; visits++) {
        if (visits == budget) return -1;
        if (!bvh4_descend(V, sr, INFINITY, stk, sp, c, n)) return 0;
        if (bvh4_leaf_hit(V, o, d, INFINITY, c, n)) return 1;
        if (!bvh4_pop(stk, sp, c, n)) return 0;
    }
}

// An undecided walk (stack [0, sp), entry (c, n) next) continued for at most
// `budget` more leaf visits: 1 hit, 0 no hit, -1 still undecided (state updated).
template <class STK>
RTM_HD int bvh4_any_near_resume_budget(const BvhView& V, rv3 o, rv3 d, const STK& stk, int budget, int& sp,
                                       int32_t& c, int32_t& n) {
    const SlabRay sr = slab_ray(V, o, d);
    for (int visits = 0;; visits++) {
        if (visits == budget) return -1;
        if (!bvh4_descend(V, sr, INFINITY, stk, sp, c, n)) return 0;
        if (bvh4_leaf_hit(V, o, d, INFINITY, c, n)) return 1;
        if (!bvh4_pop(stk, sp, c, n)) return 0;
    }
}

// bvh4_any_near_budget that also returns, when undecided (-1), the walk's
// state: the stack [0, sp) and the entry (c, n) it was about to descend --
// bvh4_any_near_resume continues from there (the brute list is done).
template <class STK>
RTM_HD int bvh4_any_near_budget_state(const BvhView& V, rv3 o, rv3 d, const STK& stk, int budget, int& sp,
                                      int32_t& c, int32_t& n) {
    sp = 0;
    c = 0;
    n = 0;  // root (internal)
    for (int k = 0; k < V.n_brute; k++)
        if (prim_hit_within(V.all[V.brute[k]], o, d, INFINITY)) return 1;
    if (!V.has_tree || dir_zero(d)) return 0;
    return bvh4_any_near_resume_budget(V, o, d, stk, budget, sp, c, n);
}

// The rest of an undecided bvh4_any_near_budget_state walk: the same boolean
// as the whole query (the visits are split, not changed).
template <class STK>
RTM_HD bool bvh4_any_near_resume(const BvhView& V, rv3 o, rv3 d, const STK& stk, int sp, int32_t c, int32_t n) {
    const SlabRay sr = slab_ray(V, o, d);
    for (;;) {
        if (!bvh4_descend(V, sr, INFINITY, stk, sp, c, n)) return false;
        if (bvh4_leaf_hit(V, o, d, INFINITY, c, n)) return true;
        if (!bvh4_pop(stk, sp, c, n)) return false;
    }
}

RTM_HD bool bvh4_any_near(const BvhView& V, rv3 o, rv3 d, float tmax = INFINITY) {
    RT_CNT(brute_tests, V.n_brute);
    for (int k = 0; k < V.n_brute; k++)
        if (prim_hit_within(V.all[V.brute[k]], o, d, tmax)) return true;
    if (!V.has_tree || dir_zero(d)) return false;
    const SlabRay sr = slab_ray(V, o, d);
    uint32_t stk_a[RT_BVH_STACK + 4];
    const ArrStack stk{stk_a};
    int sp = 0;
    int32_t c = 0, n = 0;  // root (internal)
    for (;;) {
        if (!bvh4_descend(V, sr, tmax, stk, sp, c, n)) return false;
        if (bvh4_leaf_hit(V, o, d, tmax, c, n)) return true;
        if (!bvh4_pop(stk, sp, c, n)) return false;
    }
}

// bvh_closest's near part (with_far = false) over the 4-wide tree: the same
// lexicographic minimum of (t, primitive index) -- a box is skipped only when
// its entry t is above the best t, and a primitive hit at the best t with a
// lower index lies in a box entered at or before that t. Stack entries carry
// their entry t for that pruning at pop time.
template <class STK, class TSTK>
RTM_HD bool bvh4_closest_near_s(const BvhView& V, rv3 o, rv3 d, Hit& h, const STK& stk, const TSTK& tstk) {
    bool found = false;
    h.t = 0; h.a = h.b = h.g = 0; h.prim = -1;
    RT_CNT(brute_tests, V.n_brute);
    for (int k = 0; k < V.n_brute; k++) {
        const int j = (int)V.brute[k];
        float t, a, b, g;
        if (prim_test_closest(V.all[j], o, d, t, a, b, g, found ? h.t : INFINITY) && lex_better(t, j, found, h)) {
            found = true;
            h.t = t; h.a = a; h.b = b; h.g = g; h.prim = j;
        }
    }
    if (!V.has_tree || dir_zero(d)) return found;
    const SlabRay sr = slab_ray(V, o, d);
    int sp = 0;
    int32_t c = 0, n = 0;  // root (internal)
    for (;;) {
        bool have = true;
        while (n == 0) {
            RT_CNT(nodes, 1);
            Node4 nd;
            float t[4];
            bool ok[4];
            node4_slab(V.nodes4 + c, sr, t, ok, nd.link);
#pragma unroll
            for (int j = 0; j < 4; j++) ok[j] = (nd.link[j] != 0xffffffffu) & ok[j] & (!found || t[j] <= h.t);
            int best = -1;
            float bt = INFINITY;
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (ok[j] & ((best < 0) | (t[j] < bt))) {
                    best = j;
                    bt = t[j];
                }
            bool take[4];
            uint32_t tb[4];
#pragma unroll
            for (int j = 0; j < 4; j++) {
                take[j] = ok[j] & (j != best);
                tb[j] = rt_f32_bits(t[j]);
            }
            int sp2 = sp;
            stk.push4(sp2, nd.link, take);
            tstk.push4(sp, tb, take);
            if (best >= 0) {
                const uint32_t e = best == 0 ? nd.link[0] : best == 1 ? nd.link[1] : best == 2 ? nd.link[2] : nd.link[3];
                c = (int32_t)(e & 0x7ffffffu);
                n = (int32_t)(e >> 27);
                continue;
            }
            have = false;
            while (sp > 0) {
                sp--;
                if (found && rt_bits_f32(tstk.get_lds_first(sp)) > h.t) continue;
                const uint32_t e = stk.get_lds_first(sp);
                c = (int32_t)(e & 0x7ffffffu);
                n = (int32_t)(e >> 27);
                have = true;
                break;
            }
            if (!have) return found;
        }
        RT_CNT(leaf_tris, n);
        for (int k = c; k < c + n; k++) {
            rt_prim P;
            load_prim(V.prims + k, P);
            float t, a, b, g;
            if (tri_test<true, true>(P, o, d, t, a, b, g, found ? h.t : INFINITY)) {
                const int id = (int)V.ids[k];
                if (lex_better(t, id, found, h)) {
                    found = true;
                    h.t = t; h.a = a; h.b = b; h.g = g; h.prim = id;
                }
            }
        }
        have = false;
        while (sp > 0) {
            sp--;
            if (found && rt_bits_f32(tstk.get(sp)) > h.t) continue;
            const uint32_t e = stk.get(sp);
            c = (int32_t)(e & 0x7ffffffu);
            n = (int32_t)(e >> 27);
            have = true;
            break;
        }
        if (!have) return found;
    }
}

RTM_HD bool bvh4_closest_near(const BvhView& V, rv3 o, rv3 d, Hit& h) {
    uint32_t stk_a[RT_BVH_STACK + 4], tstk_a[RT_BVH_STACK + 4];
    return bvh4_closest_near_s(V, o, d, h, ArrStack{stk_a}, ArrStack{tstk_a});
}

// The near closest-hit query: 4-wide tree when present, else the binary one.
RTM_HD bool bvh_closest_near(const BvhView& V, rv3 o, rv3 d, Hit& h) {
    return V.nodes4 ? bvh4_closest_near(V, o, d, h) : bvh_closest(V, o, d, h, /*with_far=*/false);
}

// The near any-hit query: 4-wide tree when present, else the binary one.
RTM_HD bool bvh_any_near(const BvhView& V, rv3 o, rv3 d, float tmax = INFINITY) {
    return V.nodes4 ? bvh4_any_near(V, o, d, tmax) : bvh_any(V, o, d, /*with_far=*/false, tmax);
}

}  // namespace rt580

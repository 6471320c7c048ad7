// rt_bvh.cpp — builders for the exact-semantics triangle structures (see
// rt_bvh.h for the error analysis that makes culling exact). Host C++, run
// once per scene upload.
#include "rt_bvh.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace rt580 {
namespace {

constexpr int kBins = 16;
// triangles per spatial leaf. 2: a wave's lanes test fewer triangles per leaf
// step (tools/simd_sim.cpp); AO cornell10k 82.5 -> 80.9 ms, field100k 1080p
// 61.4 -> 59.1 ms against 4.
static int leaf_max() { return 2; }
constexpr int kFarLeaf = 8;   // planes per far-tree leaf
constexpr int kSahDepth = 40; // below this depth: median splits (bounded stack)
constexpr double kU = 5.9604644775390625e-08;  // 2^-24

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY};
    float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box& b) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    void grow(const float p[3]) {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], p[k]);
            hi[k] = std::max(hi[k], p[k]);
        }
    }
    double area() const {
        double e[3];
        for (int k = 0; k < 3; k++) e[k] = hi[k] >= lo[k] ? (double)hi[k] - lo[k] : 0.0;
        return 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
    }
};

struct Ref {
    Box box;
    float c[3];
    uint32_t id;
};

float max_abs3(const float* p) { return std::max(std::fabs(p[0]), std::max(std::fabs(p[1]), std::fabs(p[2]))); }

// ---------------------------------------------------------------- analysis
struct TriBounds {
    bool ok;
    double dhi, dlo, delta;
};

double dist3(const float* a, const float* b) {
    const double x = (double)a[0] - b[0], y = (double)a[1] - b[1], z = (double)a[2] - b[2];
    return std::sqrt(x * x + y * y + z * z);
}

double angle_at(const float* p, const float* q, const float* r) {  // angle at p of triangle (p, q, r)
    double a[3], b[3];
    for (int k = 0; k < 3; k++) { a[k] = (double)q[k] - p[k]; b[k] = (double)r[k] - p[k]; }
    const double la = std::sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
    const double lb = std::sqrt(b[0] * b[0] + b[1] * b[1] + b[2] * b[2]);
    if (!(la > 0) || !(lb > 0)) return 0.0;
    double c = (a[0] * b[0] + a[1] * b[1] + a[2] * b[2]) / (la * lb);
    c = std::min(1.0, std::max(-1.0, c));
    return std::acos(c);
}

TriBounds analyse(const rt_prim& p, double S, double inflate) {
    TriBounds r{false, 0, 0, 0};
    const double e01 = dist3(p.p0, p.p1), e12 = dist3(p.p1, p.p2), e20 = dist3(p.p2, p.p0);
    const double emin = std::min(e01, std::min(e12, e20)), emax = std::max(e01, std::max(e12, e20));
    const double a0 = angle_at(p.p0, p.p1, p.p2), a1 = angle_at(p.p1, p.p2, p.p0), a2 = angle_at(p.p2, p.p0, p.p1);
    if (!(emin > 0) || !(std::min(a0, std::min(a1, a2)) > 1e-6) || !std::isfinite(emax) || !(a0 > 1e-6)) return r;
    // Signal: a point at in-plane distance D outside the triangle whose closest
    // triangle point is in an edge's interior is at distance D from that edge's
    // line; if it is a vertex v (angle a_v), at distance >= D sin(a_v/2) from the
    // line of one of v's two edges. So the most negative exact sub-area is
    // <= -G D / 2 with G = min(e_min, min_v min(adjacent edges) sin(a_v/2)).
    const double g0 = std::min(e01, e20) * std::sin(0.5 * a0);
    const double g1 = std::min(e01, e12) * std::sin(0.5 * a1);
    const double g2 = std::min(e12, e20) * std::sin(0.5 * a2);
    const double G = std::min(emin, std::min(g0, std::min(g1, g2)));
    // Error of a computed sub-area s = dot(cross(A, B), N) (twice the area;
    // A = fl(v_i - Pp), B = fl(v_j - Pp) or one short edge), standard model,
    // u = 2^-24: each cross component is off by <= gamma3 (|A_j B_k| + |A_k B_j|)
    // + u |X_i|, the dot adds gamma3 sum |c_i N_i|; with sum_i |N_i| <= sqrt3 |N|
    // and |X| <= |A||B|: |s - S| <= (3 sqrt3 + 4)(1 + 10u) u |A||B| < 9.25 u |A||B|.
    // S (exact, float inputs) is twice the signed area of the projection onto
    // the plane normal to the float N: Pp's offset along N cancels, and the
    // float N's tilt (~u / sin a0) changes the projected geometry only at
    // second order, so G below (from the exact triangle) applies.
    const double kappa = 9.25 * (1.0 + 1e-6);
    const double ep = emax + std::ldexp(S, -10);  // + off-plane height and rounding slack
    const double a = kappa * kU, b = G;
    const double bb = b - 2 * a * ep;
    const double disc = bb * bb - 4 * a * a * ep * ep;
    if (!(bb > 0) || !(disc > 0)) return r;
    r.dhi = (bb + std::sqrt(disc)) / (2 * a);
    r.dlo = ep * ep / r.dhi;  // product of the roots
    // near hit points lie within D_lo of the triangle; the rest of the float
    // error budget is carried by the fat-ray slab test (rt_isect.h)
    r.delta = std::max(std::max(inflate * emin, std::ldexp(S, -20)), 2.0 * r.dlo);
    // D_hi must clear the origin distances of rays from inside the scene
    // (|o| + sqrt3 S), else the triangle is simply tested for every ray
    r.ok = std::isfinite(r.dhi) && std::isfinite(r.delta) && r.dhi > 8.0 * S;
    return r;
}

// ---------------------------------------------------------------- spatial BVH
struct Builder {
    const rt_prim* prims;
    std::vector<Ref> refs;
    BvhBuild* out;

    Box bounds(int b, int e) const {
        Box x;
        for (int i = b; i < e; i++) x.grow(refs[i].box);
        return x;
    }

    int32_t leaf(int b, int e) {
        const int32_t first = (int32_t)out->prims.size();
        for (int i = b; i < e; i++) {
            out->prims.push_back(prims[refs[i].id]);
            out->ids.push_back(refs[i].id);
        }
        out->max_leaf = std::max(out->max_leaf, e - b);
        return first;
    }

    int split(int b, int e, int depth) {
        const int n = e - b;
        Box cb;
        for (int i = b; i < e; i++) cb.grow(refs[i].c);
        int axis = 0;
        for (int k = 1; k < 3; k++)
            if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
        auto median = [&](int ax) {
            const int m = b + n / 2;
            std::nth_element(refs.begin() + b, refs.begin() + m, refs.begin() + e, [ax](const Ref& x, const Ref& y) {
                return x.c[ax] < y.c[ax] || (x.c[ax] == y.c[ax] && x.id < y.id);
            });
            return m;
        };
        if (!(cb.hi[axis] > cb.lo[axis])) return b + n / 2;  // coincident centroids: any split
        if (depth >= kSahDepth) return median(axis);
        double best = INFINITY;
        int best_axis = -1, best_bin = -1;
        for (int k = 0; k < 3; k++) {
            const float ext = cb.hi[k] - cb.lo[k];
            if (!(ext > 0)) continue;
            Box bb[kBins];
            int cnt[kBins] = {0};
            const float scale = kBins / ext;
            for (int i = b; i < e; i++) {
                int t = (int)((refs[i].c[k] - cb.lo[k]) * scale);
                t = std::min(std::max(t, 0), kBins - 1);
                cnt[t]++;
                bb[t].grow(refs[i].box);
            }
            double right_area[kBins];
            int right_cnt[kBins];
            Box acc;
            int c = 0;
            for (int t = kBins - 1; t > 0; t--) {
                acc.grow(bb[t]);
                c += cnt[t];
                right_area[t] = acc.area();
                right_cnt[t] = c;
            }
            Box lacc;
            int lc = 0;
            for (int t = 0; t < kBins - 1; t++) {
                lacc.grow(bb[t]);
                lc += cnt[t];
                if (lc == 0 || right_cnt[t + 1] == 0) continue;
                const double cost = lacc.area() * lc + right_area[t + 1] * right_cnt[t + 1];
                if (cost < best) { best = cost; best_axis = k; best_bin = t; }
            }
        }
        if (best_axis < 0) return median(axis);
        const int k = best_axis;
        const float scale = kBins / (cb.hi[k] - cb.lo[k]);
        const float lo = cb.lo[k];
        auto it = std::partition(refs.begin() + b, refs.begin() + e, [&](const Ref& r) {
            int t = (int)((r.c[k] - lo) * scale);
            t = std::min(std::max(t, 0), kBins - 1);
            return t <= best_bin;
        });
        const int m = (int)(it - refs.begin());
        return (m > b && m < e) ? m : median(axis);
    }

    void build_child(int b, int e, int depth, int32_t& c, int32_t& n, Box& box) {
        box = bounds(b, e);
        if (e - b <= leaf_max()) {
            c = leaf(b, e);
            n = e - b;
            return;
        }
        const int32_t id = (int32_t)out->nodes.size();
        out->nodes.emplace_back();
        c = id;
        n = 0;
        build_node(id, b, e, depth + 1);
    }

    void build_node(int32_t id, int b, int e, int depth) {
        out->depth = std::max(out->depth, depth);
        const int m = split(b, e, depth);
        Box lb, rb;
        int32_t c0, n0, c1, n1;
        build_child(b, m, depth, c0, n0, lb);
        build_child(m, e, depth, c1, n1, rb);
        BvhNode& nd = out->nodes[id];
        for (int k = 0; k < 3; k++) {
            nd.lo0[k] = lb.lo[k]; nd.hi0[k] = lb.hi[k];
            nd.lo1[k] = rb.lo[k]; nd.hi1[k] = rb.hi[k];
        }
        nd.c0 = c0; nd.n0 = n0;
        nd.c1 = c1; nd.n1 = n1;
    }
};

// ---------------------------------------------------------------- plane tree
struct FarBuilder {
    std::vector<FarTri>& tris;
    std::vector<FarNode>& nodes;
    int depth = 0;

    void fill(FarNode& nd, int b, int e) {
        for (int k = 0; k < 3; k++) { nd.nlo[k] = INFINITY; nd.nhi[k] = -INFINITY; }
        nd.dlo = INFINITY; nd.dhi = -INFINITY;
        nd.min_dhi = INFINITY; nd.min_delta = INFINITY;
        for (int i = b; i < e; i++) {
            const FarTri& t = tris[i];
            for (int k = 0; k < 3; k++) {
                nd.nlo[k] = std::min(nd.nlo[k], t.n[k]);
                nd.nhi[k] = std::max(nd.nhi[k], t.n[k]);
            }
            nd.dlo = std::min(nd.dlo, t.d);
            nd.dhi = std::max(nd.dhi, t.d);
            nd.min_dhi = std::min(nd.min_dhi, t.dhi);
            nd.min_delta = std::min(nd.min_delta, t.delta);
        }
    }

    // Node `id` covers [b, e). The far test's interval of N.q + D (q ~ T d away)
    // has width ~ T_typ * |normal box| + |D range|: median-split the widest of
    // the four, so leaves are tight in both normal and offset.
    float t_typ = 1.0f;

    void build(int32_t id, int b, int e, int d) {
        depth = std::max(depth, d);
        fill(nodes[id], b, e);
        if (e - b <= kFarLeaf) {
            nodes[id].first = b;
            nodes[id].count = e - b;
            return;
        }
        int axis = 3;
        float w = nodes[id].dhi - nodes[id].dlo;
        for (int k = 0; k < 3; k++) {
            const float x = t_typ * (nodes[id].nhi[k] - nodes[id].nlo[k]);
            if (x > w) { w = x; axis = k; }
        }
        const int m = b + (e - b) / 2;
        std::nth_element(tris.begin() + b, tris.begin() + m, tris.begin() + e, [axis](const FarTri& x, const FarTri& y) {
            const float kx = axis < 3 ? x.n[axis] : x.d, ky = axis < 3 ? y.n[axis] : y.d;
            return kx < ky || (kx == ky && x.id < y.id);
        });
        const int32_t c = (int32_t)nodes.size();
        nodes.emplace_back();
        nodes.emplace_back();
        nodes[id].first = c;
        nodes[id].count = 0;
        build(c, b, m, d + 1);
        build(c + 1, m, e, d + 1);
    }
};

}  // namespace

bool build_bvh(const rt_prim* prims, int n, BvhBuild& out) {
    const auto t0 = std::chrono::steady_clock::now();
    out = BvhBuild();
    out.inflate = 0.0;
    float S = 0.0f;
    for (int i = 0; i < n; i++) {
        const rt_prim& p = prims[i];
        if (p.kind == RT_PRIM_TRIANGLE) {
            out.n_tri++;
            S = std::max(S, std::max(max_abs3(p.p0), std::max(max_abs3(p.p1), max_abs3(p.p2))));
        } else {
            S = std::max(S, max_abs3(p.p0) + std::sqrt(std::max(p.d, 0.0f)));
        }
    }
    // S <= 2^90: the quantized nodes' scales (<= 2^98 for any extent below 2S) times
    // the slab reciprocals (<= 2^20) stay finite (node4_slab)
    if (out.n_tri == 0 || !(S > 0.0f) || !(S <= 0x1p90f)) return false;
    out.scale = S;
    Builder B;
    B.prims = prims;
    B.out = &out;
    for (int i = 0; i < n; i++) {
        const rt_prim& p = prims[i];
        TriBounds tb{false, 0, 0, 0};
        if (p.kind == RT_PRIM_TRIANGLE) tb = analyse(p, S, out.inflate);
        if (!tb.ok) {
            out.brute.push_back((uint32_t)i);
            continue;
        }
        const float delta = (float)tb.delta;
        Ref r;
        r.box.grow(p.p0);
        r.box.grow(p.p1);
        r.box.grow(p.p2);
        for (int k = 0; k < 3; k++) {
            // rounded outward: the float box contains the exact [lo - delta, hi + delta]
            r.box.lo[k] = std::nextafter(r.box.lo[k] - delta, -INFINITY);
            r.box.hi[k] = std::nextafter(r.box.hi[k] + delta, INFINITY);
            r.c[k] = 0.5f * (r.box.lo[k] + r.box.hi[k]);
        }
        r.id = (uint32_t)i;
        B.refs.push_back(r);
        FarTri ft;
        std::memcpy(ft.n, p.nrm, sizeof ft.n);
        ft.d = p.d;
        ft.dhi = (float)tb.dhi;  // rounded: the device subtracts margins (see rt_kernels.hip)
        ft.delta = delta;
        ft.id = (uint32_t)i;
        ft.pad = 0;
        out.far_tris.push_back(ft);
    }
    const int nt = (int)B.refs.size();
    if (nt > 0) {
        out.nodes.reserve(nt);
        out.prims.reserve(nt);
        out.ids.reserve(nt);
        out.nodes.emplace_back();  // root
        if (nt <= leaf_max()) {
            Box b = B.bounds(0, nt);
            BvhNode& r = out.nodes[0];
            std::memset(&r, 0, sizeof r);
            for (int k = 0; k < 3; k++) {
                r.lo0[k] = b.lo[k]; r.hi0[k] = b.hi[k];
                r.lo1[k] = INFINITY; r.hi1[k] = -INFINITY;
            }
            r.c0 = B.leaf(0, nt);
            r.n0 = nt;
            r.c1 = 0;
            r.n1 = -1;
        } else {
            B.build_node(0, 0, nt, 0);
        }
        out.far_nodes.reserve(nt / 4 + 2);
        out.far_nodes.emplace_back();
        FarBuilder F{out.far_tris, out.far_nodes};
        {   // typical far threshold: median over triangles of min(0.45 delta / 8u, D_hi)
            std::vector<float> ts;
            ts.reserve(out.far_tris.size());
            for (const FarTri& t : out.far_tris) ts.push_back(t.dhi);
            std::nth_element(ts.begin(), ts.begin() + ts.size() / 2, ts.end());
            F.t_typ = std::max(ts[ts.size() / 2], 1.0f);
            out.dhi_median = ts[ts.size() / 2];
        }
        F.build(0, 0, nt, 0);
        out.far_depth = F.depth;
    }
    out.build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return out.depth + 2 <= RT_BVH_STACK && out.far_depth + 2 <= RT_BVH_STACK;
}

bool bvh_usable(const BvhBuild& b, const float cam_from[3]) {
    if (!(b.scale > 0.0f) || b.n_tri == 0) return false;
    // the bounds hold for any origin; keep the float ranges sane
    return max_abs3(cam_from) <= 1e6f * b.scale;
}

// ---------------------------------------------------------------- 4-wide collapse
namespace {
int32_t collapse4(const std::vector<BvhNode>& bin, int32_t b, std::vector<Bvh4Node>& out, int level, int& depth) {
    depth = std::max(depth, level);
    struct Entry {
        int32_t c, n;
        float lo[3], hi[3];
    };
    Entry e[4];
    int ne = 0;
    auto add = [&](int32_t c, int32_t n, const float* lo, const float* hi) {
        if (n < 0) return;  // empty
        Entry& x = e[ne++];
        x.c = c;
        x.n = n;
        for (int k = 0; k < 3; k++) { x.lo[k] = lo[k]; x.hi[k] = hi[k]; }
    };
    const BvhNode& nd = bin[b];
    for (int side = 0; side < 2; side++) {
        const int32_t c = side ? nd.c1 : nd.c0, n = side ? nd.n1 : nd.n0;
        const float* lo = side ? nd.lo1 : nd.lo0;
        const float* hi = side ? nd.hi1 : nd.hi0;
        if (n == 0) {  // internal: take its two children (their boxes as stored in it)
            const BvhNode& m = bin[c];
            add(m.c0, m.n0, m.lo0, m.hi0);
            add(m.c1, m.n1, m.lo1, m.hi1);
        } else {
            add(c, n, lo, hi);
        }
    }
    const int32_t id = (int32_t)out.size();
    out.emplace_back();
    Bvh4Node q;
    for (int j = 0; j < 4; j++) {
        for (int k = 0; k < 3; k++) { q.lo[k][j] = 0.0f; q.hi[k][j] = 0.0f; }
        q.c[j] = 0;
        q.n[j] = -1;
    }
    for (int j = 0; j < ne; j++) {
        for (int k = 0; k < 3; k++) { q.lo[k][j] = e[j].lo[k]; q.hi[k][j] = e[j].hi[k]; }
        q.n[j] = e[j].n;
        q.c[j] = e[j].n == 0 ? collapse4(bin, e[j].c, out, level + 1, depth) : e[j].c;
    }
    out[id] = q;
    return id;
}
}  // namespace

// One node of nodes4 quantized (Bvh4QNode). Per axis: origin = the smallest
// child lo, scale = 2^e with 255 * scale >= the children's extent; q_lo the
// largest and q_hi the smallest code whose decoded plane fmaf(q, scale, origin)
// (the device's exact arithmetic: q * scale is exact, one rounding) lies
// outside the float plane; a larger scale when q_hi would not fit 8 bits.
static Bvh4QNode quantize4(const Bvh4Node& nd) {
    Bvh4QNode q;
    std::memset(&q, 0, sizeof q);
    bool any = false;
    for (int j = 0; j < 4; j++) any = any || nd.n[j] >= 0;
    for (int a = 0; a < 3; a++) {
        float o = INFINITY, top = -INFINITY;
        for (int j = 0; j < 4; j++)
            if (nd.n[j] >= 0) {
                o = std::min(o, nd.lo[a][j]);
                top = std::max(top, nd.hi[a][j]);
            }
        if (!any) o = top = 0.0f;
        int e;
        (void)std::frexp(((double)top - (double)o) / 255.0, &e);  // 2^e >= extent / 255
        e = std::max(e, -100);  // scale >= 2^-100: scale / c stays a normal, exact product (node4_slab)
        for (;; e++) {
            const float scale = std::ldexp(1.0f, e);
            bool fit = true;
            for (int j = 0; j < 4 && fit; j++) {
                if (nd.n[j] < 0) continue;
                long lo = (long)std::floor(((double)nd.lo[a][j] - o) / scale);
                lo = std::max(0L, std::min(255L, lo));
                while (lo > 0 && std::fma((float)lo, scale, o) > nd.lo[a][j]) lo--;
                while (lo < 255 && std::fma((float)(lo + 1), scale, o) <= nd.lo[a][j]) lo++;
                long hi = (long)std::ceil(((double)nd.hi[a][j] - o) / scale);
                hi = std::max(lo, std::min(256L, hi));
                while (hi <= 255 && std::fma((float)hi, scale, o) < nd.hi[a][j]) hi++;
                while (hi > lo && hi <= 255 && std::fma((float)(hi - 1), scale, o) >= nd.hi[a][j]) hi--;
                if (hi > 255 || std::fma((float)lo, scale, o) > nd.lo[a][j]) {
                    fit = false;
                    break;
                }
                q.qlo[a][j] = (uint8_t)lo;
                q.qhi[a][j] = (uint8_t)hi;
            }
            if (fit) break;
        }
        q.origin[a] = o;
        q.exps |= (uint32_t)(e + 127) << (8 * a);
    }
    for (int j = 0; j < 4; j++)
        q.link[j] = nd.n[j] < 0 ? 0xffffffffu : (((uint32_t)nd.n[j] << 27) | (uint32_t)nd.c[j]);
    return q;
}

void collapse_bvh4(BvhBuild& out) {
    out.nodes4.clear();
    out.nodes4q.clear();
    if (out.nodes.empty()) return;
    out.nodes4.reserve(out.nodes.size() / 2 + 8);
    int depth = 0;
    collapse4(out.nodes, 0, out.nodes4, 1, depth);
    // a traversal stacks at most 3 entries per level
    if (3 * depth + 1 > RT_BVH_STACK) {
        out.nodes4.clear();
        return;
    }
    out.nodes4q.reserve(out.nodes4.size());
    for (const Bvh4Node& nd : out.nodes4) out.nodes4q.push_back(quantize4(nd));
}

}  // namespace rt580

namespace rt580 {

// ---------------------------------------------------------------- direction grid
// A far hit of triangle j (t >= T_j, rt_isect.h far_candidate) for a ray with
// |o| <= R needs, besides the reference's own t test:
//  (band)  |N.d| <= eps_j = |num| / (t nd-rounding) <= (R + |D|)(1 + 1e-5) / T_j + 2e-7;
//  (wedge) the sub-areas through v0 not negative: bb = 0.5 dot(cross(Q, E2), N),
//          Q = fl(Pp - v0), E2 = fl(v2 - v0) (gg alike with E1 = fl(v1 - v0)). With
//          the 9.25u|Q||E| arithmetic bound (analyse), Pp = o + d t + dP,
//          |dP| <= u(2t + |o|), |Q - (Pp - v0)| <= u|Pp - v0|, and t >= T_j:
//            (d x E2).N >= -|E2| zeta_j,  (E1 x d).N >= -|E1| zeta_j,
//            zeta_j = ((R + |v0|)(1 + 11u) + uR) / T_j + 12.4u  (x 1.001).
// (The reference's acceptance is !(bb/area < 0); area > 0 for every far-set
// triangle, and a quotient rounding to -0 only admits bb >= -area 2^-149, far
// inside the slack.) So d lies in a thin arc-shaped patch: nearly in the plane
// and inside the triangle's angle at v0 widened by ~zeta_j.
// A direction d within chord rho of a cell centre c satisfies each condition
// only if c does with rho|N| (resp. rho|E||N|) added to the bound; cell radii
// come from the octahedral decode's Lipschitz bound (<= 3 per map unit: sqrt3
// for the unnormalised vector -- (a, b, 1 - |a| - |b|) moves by
// sqrt(da^2 + db^2 + (da +- db)^2) <= sqrt3 |(da, db)|, the folded half alike --
// and sqrt3 for normalising it, |v|_2 >= |v|_1 / sqrt3 = 1 / sqrt3) times the
// cell's half diagonal, plus 1e-6 map units for the device's float cell
// computation. (Rounds 2-5 used sqrt6, taking sqrt2 for the first factor: a
// quadtree node whose centre was 2.6 half diagonals from a direction inside it
// was pruned, and the north-star frame lost 34 far hits -- tools/pixel_tree_check.cpp,
// DESIGN.md "Full-frame parity".) A quadtree over the map lists every triangle in every cell
// its patch can reach; the device tests far_candidate + the full reference
// test on the listed triangles only.

namespace {

constexpr double kOctLipschitz = 3.0 * (1.0 + 1e-9);  // chord per map unit (above), with the doubles' rounding

void oct_decode(double a, double b, double out[3]) {
    double x = a, y = b;
    const double z = 1.0 - std::fabs(a) - std::fabs(b);
    if (z < 0) {
        x = (1.0 - std::fabs(b)) * (a < 0 ? -1.0 : 1.0);
        y = (1.0 - std::fabs(a)) * (b < 0 ? -1.0 : 1.0);
    }
    const double l = std::sqrt(x * x + y * y + z * z);
    out[0] = x / l; out[1] = y / l; out[2] = z / l;
}

struct GridTri {
    double n[3], ea[3], eb[3];  // N, E2 x N, N x E1
    double band, wa, wb;        // eps, |E2| zeta, |E1| zeta
    double nn, na, nb;          // |N|, |E2||N|, |E1||N|
};

bool grid_tri(const rt_prim& p, const FarTri& ft, double R, double S, GridTri& g) {
    const double T = ((double)ft.dhi - (R * 1.0002 + 1.7322 * S)) * 0.9998;
    if (!(T > 0)) return false;
    double n[3], e1[3], e2[3], v0 = 0;
    for (int k = 0; k < 3; k++) {
        n[k] = p.nrm[k];
        e1[k] = (double)(p.p1[k] - p.p0[k]);  // fl(v1 - v0), as the reference computes it
        e2[k] = (double)(p.p2[k] - p.p0[k]);
        v0 += (double)p.p0[k] * p.p0[k];
    }
    v0 = std::sqrt(v0);
    const double l1 = std::sqrt(e1[0] * e1[0] + e1[1] * e1[1] + e1[2] * e1[2]) * (1 + 1e-9);
    const double l2 = std::sqrt(e2[0] * e2[0] + e2[1] * e2[1] + e2[2] * e2[2]) * (1 + 1e-9);
    g.nn = std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]) * (1 + 1e-9);
    const double u = std::ldexp(1.0, -24);
    g.band = (R + std::fabs((double)p.d)) * (1 + 1e-5) / T + 2e-7;
    const double zeta = (((R + v0) * (1 + 11 * u) + u * R) / T + 12.4 * u) * 1.001;
    g.wa = l2 * zeta + 1e-12;
    g.wb = l1 * zeta + 1e-12;
    g.na = l2 * g.nn;
    g.nb = l1 * g.nn;
    for (int k = 0; k < 3; k++) g.n[k] = n[k];
    // ea = E2 x N: (c x E2).N = c.(E2 x N); eb = N x E1: (E1 x c).N = c.(N x E1)
    g.ea[0] = e2[1] * n[2] - e2[2] * n[1];
    g.ea[1] = e2[2] * n[0] - e2[0] * n[2];
    g.ea[2] = e2[0] * n[1] - e2[1] * n[0];
    g.eb[0] = n[1] * e1[2] - n[2] * e1[1];
    g.eb[1] = n[2] * e1[0] - n[0] * e1[2];
    g.eb[2] = n[0] * e1[1] - n[1] * e1[0];
    return true;
}

// Can a direction within chord rho of c satisfy triangle g's band and wedge?
bool grid_reach(const GridTri& g, const double c[3], double rho) {
    const double dn = g.n[0] * c[0] + g.n[1] * c[1] + g.n[2] * c[2];
    if (std::fabs(dn) > g.band + rho * g.nn + 1e-12) return false;
    const double da = g.ea[0] * c[0] + g.ea[1] * c[1] + g.ea[2] * c[2];
    if (da < -(g.wa + rho * g.na)) return false;
    const double db = g.eb[0] * c[0] + g.eb[1] * c[1] + g.eb[2] * c[2];
    return !(db < -(g.wb + rho * g.nb));
}

}  // namespace

void oct_node_centre(int level, int i, int j, double out[3]) {
    const double side = 2.0 / (double)(1 << level);
    oct_decode(-1.0 + (i + 0.5) * side, -1.0 + (j + 0.5) * side, out);
}

// node radius (chord) of a map square of side 2/2^level, centre decoded
double oct_node_radius(int level) { return kOctLipschitz * (std::sqrt(0.5) * 2.0 / (double)(1 << level) + 1e-6); }

void build_dir_grid(const rt_prim* prims, BvhBuild& out, int log2_cells) {
    const auto t0 = std::chrono::steady_clock::now();
    out.grid_log2 = 0;
    out.grid_start.clear();
    out.grid_items.clear();
    out.grid_always.clear();
    if (out.far_tris.empty() || log2_cells <= 0) return;
    const int L = log2_cells, M = 1 << L;
    const double S = out.scale;
    constexpr double rmul = 4.0;  // the origin radius, in units of S
    const double R = rmul * S;  // origins on (or 0.2 off) the scene's surfaces; farther ones walk the plane tree
    std::vector<GridTri> gt(out.far_tris.size());
    std::vector<uint8_t> ok(out.far_tris.size());
    for (size_t k = 0; k < out.far_tris.size(); k++) {
        const FarTri& ft = out.far_tris[k];
        ok[k] = prims[ft.id].area > 0.0f && grid_tri(prims[ft.id], ft, R, S, gt[k]);
        if (!ok[k]) out.grid_always.push_back((uint32_t)k);
    }
    auto rho_of = [](int level) { return oct_node_radius(level); };
    unsigned nt = std::thread::hardware_concurrency();
    if (nt < 1) nt = 1;
    if (nt > 16) nt = 16;
    const size_t n = out.far_tris.size(), ncell = (size_t)M * M;
    // two passes over the same deterministic descent: per-thread counts per
    // cell, then each thread fills its slice of every cell (ascending k per cell)
    std::vector<std::vector<uint32_t>> cnt(nt, std::vector<uint32_t>(ncell, 0));
    auto descend = [&](unsigned w, bool fill, std::vector<uint32_t>& cursor) {
        const size_t lo = n * w / nt, hi = n * (w + 1) / nt;
        struct Node { int level, i, j; };
        std::vector<Node> stk;
        for (size_t k = lo; k < hi; k++) {
            if (!ok[k]) continue;
            const GridTri& g = gt[k];
            stk.clear();
            for (int i = 0; i < 2; i++)
                for (int j = 0; j < 2; j++) stk.push_back({1, i, j});
            while (!stk.empty()) {
                const Node nd = stk.back();
                stk.pop_back();
                double c[3];
                oct_node_centre(nd.level, nd.i, nd.j, c);
                if (!grid_reach(g, c, rho_of(nd.level))) continue;
                if (nd.level == L) {
                    const size_t cell = (size_t)nd.i * M + nd.j;
                    if (fill) out.grid_items[cursor[cell]++] = (uint32_t)k;
                    else cnt[w][cell]++;
                    continue;
                }
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++) stk.push_back({nd.level + 1, 2 * nd.i + a, 2 * nd.j + b});
            }
        }
    };
    {
        std::vector<std::thread> th;
        std::vector<uint32_t> none;
        for (unsigned w = 0; w < nt; w++) th.emplace_back([&, w] { std::vector<uint32_t> c; descend(w, false, c); });
        for (auto& t : th) t.join();
    }
    out.grid_start.assign(ncell + 1, 0);
    uint64_t total = 0;
    for (size_t c = 0; c < ncell; c++) {
        out.grid_start[c] = (uint32_t)total;
        for (unsigned w = 0; w < nt; w++) total += cnt[w][c];
        if (total > 0xffffffffull) {  // beyond 32-bit offsets: keep the plane tree
            out.grid_start.clear();
            return;
        }
    }
    out.grid_start[ncell] = (uint32_t)total;
    out.grid_items.assign(total, 0);
    {
        std::vector<std::thread> th;
        for (unsigned w = 0; w < nt; w++)
            th.emplace_back([&, w] {
                std::vector<uint32_t> cursor(ncell);
                for (size_t c = 0; c < ncell; c++) {
                    uint32_t off = out.grid_start[c];
                    for (unsigned v = 0; v < w; v++) off += cnt[v][c];
                    cursor[c] = off;
                }
                descend(w, true, cursor);
            });
        for (auto& t : th) t.join();
    }
    out.grid_log2 = L;
    out.grid_r = (float)R;
    out.grid_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

void coarsen_dir_grid(BvhBuild& out) {
    out.grid2_start.clear();
    out.grid2_items.clear();
    if (out.grid_log2 < 2 || out.grid_start.empty()) return;
    const int L = out.grid_log2, M = 1 << L, Mc = M / 2;
    const size_t nc = (size_t)Mc * Mc;
    unsigned nt = std::thread::hardware_concurrency();
    if (nt < 1) nt = 1;
    if (nt > 16) nt = 16;
    // per thread: a band of coarse rows, its merged lists back to back
    std::vector<std::vector<uint32_t>> items(nt), lens(nt);
    {
        std::vector<std::thread> th;
        for (unsigned w = 0; w < nt; w++)
            th.emplace_back([&, w] {
                const int i0 = (int)((int64_t)Mc * w / nt), i1 = (int)((int64_t)Mc * (w + 1) / nt);
                std::vector<uint32_t> u;
                for (int ic = i0; ic < i1; ic++)
                    for (int jc = 0; jc < Mc; jc++) {
                        u.clear();
                        for (int a = 0; a < 2; a++)
                            for (int b = 0; b < 2; b++) {
                                const size_t c = ((size_t)(2 * ic + a) << L) | (size_t)(2 * jc + b);
                                u.insert(u.end(), out.grid_items.begin() + out.grid_start[c],
                                         out.grid_items.begin() + out.grid_start[c + 1]);
                            }
                        std::sort(u.begin(), u.end());
                        u.erase(std::unique(u.begin(), u.end()), u.end());
                        items[w].insert(items[w].end(), u.begin(), u.end());
                        lens[w].push_back((uint32_t)u.size());
                    }
            });
        for (auto& t : th) t.join();
    }
    out.grid2_start.assign(nc + 1, 0);
    uint64_t total = 0;
    size_t c = 0;
    for (unsigned w = 0; w < nt; w++)
        for (uint32_t n : lens[w]) {
            out.grid2_start[c++] = (uint32_t)total;
            total += n;
        }
    out.grid2_start[nc] = (uint32_t)total;
    out.grid2_items.reserve(total);
    for (unsigned w = 0; w < nt; w++) {
        out.grid2_items.insert(out.grid2_items.end(), items[w].begin(), items[w].end());
        std::vector<uint32_t>().swap(items[w]);
    }
}

}  // namespace rt580

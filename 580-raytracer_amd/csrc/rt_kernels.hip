// rt_kernels.hip — MI355X (gfx950) kernels for the reference's per-pixel path:
//   Render loop (Raytracer.cpp:916-935) -> GenerateRay (:832-858) -> Raycast
//   (:28-129) -> IntersectScene (:473-526) / IntersectTriangle (:348-409) /
//   IntersectSphere (:419-464) / CalculateLocalColor (:213-267) /
//   CalculateAmbientOcclusion (:269-330) / ComputeFresnel (:131-166) /
//   CalculateRefraction (:168-203).
//
// Wavefront organisation of one frame (or one rank's interleaved rows):
//   trace_kernel x (depth+1)  breadth-first over the levels of Raycast's binary
//        recursion tree: level 0 = camera rays, level L+1 = the reflection and
//        refraction children of level L's hits, kept in compacted queues (wave-
//        aggregated atomics). Each tree ray: closest hit, shadow rays, the
//        non-ambient local colour, Fresnel, children -> one NodeRec.
//   row_counts_kernel / row_scan_kernel  AO calls per pixel (hits x ambient
//        lights) -> in-row prefixes, per-row totals, scan over this call's rows.
//   rank_kernel   per pixel: pre-order walk of the pixel's tree numbers its AO
//        calls exactly as the reference's serial RNG consumes them (raster order,
//        then pre-order, then lights) and records each call's RNG position.
//   ao_kernel     flat over (AO call, sample): every lane one hemisphere sample,
//        any-hit against the scene; perfectly balanced (95% of all rays).
//   resolve_kernel per pixel: post-order int16 blend of the tree (the blend is
//        non-linear, so it runs bottom-up after AO is known).
// Scene loops stage primitives in LDS tiles read uniformly by the workgroup.
//
// Bit-exactness rules: -ffp-contract=off; correctly rounded fp32
// division/sqrt (hipcc default); denormals preserved; glibc powf/sincos restated
// in rt_libm.h; double precision only where the reference uses double.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <hipcub/hipcub.hpp>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/rt580.h"
#include "rt_kernels.h"
#include "rt_mt.h"
#include "rt_isect.h"
#include "rt_libm.h"
#include "rt_math.h"

namespace rt580 {

#define TB 256    // threads per workgroup (4 waves)
#define TILE 64   // primitives per LDS tile (4 KiB)
#define NEAR_LDS 16  // traversal-stack entries per lane in LDS (trace_kernel's near phases)
#define LVL_BASE (RT_MAX_DEPTH + 2)

// A frame whose replayed count differed from its own (count_check_kernel set
// the slot's check word, DevWork::poison). Launches enqueued after a replayed
// count are sized by it; every kernel of a BVH frame that such a launch can
// reach returns at entry once the word is set, so a wrong count (and the stale
// queue entries it would cover) is never used to index anything. The word is
// uniform over the grid: the whole launch returns. The call ends as RT_FAILURE
// (rt_shim.cpp check_replay).
__device__ __forceinline__ bool frame_poisoned(const DevWork& W) {
    return W.poison != nullptr && __builtin_expect(*W.poison != 0u, 0);
}

// ---------------------------------------------------------------- RNG
// minstd_rand0: x' = 16807 x mod (2^31-1), seed 1 (libstdc++ default_random_engine).
__device__ __forceinline__ uint32_t mersenne31_mul(uint32_t a, uint32_t b) {
    uint64_t p = (uint64_t)a * (uint64_t)b;       // < 2^62
    uint64_t r = (p & 0x7fffffffull) + (p >> 31);  // < 2^32
    r = (r & 0x7fffffffull) + (r >> 31);           // <= 2^31
    uint32_t v = (uint32_t)r;
    return v >= 0x7fffffffu ? v - 0x7fffffffu : v;
}

__constant__ uint32_t c_minstd_j1[512];    // 16807^(2s+1) mod m: state offset of sample s's first draw


// generate_canonical<float,24> (libstdc++ random.tcc:3348-3378) for one draw.
__device__ __forceinline__ float canon_minstd(uint32_t x) {  // r = 2^31-2 -> tmp = 2^31 (float)
    float r = (float)(x - 1u) / 2147483648.0f;
    return r >= 1.0f ? 0x1.fffffep-1f : r;
}
__device__ __forceinline__ float canon_mt(uint32_t x) {      // r = 2^32
    float r = (float)x / 4294967296.0f;
    return r >= 1.0f ? 0x1.fffffep-1f : r;
}

// ---------------------------------------------------------------- scene queries
// Hit, tri_test, sph_test and the BVH queries (bvh_closest / bvh_any) live in
// rt_isect.h, shared with the host-side BVH checker.

// Stage primitives [base, base+n) in LDS (every thread of the workgroup calls it).
__device__ __forceinline__ void load_tile(const rt_prim* __restrict__ prims, int base, int n, rt_prim* tile) {
    const float4* src = reinterpret_cast<const float4*>(prims + base);
    float4* dst = reinterpret_cast<float4*>(tile);
    for (int i = threadIdx.x; i < n * 4; i += blockDim.x) dst[i] = src[i];
}

// IntersectScene, closest hit (Raytracer.cpp:473-526): primitives in the
// reference's order; the first hit is taken unconditionally, later ones only if
// strictly closer. Workgroup-uniform call; `active` lanes test.
// With resident == true the whole scene (<= TILE primitives) is already in the
// tile and no barrier is needed.
__device__ bool closest_hit(const DevScene& S, rt_prim* tile, bool resident, bool active, rv3 o, rv3 d, Hit& h) {
    bool found = false;
    for (int base = 0; base < S.n_prims; base += TILE) {
        const int n = min(TILE, S.n_prims - base);
        if (!resident) {
            __syncthreads();
            load_tile(S.prims, base, n, tile);
            __syncthreads();
        }
        if (active) {
            for (int j = 0; j < n; j++) {
                const rt_prim& P = tile[j];
                float t, a = 0, b = 0, g = 0;
                bool hit = P.kind == RT_PRIM_TRIANGLE ? tri_test<true>(P, o, d, t, a, b, g, found ? h.t : INFINITY)
                                                      : sph_test(P, o, d, t);
                if (hit && (!found || t < h.t)) {
                    found = true;
                    h.t = t; h.a = a; h.b = b; h.g = g; h.prim = base + j;
                }
            }
        }
    }
    return found;
}

// IntersectScene where only the boolean is read (directional shadows, AO rays):
// any hit, with a workgroup-wide early exit once every active lane has hit.
template <bool SIGN = false>
__device__ bool any_hit(const DevScene& S, rt_prim* tile, bool resident, bool active, rv3 o, rv3 d) {
    bool hit = false;
    for (int base = 0; base < S.n_prims; base += TILE) {
        const int n = min(TILE, S.n_prims - base);
        if (!resident) {
            __syncthreads();
            load_tile(S.prims, base, n, tile);
            __syncthreads();
        }
        if (active && !hit) {
            for (int j = 0; j < n; j++) {
                const rt_prim& P = tile[j];
                float t, a, b, g;
                if (P.kind == RT_PRIM_TRIANGLE ? tri_test<false, SIGN>(P, o, d, t, a, b, g) : sph_test(P, o, d, t)) {
                    hit = true;
                    break;
                }
            }
        }
        if (base + TILE < S.n_prims && __syncthreads_and(!active || hit)) break;
    }
    return hit;
}

// Scene records read through the constant address space: with a wave-uniform
// index the compiler emits s_load (primitive fields land in SGPRs and every
// per-primitive branch is uniform; the scalar cache holds small scenes).
typedef const uint32_t __attribute__((address_space(4)))* cu32_ptr;

__device__ __forceinline__ rt_prim load_prim_scalar(const rt_prim* prims, int j) {
    const cu32_ptr src = (cu32_ptr)(prims + j);
    rt_prim P;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&P);
#pragma unroll
    for (int k = 0; k < 16; k++) dst[k] = src[k];
    return P;
}

template <bool SIGN = false>
__device__ bool closest_hit_scalar(const DevScene& S, bool active, rv3 o, rv3 d, Hit& h) {
    bool found = false;
    for (int j = 0; j < S.n_prims; j++) {
        const rt_prim P = load_prim_scalar(S.prims, j);
        float t, a = 0, b = 0, g = 0;
        const bool hit = active && (P.kind == RT_PRIM_TRIANGLE
                                        ? tri_test<true, SIGN>(P, o, d, t, a, b, g, found ? h.t : INFINITY)
                                        : sph_test(P, o, d, t));
        if (hit && (!found || t < h.t)) {
            found = true;
            h.t = t; h.a = a; h.b = b; h.g = g; h.prim = j;
        }
    }
    return found;
}

template <bool SIGN = false>
__device__ bool any_hit_scalar(const DevScene& S, bool active, rv3 o, rv3 d) {
    bool hit = !active;
    for (int j = 0; j < S.n_prims; j++) {
        const rt_prim P = load_prim_scalar(S.prims, j);
        float t, a, b, g;
        if (!hit) hit = P.kind == RT_PRIM_TRIANGLE ? tri_test<false, SIGN>(P, o, d, t, a, b, g) : sph_test(P, o, d, t);
        if (__builtin_amdgcn_read_exec() == __ballot(hit)) break;  // every lane of the wave done
    }
    return active && hit;
}

// any_hit_scalar for two rays per lane: each primitive is loaded once for
// both; both tests run unconditionally (straight-line code the compiler can
// interleave; an any-hit answer is the OR over the primitives, so testing a ray
// already hit changes nothing). Early exit once every lane has both answers.
template <bool SIGN = false>
__device__ void any_hit_scalar2(const DevScene& S, bool a0, rv3 o0, rv3 d0, bool a1, rv3 o1, rv3 d1, bool& h0,
                                bool& h1) {
    bool x0 = !a0, x1 = !a1;
    for (int j = 0; j < S.n_prims; j++) {
        const rt_prim P = load_prim_scalar(S.prims, j);
        float t0, t1, a, b, g;
        if (P.kind == RT_PRIM_TRIANGLE) {
            const bool y0 = tri_test<false, SIGN>(P, o0, d0, t0, a, b, g);
            const bool y1 = tri_test<false, SIGN>(P, o1, d1, t1, a, b, g);
            x0 = x0 || y0;
            x1 = x1 || y1;
        } else {
            const bool y0 = sph_test(P, o0, d0, t0);
            const bool y1 = sph_test(P, o1, d1, t1);
            x0 = x0 || y0;
            x1 = x1 || y1;
        }
        if (__builtin_amdgcn_read_exec() == __ballot(x0 && x1)) break;  // every lane of the wave done
    }
    h0 = a0 && x0;
    h1 = a1 && x1;
}

// Small scenes (<= TILE primitives) are staged once per workgroup and stay resident.
__device__ __forceinline__ bool stage_resident(const DevScene& S, rt_prim* tile) {
    const bool resident = S.n_prims <= TILE;
    if (resident) {
        load_tile(S.prims, 0, S.n_prims, tile);
        __syncthreads();
    }
    return resident;
}

// ---------------------------------------------------------------- camera
// GenerateRay (Raytracer.cpp:832-858): double NDC, no +0.5 pixel centre.
__device__ __forceinline__ void generate_ray(const DevFrame& F, int x, int y, rv3& o, rv3& d) {
    double ndcx = (2.0 * x) / F.width - 1;
    double ndcy = 1 - (2.0 * y) / F.height;
    ndcx *= F.ndc_kx;
    ndcy *= F.ndc_ky;
    o = v3(F.cam_from[0], F.cam_from[1], F.cam_from[2]);
    rv3 dir = v3((float)ndcx, (float)ndcy, -1.0f);
    if (F.view_inverse_ok) {
        const float* m = F.view_inv;
        d = v3_normalize(v3(m[0] * dir.x + m[1] * dir.y + m[2] * dir.z,
                            m[3] * dir.x + m[4] * dir.y + m[5] * dir.z,
                            m[6] * dir.x + m[7] * dir.y + m[8] * dir.z));
    } else {
        d = v3(0, 0, 0);  // the reference leaves the direction zeroed (:854-857)
    }
}

// ---------------------------------------------------------------- shading
struct HitInfo {
    rv3 p, n;  // world hit point, geometric normal (hitInfo.normal)
    int prim, kind;
    float a, b, g;
};

__device__ __forceinline__ void resolve_hit(const DevScene& S, rv3 o, rv3 d, const Hit& h, HitInfo& hi) {
    const rt_prim P = S.prims[h.prim];
    hi.p = v3_add(o, v3_scale(d, h.t));
    hi.prim = h.prim;
    hi.kind = P.kind;
    hi.a = h.a; hi.b = h.b; hi.g = h.g;
    if (P.kind == RT_PRIM_TRIANGLE) hi.n = ld3(S.shade[h.prim].hit_nrm);
    else hi.n = v3_normalize(v3_sub(hi.p, ld3(P.p0)));
}

// CalculateLocalColor (Raytracer.cpp:213-267); L is the normalized to-light vector.
__device__ rpix local_color(const DevScene& S, const DevFrame& F, const HitInfo& h, const rt_light& l,
                            const rt_material& m, rv3 L) {
    rv3 n;
    if (h.kind == RT_PRIM_TRIANGLE) {
        const rt_prim_shade& sh = S.shade[h.prim];
        rv3 in = v3_add(v3_add(v3_scale(ld3(sh.vn0), h.a), v3_scale(ld3(sh.vn1), h.b)), v3_scale(ld3(sh.vn2), h.g));
        n = v3_normalize(v3_normalize(in));  // InterpolateVector3 (:333-338) + :237
    } else {
        n = v3_normalize(h.n);
    }
    rv3 lc = ld3(l.color);
    float ds = rt_fmax0(v3_dot(L, n));
    rv3 diffuse = v3_scale(v3_scale(lc, ds), l.intensity);
    rv3 R = v3_normalize(v3_reflect(L, n));
    rv3 V = v3_normalize(v3_sub(v3(F.cam_from[0], F.cam_from[1], F.cam_from[2]), h.p));
    float ss = rt_fmax0(v3_dot(V, R));
    ss = rt_glibc_powf(ss, m.spec_exp);
    rv3 spec = v3_scale(v3_scale(lc, ss), l.intensity);
    rv3 lighting = v3_add(v3_scale(diffuse, m.kd), v3_scale(spec, m.ks));
    rv3 col = v3_mul(ld3(m.cs), lighting);
    col.x = rt_clipf(col.x, 0.0f, 1.0f);
    col.y = rt_clipf(col.y, 0.0f, 1.0f);
    col.z = rt_clipf(col.z, 0.0f, 1.0f);
    return px_from(col);
}

// CalculateRefraction (Raytracer.cpp:168-203)
__device__ __forceinline__ rv3 refraction_dir(rv3 I, rv3 N, float ior) {
    float cosi = v3_dot(I, N);
    if (cosi < -1) cosi = -1;
    else if (cosi > 1) cosi = 1;
    float n1 = 1, n2 = ior;
    rv3 n = N;
    if (cosi < 0) {
        cosi = -1 * cosi;
    } else {
        float t = n1; n1 = n2; n2 = t;
        n = v3_neg(N);
    }
    float eta = n1 / n2;
    float k = 1 - eta * eta * (1 - cosi * cosi);
    if (k < 0) return v3(0, 0, 0);
    return v3_add(v3_scale(I, eta), v3_scale(n, (eta * cosi - sqrtf(k))));
}

// ComputeFresnel (Raytracer.cpp:131-166)
__device__ __forceinline__ void fresnel(float ior, rv3 N, rv3 I, float& kr, float& kt) {
    float cosi = rt_clipf(v3_dot(I, N), -1.0f, 1.0f);
    bool inside = cosi > 0;
    float ei = 1, et = ior;
    if (inside) { float t = ei; ei = et; et = t; cosi = -cosi; }
    float s = 1 - cosi * cosi;
    float sint = ei / et * sqrtf(0.f < s ? s : 0.f);
    if (sint >= 1) {
        kr = 1; kt = 0;
    } else {
        float s2 = 1 - sint * sint;
        float cost = sqrtf(0.f < s2 ? s2 : 0.f);
        cosi = fabsf(cosi);
        float Rs = ((et * cosi) - (ei * cost)) / ((et * cosi) + (ei * cost));
        float Rp = ((ei * cosi) - (et * cost)) / ((ei * cosi) + (et * cost));
        kr = (Rs * Rs + Rp * Rp) / 2;
        kt = 1 - kr;
    }
}

// Raycast's blend (Raytracer.cpp:114-128)
__device__ __forceinline__ rpix combine(rpix local, rpix refl, rpix refr, float kr, float kt, float ks, float ktm) {
    rpix fR = px_mul(px_mul(refl, kr), ks);
    rpix fT = px_mul(px_mul(refr, kt), ktm);
    float alb = 1 - ks - ktm;
    alb = alb > 0.0f ? alb : 0.0f;  // std::max(alb, 0.0f)
    return px_clamp(px_add(px_add(px_mul(local, alb), px_mul(fR, ks)), px_mul(fT, ktm)));
}

// ---------------------------------------------------------------- wave utilities
__device__ __forceinline__ uint64_t lanemask_lt() {
    const int lane = threadIdx.x & 63;
    return lane ? (~0ull >> (64 - lane)) : 0ull;
}

// Allocate one slot per set flag (two flags per lane) from *counter, one atomic per wave.
__device__ __forceinline__ void wave_alloc2(uint32_t* counter, bool fa, bool fb, uint32_t& sa, uint32_t& sb) {
    const uint64_t ma = __ballot(fa), mb = __ballot(fb);
    const uint32_t na = (uint32_t)__popcll(ma), nb = (uint32_t)__popcll(mb);
    const uint64_t active = __ballot(1);
    const int leader = __ffsll((unsigned long long)active) - 1;
    uint32_t base = 0;
    if ((threadIdx.x & 63) == leader && na + nb) base = atomicAdd(counter, na + nb);
    base = __shfl(base, leader);
    const uint64_t lt = lanemask_lt();
    sa = base + (uint32_t)__popcll(ma & lt);
    sb = base + na + (uint32_t)__popcll(mb & lt);
}

// Same, one atomic per workgroup: the waves' totals meet in LDS (every thread
// of the block must call it, in the same iteration).
__device__ __forceinline__ void block_alloc2(uint32_t* counter, bool fa, bool fb, uint32_t& sa, uint32_t& sb) {
    __shared__ uint32_t wtot[TB / 64 + 1];
    const uint64_t ma = __ballot(fa), mb = __ballot(fb);
    const uint32_t na = (uint32_t)__popcll(ma), nb = (uint32_t)__popcll(mb);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane == 0) wtot[wave] = na + nb;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t sum = 0;
        for (int w = 0; w < TB / 64; w++) {
            const uint32_t c = wtot[w];
            wtot[w] = sum;
            sum += c;
        }
        wtot[TB / 64] = sum ? atomicAdd(counter, sum) : 0u;
    }
    __syncthreads();
    const uint32_t base = wtot[TB / 64] + wtot[wave];
    __syncthreads();  // wtot is reused by the next call
    const uint64_t lt = lanemask_lt();
    sa = base + (uint32_t)__popcll(ma & lt);
    sb = base + na + (uint32_t)__popcll(mb & lt);
}

// Sort keys of the far-hit queues (grouping only; never affects a result):
// grid-origin rays: their direction-grid cell (< 2^24, rt_isect.h grid_cell,
// scaled to 24 bits); plane-tree rays: RT_KEY_TREE | a 12 + 12-bit octahedral
// direction key; far-origin rays (brute scan): RT_KEY_BRUTE, sorted last.
#define RT_DIR_KEY_BITS 26
#define RT_KEY_TREE (1u << 24)
#define RT_KEY_BRUTE (1u << 25)

// Rays whose origin is so far out (a child of one of the reference's far hits)
// that a typical triangle cannot be culled (T <= 0) or the fat-ray margin
// covers the scene: the reference's own loop over every primitive
// (far_scan_kernel) is cheaper than any traversal for them. Routing only; the
// results are the same.
__device__ __forceinline__ bool far_origin(const DevScene& S, rv3 o) {
    const float oi = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
    return oi > 64.0f * S.bv.scale || !(far_T(far_ray(S.bv, o), 0.5f * S.bv.dhi_median) > 0.0f);
}
__device__ __forceinline__ uint32_t dir_key(rv3 d);
// Sort key of a far-pass ray: its direction-grid cell (rays of one cell are
// then contiguous: one candidate list serves them all) when the origin uses
// the grid, else RT_KEY_TREE | the 4096^2 direction key. Below RT_KEY_BRUTE.
__device__ __forceinline__ uint32_t far_key(const BvhView& V, rv3 o, rv3 d) {
    if (grid_origin(V, o)) return grid_cell(d, V.grid_log2) << (24 - 2 * V.grid_log2);
    return RT_KEY_TREE | dir_key(d);
}
// false: a grid-origin ray whose direction-grid cell lists no candidate (and
// the scene has no always-tested plane) -- it cannot have a far hit, and the
// far pass would only find that out after sorting it (routing only: an any-hit
// ray that skips the far queue stays a miss, as it would there)
// The cell's bit in a bitmap of the non-empty cells (512 KB for 2048^2 cells:
// L2-resident) rather than its two offsets (16.8 MB of grid_start: one fabric
// line per AO miss, ~60 of round 5's 273 bytes per AO ray).
__device__ __forceinline__ bool far_live(const BvhView& V, rv3 o, rv3 d) {
    if (V.n_always > 0 || !grid_origin(V, o)) return true;
    const uint32_t cell = grid_cell(d, V.grid_log2);
    return (V.grid_live[cell >> 5] >> (cell & 31u)) & 1u;
}
__device__ __forceinline__ uint32_t dir_key(rv3 d) {
    const float s = fabsf(d.x) + fabsf(d.y) + fabsf(d.z);
    float x = d.x / s, y = d.y / s;
    if (d.z < 0.0f) {
        const float ax = fabsf(x), ay = fabsf(y);
        x = (1.0f - ay) * (x < 0.0f ? -1.0f : 1.0f);
        y = (1.0f - ax) * (y < 0.0f ? -1.0f : 1.0f);
    }
    const uint32_t u = (uint32_t)fminf(fmaxf((x * 0.5f + 0.5f) * 4095.0f, 0.0f), 4095.0f);
    const uint32_t v = (uint32_t)fminf(fmaxf((y * 0.5f + 0.5f) * 4095.0f, 0.0f), 4095.0f);
    return (u << 12) | v;
}

// Wave-uniform loads of the plane tree (the node index is uniform: every lane
// of the wave walks the same node sequence).
__device__ __forceinline__ FarNode load_far_node(const FarNode* nodes, int j) {
    const cu32_ptr src = (cu32_ptr)(nodes + j);
    FarNode n;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&n);
#pragma unroll
    for (int k = 0; k < 12; k++) dst[k] = src[k];
    return n;
}
__device__ __forceinline__ FarTri load_far_tri(const FarTri* tris, int j) {
    const cu32_ptr src = (cu32_ptr)(tris + j);
    FarTri t;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&t);
#pragma unroll
    for (int k = 0; k < 8; k++) dst[k] = src[k];
    return t;
}

// ---------------------------------------------------------------- trace (one tree level)
__device__ __forceinline__ int pixel_frame_row(const DevFrame& F, int lr) { return F.row_begin + lr * F.row_step; }

// PHASE 0: the whole level in one pass (brute force, or BVH without sorted far
// pass). BVH scenes with a plane tree split it: PHASE 1 = near closest hit,
// provisional hit stored per node and rays that may still have a far hit
// queued (sorted far_closest_kernel in between); PHASE 3 = the shadow ray of
// directional light `light` (its index among the directional lights: `dl`):
// near any-hit, the undecided rays queued for the sorted far pass, flags in
// W.shadow; PHASE 2 = shading from the stored hit and shadow flags. Items
// [i0, i1) of the level.
// SCALAR (small brute-force scenes): wave-uniform scalar scene loads and the
// division-free sign rejections (tri_test<SIGN>) instead of the LDS tile.

template <int HOLD2, bool BOUND, class STK>
__device__ int bvh4_any_spec_budget_state(const BvhView& V, rv3 o, rv3 d, const STK& stk, int budget, bool live,
                                          int& sp, int32_t& c, int32_t& n, float tmax = INFINITY);

// PHASE 3 (shadow rays) walks the 4-wide tree in speculative while-while form
// (bvh4_any_spec_budget_state, the whole wave; profiles/r05/ab/trace_spec.txt:
// 283.5 -> 271.9 us per launch on the north-star frame, 451 -> 404 us on
// Cornell). The closest-hit walk of PHASE 1 stays per lane: its speculative
// form was slower (392 -> 526 us), its descents running with the bound of
// before the held leaf's test, which is what prunes most of the tree.
template <bool BVH, int PHASE, bool SCALAR = false>
__global__ void __launch_bounds__(TB) trace_kernel(DevScene S, DevFrame F, DevWork W, int level, uint32_t i0,
                                                   uint32_t i1, int light = 0, int dl = 0) {
    if (BVH && frame_poisoned(W)) return;
    __shared__ rt_prim tile[TILE];
    // the near queries' traversal stacks (4-wide tree): the first NEAR_LDS
    // entries of each lane in LDS, one column per lane (PHASE 1: node links
    // and entry distances; PHASE 3: node links), the rest in scratch
    constexpr int NL = (BVH && (PHASE == 1 || PHASE == 3)) ? NEAR_LDS : 1;
    __shared__ uint32_t nstk[NL][TB];
    __shared__ uint32_t ntstk[PHASE == 1 && BVH ? NEAR_LDS : 1][TB];
    const uint32_t npix = (uint32_t)F.n_rows * (uint32_t)F.width;
    const uint32_t base_id = level == 0 ? 0u : W.lvl[LVL_BASE + level];
    // Children beyond the node capacity were not stored (the frame is re-rendered
    // with a larger capacity, rt_shim.cpp check_capacity): never touch their ids.
    const uint32_t room = W.node_cap > base_id ? W.node_cap - base_id : 0u;
    const uint32_t count_req = level == 0 ? npix : W.lvl[level];
    const uint32_t count_all = count_req < room ? count_req : room;
    const uint32_t count = i1 < count_all ? i1 : count_all;
    const uint32_t next_base = base_id + count_all;
    if (blockIdx.x == 0 && threadIdx.x == 0) W.lvl[LVL_BASE + level + 1] = next_base;
    const int bounces = F.depth - level;
    const bool resident = (BVH || SCALAR) ? false : stage_resident(S, tile);

    for (uint32_t b0 = i0 + blockIdx.x * TB; b0 < count; b0 += gridDim.x * TB) {
        const uint32_t item = b0 + threadIdx.x;
        const bool active = item < count;
        const uint32_t node = base_id + item;
        rv3 o = v3(0, 0, 0), d = v3(0, 0, 0);
        int pixel = 0;
        if (active) {
            if (level == 0) {
                pixel = (int)item;
                const int lr = pixel / F.width;
                generate_ray(F, pixel - lr * F.width, pixel_frame_row(F, lr), o, d);
            } else {
                const RayItem r = W.rays[node];
                o = v3(r.o[0], r.o[1], r.o[2]);
                d = v3(r.d[0], r.d[1], r.d[2]);
                pixel = r.pixel;
            }
        }
        Hit h;
        h.t = 0; h.prim = 0;
        if (PHASE == 1) {
            const FarNode root = load_far_node(S.bv.far_nodes, 0);
            const bool brute = active && far_origin(S, o);
            bool nh = false;
            if (active && !brute) {
                if (S.bv.nodes4) {
                    uint32_t sa[RT_BVH_STACK + 4 - NEAR_LDS], ta[RT_BVH_STACK + 4 - NEAR_LDS];
                    nh = bvh4_closest_near_s(S.bv, o, d, h, LdsStack<NEAR_LDS, TB>{&nstk[0][threadIdx.x], sa},
                                             LdsStack<NEAR_LDS, TB>{&ntstk[0][threadIdx.x], ta});
                } else {
                    nh = bvh_closest_near(S.bv, o, d, h);
                }
            }
            bool q = false;
            if (active) {
                W.hit4[node] = make_float4(h.t, h.a, h.b, h.g);
                W.hit_prim[node] = nh ? h.prim : -1;
                q = brute || (!dir_zero(d) && !(nh && h.t < far_T(far_ray(S.bv, o), root.min_dhi)) &&
                              far_live(S.bv, o, d));
            }
            const uint64_t bm = __ballot(brute);
            if (bm && (threadIdx.x & 63) == 0) atomicAdd(W.far_count + 1, (uint32_t)__popcll(bm));
            const uint64_t qm = __ballot(q);
            if (qm) {
                const int leader = __ffsll((unsigned long long)qm) - 1;
                uint32_t qb = 0;
                if ((threadIdx.x & 63) == leader) qb = atomicAdd(W.far_count, (uint32_t)__popcll(qm));
                qb = __shfl(qb, leader);
                if (q) {
                    const uint32_t slot = qb + (uint32_t)__popcll(qm & lanemask_lt());
                    W.far_rays[2 * (size_t)slot] = make_float4(o.x, o.y, o.z, __uint_as_float(node));
                    W.far_rays[2 * (size_t)slot + 1] = make_float4(d.x, d.y, d.z, 0.0f);
                    W.far_keys[slot] = brute ? RT_KEY_BRUTE : far_key(S.bv, o, d);
                    W.far_vals[slot] = slot;
                }
            }
            continue;
        }
        if (PHASE == 3) {
            // the shadow ray of the shading phase (Raytracer.cpp:59-75), same
            // float operations as below: hit point o + d t, origin hp + L * 0.2.
            // Directional: occluded iff any hit. Point: iff the closest hit has
            // !(t > dist), i.e. some hit has !(t > dist) (tmax); a far hit
            // (t >= T, rt_bvh.h) cannot have t <= dist unless dist >= T, and
            // those rare rays go to the brute scan, which applies the bound.
            bool q = false, brute = false, lit = false;
            uint8_t flag = 0;
            rv3 so = v3(0, 0, 0), L2 = v3(1, 0, 0);
            float tmax = INFINITY;
            if (active && W.hit_prim[node] >= 0) {
                const float t = W.hit4[node].x;
                const rt_light l = S.lights[light];
                const rv3 hp = v3_add(o, v3_scale(d, t));
                rv3 L;
                if (l.kind == RT_LIGHT_DIRECTIONAL) {
                    L = ld3(l.L);
                    L2 = ld3(l.L2);
                } else {
                    const rv3 tl = v3_sub(ld3(l.position), hp);
                    L = v3_normalize(tl);
                    L2 = v3_normalize(L);
                    tmax = v3_length(tl);
                }
                so = v3_add(hp, v3_scale(L, 0.2f));
                brute = far_origin(S, so);
                if (!brute && l.kind != RT_LIGHT_DIRECTIONAL) {
                    const FarNode root = load_far_node(S.bv.far_nodes, 0);
                    brute = !(tmax < far_T(far_ray(S.bv, so), root.min_dhi));
                }
                lit = true;
            }
            bool nh;
            if (S.bv.nodes4) {  // the whole wave walks (speculative form)
                uint32_t sa[RT_BVH_STACK + 4 - NEAR_LDS];
                int ssp = 0;
                int32_t sc = 0, sn = 0;
                nh = bvh4_any_spec_budget_state<0, true>(S.bv, so, L2, LdsStack<NEAR_LDS, TB>{&nstk[0][threadIdx.x], sa},
                                                         1 << 30, lit && !brute, ssp, sc, sn, tmax) > 0;
            } else {
                nh = lit && !brute && bvh_any_near(S.bv, so, L2, tmax);
            }
            if (nh) flag = 1;
            else q = lit && (brute || (!dir_zero(L2) && isinf(tmax) && far_live(S.bv, so, L2)));
            if (active) W.shadow[(size_t)dl * W.far_cap + (item - i0)] = flag;
            const uint64_t bm = __ballot(brute);
            if (bm && (threadIdx.x & 63) == 0) atomicAdd(W.far_count + 1, (uint32_t)__popcll(bm));
            const uint64_t qm = __ballot(q);
            if (qm) {
                const int leader = __ffsll((unsigned long long)qm) - 1;
                uint32_t qb = 0;
                if ((threadIdx.x & 63) == leader) qb = atomicAdd(W.far_count, (uint32_t)__popcll(qm));
                qb = __shfl(qb, leader);
                if (q) {
                    const uint32_t slot = qb + (uint32_t)__popcll(qm & lanemask_lt());
                    W.far_rays[2 * (size_t)slot] = make_float4(so.x, so.y, so.z, __uint_as_float(item - i0));
                    W.far_rays[2 * (size_t)slot + 1] = make_float4(L2.x, L2.y, L2.z, tmax);
                    W.far_keys[slot] = brute ? RT_KEY_BRUTE : far_key(S.bv, so, L2);
                    W.far_vals[slot] = slot;
                }
            }
            continue;
        }
        bool hit;
        if (PHASE == 2) {
            hit = false;
            if (active) {
                const int32_t hp = W.hit_prim[node];
                const float4 hv = W.hit4[node];
                hit = hp >= 0;
                h.t = hv.x; h.a = hv.y; h.b = hv.z; h.g = hv.w; h.prim = hp;
            }
        } else {
            hit = BVH ? (active && bvh_closest(S.bv, o, d, h))
                      : SCALAR ? closest_hit_scalar<true>(S, active, o, d, h)
                               : closest_hit(S, tile, resident, active, o, d, h);
        }

        HitInfo hi;
        rt_material m;
        hi.p = hi.n = v3(0, 0, 0);
        hi.kind = 0;
        m.ks = m.kt = 0.0f;
        m.ior = 2.5f;
        int shape = 0;
        if (hit) {
            resolve_hit(S, o, d, h, hi);
            shape = S.prims[h.prim].shape;
            m = S.mats[shape];
        }
        // Raycast's light loop (Raytracer.cpp:39-82) without the ambient terms
        // (those need AO; int16 wrap-around addition commutes, so they are added
        // in resolve_kernel).
        rpix local = px(0, 0, 0);
        int dli = 0;  // index among the shadow-casting lights
        for (int li = 0; li < S.n_lights; li++) {
            const rt_light l = S.lights[li];
            if (l.kind == RT_LIGHT_AMBIENT) continue;
            rv3 L = v3(0, 0, 0), L2 = v3(0, 0, 0), so = v3(0, 0, 0);
            float dist = 0.0f;
            if (hit) {
                if (l.kind == RT_LIGHT_DIRECTIONAL) {
                    L = ld3(l.L);
                    L2 = ld3(l.L2);
                } else {
                    rv3 tl = v3_sub(ld3(l.position), hi.p);
                    L = v3_normalize(tl);
                    L2 = v3_normalize(L);
                    dist = v3_length(tl);
                }
                so = v3_add(hi.p, v3_scale(L, 0.2f));
            }
            bool occluded;
            if (PHASE == 2 && W.shadow) {
                occluded = hit && W.shadow[(size_t)dli * W.far_cap + (item - i0)] != 0;  // decided by PHASE 3
                dli++;
            } else if (l.kind == RT_LIGHT_DIRECTIONAL) {
                occluded = BVH ? (hit && bvh_any(S.bv, so, L2))
                               : SCALAR ? any_hit_scalar<true>(S, hit, so, L2)
                                        : any_hit(S, tile, resident, hit, so, L2);
            } else {
                Hit sh;
                sh.t = 0;
                const bool shit = BVH ? (hit && bvh_closest(S.bv, so, L2, sh))
                                  : SCALAR ? closest_hit_scalar<true>(S, hit, so, L2, sh)
                                           : closest_hit(S, tile, resident, hit, so, L2, sh);
                occluded = shit && !(sh.t > dist);
            }
            if (hit && !occluded) local = px_add(local, local_color(S, F, hi, l, m, L));
        }
        // children (Raytracer.cpp:87-112)
        bool want_refl = false, want_refr = false;
        RayItem crefl, crefr;
        float kr = 0.0f, kt = 0.0f;
        if (hit && bounces > 0) {
            fresnel(m.ior, hi.n, d, kr, kt);
            if (m.ks > 0) {
                rv3 rd = v3_normalize(v3_reflect(d, hi.n));
                rv3 ro = v3_add(hi.p, v3_scale(rd, 0.2f));
                rd = v3_normalize(rd);
                crefl.o[0] = ro.x; crefl.o[1] = ro.y; crefl.o[2] = ro.z;
                crefl.d[0] = rd.x; crefl.d[1] = rd.y; crefl.d[2] = rd.z;
                crefl.pixel = pixel;
                crefl.pad = 0;
                want_refl = true;
            }
            if (m.kt > 0) {
                rv3 td = refraction_dir(d, hi.n, m.ior);
                rv3 to = v3_add(hi.p, v3_scale(td, 0.2f));
                td = v3_normalize(td);
                crefr.o[0] = to.x; crefr.o[1] = to.y; crefr.o[2] = to.z;
                crefr.d[0] = td.x; crefr.d[1] = td.y; crefr.d[2] = td.z;
                crefr.pixel = pixel;
                crefr.pad = 0;
                want_refr = true;
            }
        }
        uint32_t sa, sb;
        block_alloc2(&W.lvl[level + 1], want_refl, want_refr, sa, sb);
        int32_t child0 = -1, child1 = -1;
        if (want_refl) {
            const uint32_t id = next_base + sa;
            if (id < W.node_cap) { W.rays[id] = crefl; child0 = (int32_t)id; }
            else atomicMax(W.needed, id + 1);
        }
        if (want_refr) {
            const uint32_t id = next_base + sb;
            if (id < W.node_cap) { W.rays[id] = crefr; child1 = (int32_t)id; }
            else atomicMax(W.needed, id + 1);
        }
        if (active) {
            NodeRec rec;
            rec.hp[0] = hi.p.x; rec.hp[1] = hi.p.y; rec.hp[2] = hi.p.z;
            rec.n[0] = hi.n.x; rec.n[1] = hi.n.y; rec.n[2] = hi.n.z;
            const int flags = (hit ? RT_NODE_HIT : 0) | (bounces == 0 ? RT_NODE_LEAF : 0);
            rec.local_rg = (int32_t)(((uint32_t)local.r & 0xffffu) | ((uint32_t)local.g << 16));
            rec.local_b_flags = (int32_t)(((uint32_t)local.b & 0xffffu) | ((uint32_t)flags << 16));
            rec.kr = kr;
            rec.kt = kt;
            rec.shape = shape;
            rec.spare = 0;
            W.nodes[node] = rec;
            W.topo[node] = make_int4(child0, child1, flags, 0);
            if (level == 0) {
                W.pix_hits[pixel] = hit ? 1u : 0u;
                W.pix_nodes[pixel] = 1u;
            } else {
                if (hit) atomicAdd(&W.pix_hits[pixel], 1u);
                atomicAdd(&W.pix_nodes[pixel], 1u);
            }
        }
    }
}

// ---------------------------------------------------------------- AO-call bookkeeping
// One workgroup per local row: AO calls per pixel (hits x ambient lights), their
// in-row exclusive prefix, and the row's totals. Each thread takes a run of
// consecutive pixels; the runs' sums are scanned across the wave (shuffles)
// and the workgroup's four waves (LDS), then each run writes its prefixes.
__global__ void __launch_bounds__(TB) row_counts_kernel(DevScene S, DevFrame F, DevWork W) {
    if (frame_poisoned(W)) return;
    __shared__ uint32_t wsum[TB / 64][3];
    const int lr = blockIdx.x;
    const uint32_t off = (uint32_t)lr * (uint32_t)F.width;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int per = (F.width + TB - 1) / TB;
    const int x0 = threadIdx.x * per, x1 = min(x0 + per, F.width);
    const uint32_t na = (uint32_t)S.n_ambient;
    uint32_t calls = 0, hits = 0, nodes = 0;
    for (int x = x0; x < x1; x++) {
        const uint32_t h = W.pix_hits[off + x];
        hits += h;
        calls += h * na;
        nodes += W.pix_nodes[off + x];
    }
    // inclusive scan of calls over the wave; sums of hits and nodes
    uint32_t inc = calls, hs = hits, ns = nodes;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)inc, k);
        if (lane >= k) inc += v;
        hs += (uint32_t)__shfl_xor((int)hs, k);
        ns += (uint32_t)__shfl_xor((int)ns, k);
    }
    if (lane == 63) {
        wsum[wave][0] = inc;
        wsum[wave][1] = hs;
        wsum[wave][2] = ns;
    }
    __syncthreads();
    uint32_t base = 0, tot = 0, th = 0, tn = 0;
#pragma unroll
    for (int w = 0; w < TB / 64; w++) {
        if (w < wave) base += wsum[w][0];
        tot += wsum[w][0];
        th += wsum[w][1];
        tn += wsum[w][2];
    }
    uint32_t acc = base + inc - calls;
    for (int x = x0; x < x1; x++) {
        W.pix_prefix[off + x] = acc;
        acc += W.pix_hits[off + x] * na;
    }
    if (threadIdx.x == 0) {
        W.row_calls[lr] = tot;
        W.row_hits[lr] = th;
        W.row_nodes[lr] = tn;
    }
}

// Exclusive scan of this call's per-row AO calls (one workgroup) + the total.
__global__ void __launch_bounds__(1024) row_scan_kernel(DevFrame F, DevWork W) {
    if (frame_poisoned(W)) return;
    __shared__ uint64_t part[1024];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int b = 0; b < F.n_rows; b += 1024) {
        const int i = b + threadIdx.x;
        const uint64_t v = i < F.n_rows ? W.row_calls[i] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int s = 1; s < 1024; s <<= 1) {
            uint64_t add = threadIdx.x >= s ? part[threadIdx.x - s] : 0;
            __syncthreads();
            part[threadIdx.x] += add;
            __syncthreads();
        }
        if (i < F.n_rows) W.row_base_local[i] = carry + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += part[1023];
        __syncthreads();
    }
    if (threadIdx.x == 0) W.totals[0] = carry;
}

// Per pixel: number the pixel's AO calls in the reference's draw order (pre-order
// of the recursion tree, lights in JSON order) and record each call's RNG position.
__global__ void __launch_bounds__(TB) rank_kernel(DevScene S, DevFrame F, DevWork W,
                                                  const uint64_t* __restrict__ row_base_global) {
    if (frame_poisoned(W)) return;
    const uint32_t npix = (uint32_t)F.n_rows * (uint32_t)F.width;
    const uint32_t p = blockIdx.x * TB + threadIdx.x;
    if (p >= npix || S.n_ambient == 0) return;
    if (W.pix_hits[p] == 0) return;
    const int lr = (int)(p / (uint32_t)F.width);
    const uint64_t lbase = W.row_base_local[lr] + W.pix_prefix[p];
    const uint64_t gbase = (row_base_global ? row_base_global[lr] : W.row_base_local[lr]) + W.pix_prefix[p];
    uint64_t rng = 0;
    const uint32_t step = F.step_pow2[0];
    if (F.rng_engine == RT_RNG_MINSTD_RAND0) {
        // seed * step^gbase (the order of step divides the period 2^31 - 2)
        uint64_t k = gbase < 2147483646ull ? gbase : gbase % 2147483646ull;
        uint32_t st = F.rng_seed;
        for (int i = 0; k; i++, k >>= 1)
            if (k & 1) st = mersenne31_mul(st, F.step_pow2[i]);
        rng = st;
    } else {
        rng = gbase;
    }
    int stack[2 * RT_MAX_DEPTH + 4];
    int sp = 0;
    stack[sp++] = (int)p;
    uint32_t call = (uint32_t)lbase;
    while (sp > 0) {
        const int n = stack[--sp];
        const int4 tp = W.topo[n];  // child[0], child[1], flags
        if (!(tp.z & RT_NODE_HIT)) continue;
        W.node_call0[n] = call;
        for (int a = 0; a < S.n_ambient; a++) {
            W.call_node[call] = (uint32_t)n;
            W.call_rng[call] = rng;
            W.occ[call] = 0;
            call++;
            if (F.rng_engine == RT_RNG_MINSTD_RAND0) rng = mersenne31_mul((uint32_t)rng, step);
            else rng++;
        }
        if (tp.y >= 0) stack[sp++] = tp.y;  // refraction after
        if (tp.x >= 0) stack[sp++] = tp.x;  // reflection first
    }
}

// ---------------------------------------------------------------- AO
// The two draws of sample s of the AO call whose first draw's RNG position is
// rbase (minstd state / mt19937 call index): z's, then the angle's.
__device__ __forceinline__ void ao_draws(const DevFrame& F, const DevWork& W, uint64_t rbase, uint32_t s, float& u0,
                                         float& u1) {
    if (F.rng_engine == RT_RNG_MINSTD_RAND0) {
        uint32_t st = mersenne31_mul((uint32_t)rbase, c_minstd_j1[s]);
        u0 = canon_minstd(st);
        st = mersenne31_mul(st, 16807u);
        u1 = canon_minstd(st);
    } else {
        const uint64_t k = rbase * 2ull * (uint64_t)F.ao_samples + 2ull * s - W.mt_base;
        u0 = canon_mt(W.mt_stream[k]);
        u1 = canon_mt(W.mt_stream[k + 1]);
    }
}

// After an AO ray's any-hit query: BVH scenes queue the near misses for the
// sorted far-hit pass (and count the far-origin rays); hits count towards the
// call's occlusion (W.occ). With N a multiple of 64 a wave holds one call's
// samples (items are aligned chunks), so one atomic per wave.
template <bool BVH>
__device__ __forceinline__ void ao_finish(const DevScene& S, const DevWork& W, uint32_t N, bool active, bool ao_brute,
                                          bool hit, uint64_t c, rv3 o, rv3 d) {
    if (BVH) {
        // rays that miss every near triangle go to the sorted far-hit pass,
        // unless their direction-grid cell is empty
        const bool q = active && !hit && S.bv.has_far && (ao_brute || far_live(S.bv, o, d));
        const uint64_t qm = __ballot(q);
        const uint64_t bm = __ballot(ao_brute);
        if (bm && (threadIdx.x & 63) == 0) atomicAdd(W.far_count + 1, (uint32_t)__popcll(bm));
        if (qm) {
            const int leader = __ffsll((unsigned long long)qm) - 1;
            uint32_t base = 0;
            if ((threadIdx.x & 63) == leader) base = atomicAdd(W.far_count, (uint32_t)__popcll(qm));
            base = __shfl(base, leader);
            if (q) {
                const uint32_t slot = base + (uint32_t)__popcll(qm & lanemask_lt());
                W.far_rays[2 * (size_t)slot] = make_float4(o.x, o.y, o.z, __uint_as_float((uint32_t)c));
                W.far_rays[2 * (size_t)slot + 1] = make_float4(d.x, d.y, d.z, INFINITY);  // .w: t bound
                W.far_keys[slot] = ao_brute ? RT_KEY_BRUTE : far_key(S.bv, o, d);
                W.far_vals[slot] = slot;
            }
        }
    }
    if ((N & 63u) == 0) {
        const uint64_t m = __ballot(active && hit);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(&W.occ[c], (uint32_t)__popcll(m));
    } else if (active && hit) {
        atomicAdd(&W.occ[c], 1u);
    }
}

// CalculateAmbientOcclusion (Raytracer.cpp:315-330) + RandomInHemisphere (:283-292)
// + RandomUnitVector (:269-281): one lane per (call, sample).
// VARIANT bits (A/B switches, results identical): 1 = sincos table in LDS,
// 2 = scalar per-call data (readfirstlane), 4 = sign-decided triangle rejects,
// 8 = scalar (wave-uniform) scene loop, 16 = 8-waves/SIMD register cap,
// 512 = exact BVH queries (triangle scenes; rt_isect.h), 1024 = polynomial
// sincos with exact glibc fallback (rt_ao_dir_xy), 2048 = range-restricted
// sqrt/division sequences for the unit vectors (v3_normalize_unit), 4096 = with
// 1024: samples whose fast rounding test fails are queued (W.aofix_*) for
// ao_fix_kernel instead of running glibc's sincos inline (keeps the rarely
// taken fallback's registers out of the hot loop).
// AO items [item_begin, item_end) (item = call * N + sample).
// One AO sample of ao_body: item -> its call c and the ray (o, d) of
// CalculateAmbientOcclusion's hemisphere sample (RandomInHemisphere /
// RandomUnitVector with the serial RNG's draws); ao_brute: a far-origin ray;
// fix: the fast sincos's rounding test failed (VARIANT & 4096).
template <int VARIANT>
__device__ __forceinline__ void ao_sample(const DevScene& S, const DevFrame& F, const DevWork& W, const double* sct,
                                          uint32_t N, bool pow2, int log2n, bool wave_per_call, uint64_t item,
                                          bool active, uint64_t& c, rv3& o, rv3& d, bool& ao_brute, bool& fix,
                                          rv3& vo, rv3& hpo, uint32_t& so) {
    c = 0;
    uint32_t s = 0;
    vo = v3(0, 0, 0);
    hpo = v3(0, 0, 0);
    if (active) {
        if (pow2) { c = item >> log2n; s = (uint32_t)(item & (N - 1)); }
        else { c = item / N; s = (uint32_t)(item - c * N); }
    }
    o = v3(0, 0, 0);
    d = v3(0, 0, 0);
    ao_brute = false;
    fix = false;  // VARIANT & 4096: this sample goes to ao_fix_kernel
    if (active) {
        // With N a multiple of 64 a wave serves one call: keep its data scalar.
        uint32_t cc = (uint32_t)c;
        if (wave_per_call) cc = __builtin_amdgcn_readfirstlane(cc);
        uint32_t node = W.call_node[cc];
        if (wave_per_call) node = __builtin_amdgcn_readfirstlane(node);
        const NodeRec& nd = W.nodes[node];
        rv3 hp = ld3(nd.hp), n = ld3(nd.n);
        uint64_t rbase = W.call_rng[cc];
        if (wave_per_call) {
            hp = v3(__builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, hp.x))),
                    __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, hp.y))),
                    __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, hp.z))));
            n = v3(__builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, n.x))),
                   __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, n.y))),
                   __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(uint32_t, n.z))));
            rbase = ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(rbase >> 32)) << 32) |
                    __builtin_amdgcn_readfirstlane((uint32_t)rbase);
        }
        float u0, u1;
        ao_draws(F, W, rbase, s, u0, u1);
        // uniform_real_distribution<float>: canonical * (b - a) + a
        const float z = u0 * (1.0f - (-1.0f)) + (-1.0f);
        const float ang = u1 * (F.ao_angle_max - 0.0f) + 0.0f;
        // Ranges for the 2048 sequences (rt_math.h): z is 0 or a multiple of
        // 2^-30 in [-1, 1), so 1 - z*z (float) is +0 or >= 2^-24 and r is 0 or
        // >= 2^-12; |cos|, |sin| of a float angle in [0, 2pi) are 0 or > 2^-27,
        // so v's components are 0 or in [2^-39, 1] and |v| ~ 1 (also after the
        // first normalize).
        const float r = (VARIANT & 2048) ? rt_sqrt_nr(1 - z * z) : sqrtf(1 - z * z);
        rv3 v;
        if (VARIANT & 4096) {
            double sa, ca;
            rt_fast_sincos((double)ang, &sa, &ca);
            const double X = (double)r * ca, Y = (double)r * sa;
            const float fx = (float)X, fy = (float)Y;
            fix = !(rt_f32_round_safe(X, fx) && rt_f32_round_safe(Y, fy));
            v = v3(fx, fy, z);
        } else if (VARIANT & 1024) {
            float vx, vy;
            rt_ao_dir_xy(rt_dev::rt_sincostab, r, ang, &vx, &vy);
            v = v3(vx, vy, z);
        } else {
            double sa, ca;
            rt_glibc_sincos_simd_t(sct, (double)ang, &sa, &ca);
            v = v3((float)((double)r * ca), (float)((double)r * sa), z);
        }
        v = (VARIANT & 2048) ? v3_normalize_unit(v) : v3_normalize(v);
        if (!(v3_dot(v, n) > 0.0f)) v = v3_neg(v);
        o = v3_add(hp, v3_scale(v, 0.2f));
        // Ray constructor (Raytracer.h:431-433)
        d = (VARIANT & 2048) ? v3_normalize_unit(v) : v3_normalize(v);
        if ((VARIANT & 512) && S.bv.has_far) ao_brute = far_origin(S, o);
        vo = v;
        hpo = hp;
    }
    so = s;
}

template <int VARIANT>
__device__ __forceinline__ void ao_body(const DevScene& S, const DevFrame& F, const DevWork& W,
                                        uint64_t item_begin = 0, uint64_t item_end = ~0ull) {
    __shared__ rt_prim tile[TILE];
    __shared__ double sct_lds[440];  // glibc __sincostab, staged once per workgroup
    const double* sct = rt_dev::rt_sincostab;
    if (VARIANT & 1) {
        for (int i = threadIdx.x; i < 440; i += TB) sct_lds[i] = rt_dev::rt_sincostab[i];
        __syncthreads();
        sct = sct_lds;
    }
    const uint32_t N = (uint32_t)F.ao_samples;
    const uint64_t items_all = W.totals[0] * (uint64_t)N;
    const uint64_t items = item_end < items_all ? item_end : items_all;
    const bool pow2 = (N & (N - 1)) == 0;
    const int log2n = 31 - __clz((int)N);
    const bool wave_per_call = (VARIANT & 2) && (N & 63u) == 0;
    const bool resident = (VARIANT & (8 | 512)) ? true : stage_resident(S, tile);
    // VARIANT & 32768: two samples per lane (items b0 + threadIdx.x and
    // b0 + TB + threadIdx.x): the scene loop loads each primitive once for both
    // rays, and the two rays' arithmetic is independent (more work in flight per
    // wave, half the per-sample scalar loads and loop control)
    constexpr int SPL = (VARIANT & 32768) ? 2 : 1;
    for (uint64_t b0 = item_begin + (uint64_t)blockIdx.x * TB * SPL; b0 < items; b0 += (uint64_t)gridDim.x * TB * SPL) {
        bool active[SPL], ao_brute[SPL], fix[SPL], hit[SPL];
        uint64_t c[SPL];
        rv3 o[SPL], d[SPL], vv[SPL], hh[SPL];
        uint32_t ss[SPL];
#pragma unroll
        for (int k = 0; k < SPL; k++) {
            const uint64_t item = b0 + (uint64_t)k * TB + threadIdx.x;
            active[k] = item < items;
            ao_sample<VARIANT>(S, F, W, sct, N, pow2, log2n, wave_per_call, item, active[k], c[k], o[k], d[k],
                               ao_brute[k], fix[k], vv[k], hh[k], ss[k]);
        }
#pragma unroll
        for (int k = 0; k < SPL; k++) {
            const uint64_t item = b0 + (uint64_t)k * TB + threadIdx.x;
            if (VARIANT & 4096) {
                const uint64_t fm = __ballot(fix[k]);
                if (fm) {
                    const int leader = __ffsll((unsigned long long)fm) - 1;
                    uint32_t fb = 0;
                    if ((threadIdx.x & 63) == leader) fb = atomicAdd(W.aofix_count, (uint32_t)__popcll(fm));
                    fb = __shfl(fb, leader);
                    if (fix[k]) {
                        const uint32_t slot = fb + (uint32_t)__popcll(fm & lanemask_lt());
                        if (slot < W.aofix_cap) W.aofix_items[slot] = item;
                        active[k] = false;
                        ao_brute[k] = false;
                    }
                }
            }
            if (VARIANT & 16384) {
                // generation only: the 16-byte ray record for ao_trace_kernel -- the
                // sample's hemisphere vector v and (call - the chunk's first call) |
                // flag << 30 (0: no ray, 1: near query, 2: far origin) -- and the
                // call's hit point once per call (ao_record rebuilds o and d)
                if (item < items) {
                    const uint64_t c0 = item_begin / N;
                    const uint32_t flag = active[k] ? (ao_brute[k] ? 2u : 1u) : 0u;
                    W.ao_rays[item - item_begin] =
                        make_float4(vv[k].x, vv[k].y, vv[k].z, __uint_as_float((uint32_t)(c[k] - c0) | (flag << 30)));
                    if (ss[k] == 0u || item == item_begin)
                        W.ao_hp[c[k] - c0] = make_float4(hh[k].x, hh[k].y, hh[k].z, 0.0f);
                }
            }
        }
        if (VARIANT & 16384) continue;
        if (SPL == 2 && (VARIANT & 8) && !(VARIANT & 512)) {
            any_hit_scalar2<(VARIANT & 4) != 0>(S, active[0], o[0], d[0], active[SPL - 1], o[SPL - 1], d[SPL - 1],
                                                hit[0], hit[SPL - 1]);
        } else {
#pragma unroll
            for (int k = 0; k < SPL; k++)
                hit[k] =
#ifdef RT580_DIAG_NO_NEAR
                    (VARIANT & 512) ? (active[k] && !ao_brute[k]) :  // DIAGNOSTIC build only: every AO ray occluded, no traversal
#endif
                    (VARIANT & 512) ? (active[k] && !ao_brute[k] && bvh_any_near(S.bv, o[k], d[k]))
                  : (VARIANT & 8) ? any_hit_scalar<(VARIANT & 4) != 0>(S, active[k], o[k], d[k])
                                  : any_hit<(VARIANT & 4) != 0>(S, tile, resident, active[k], o[k], d[k]);
        }
#pragma unroll
        for (int k = 0; k < SPL; k++)
            ao_finish<(VARIANT & 512) != 0>(S, W, N, active[k], ao_brute[k], hit[k], c[k], o[k], d[k]);
    }
}


// ---------------------------------------------------------------- AO fix-up
// Samples of ao_body<... | 4096> whose fast rounding test failed (rt_libm.h
// rt_f32_round_safe; ~3e-5 of samples): the exact sample with glibc's sincos,
// then the main pass's scene query. Brute-force scenes test every primitive;
// BVH scenes run the near query and send misses (and far-origin rays) to the
// chunk's sorted far queue, like ao_body's own misses.
__device__ void ao_fix_item(const DevScene& S, const DevFrame& F, const DevWork& W, uint64_t item) {
    const uint32_t N = (uint32_t)F.ao_samples;
    const uint64_t c = item / N;
    const uint32_t s = (uint32_t)(item - c * N);
    const NodeRec& nd = W.nodes[W.call_node[c]];
    const rv3 hp = ld3(nd.hp), n = ld3(nd.n);
    float u0, u1;
    ao_draws(F, W, W.call_rng[c], s, u0, u1);
    const float z = u0 * (1.0f - (-1.0f)) + (-1.0f);
    const float ang = u1 * (F.ao_angle_max - 0.0f) + 0.0f;
    const float r = sqrtf(1 - z * z);
    double sa, ca;
    rt_glibc_sincos_simd_t(rt_dev::rt_sincostab, (double)ang, &sa, &ca);
    rv3 v = v3_normalize(v3((float)((double)r * ca), (float)((double)r * sa), z));
    if (!(v3_dot(v, n) > 0.0f)) v = v3_neg(v);
    const rv3 o = v3_add(hp, v3_scale(v, 0.2f));
    const rv3 d = v3_normalize(v);
    bool hit = false;
    if (S.use_bvh) {
        const bool brute = S.bv.has_far && far_origin(S, o);
        hit = !brute && bvh_any_near(S.bv, o, d);
        if (!hit && S.bv.has_far && (brute || far_live(S.bv, o, d))) {
            if (brute) atomicAdd(W.far_count + 1, 1u);
            const uint32_t slot = atomicAdd(W.far_count, 1u);
            W.far_rays[2 * (size_t)slot] = make_float4(o.x, o.y, o.z, __uint_as_float((uint32_t)c));
            W.far_rays[2 * (size_t)slot + 1] = make_float4(d.x, d.y, d.z, INFINITY);
            W.far_keys[slot] = brute ? RT_KEY_BRUTE : far_key(S.bv, o, d);
            W.far_vals[slot] = slot;
            return;
        }
    } else {
        for (int j = 0; j < S.n_prims && !hit; j++) hit = prim_test_any(S.prims[j], o, d);
    }
    if (hit) atomicAdd(&W.occ[c], 1u);
}

// The queued items; if the queue overflowed (more failing samples than slots),
// every item of [b, e) is re-tested and the failing ones recomputed instead.
__global__ void __launch_bounds__(TB) ao_fix_kernel(DevScene S, DevFrame F, DevWork W, uint64_t b, uint64_t e,
                                                    const uint64_t* call_lo, const uint64_t* call_hi) {
    if (frame_poisoned(W)) return;
    if (call_lo) b = *call_lo * (uint64_t)F.ao_samples;
    if (call_hi) e = *call_hi * (uint64_t)F.ao_samples;
    const uint32_t n = *W.aofix_count;
    if (n == 0) return;
    if (n <= W.aofix_cap) {
        for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < n; i += gridDim.x * TB)
            ao_fix_item(S, F, W, W.aofix_items[i]);
        return;
    }
    const uint64_t items_all = W.totals[0] * (uint64_t)F.ao_samples;
    if (e > items_all) e = items_all;
    const uint32_t N = (uint32_t)F.ao_samples;
    for (uint64_t item = b + (uint64_t)blockIdx.x * TB + threadIdx.x; item < e; item += (uint64_t)gridDim.x * TB) {
        const uint64_t c = item / N;
        const uint32_t s = (uint32_t)(item - c * N);
        float u0, u1;
        ao_draws(F, W, W.call_rng[c], s, u0, u1);
        const float z = u0 * (1.0f - (-1.0f)) + (-1.0f);
        const float ang = u1 * (F.ao_angle_max - 0.0f) + 0.0f;
        const float r = rt_sqrt_nr(1 - z * z);
        double sa, ca;
        rt_fast_sincos((double)ang, &sa, &ca);
        const double X = (double)r * ca, Y = (double)r * sa;
        if (!(rt_f32_round_safe(X, (float)X) && rt_f32_round_safe(Y, (float)Y))) ao_fix_item(S, F, W, item);
    }
}

// Occupancy-capped flavours of ao_near_kernel (RT580_NEAR_WPE=0|5|6|8 for A/B;
// 100k 1080p AO time: uncapped 169 ms (103 VGPRs, 4 waves/SIMD), 5: 161 ms, 6: 158 ms,
// 8: 149 ms; the spills of the capped builds cost less than the latency they hide).
template <int WPE, int V = 512 | 1024 | 2048 | 4096>
__global__ void __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(WPE)))
ao_near_kernel_w(DevScene S, DevFrame F, DevWork W, uint64_t b, uint64_t e) {
    if (frame_poisoned(W)) return;
    ao_body<V>(S, F, W, b, e);
}

// bvh4_any_near_budget_state in speculative while-while form (Aila & Laine's
// postponed leaves): the wave descends until every lane holds a leaf; a lane
// that reaches one first keeps it and goes on descending from its stack in the
// node iterations the wave spends on the others, so its next leaf is found in
// steps that would otherwise idle; the leaf phase then tests the held leaf and,
// when the lane's current entry is a leaf too, that one. The same nodes and
// leaves as the ordinary walk, visited in another order and stopped at the
// first hit: the same boolean. tools/simd_sim.cpp (100k field, budget 4): wave
// node iterations 45.5 -> 32.8, leaf tests 7.8 -> 8.8. Needs the whole wave
// (a vote ends the node phase): inactive lanes pass live = false.
// 1 hit, 0 no hit, -1 undecided after `budget` leaf tests: the stack [0, sp) and
// the entry (c, n) next (n > 0 a leaf) are the walk's state for ao_late_kernel.
template <class STK>
__device__ __forceinline__ bool spec_pop(const STK& stk, int& sp, int32_t& c, int32_t& n) {
    if (sp == 0) return false;
    sp--;
    const uint32_t e = stk.get_lds_first(sp);
    c = (int32_t)(e & 0x7ffffffu);
    n = (int32_t)(e >> 27);
    return true;
}

// bvh4_any_spec_walk: the walk from the state (stack [0, sp), entry (c, n)),
// as bvh4_any_near_resume_budget; bvh4_any_spec_budget_state: from the root,
// after the brute list, as bvh4_any_near_budget_state.
// HOLD2: a lane holds up to two leaves (the second taken while it goes on
// descending with one held); the leaf phase tests them in order, then the
// current entry if it is a leaf. tools/simd_sim.cpp, 100k field, budget 4: wave
// node iterations 32.6 -> 29.2, leaf tests 8.8 -> 9.1.
template <int HOLD2 = 0, bool BOUND = false, class STK>
__device__ int bvh4_any_spec_walk(const BvhView& V, rv3 o, rv3 d, const STK& stk, int budget, bool live, int& sp,
                                  int32_t& c, int32_t& n, float tmax = INFINITY) {
    if (!live) return 0;
    int r = 0;
    const SlabRay sr = slab_ray(V, o, d);
    int32_t pc = 0, pn = 0;  // the held leaf (pn > 0)
    int32_t qc = 0, qn = 0;  // the second held leaf (HOLD2)
    int visits = 0;
    while (live) {
        for (;;) {  // node phase
            if (pn == 0 && n > 0) {
                pc = c;
                pn = n;
                if (!spec_pop(stk, sp, c, n)) n = -1;
            }
            if (HOLD2 && qn == 0 && pn > 0 && n > 0) {
                qc = c;
                qn = n;
                if (!spec_pop(stk, sp, c, n)) n = -1;
            }
            if (!__any(pn == 0 && n == 0)) break;  // every lane holds a leaf or has none left
            if (n == 0 && (!HOLD2 || qn == 0)) {  // one node iteration (speculative when the lane holds a leaf)
                Node4 nd;
                float t[4];
                bool ok[4];
                node4_slab(V.nodes4 + c, sr, t, ok, nd.link);
#pragma unroll
                for (int j = 0; j < 4; j++) ok[j] = (nd.link[j] != 0xffffffffu) & ok[j] & (!BOUND || !(t[j] > tmax));
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
                } else if (!spec_pop(stk, sp, c, n)) {
                    n = -1;
                }
            }
        }
        // leaf phase
        bool h = false;
        if (pn > 0) {
            h = bvh4_leaf_hit(V, o, d, BOUND ? tmax : INFINITY, pc, pn);
            visits++;
            pn = 0;
            if (HOLD2 && !h && qn > 0 && visits < budget) {
                h = bvh4_leaf_hit(V, o, d, BOUND ? tmax : INFINITY, qc, qn);
                visits++;
                qn = 0;
            }
            if (!h && n > 0 && (!HOLD2 || qn == 0) && visits < budget) {  // the current entry is a leaf too
                h = bvh4_leaf_hit(V, o, d, BOUND ? tmax : INFINITY, c, n);
                visits++;
                if (!spec_pop(stk, sp, c, n)) n = -1;
            }
        }
        if (h) {
            r = 1;
            live = false;
        } else if (n < 0 && (!HOLD2 || qn == 0)) {
            r = 0;
            live = false;
        } else if (visits >= budget) {
            if (HOLD2 && qn > 0) {  // the untested held leaf back into the walk's state
                if (n < 0) {
                    c = qc;
                    n = qn;
                } else {
                    stk.put(sp, ((uint32_t)qn << 27) | (uint32_t)qc);
                    sp++;
                }
                qn = 0;
            }
            r = -1;
            live = false;
        }
    }
    return r;
}

template <int HOLD2 = 0, bool BOUND = false, class STK>
__device__ int bvh4_any_spec_budget_state(const BvhView& V, rv3 o, rv3 d, const STK& stk, int budget, bool live,
                                          int& sp, int32_t& c, int32_t& n, float tmax) {
    sp = 0;
    c = 0;
    n = 0;  // root (internal); n < 0: nothing left on this lane
    if (live)
        for (int k = 0; k < V.n_brute; k++)
            if (prim_hit_within(V.all[V.brute[k]], o, d, BOUND ? tmax : INFINITY)) return 1;
    if (live && (!V.has_tree || dir_zero(d))) live = false;
    return bvh4_any_spec_walk<HOLD2, BOUND>(V, o, d, stk, budget, live, sp, c, n, tmax);
}

// The AO ray of a 16-byte record of the generation pass (ao_body, VARIANT &
// 16384): origin hp + 0.2 v and direction normalize(v) by the generation's own
// float operations (CalculateAmbientOcclusion, Raytracer.cpp:323-326; the Ray
// constructor, Raytracer.h:431-433), so (o, d) are the bits the generation
// computed; c = the call. Returns the flag (0: no ray, 1: near query, 2: far
// origin). c0: the chunk's first call (its first item / N).
__device__ __forceinline__ uint32_t ao_record(const DevWork& W, float4 r, uint64_t c0, rv3& o, rv3& d, uint64_t& c) {
    const uint32_t w = __float_as_uint(r.w), rel = w & 0x3fffffffu, flag = w >> 30;
    c = c0 + rel;
    o = v3(0, 0, 0);
    d = v3(0, 0, 0);
    if (flag) {
        const float4 h = W.ao_hp[rel];
        const rv3 v = v3(r.x, r.y, r.z);
        o = v3_add(v3(h.x, h.y, h.z), v3_scale(v, 0.2f));
        d = v3_normalize_unit(v);
    }
    return flag;
}

// Split AO pass of BVH scenes: ao_near_kernel_w<.., V | 16384> writes each
// item's ray (W.ao_rays); this kernel runs the near any-hit query over the
// 4-wide tree with nothing else live, then ao_finish. Rays [0, n) of the chunk.
// LDS_D: the first LDS_D traversal-stack entries of each lane live in LDS (a
//   column per lane), the rest in scratch.
// SORT: the workgroup takes SORT * TB consecutive samples (SORT * TB / N calls
//   of neighbouring pixels) at a time and traces them in the order of an LDS
//   counting sort by octahedral direction cell (2^KL x 2^KL): a wave then holds
//   rays of similar direction from nearby origins, which share more of their
//   paths (tools/simd_sim.cpp "block sort"). Hits are counted per lane.
// BUDGET: a lane gives up after BUDGET leaf visits; its item and its walk so
//   far (W.ao_state) go to W.ao_late, and ao_late_kernel resumes the walk, so
//   a wave is not held by its few long traversals (tools/simd_sim.cpp "budget").
// The walk is in speculative while-while form (bvh4_any_spec_budget_state).
template <int WPE, int LDS_D, int SORT, int KL, int BUDGET>
__global__ void __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(WPE)))
ao_trace_kernel(DevScene S, DevWork W, uint64_t n, uint64_t c0) {
    static_assert(LDS_D > 0 && SORT > 0 && BUDGET > 0, "LDS stack, block sort, step budget");
    if (frame_poisoned(W)) return;
    __shared__ uint32_t lstk[LDS_D][TB];
    constexpr int SN = SORT * TB;
    constexpr int NB = 1 << (2 * KL);  // direction cells
    __shared__ uint32_t s_order[SN];
    __shared__ uint32_t s_bin[NB + 1];
    __shared__ uint32_t s_wsum[TB / 64];
    for (uint64_t blk = (uint64_t)blockIdx.x * SN; blk < n; blk += (uint64_t)gridDim.x * SN)
    for (int round = 0; round < SORT; round++) {
        if (round == 0) {
            // counting sort of the block's samples by direction cell
            __syncthreads();
            for (int k = threadIdx.x; k < NB + 1; k += TB) s_bin[k] = 0;
            __syncthreads();
            uint32_t key[SORT];
#pragma unroll
            for (int q = 0; q < SORT; q++) {
                const uint64_t j = blk + (uint64_t)q * TB + threadIdx.x;
                key[q] = NB;  // past the end (or no ray): last
                if (j < n) {
                    const float4 r = W.ao_rays[j];  // grouping only: v's cell (d = normalize(v))
                    if (__float_as_uint(r.w) >> 30) key[q] = grid_cell(v3(r.x, r.y, r.z), KL);
                }
                atomicAdd(&s_bin[key[q]], 1u);
            }
            __syncthreads();
            {   // exclusive scan of the NB + 1 bins: runs of PER bins per thread,
                // their sums scanned across the wave (shuffles) and the waves (LDS)
                constexpr int PER = (NB + 1 + TB - 1) / TB;
                const int k0 = threadIdx.x * PER;
                uint32_t run = 0;
#pragma unroll
                for (int q = 0; q < PER; q++)
                    if (k0 + q < NB + 1) run += s_bin[k0 + q];
                const int ln = threadIdx.x & 63, wv = threadIdx.x >> 6;
                uint32_t inc = run;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t v = (uint32_t)__shfl_up((int)inc, o);
                    if (ln >= o) inc += v;
                }
                if (ln == 63) s_wsum[wv] = inc;
                __syncthreads();
                uint32_t acc = inc - run;
                for (int w2 = 0; w2 < wv; w2++) acc += s_wsum[w2];
#pragma unroll
                for (int q = 0; q < PER; q++)
                    if (k0 + q < NB + 1) {
                        const uint32_t c = s_bin[k0 + q];
                        s_bin[k0 + q] = acc;
                        acc += c;
                    }
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < SORT; q++) {
                const uint32_t pos = atomicAdd(&s_bin[key[q]], 1u);
                s_order[pos] = (uint32_t)(q * TB + threadIdx.x);
            }
            __syncthreads();
        }
        const uint64_t i = blk + s_order[round * TB + threadIdx.x];
        rv3 o, d;
        uint64_t call = 0;
        const uint32_t flag = ao_record(W, i < n ? W.ao_rays[i] : make_float4(0, 0, 0, 0), c0, o, d, call);
        const bool active = flag != 0u, ao_brute = flag == 2u;
        uint32_t stk_a[RT_BVH_STACK + 4 - LDS_D];
        const LdsStack<LDS_D, TB> stk{&lstk[0][threadIdx.x], stk_a};
        int sp = 0;
        int32_t wc = 0, wn = 0;
        const int r = bvh4_any_spec_budget_state<0>(S.bv, o, d, stk, BUDGET, flag == 1u, sp, wc, wn);
        const bool hit = r > 0, late = r < 0;
        const uint64_t lm = __ballot(late);
        if (lm) {
            const int leader = __ffsll((unsigned long long)lm) - 1;
            uint32_t base = 0;
            if ((threadIdx.x & 63) == leader) base = atomicAdd(W.ao_late_count, (uint32_t)__popcll(lm));
            base = __shfl(base, leader);
            if (late) {
                const uint32_t slot = base + (uint32_t)__popcll(lm & lanemask_lt());
                W.ao_late[slot] = (uint32_t)i;
                if (slot < W.ao_state_cap) {  // the walk so far, for ao_late_kernel to resume
                    uint32_t* rec = W.ao_state + (size_t)slot * kLateWords;
                    rec[0] = (uint32_t)wc;
                    rec[1] = sp <= kLateSaved ? ((uint32_t)wn | ((uint32_t)sp << 8)) : 0xffffffffu;
                    if (sp <= kLateSaved)
                        for (int t = 0; t < sp; t++) rec[2 + t] = stk.get(t);
                }
            }
        }
        // sorted: a wave's lanes are no longer one call's samples
        ao_finish<true>(S, W, 1u, active && !late, ao_brute, hit, call, o, d);
    }
}

// The chunk's AO rays that ran out of ao_trace_kernel's step budget: the full
// near query (resuming the walk saved for the ray, or from the root when its
// stack was too deep to save), in speculative form, then the same bookkeeping
// (hits counted per call, misses queued for the far pass). Grid-stride over the
// device-side count.
// The ray's record is read again after the walk (a volatile load, not the
// registers of the first read), so that nothing of the ray but its index is
// live across the traversal. History: round 4's 64-VGPR build of this kernel
// (8 waves per SIMD, since removed) queued ~2 % of its far-pass rays with
// origins not their own when the origin stayed live across the walk; every
// answer it computed was right ("The 8-wave late-pass defect").
template <int WPE, int LDS_D>
__global__ void __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(WPE)))
ao_late_kernel(DevScene S, DevWork W, uint64_t c0) {
    if (frame_poisoned(W)) return;
    __shared__ uint32_t lstk[LDS_D][TB];
    const uint32_t cnt = W.ao_late_count[0];
    for (uint32_t b0 = blockIdx.x * TB; b0 < cnt; b0 += gridDim.x * TB) {
        const uint32_t k = b0 + threadIdx.x;
        const bool live = k < cnt;
        uint32_t i = 0;
        float4 r = make_float4(0, 0, 0, 0);
        if (live) {
            i = W.ao_late[k];
            r = W.ao_rays[i];
        }
        rv3 o, d;
        uint64_t call = 0;
        (void)ao_record(W, r, c0, o, d, call);
        uint32_t stk_a[RT_BVH_STACK + 4 - LDS_D];
        const LdsStack<LDS_D, TB> stk{&lstk[0][threadIdx.x], stk_a};
        // the walk ao_trace_kernel saved for this ray
        int sp = 0;
        int32_t wc = 0, wn = 0;
        bool saved = false;
        if (live && k < W.ao_state_cap) {
            const uint32_t* rec = W.ao_state + (size_t)k * kLateWords;
            const uint32_t h1 = rec[1];
            if (h1 != 0xffffffffu) {
                saved = true;
                sp = (int)(h1 >> 8);
                wn = (int32_t)(h1 & 255u);
                wc = (int32_t)rec[0];
                for (int t = 0; t < sp; t++) stk.put(t, rec[2 + t]);
            }
        }
        // one walk for the saved and the restarted rays (the wave votes together)
        bool go = live, pre = false;
        if (live && !saved) {  // from the root, after the brute list
            for (int t = 0; t < S.bv.n_brute && !pre; t++) pre = prim_hit_within(S.bv.all[S.bv.brute[t]], o, d, INFINITY);
            go = !pre && S.bv.has_tree && !dir_zero(d);
        }
        const bool hit = pre || bvh4_any_spec_walk<0>(S.bv, o, d, stk, 1 << 30, go, sp, wc, wn) > 0;
        if (live) {
            const volatile float4* rv = W.ao_rays + i;
            r = make_float4(rv->x, rv->y, rv->z, rv->w);
        }
        rv3 o2, d2;
        (void)ao_record(W, r, c0, o2, d2, call);
        ao_finish<true>(S, W, 1u, live, false, hit, call, o2, d2);
    }
}

// (A wave per late ray, its lanes sharing the ray's traversal stack -- 64
// entries popped at a time, children pushed with wave prefix sums: correct,
// but north-star 38.8 -> 56-58 ms; the late rays' frontiers are narrow. Not
// kept. Persistent forms of ao_trace_kernel -- lanes refilled from the chunk as
// they finish, per-iteration atomic fetch, static per-wave ranges, or batched
// fetch with prefetched records -- measured 94 / 137 / 133 ms against 89 ms
// for this kernel on cornell10k's AO; the SIMD-efficiency model
// tools/simd_sim.cpp predicts fewer lock-step iterations for them, but their
// extra live state spills. Not kept.)

#ifdef RT580_DIAGNOSTICS
// DIAGNOSTIC build only (RT580_AO_VERIFY=1): an audit of the budgeted AO
// trace + late passes of each chunk that does not touch those kernels (their
// code is the product's). Every near-query AO ray of the chunk (flag 1) is
// answered again by the unbudgeted 4-wide query with a plain per-lane stack
// (ao_audit_expect_kernel): the near hits it implies per AO call, and the far
// queue it implies (every miss and every far-origin ray: count, and an
// order-free checksum of each entry's ray, call and key). ao_audit_compare_kernel
// then checks the occlusion counts the passes added and the queue they wrote.
// out[0] rays checked, [1] calls whose near hits differ, [2] far-queue count
// differs (chunks), [3] far-queue checksum differs (chunks), [4] chunks
// audited, [5] expected near hits, [6] queued rays, [7] queue entries that no
// ray of the chunk explains; [8 + 2k], [9 + 2k]: the first 8 differing calls
// (call | got << 32, want); [24] the OR of those entries' reasons, [25] their
// count, [26 + 18k]: the first 2 such entries (ao_audit_compare_kernel).
__device__ __forceinline__ unsigned long long audit_mix(float4 a, float4 b, uint32_t key) {
    unsigned long long h = 0x9e3779b97f4a7c15ull;
    const uint32_t w[8] = {__float_as_uint(a.x), __float_as_uint(a.y), __float_as_uint(a.z), __float_as_uint(a.w),
                           __float_as_uint(b.x), __float_as_uint(b.y), __float_as_uint(b.z), key};
#pragma unroll
    for (int k = 0; k < 8; k++) {
        h ^= w[k];
        h *= 0xff51afd7ed558ccdull;
        h ^= h >> 33;
    }
    return h;
}

// exp[c - c_lo]: near hits of call c among the chunk's rays [0, n); aud[0..1]:
// expected queue length and checksum
__global__ void __launch_bounds__(TB) ao_audit_expect_kernel(DevScene S, DevWork W, uint64_t n, uint32_t c_lo,
                                                             uint32_t* exp, unsigned long long* aud,
                                                             unsigned long long* out) {
    if (frame_poisoned(W)) return;
    for (uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * TB) {
        rv3 o, d;
        uint64_t c64 = 0;
        const uint32_t flag = ao_record(W, W.ao_rays[i], c_lo, o, d, c64);
        if (flag == 0u) continue;
        const uint32_t c = (uint32_t)c64;
        const bool hit = flag == 1u && bvh4_any_near(S.bv, o, d);
        if (flag == 1u) atomicAdd(&out[0], 1ull);
        if (hit) {
            atomicAdd(&exp[c - c_lo], 1u);
            atomicAdd(&out[5], 1ull);
        } else if (S.bv.has_far && (flag == 2u || far_live(S.bv, o, d))) {
            const uint32_t key = flag == 2u ? RT_KEY_BRUTE : far_key(S.bv, o, d);
            atomicAdd(&aud[0], 1ull);
            atomicAdd(&aud[1], audit_mix(make_float4(o.x, o.y, o.z, __uint_as_float(c)), make_float4(d.x, d.y, d.z, INFINITY),
                                         key));
        }
    }
}

// occ_before: W.occ[c_lo, c_lo + nc) before the chunk's passes
__global__ void __launch_bounds__(TB) ao_audit_compare_kernel(DevScene S, DevWork W, uint32_t c_lo, uint32_t nc,
                                                              uint32_t N, uint64_t item0, uint64_t n,
                                                              const uint32_t* occ_before, const uint32_t* exp,
                                                              unsigned long long* aud, unsigned long long* out) {
    if (frame_poisoned(W)) return;
    const uint32_t nq = S.bv.has_far ? W.far_count[0] : 0u;
    for (uint32_t j = blockIdx.x * TB + threadIdx.x; j < nc; j += gridDim.x * TB) {
        const uint32_t got = W.occ[c_lo + j] - occ_before[j];
        if (got != exp[j]) {
            const unsigned long long k = atomicAdd(&out[1], 1ull);
            if (k < 8) {
                out[8 + 2 * k] = (unsigned long long)(c_lo + j) | ((unsigned long long)got << 32);
                out[9 + 2 * k] = exp[j];
            }
        }
    }
    for (uint32_t s = blockIdx.x * TB + threadIdx.x; s < nq; s += gridDim.x * TB) {
        const float4 a = W.far_rays[2 * (size_t)s], b = W.far_rays[2 * (size_t)s + 1];
        const uint32_t key = W.far_keys[s];
        atomicAdd(&aud[2], audit_mix(a, b, key));
        // the entry against the rays of its call in this chunk: which part of it
        // (if any) no ray of the chunk has -- 1 call out of the chunk, 2 no
        // sample of the call with this origin, 4 the origin's sample has another
        // direction, 8 the key is not the ray's own
        const uint32_t c = __float_as_uint(a.w);
        uint32_t why = 0u;
        int64_t found = -1;
        if (c < c_lo || c >= c_lo + nc) {
            why = 1u;
        } else {
            const int64_t j0 = (int64_t)c * N - (int64_t)item0, j1 = j0 + N;
            why = 2u;
            for (int64_t j = j0 < 0 ? 0 : j0; j < j1 && j < (int64_t)n; j++) {
                rv3 oj, dj;
                uint64_t cj = 0;
                const uint32_t flag = ao_record(W, W.ao_rays[j], c_lo, oj, dj, cj);
                const float4 r0 = make_float4(oj.x, oj.y, oj.z, __uint_as_float((uint32_t)cj)),
                             r1 = make_float4(dj.x, dj.y, dj.z, __uint_as_float(flag));
                if (why == 2u && a.x != a.z && __float_as_uint(r0.z) == __float_as_uint(a.x) &&
                    __float_as_uint(r0.y) == __float_as_uint(a.y) && __float_as_uint(r0.x) == __float_as_uint(a.z))
                    why = 16u;  // a sample of the call has this origin with x and z exchanged
                if (why == 16u) { found = j; continue; }
                if (why == 2u && found < 0 && __float_as_uint(r1.x) == __float_as_uint(b.x) &&
                    __float_as_uint(r1.y) == __float_as_uint(b.y) && __float_as_uint(r1.z) == __float_as_uint(b.z))
                    found = j;  // (reported: the sample with this direction, when no origin matches)
                if (__float_as_uint(r0.x) != __float_as_uint(a.x) || __float_as_uint(r0.y) != __float_as_uint(a.y) ||
                    __float_as_uint(r0.z) != __float_as_uint(a.z))
                    continue;
                found = j;
                const bool dsame = __float_as_uint(r1.x) == __float_as_uint(b.x) &&
                                   __float_as_uint(r1.y) == __float_as_uint(b.y) &&
                                   __float_as_uint(r1.z) == __float_as_uint(b.z);
                if (!dsame) { why = 4u; continue; }
                const uint32_t want = flag == 2u ? RT_KEY_BRUTE : far_key(S.bv, v3(r0.x, r0.y, r0.z), v3(r1.x, r1.y, r1.z));
                why = want == key ? 0u : 8u;
                if (!why) break;
            }
        }
        if (why) {
            atomicAdd(&out[7], 1ull);
            atomicOr(&out[24], (unsigned long long)why);
            const unsigned long long k = atomicAdd(&out[25], 1ull);
            if (k < 2) {  // the entry and the ray it was matched with (or none)
                unsigned long long* d = out + 26 + 18 * k;
                rv3 of = v3(0, 0, 0), df = v3(0, 0, 0);
                uint64_t cf = 0;
                const uint32_t ff = found >= 0 ? ao_record(W, W.ao_rays[found], c_lo, of, df, cf) : 0u;
                const float4 r0 = make_float4(of.x, of.y, of.z, __uint_as_float((uint32_t)cf));
                const float4 r1 = make_float4(df.x, df.y, df.z, __uint_as_float(ff));
                const float v[16] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
                for (int t = 0; t < 16; t++) d[t] = __float_as_uint(v[t]);
                d[16] = key | ((unsigned long long)why << 32);
                d[17] = (unsigned long long)s | ((unsigned long long)(found >= 0 ? (uint32_t)found : 0xffffffffu) << 32);
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(&out[4], 1ull);
        atomicAdd(&out[6], (unsigned long long)nq);
    }
}

__global__ void ao_audit_finish_kernel(const DevScene S, const DevWork W, const unsigned long long* aud,
                                       unsigned long long* out) {
    if (threadIdx.x != 0) return;
    const uint32_t nq = S.bv.has_far ? W.far_count[0] : 0u;
    if (aud[0] != nq) out[2]++;
    if (aud[1] != aud[2]) out[3]++;
}

static bool ao_verify_on() {
    static int v = -1;
    if (v < 0) {
        const char* e = getenv("RT580_AO_VERIFY");
        v = e ? atoi(e) : 0;
    }
    return v != 0;
}

static unsigned long long* g_verify_out = nullptr;  // device, 64 words
// per slot (keyed by its W.ao_rays): expected near hits per call, the calls'
// counts before the chunk, the queue sums
struct AuditBuf {
    const void* key;
    uint32_t cap;
    uint32_t* exp;
    uint32_t* before;
    unsigned long long* aud;
};
static std::vector<AuditBuf*> g_audit_bufs;  // (never freed: diagnostic runs only)

static const AuditBuf* audit_for(const DevWork& W) {
    if (!ao_verify_on() || !W.ao_rays) return nullptr;
    if (!g_verify_out) {
        if (hipMalloc((void**)&g_verify_out, 64 * 8) != hipSuccess) return nullptr;
        if (hipMemset(g_verify_out, 0, 64 * 8) != hipSuccess) return nullptr;
    }
    for (const AuditBuf* b : g_audit_bufs)
        if (b->key == W.ao_rays && b->cap >= W.ao_cap) return b;
    AuditBuf b{W.ao_rays, W.ao_cap, nullptr, nullptr, nullptr};
    // a chunk of ao_cap rays spans at most ao_cap + 1 calls
    if (hipMalloc((void**)&b.exp, ((size_t)W.ao_cap + 2) * 4) != hipSuccess ||
        hipMalloc((void**)&b.before, ((size_t)W.ao_cap + 2) * 4) != hipSuccess ||
        hipMalloc((void**)&b.aud, 4 * 8) != hipSuccess)
        return nullptr;
    g_audit_bufs.push_back(new AuditBuf(b));
    return g_audit_bufs.back();
}
#endif

// ---------------------------------------------------------------- far-hit pass
// Direction-grid candidates (rt_bvh.h build_dir_grid) of a lane whose origin is
// within grid_r: the "always" entries, then its cell's list. When every grid
// lane of the wave shares one cell (queues are sorted by cell, far_key), the
// list is read 64 planes at a time: each lane gathers one plane into the
// wave's LDS tile, then every lane walks the tile by broadcast reads; else
// each lane walks its own cell's list. (Walking a wave's distinct cells one
// after the other instead: field1m AO 2.26 -> 5.54 s -- waves hold many.)
// Each candidate gets far_candidate + the full reference test. Must be called
// by the whole wave.
#ifdef RT580_DIAGNOSTICS
// DIAGNOSTIC build only: far_any_kernel statistics -- rays, grid rays, uniform
// waves, per-lane waves, lanes' list entries, lock-step list steps (per wave:
// the longest lane list / U), plane-tree rays, candidates passing
// far_candidate, full tests that hit
__device__ unsigned long long g_far_stats[9];
#ifdef RT580_DIAG_NO_STATS  // timing ablations: no per-pair atomics
#define RT_FAR_STAT(k, v) ((void)0)
#else
#define RT_FAR_STAT(k, v) atomicAdd(&g_far_stats[k], (unsigned long long)(v))
#endif
// far_cell_any_kernel: rays of items whose cell has no candidate, (ray,
// candidate) pairs of the other items, pairs passing far_candidate
__device__ unsigned long long g_cell_stats[3];
#ifdef RT580_DIAG_NO_STATS
#define RT_CELL_STAT(k, v) ((void)0)
#else
#define RT_CELL_STAT(k, v) atomicAdd(&g_cell_stats[k], (unsigned long long)(v))
#endif
// RT580_CELL_SKIP (timing attribution only; results wrong): 1 no candidate
// loop, 2 no full tests, 3 no far_candidate either (the loop's LDS reads kept)
__device__ int g_cell_skip;
#define CELL_SKIP(k) (g_cell_skip == (k))
#else
#define CELL_SKIP(k) false
#define RT_CELL_STAT(k, v) ((void)0)
#define RT_FAR_STAT(k, v) ((void)0)
#endif

// The queued AO rays, sorted by direction key, 64 per wave: the wave walks the
// plane tree once for all its lanes (a node is entered if any live lane may
// have a far hit below it), each lane evaluating the exact tests of rt_isect.h
// for its own ray. Same candidates, same full tests as bvh_any's far search.
#ifndef FAR_ANY_WPE
// 6 waves/SIMD for the far any-hit and cell passes (their 8-wave build spills):
// north-star 36.36 / 36.52 vs 36.75 / 37.11 ms (profiles/r04/ab/w6_*.json)
#define FAR_ANY_WPE 6
#endif
// flag != null: shadow rays (tag = flag index, the flag is set on a hit);
// else AO rays (tag = AO call, its occlusion count is incremented).
__device__ __forceinline__ void any_hit_out(const DevWork& W, uint8_t* flag, uint32_t tag) {
    if (flag) flag[tag] = 1;
    else atomicAdd(&W.occ[tag], 1u);
}

// The plane-tree far search of the live lanes (bvh_any's far part): the wave
// walks the tree once for all of them (a node is entered if any live lane may
// have a far hit below it; node index wave-uniform), each lane evaluating the
// exact tests for its own ray. stk: the wave's LDS stack. Whole wave.
__device__ __forceinline__ bool far_tree_any_wave(const DevScene& S, bool live, rv3 o, rv3 d, const FarRay& fr,
                                                  int32_t* stk) {
    bool hit = false;
    int sp = 0;
    stk[sp++] = 0;  // every lane writes the same value: no cross-lane ordering needed
    while (sp > 0) {
        if (__ballot(live) == 0) break;
        const int node = __builtin_amdgcn_readfirstlane(stk[--sp]);
        const FarNode fn = load_far_node(S.bv.far_nodes, node);
        float T;
        const bool may = live && far_node_may(fn, fr, o, d, T);
        if (__ballot(may) == 0) continue;
        if (fn.count == 0) {
            stk[sp++] = fn.first + 1;
            stk[sp++] = fn.first;
            continue;
        }
        for (int k = fn.first; k < fn.first + fn.count; k++) {
            const FarTri ft = load_far_tri(S.bv.far_tris, k);
            bool cand = may && live && far_candidate(ft, fr, o, d);
            if (__ballot(cand) == 0) continue;
            const rt_prim P = load_prim_scalar(S.prims, (int)ft.id);
            if (cand && prim_test_any(P, o, d)) {
                hit = true;
                live = false;
            }
        }
    }
    return hit;
}

// The plane-tree far search of bvh_closest for the lanes with `walk` set
// (far_closest's tree part): the wave walks the tree once for all of them,
// merging into (h, found) with the lexicographic rule. Returns whether h
// changed. stk: the wave's LDS stack. Whole wave.
__device__ __forceinline__ bool far_tree_closest_wave(const DevScene& S, bool walk, rv3 o, rv3 d, const FarRay& fr,
                                                      Hit& h, bool& found, int32_t* stk) {
    bool changed = false;
    int sp = 0;
    stk[sp++] = 0;
    while (sp > 0) {
        const int fnode = __builtin_amdgcn_readfirstlane(stk[--sp]);
        const FarNode fn = load_far_node(S.bv.far_nodes, fnode);
        float T;
        const bool may = walk && far_node_may(fn, fr, o, d, T) && !(found && h.t < T);
        if (__ballot(may) == 0) continue;
        if (fn.count == 0) {
            stk[sp++] = fn.first + 1;
            stk[sp++] = fn.first;
            continue;
        }
        for (int k = fn.first; k < fn.first + fn.count; k++) {
            const FarTri ft = load_far_tri(S.bv.far_tris, k);
            const bool cand = may && far_candidate(ft, fr, o, d);
            if (__ballot(cand) == 0) continue;
            const rt_prim P = load_prim_scalar(S.prims, (int)ft.id);
            float t, a, b, g;
            if (cand && prim_test_closest(P, o, d, t, a, b, g, found ? h.t : INFINITY) &&
                lex_better(t, (int)ft.id, found, h)) {
                found = true;
                changed = true;
                h.t = t; h.a = a; h.b = b; h.g = g; h.prim = (int)ft.id;
            }
        }
    }
    return changed;
}

// Cell-major any-hit far pass over the sorted queue [0, n) (far-origin rays
// excluded), cut into segments of one sort key (far_seg_off / far_keys, see
// launch_far_cells). A wave takes a segment: a grid cell's rays share one
// candidate list (rt_bvh.h build_dir_grid), so the list is read once per
// segment, not once per ray. The wave stages up to 64 of the segment's rays in
// LDS; the lanes hold candidates (the "always" entries, then the cell's list;
// lists shorter than 64 are replicated 64 / Lp times, Lp = the list length
// rounded up to a power of two, so each step tests 64 / Lp rays) and step
// through the staged rays: far_candidate, then the full reference test
// (prim_test_any) -- the tests far_any / far_grid_lane make, on the same pairs.
// A plane-tree segment (RT_KEY_TREE keys) runs far_tree_any_wave over its
// staged rays instead. Hit rays: any_hit_out. A wave's work item is one chunk
// of <= 64 rays of one segment (a directional light's shadow rays all share a
// cell); grid-stride over the work items (their count is read on the device).
// A ray already hit is not re-checked per step (hits are ~1e-3 of the rays; a
// second accepting candidate only repeats the flag). Pairs passing
// far_candidate (~1 % of the north-star frame's 2.4e9 pairs) are queued in LDS
// and get their full tests 64 at a time (cell_full_tests): tested in place,
// each cost a whole divergent wave step (3.0 of the frame's 5.0 candidate-loop
// ms, measured with RT580_CELL_SKIP). (Software-pipelining the items' load
// chains -- next item's indices and descriptor in flight during the current
// item -- measured slower: 41.7 vs 38.8 ms, 9.8 vs 8.4 ms at a 1/8 share.)
struct CellItem {
    uint32_t r0, nr, lb, n_list;
    bool tree, skip;
};
__device__ __forceinline__ CellItem cell_item(const BvhView& V, uint4 wd) {
    CellItem it;
    it.r0 = __builtin_amdgcn_readfirstlane(wd.x);
    const uint32_t r1 = __builtin_amdgcn_readfirstlane(wd.y);
    it.lb = __builtin_amdgcn_readfirstlane(wd.z);
    const uint32_t lw = __builtin_amdgcn_readfirstlane(wd.w);
    it.nr = r1 - it.r0 < 64u ? r1 - it.r0 : 64u;
    it.tree = lw == 0xffffffffu;
    it.n_list = it.tree ? 0u : lw;
    it.skip = !it.tree && V.n_always + (int)it.n_list == 0;  // no candidate: no far hit in this cell
    return it;
}
// lane j's value of x (j wave-uniform)
__device__ __forceinline__ float lane_f32(float x, int j) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j));
}
__device__ __forceinline__ int cell_lg(int lt) {
    return lt > 32 ? 6 : lt > 16 ? 5 : lt > 8 ? 4 : lt > 4 ? 3 : lt > 2 ? 2 : lt > 1 ? 1 : 0;
}
// The item's index loads for this lane: its ray's queue entry (q) and its
// first-chunk candidate's far_tris index (gi).
__device__ __forceinline__ void cell_indices(const BvhView& V, const DevWork& W, const CellItem& it, int lane,
                                             uint32_t& q, uint32_t& gi) {
    q = 0u;
    gi = 0u;
    if (it.skip) return;
    if ((uint32_t)lane < it.nr) q = W.far_vals_alt[it.r0 + lane];
    if (it.tree) return;
    const int n_cand = V.n_always + (int)it.n_list;
    const int lt = n_cand < 64 ? n_cand : 64, lg = cell_lg(lt);
    const int kk = lane & ((1 << lg) - 1);
    if (kk < lt) {
        const int k = kk - V.n_always;
        gi = k < 0 ? V.grid_always[k + V.n_always] : V.grid_items[it.lb + (uint32_t)k];
    }
}

// The queued pairs [0, qn) of far_cell_any_kernel (qn < 128): the full
// reference test of each, one pair per lane; a hit flags the ray. Whole wave.
__device__ __forceinline__ void cell_full_tests(const DevScene& S, const float4 (*sray)[2], uint32_t* shit,
                                                const uint32_t* pq_id, const uint8_t* pq_j, uint32_t qn) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = lane; i < qn; i += 64) {
        const uint32_t j = pq_j[i];
        if (CELL_SKIP(2) || shit[j] != 0u) continue;
        const float4 a = sray[j][0], b = sray[j][1];
        if (prim_test_any(S.prims[pq_id[i]], v3(a.x, a.y, a.z), v3(b.x, b.y, b.z))) shit[j] = 1u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// (A ray-per-lane form -- each lane's ray in registers, the cell's candidates
// as wave-uniform scalar loads one after the other -- measured slower on the
// north-star frame for items of >= 16 rays, 39.7-39.9 vs 37.5-38.1 ms, and
// equal for >= 32: the scalar loads' latency is exposed per candidate. Not kept.)
__global__ void __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(FAR_ANY_WPE)))
far_cell_any_kernel(DevScene S, DevWork W, uint32_t n, uint8_t* flag) {
    if (frame_poisoned(W)) return;
    __shared__ float4 sray[TB / 64][64][2];
    __shared__ uint32_t shit[TB / 64][64];
    __shared__ int32_t stk[TB / 64][RT_BVH_STACK];
    __shared__ uint32_t pq_id[TB / 64][128];
    __shared__ uint8_t pq_j[TB / 64][128];
    const BvhView& V = S.bv;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t nwork = W.far_seg_n[1];
    const uint32_t stride = gridDim.x * (TB / 64);
    uint32_t w = blockIdx.x * (TB / 64) + wave;
    if (w >= nwork) return;
    for (;;) {
        const CellItem cur = cell_item(V, W.far_work[w]);
        uint32_t q, gi;
        cell_indices(V, W, cur, lane, q, gi);
        const bool live = !cur.skip && (uint32_t)lane < cur.nr;
        float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b = make_float4(1.0f, 0.0f, 0.0f, 0.0f);
        if (live) {
            a = W.far_rays[2 * (size_t)q];
            b = W.far_rays[2 * (size_t)q + 1];
        }
        const int n_cand = V.n_always + (int)cur.n_list;
        FarTri ft0;
        if (!cur.skip && !cur.tree) ft0 = V.far_tris[gi];
        const uint32_t wn = w + stride;
        if (cur.skip) {
            RT_CELL_STAT(0, lane == 0 ? (uint64_t)cur.nr : 0ull);
        } else {
            const uint32_t nr = cur.nr;
            // the previous item's LDS reads are done before it is overwritten
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (live) {
                sray[wave][lane][0] = a;
                sray[wave][lane][1] = make_float4(b.x, b.y, b.z, far_ray(V, v3(a.x, a.y, a.z)).R);
                shit[wave][lane] = 0u;
            }
            bool hit = false;
            if (cur.tree) {
                // the rays back from LDS (registers are short across the candidate loop)
                const float4 at = sray[wave][lane][0], bt = sray[wave][lane][1];
                FarRay fr;
                fr.R = bt.w;
                hit = far_tree_any_wave(S, live, v3(at.x, at.y, at.z), v3(bt.x, bt.y, bt.z), fr, stk[wave]);
            } else {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                uint32_t qn = 0;  // queued (candidate, ray) pairs, wave-uniform
                // this lane's ray, for the full chunks' register broadcasts
                const float rR = far_ray(V, v3(a.x, a.y, a.z)).R;
                uint64_t hitm = 0;  // rays flagged by the full tests so far (refreshed after each batch)
                for (int kc = 0; kc < (CELL_SKIP(1) ? 0 : n_cand); kc += 64) {
                    const int lt = n_cand - kc < 64 ? n_cand - kc : 64;
                    const int lg = cell_lg(lt);
                    const int kk = lane & ((1 << lg) - 1), g = lane >> lg;
                    const bool has = kk < lt;
                    FarTri ft = ft0;
                    if (kc > 0 && has) {
                        const int k = kc + kk - V.n_always;
                        ft = V.far_tris[k < 0 ? V.grid_always[k + V.n_always] : V.grid_items[cur.lb + (uint32_t)k]];
                    }
                    if (lg == 6 && !CELL_SKIP(3)) {
                        // 64 candidates, one ray a step: the ray is wave-uniform, read
                        // from its lane's registers (7 readlanes) instead of LDS (two
                        // b128 reads and the flag: the LDS pipe, not the VALU, bound
                        // this loop), and rays already hit are skipped as a whole step.
                        uint64_t todo = __ballot(live) & ~hitm;
                        while (todo) {
                            const int j = __builtin_ctzll(todo);
                            todo &= todo - 1;
                            FarRay fj;
                            fj.R = lane_f32(rR, j);
                            const rv3 oj = v3(lane_f32(a.x, j), lane_f32(a.y, j),
                                              lane_f32(a.z, j));
                            const rv3 dj = v3(lane_f32(b.x, j), lane_f32(b.y, j),
                                              lane_f32(b.z, j));
                            const bool fc = far_candidate_filter(ft, fj, oj, dj);
                            RT_CELL_STAT(2, fc ? 1 : 0);
                            const uint64_t m = __ballot(fc);
                            if (m == 0) continue;
                            if (fc) {
                                const uint32_t slot = qn + (uint32_t)__popcll(m & lanemask_lt());
                                pq_id[wave][slot] = ft.id;
                                pq_j[wave][slot] = (uint8_t)j;
                            }
                            qn += (uint32_t)__popcll(m);
                            if (qn >= 64u) {
                                cell_full_tests(S, sray[wave], shit[wave], pq_id[wave], pq_j[wave], qn);
                                qn = 0;
                                hitm = __ballot(live && shit[wave][lane] != 0u);
                                todo &= ~hitm;
                            }
                        }
                        continue;
                    }
                    const uint32_t step = 64u >> lg;
                    for (uint32_t j0 = 0; j0 < nr; j0 += step) {
                        const uint32_t j = j0 + (uint32_t)g;
                        bool fc = false;
                        if (has && j < nr && !((hitm >> j) & 1u)) {  // (rays hit so far: hitm, refreshed after each batch)
                            const float4 aj = sray[wave][j][0], bj = sray[wave][j][1];
                            FarRay fj;
                            fj.R = bj.w;
                            if (CELL_SKIP(3)) {
                                if (aj.x == ft.n[0] && bj.w == ft.d) shit[wave][j] = 1u;
                                continue;
                            }
                            fc = far_candidate_filter(ft, fj, v3(aj.x, aj.y, aj.z), v3(bj.x, bj.y, bj.z));
                        }
                        RT_CELL_STAT(2, fc ? 1 : 0);
                        // passing pairs are queued; their full tests run 64 at a time
                        // (~1 % of pairs pass: tested in place they would each cost a
                        // whole wave step)
                        const uint64_t m = __ballot(fc);
                        if (m == 0) continue;
                        if (fc) {
                            const uint32_t slot = qn + (uint32_t)__popcll(m & lanemask_lt());
                            pq_id[wave][slot] = ft.id;
                            pq_j[wave][slot] = j;
                        }
                        qn += (uint32_t)__popcll(m);
                        if (qn >= 64u) {
                            cell_full_tests(S, sray[wave], shit[wave], pq_id[wave], pq_j[wave], qn);
                            qn = 0;
                            hitm = __ballot(live && shit[wave][lane] != 0u);
                        }
                    }
                }
                if (qn) cell_full_tests(S, sray[wave], shit[wave], pq_id[wave], pq_j[wave], qn);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                hit = live && shit[wave][lane] != 0u;
            }
            RT_FAR_STAT(0, live ? 1 : 0);
            RT_CELL_STAT(1, lane == 0 && !cur.tree ? (uint64_t)nr * (uint64_t)n_cand : 0ull);
            RT_FAR_STAT(8, hit ? 1 : 0);
            if (hit) any_hit_out(W, flag, __float_as_uint(sray[wave][lane][0].w));
        }
        if (wn >= nwork) break;
        w = wn;
    }
}

// (t, primitive) as one ordered key: t > 0 for every accepted hit (tri_test
// rejects t <= EPSILON), so its bits order like the floats; the lexicographic
// rule lex_better is then the minimum of the keys.
__device__ __forceinline__ unsigned long long hit_key(float t, int prim) {
    return ((unsigned long long)rt_f32_bits(t) << 32) | (uint32_t)prim;
}

// The queued pairs [0, qn) of far_cell_closest_kernel (qn < 128): the full
// closest test of each, one pair per lane, bounded by the ray's best so far
// (any bound >= the final best gives the same minimum); an accepted hit
// lowers the ray's key. Whole wave.
__device__ __forceinline__ void cell_closest_tests(const DevScene& S, const float4 (*sray)[2],
                                                   unsigned long long* sbest, const uint32_t* pq_id,
                                                   const uint8_t* pq_j, uint32_t qn) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i = lane; i < qn; i += 64) {
        const uint32_t j = pq_j[i], id = pq_id[i];
        const unsigned long long kb = sbest[j];
        const float tcut = kb == ~0ull ? INFINITY : rt_bits_f32((uint32_t)(kb >> 32));
        const float4 a = sray[j][0], b = sray[j][1];
        float t, ba, bb, bg;
        if (prim_test_closest(S.prims[id], v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), t, ba, bb, bg, tcut))
            atomicMin(&sbest[j], hit_key(t, (int)id));
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Cell-major closest-hit far pass over the sorted queue [0, n) of a trace
// level (far-origin rays excluded), on the work items of launch_far_cells:
// far_cell_any_kernel's shape with bvh_closest's far part per ray. A wave
// stages an item's rays and their provisional hits (hit4 / hit_prim) in LDS;
// lanes hold the cell's candidates and step through the rays (far_candidate);
// passing pairs are queued and tested 64 at a time, each hit folded into the
// ray's (t, primitive) key with an LDS atomicMin (= lex_better's order). The
// winner's barycentrics are then recomputed (tri_test's outputs do not depend
// on its bound) and stored if it changed. Plane-tree items walk the tree
// (far_tree_closest_wave). Against far_closest_kernel, whose per-lane list
// walk makes a wave as slow as its longest cell list, one dependent
// entry -> plane -> record chain per step.
__global__ void __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(FAR_ANY_WPE)))
far_cell_closest_kernel(DevScene S, DevWork W) {
    if (frame_poisoned(W)) return;
    __shared__ float4 sray[TB / 64][64][2];
    __shared__ unsigned long long sbest[TB / 64][64];
    __shared__ int32_t stk[TB / 64][RT_BVH_STACK];
    __shared__ uint32_t pq_id[TB / 64][128];
    __shared__ uint8_t pq_j[TB / 64][128];
    const BvhView& V = S.bv;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t nwork = W.far_seg_n[1];
    const uint32_t stride = gridDim.x * (TB / 64);
    for (uint32_t w = blockIdx.x * (TB / 64) + wave; w < nwork; w += stride) {
        const CellItem cur = cell_item(V, W.far_work[w]);
        if (cur.skip) continue;  // no candidate: no far hit in this cell
        uint32_t q, gi;
        cell_indices(V, W, cur, lane, q, gi);
        const bool live = (uint32_t)lane < cur.nr;
        float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b = make_float4(1.0f, 0.0f, 0.0f, 0.0f);
        uint32_t node = 0;
        if (live) {
            a = W.far_rays[2 * (size_t)q];
            b = W.far_rays[2 * (size_t)q + 1];
            node = __float_as_uint(a.w);
        }
        if (cur.tree) {
            Hit h;
            h.t = 0; h.a = h.b = h.g = 0; h.prim = -1;
            if (live) {
                const float4 hv = W.hit4[node];
                h.prim = W.hit_prim[node];
                h.t = hv.x; h.a = hv.y; h.b = hv.z; h.g = hv.w;
            }
            bool found = h.prim >= 0;
            const rv3 o = v3(a.x, a.y, a.z), d = v3(b.x, b.y, b.z);
            if (far_tree_closest_wave(S, live, o, d, far_ray(V, o), h, found, stk[wave])) {
                W.hit4[node] = make_float4(h.t, h.a, h.b, h.g);
                W.hit_prim[node] = h.prim;
            }
            continue;
        }
        const int n_cand = V.n_always + (int)cur.n_list;
        const FarTri ft0 = V.far_tris[gi];
        // the ray's best so far as a key (hit4.x = t, hit_prim)
        unsigned long long k0 = ~0ull;
        if (live) {
            const int hp = W.hit_prim[node];
            if (hp >= 0) k0 = hit_key(W.hit4[node].x, hp);
        }
        // the previous item's LDS reads are done before it is overwritten
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (live) {
            sray[wave][lane][0] = a;
            sray[wave][lane][1] = make_float4(b.x, b.y, b.z, far_ray(V, v3(a.x, a.y, a.z)).R);
            sbest[wave][lane] = k0;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const uint32_t nr = cur.nr;
        uint32_t qn = 0;  // queued (candidate, ray) pairs, wave-uniform
        for (int kc = 0; kc < n_cand; kc += 64) {
            const int lt = n_cand - kc < 64 ? n_cand - kc : 64;
            const int lg = cell_lg(lt);
            const int kk = lane & ((1 << lg) - 1), g = lane >> lg;
            const bool has = kk < lt;
            FarTri ft = ft0;
            if (kc > 0 && has) {
                const int k = kc + kk - V.n_always;
                ft = V.far_tris[k < 0 ? V.grid_always[k + V.n_always] : V.grid_items[cur.lb + (uint32_t)k]];
            }
            const uint32_t step = 64u >> lg;
            for (uint32_t j0 = 0; j0 < nr; j0 += step) {
                const uint32_t j = j0 + (uint32_t)g;
                bool fc = false;
                if (has && j < nr) {
                    const float4 aj = sray[wave][j][0], bj = sray[wave][j][1];
                    FarRay fj;
                    fj.R = bj.w;
                    fc = far_candidate_filter(ft, fj, v3(aj.x, aj.y, aj.z), v3(bj.x, bj.y, bj.z));
                }
                const uint64_t m = __ballot(fc);
                if (m == 0) continue;
                if (fc) {
                    const uint32_t slot = qn + (uint32_t)__popcll(m & lanemask_lt());
                    pq_id[wave][slot] = ft.id;
                    pq_j[wave][slot] = j;
                }
                qn += (uint32_t)__popcll(m);
                if (qn >= 64u) {
                    cell_closest_tests(S, sray[wave], sbest[wave], pq_id[wave], pq_j[wave], qn);
                    qn = 0;
                }
            }
        }
        if (qn) cell_closest_tests(S, sray[wave], sbest[wave], pq_id[wave], pq_j[wave], qn);
        if (live) {
            const unsigned long long kb = sbest[wave][lane];
            if (kb != k0) {  // a far hit won: its full record
                const int id = (int)(uint32_t)kb;
                const float4 ar = sray[wave][lane][0], br = sray[wave][lane][1];
                float t, ba, bb, bg;
                (void)prim_test_closest(S.prims[id], v3(ar.x, ar.y, ar.z), v3(br.x, br.y, br.z), t, ba, bb, bg);
                W.hit4[node] = make_float4(t, ba, bb, bg);
                W.hit_prim[node] = id;
            }
        }
    }
}

// One wave per ray: the lanes stride over every plane with the exact candidate
// test (a superset of what the tree visits: its pruning is only conservative),
// full tests on the candidates, lexicographic wave reduction. Latency-friendly
// for sparse queues, where sorted waves no longer share directions.
// brute != 0: every primitive in scene order with the plain tests (the
// reference's IntersectScene loop), for the far-origin rays.
#ifdef RT580_DIAGNOSTICS
// DIAGNOSTIC build only: brute any-hit scan statistics (rays, steps, rays
// without an acceptor, their steps, rays decided by the call hint)
__device__ unsigned long long g_brute_stats[5];
#endif
#ifndef BRUTE_ANY_U
#define BRUTE_ANY_U 2  // far_scan_kernel brute any-hit: records per lane per ballot step
#endif
__global__ void __launch_bounds__(TB) far_scan_kernel(DevScene S, DevWork W, uint32_t first, uint32_t n, int closest,
                                                      int n_far, int brute, uint8_t* flag) {
    if (frame_poisoned(W)) return;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n_scan = brute ? S.n_prims : n_far;
    for (uint32_t i = first + blockIdx.x * (TB / 64) + wave; i < n; i += gridDim.x * (TB / 64)) {
        const uint32_t r = W.far_vals_alt[i];
        const float4 a = W.far_rays[2 * (size_t)r], b = W.far_rays[2 * (size_t)r + 1];
        const rv3 o = v3(a.x, a.y, a.z), d = v3(b.x, b.y, b.z);
        const uint32_t tag = __float_as_uint(a.w);  // AO call / shadow flag (any) or tree node (closest)
        const float tmax = b.w;                     // any-hit: count a hit only if !(t > tmax)
        if (!brute && dir_zero(d)) continue;
        const FarRay fr = far_ray(S.bv, o);
        if (!closest) {
            bool hit = false;
            // AO rays (flag null, tag = call): the record that accepted another
            // sample of the same call, first (its samples share the far origin and
            // mostly share an acceptor, tools/far_origin_study.cpp)
            uint32_t* hintp = (brute && !flag && W.call_hint) ? W.call_hint + tag : nullptr;
            if (hintp) {
                const uint32_t hk = __builtin_amdgcn_readfirstlane(*hintp);
                if (hk < (uint32_t)n_scan && lane == 0 && prim_hit_within(S.scan_prims[hk], o, d, tmax)) hit = true;
            }
#ifdef RT580_DIAGNOSTICS
            if (brute && lane == 0) {
                atomicAdd(&g_brute_stats[0], 1ull);
                if (hit) atomicAdd(&g_brute_stats[4], 1ull);
            }
            int diag_steps = 0;
#endif
            if (brute && !__ballot(hit)) {
                // BRUTE_ANY_U records per lane in flight per step, then one
                // ballot; any order gives the same boolean
                // in the shuffled order (DevScene::scan_prims): the first acceptor
                // is then ~N / (acceptors + 1) records in instead of up to N
                for (int k0 = 0; k0 < n_scan; k0 += BRUTE_ANY_U * 64) {
                    rt_prim p[BRUTE_ANY_U];
#pragma unroll
                    for (int u = 0; u < BRUTE_ANY_U; u++) {
                        const int k = k0 + u * 64 + lane;
                        if (k < n_scan) p[u] = S.scan_prims[k];
                    }
#ifdef RT580_DIAGNOSTICS
                    diag_steps++;
#endif
                    int found_k = -1;
#pragma unroll
                    for (int u = 0; u < BRUTE_ANY_U; u++) {
                        const int k = k0 + u * 64 + lane;
                        if (k < n_scan && prim_hit_within(p[u], o, d, tmax)) {
                            hit = true;
                            if (found_k < 0) found_k = k;
                        }
                    }
                    const uint64_t fm = __ballot(found_k >= 0);
                    if (fm) {
                        if (hintp && lane == __ffsll((unsigned long long)fm) - 1) *hintp = (uint32_t)found_k;
                        break;
                    }
                }
            }
            for (int k0 = 0; !brute && k0 < n_scan; k0 += 64) {
                const int k = k0 + lane;
                if (k < n_scan) {
                    {
                        const FarTri ft = S.bv.far_tris[k];
                        if (far_candidate(ft, fr, o, d) && prim_test_any(S.prims[ft.id], o, d)) hit = true;
                    }
                }
                if (__ballot(hit)) break;
            }
#ifdef RT580_DIAGNOSTICS
            if (brute && lane == 0) {
                atomicAdd(&g_brute_stats[1], (unsigned long long)diag_steps);
                if (!__ballot(hit)) {
                    atomicAdd(&g_brute_stats[2], 1ull);
                    atomicAdd(&g_brute_stats[3], (unsigned long long)diag_steps);
                }
            }
#endif
            if (__ballot(hit) && lane == 0) any_hit_out(W, flag, tag);
            continue;
        }
        Hit h;
        h.t = 0; h.a = h.b = h.g = 0; h.prim = -1;
        bool found = false;
        for (int k = lane; k < n_scan; k += 64) {
            int id = k;
            if (!brute) {
                const FarTri ft = S.bv.far_tris[k];
                if (!far_candidate(ft, fr, o, d)) continue;
                id = (int)ft.id;
            }
            float t, aa, bb, gg;
            if (prim_test_closest(S.prims[id], o, d, t, aa, bb, gg, found ? h.t : INFINITY) && lex_better(t, id, found, h)) {
                found = true;
                h.t = t; h.a = aa; h.b = bb; h.g = gg; h.prim = id;
            }
        }
        // lexicographic (t, prim) minimum over the wave; t > EPSILON > 0, so the
        // float bits order like the values
        uint64_t key = found ? (((uint64_t)__float_as_uint(h.t) << 32) | (uint32_t)h.prim) : ~0ull;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t other = __shfl_xor(key, off);
            key = other < key ? other : key;
        }
        if (key == ~0ull) continue;
        const bool mine = found && key == ((((uint64_t)__float_as_uint(h.t)) << 32) | (uint32_t)h.prim);
        const uint64_t owner = __ballot(mine);
        if (lane == __ffsll((unsigned long long)owner) - 1) {
            const float4 hv = W.hit4[tag];
            const int32_t hp = W.hit_prim[tag];
            Hit cur;
            cur.t = hv.x; cur.prim = hp;
            if (lex_better(h.t, h.prim, hp >= 0, cur)) {
                W.hit4[tag] = make_float4(h.t, h.a, h.b, h.g);
                W.hit_prim[tag] = h.prim;
            }
        }
    }
}

// Brute closest hit of far-origin tree rays, split: wave w scans slice
// w % splits of the scene for the R rays of group w / splits (few rays, each a
// full scan: one wave per ray left most of the GPU idle and each wave waiting
// on its loads); the slices' lexicographic (t, primitive) minima meet in
// best[r] by a 64-bit atomicMin (t > EPSILON > 0: float bits order like the
// values). A lane loads each record of its stride once and tests it against
// all R rays of the group (wave-uniform: scalar registers), so the scan reads
// the scene once per R rays instead of once per ray.
template <int R>
__global__ void __launch_bounds__(TB) far_brute_split_kernel(DevScene S, DevWork W, uint32_t first, uint32_t nb,
                                                             uint32_t splits, unsigned long long* best) {
    if (frame_poisoned(W)) return;
    // the group's rays and each lane's best (t, primitive) per ray, in LDS (a
    // register copy per ray would cost the kernel its occupancy)
    __shared__ float4 sray[TB / 64][R][2];
    __shared__ float sbt[TB / 64][R][64];
    __shared__ int sbp[TB / 64][R][64];
    const int lane = threadIdx.x & 63;
    const uint32_t ng = (nb + R - 1) / R;
    const uint64_t total = (uint64_t)ng * splits;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t w = (uint64_t)blockIdx.x * (TB / 64) + wave; w < total; w += (uint64_t)gridDim.x * (TB / 64)) {
        const uint32_t gi = (uint32_t)(w / splits), sl = (uint32_t)(w % splits);
        const uint32_t nr = nb - gi * R < (uint32_t)R ? nb - gi * R : (uint32_t)R;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the previous group's LDS reads are done
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if ((uint32_t)lane < 2 * nr) {
            const uint32_t q = W.far_vals_alt[first + gi * R + (uint32_t)(lane >> 1)];
            sray[wave][lane >> 1][lane & 1] = W.far_rays[2 * (size_t)q + (lane & 1)];
        }
        for (int j = 0; j < R; j++) sbp[wave][j][lane] = -1;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        const int n = S.n_prims;
        const int k0 = (int)((uint64_t)n * sl / splits), k1 = (int)((uint64_t)n * (sl + 1) / splits);
        for (int k = k0 + lane; k < k1; k += 64) {
            rt_prim P;
            load_prim(S.prims + k, P);
#pragma unroll 1
            for (uint32_t j = 0; j < nr; j++) {
                const float4 a = sray[wave][j][0], b = sray[wave][j][1];
                const int bp = sbp[wave][j][lane];
                const float bt = sbt[wave][j][lane];
                const bool found = bp >= 0;
                float t, aa, bb, gg;
                if (prim_test_closest(P, v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), t, aa, bb, gg, found ? bt : INFINITY) &&
                    (!found || t < bt || (t == bt && k < bp))) {
                    sbt[wave][j][lane] = t;
                    sbp[wave][j][lane] = k;
                }
            }
        }
        for (uint32_t j = 0; j < nr; j++) {
            const int bp = sbp[wave][j][lane];
            uint64_t key = bp >= 0 ? (((uint64_t)__float_as_uint(sbt[wave][j][lane]) << 32) | (uint32_t)bp) : ~0ull;
            for (int off = 32; off > 0; off >>= 1) {
                const uint64_t other = __shfl_xor(key, off);
                key = other < key ? other : key;
            }
            if (lane == 0 && key != ~0ull) atomicMin(best + gi * R + j, (unsigned long long)key);
        }
    }
}

// The winners of far_brute_split_kernel: the exact test again for (t, alpha,
// beta, gamma), merged into the ray's provisional hit with the same rule.
__global__ void __launch_bounds__(TB) far_brute_merge_kernel(DevScene S, DevWork W, uint32_t first, uint32_t nb,
                                                             const unsigned long long* best) {
    if (frame_poisoned(W)) return;
    for (uint32_t r = blockIdx.x * TB + threadIdx.x; r < nb; r += gridDim.x * TB) {
        const unsigned long long key = best[r];
        if (key == ~0ull) continue;
        const uint32_t q = W.far_vals_alt[first + r];
        const float4 a = W.far_rays[2 * (size_t)q], b = W.far_rays[2 * (size_t)q + 1];
        const rv3 o = v3(a.x, a.y, a.z), d = v3(b.x, b.y, b.z);
        const uint32_t tag = __float_as_uint(a.w);
        const int id = (int)(uint32_t)key;
        Hit h;
        float t, aa, bb, gg;
        if (!prim_test_closest(S.prims[id], o, d, t, aa, bb, gg)) continue;  // (same test: cannot fail)
        h.t = t; h.a = aa; h.b = bb; h.g = gg; h.prim = id;
        const float4 hv = W.hit4[tag];
        const int32_t hp = W.hit_prim[tag];
        Hit cur;
        cur.t = hv.x; cur.prim = hp;
        if (lex_better(h.t, h.prim, hp >= 0, cur)) {
            W.hit4[tag] = make_float4(h.t, h.a, h.b, h.g);
            W.hit_prim[tag] = h.prim;
        }
    }
}

// Brute any-hit scans of far-origin rays (AO samples, shadow rays), split like
// far_brute_split_kernel: wave w scans slice w / ng of the shuffled records for
// the R rays of group w % ng (slice-major, so the first slices of every group
// run first), each record loaded once and tested against the group's rays
// still undecided. One wave per ray left the pass as long as its slowest ray's
// full serial scan (a ray no record accepts reads all of them). A wave drops a
// ray once another slice has found an acceptor for it (done[r], polled at the
// start and every 8 steps); the first slice to find one claims the ray
// (atomicOr on done[r]), so the AO call's occlusion count is raised once per
// ray as in far_scan_kernel. The boolean does not depend on which record
// accepted. AO rays test their call's hint record first (slice 0).
template <int R>
__global__ void __launch_bounds__(TB) far_brute_any_split_kernel(DevScene S, DevWork W, uint32_t first, uint32_t nb,
                                                                 uint32_t splits, uint32_t* done, uint8_t* flag) {
    if (frame_poisoned(W)) return;
    __shared__ float4 sray[TB / 64][R][2];  // the group's rays (register copies would cost occupancy)
    __shared__ int sfk[TB / 64][R];         // an accepting record per ray (the AO call hint)
    const int lane = threadIdx.x & 63;
    const uint32_t ng = (nb + R - 1) / R;
    const uint64_t total = (uint64_t)ng * splits;
    const int n = S.n_prims;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    for (uint64_t w = (uint64_t)blockIdx.x * (TB / 64) + wave; w < total; w += (uint64_t)gridDim.x * (TB / 64)) {
        const uint32_t gi = (uint32_t)(w % ng), sl = (uint32_t)(w / ng);
        const uint32_t nr = nb - gi * R < (uint32_t)R ? nb - gi * R : (uint32_t)R;
        // the group's rays still undecided (wave-uniform bit mask)
        bool und = false;
        if ((uint32_t)lane < nr)
            und = __hip_atomic_load(done + gi * R + (uint32_t)lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u;
        uint32_t live = (uint32_t)__ballot(und);
        if (!live) continue;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the previous group's LDS reads are done
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if ((uint32_t)lane < 2 * nr) {
            const uint32_t q = W.far_vals_alt[first + gi * R + (uint32_t)(lane >> 1)];
            sray[wave][lane >> 1][lane & 1] = W.far_rays[2 * (size_t)q + (lane & 1)];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        uint32_t mine = 0;  // this lane's accepted rays
        if (!flag && W.call_hint && sl == 0 && (uint32_t)lane < nr && ((live >> lane) & 1u)) {
            const float4 a = sray[wave][lane][0], b = sray[wave][lane][1];
            const uint32_t hk = W.call_hint[__float_as_uint(a.w)];
            if (hk < (uint32_t)n && prim_hit_within(S.scan_prims[hk], v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), b.w)) {
                mine = 1u << lane;
                sfk[wave][lane] = (int)hk;
            }
        }
        const int k0 = (int)((uint64_t)n * sl / splits), k1 = (int)((uint64_t)n * (sl + 1) / splits);
        uint32_t decided = 0;
        for (int kb = k0, step = 0;; kb += 64, step++) {
            if (__ballot(mine != 0u)) {  // new acceptors: drop their rays from the scan
                uint32_t m = mine;
                for (int off = 32; off > 0; off >>= 1) m |= (uint32_t)__shfl_xor((int)m, off);
                decided = __builtin_amdgcn_readfirstlane(m);
                live &= ~decided;
            }
            if (!live || kb >= k1) break;
            if ((step & 7) == 7) {
                bool gone = false;
                if ((uint32_t)lane < nr && ((live >> lane) & 1u))
                    gone = __hip_atomic_load(done + gi * R + (uint32_t)lane, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT) != 0u;
                live &= ~(uint32_t)__ballot(gone);
                if (!live) break;
            }
            const int k = kb + lane;
            if (k < k1) {
                rt_prim P;
                load_prim(S.scan_prims + k, P);
                for (uint32_t lv = live; lv;) {
                    const int j = __builtin_ctz(lv);
                    lv &= lv - 1u;
                    const float4 a = sray[wave][j][0], b = sray[wave][j][1];
                    if (prim_hit_within(P, v3(a.x, a.y, a.z), v3(b.x, b.y, b.z), b.w)) {
                        mine |= 1u << j;
                        sfk[wave][j] = k;
                    }
                }
            }
        }
        // claims: for each decided ray, its first accepting lane
        for (uint32_t dv = decided; dv;) {
            const int j = __builtin_ctz(dv);
            dv &= dv - 1u;
            const uint64_t fm = __ballot((mine >> j) & 1u);
            if (lane == __ffsll((unsigned long long)fm) - 1 && atomicOr(done + gi * R + (uint32_t)j, 1u) == 0u) {
                const uint32_t tag = __float_as_uint(sray[wave][j][0].w);
                any_hit_out(W, flag, tag);
                if (!flag && W.call_hint) W.call_hint[tag] = (uint32_t)sfk[wave][j];
            }
        }
    }
}

// Largest slice of the scene one wave scans in the split any-hit brute scan.
constexpr uint32_t kBruteSlice = 4096;

// Waves a split brute scan aims at (ray groups x slices). North-star frame,
// 8192 vs 32768 over three boxes: 38.22 / 38.69 / 36.69 vs 39.27 / 39.04 /
// 37.40 ms; the 8-way share 7.56 vs 7.59 (profiles/r04/ab/bw*, kn2_*): fewer,
// longer waves per launch. Far-origin rays per wave of the split scans: 8.
constexpr uint32_t kBruteWaves = 8192;
constexpr int kBruteRays = 8;

static int grid_for(uint64_t items, int cap);

// The brute any-hit scan of the far-origin rays [first, first + nb) of the
// sorted queue (flag: shadow flags, or null: AO occlusion counts).
static hipError_t launch_brute_any(const DevScene& S, const DevWork& W, uint32_t first, uint32_t nb, uint8_t* flag,
                                   hipStream_t s) {
    if (nb == 0) return hipSuccess;
    {
        // the sort's input keys are free now: one claim word per ray
        uint32_t* done = W.far_keys;
        hipError_t e = hipMemsetAsync(done, 0, (size_t)nb * 4, s);
        if (e != hipSuccess) return e;
        const uint32_t ng = (nb + (uint32_t)kBruteRays - 1) / (uint32_t)kBruteRays;
        uint32_t splits = kBruteWaves / ng;
        splits = splits < 1u ? 1u : (splits > 256u ? 256u : splits);
        // slices of at most kBruteSlice records: a ray no record accepts is
        // scanned in parallel slices even when the queue is long (the AO chunks
        // queue ~10^5 far-origin samples; their groups decided by the call hint
        // skip their later slices through done[])
        splits = std::max(splits, ((uint32_t)S.n_prims + kBruteSlice - 1) / kBruteSlice);
        const dim3 grid(grid_for((uint64_t)ng * splits * 64, 16384));
        hipLaunchKernelGGL(far_brute_any_split_kernel<kBruteRays>, grid, dim3(TB), 0, s, S, W, first, nb, splits, done,
                           flag);
    }
    return hipGetLastError();
}

// Same kernel with the register budget capped for 8 waves per SIMD (SGPR <= 80
// admits 8 workgroups per CU instead of 6).
// call_lo / call_hi (device, may be null): only the items of AO calls
// [*call_lo, *call_hi) (a row range of the frame: its calls are contiguous).
template <int VARIANT>
__global__ void __launch_bounds__(TB) __attribute__((amdgpu_waves_per_eu(8, 8)))
ao_kernel_occ8(DevScene S, DevFrame F, DevWork W, const uint64_t* call_lo, const uint64_t* call_hi) {
    const uint64_t N = (uint64_t)F.ao_samples;
    ao_body<VARIANT>(S, F, W, call_lo ? *call_lo * N : 0ull, call_hi ? *call_hi * N : ~0ull);
}

// ---------------------------------------------------------------- resolve

__device__ __forceinline__ rpix node_local(const DevScene& S, const DevFrame& F, const DevWork& W, const NodeRec& nd,
                                           const rt_material& m, uint32_t node) {
    rpix local = px((int16_t)(nd.local_rg & 0xffff), (int16_t)(nd.local_rg >> 16), (int16_t)(nd.local_b_flags & 0xffff));
    int a = 0;
    for (int li = 0; li < S.n_lights; li++) {
        const rt_light l = S.lights[li];
        if (l.kind != RT_LIGHT_AMBIENT) continue;
        rv3 amb = v3_scale(v3_mul(v3_scale(ld3(m.cs), m.ka), ld3(l.color)), l.intensity);
        float ao = 1.0f;
        if (F.ao_enabled) ao = 1.0f - ((float)W.occ[W.node_call0[node] + a] / (float)F.ao_samples);
        amb = v3_scale(amb, ao);
        local = px_add(local, px_from(amb));
        a++;
    }
    return local;
}


// Level-by-level form of the same blend: one launch per recursion level, from
// the deepest up. A node's value (Raycast's return) is combined from its own
// local colour and its children's values, stored by the previous launch in
// W.node_val (8 bytes per node, not the 64-byte records); level 0 writes the framebuffer. Coalesced over each
// level's contiguous node ids, no per-thread stack.
__device__ __forceinline__ rpix node_val_load(const DevWork& W, int32_t id) {
    if (id < 0) return px(0, 0, 0);
    const int2 v = W.node_val[id];
    return px((int16_t)(v.x & 0xffff), (int16_t)(v.x >> 16), (int16_t)(v.y & 0xffff));
}

// Only the nodes of pixels [p_lo, p_hi) (local pixel index; level 0 nodes are
// the pixels, deeper ones name theirs in W.rays).
__global__ void __launch_bounds__(TB) resolve_level_kernel(DevScene S, DevFrame F, DevWork W, int level,
                                                           int16_t* __restrict__ fb, uint32_t p_lo, uint32_t p_hi) {
    if (S.use_bvh && frame_poisoned(W)) return;
    uint32_t base = p_lo, count = p_hi - p_lo;
    if (level > 0) {  // the trace's own clamp to the node capacity
        base = W.lvl[LVL_BASE + level];
        const uint32_t room = W.node_cap > base ? W.node_cap - base : 0u;
        count = W.lvl[level] < room ? W.lvl[level] : room;
    }
    const bool all = p_lo == 0 && p_hi == (uint32_t)F.n_rows * (uint32_t)F.width;
    for (uint32_t i = blockIdx.x * TB + threadIdx.x; i < count; i += gridDim.x * TB) {
        const uint32_t node = base + i;
        if (level > 0 && !all) {
            const uint32_t px = (uint32_t)W.rays[node].pixel;
            if (px < p_lo || px >= p_hi) continue;
        }
        const NodeRec nd = W.nodes[node];
        const int flags = nd.local_b_flags >> 16;
        rpix v;
        if (!(flags & RT_NODE_HIT)) {
            v = px(254, 64, 205);  // BG_COLOR (Raytracer.h:597)
        } else {
            const rt_material m = S.mats[nd.shape];
            const rpix local = node_local(S, F, W, nd, m, node);
            if (flags & RT_NODE_LEAF) {
                v = px_clamp(local);
            } else {
                const int4 tp = W.topo[node];
                v = combine(local, node_val_load(W, tp.x), node_val_load(W, tp.y), nd.kr, nd.kt, m.ks, m.kt);
            }
        }
        if (level == 0) {
            fb[(size_t)node * 3 + 0] = (int16_t)v.r;
            fb[(size_t)node * 3 + 1] = (int16_t)v.g;
            fb[(size_t)node * 3 + 2] = (int16_t)v.b;
        } else {
            W.node_val[node] =
                make_int2((int32_t)(((uint32_t)v.r & 0xffffu) | ((uint32_t)v.g << 16)), (int32_t)((uint32_t)v.b & 0xffffu));
        }
    }
}

// Exclusive raster-order scan of all ranks' per-row AO calls (one workgroup),
// written out at this rank's rows (rt_gpu_row_bases).
__global__ void __launch_bounds__(1024) row_bases_kernel(const int32_t* __restrict__ gathered, int world, int n_max,
                                                         int height, int rank, uint64_t* __restrict__ out) {
    __shared__ uint64_t part[1024];
    __shared__ uint64_t carry;
    if (threadIdx.x == 0) carry = 0;
    for (int j = threadIdx.x; j < n_max; j += 1024) out[j] = 0;
    __syncthreads();
    for (int b = 0; b < height; b += 1024) {
        const int y = b + threadIdx.x;
        const uint64_t v = y < height ? (uint64_t)(uint32_t)gathered[(y % world) * n_max + y / world] : 0;
        part[threadIdx.x] = v;
        __syncthreads();
        for (int s = 1; s < 1024; s <<= 1) {
            const uint64_t add = threadIdx.x >= s ? part[threadIdx.x - s] : 0;
            __syncthreads();
            part[threadIdx.x] += add;
            __syncthreads();
        }
        if (y < height && y % world == rank) out[y / world] = carry + part[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 1023) carry += part[1023];
        __syncthreads();
    }
}

hipError_t launch_row_bases(const int32_t* gathered, int world, int n_max, int height, int rank, uint64_t* out,
                            hipStream_t s) {
    hipLaunchKernelGGL(row_bases_kernel, dim3(1), dim3(1024), 0, s, gathered, world, n_max, height, rank, out);
    return hipGetLastError();
}

static int grid_for(uint64_t items, int cap) {
    uint64_t b = (items + TB - 1) / TB;
    if (b < 1) b = 1;
    return (int)(b < (uint64_t)cap ? b : (uint64_t)cap);
}

// Workgroups of a recursion level > 0 (trace and resolve; grid-stride over the
// level's count, which only the device knows): RT580_DEEP_GRID for A/B.
constexpr int kDeepGrid = 512;  // 4096 / 1024 / 512: config 2 1.562 / 1.561 / 1.550 ms, its 8-way share 0.324 / 0.323 / 0.319

// RT580_PROGRESS=1: a stderr line per trace level / AO chunk of the BVH path
// (those already synchronize), so multi-minute frames show progress.
static void progress(const char* fmt, ...) {
    static int on = -1;
    if (on < 0) {
        const char* e = getenv("RT580_PROGRESS");
        on = e && atoi(e) > 0;
    }
    if (!on) return;
    va_list ap;
    va_start(ap, fmt);
    fprintf(stderr, "[rt580] ");
    vfprintf(stderr, fmt, ap);
    fprintf(stderr, "\n");
    fflush(stderr);
    va_end(ap);
}

// Which launcher step failed last (error messages of the shim).
static const char* g_where = "";
const char* launch_where() { return g_where; }
#define RT_STEP(what) (g_where = (what))

static thread_local CountSchedule* g_cs = nullptr;
void set_count_schedule(CountSchedule* cs) { g_cs = cs; }

// A replayed count against the frame's own. bad[0] = 1 on any mismatch; the
// first mismatch of the frame also records which count (bad[1] = its index in
// the schedule + 1) and both values (bad[2..3] the frame's, bad[4..5] the
// recorded ones), for the error message (rt_shim.cpp check_replay).
__global__ void count_check_kernel(const uint32_t* dev, uint32_t e0, uint32_t e1, int n, uint32_t* bad,
                                   uint32_t pos) {
    if (threadIdx.x != 0) return;
    const uint32_t a0 = dev[0], a1 = n > 1 ? dev[1] : 0u;
    if (a0 == e0 && (n < 2 || a1 == e1)) return;
    bad[0] = 1u;
    if (atomicCAS(&bad[1], 0u, pos + 1u) == 0u) {
        bad[2] = a0;
        bad[3] = a1;
        bad[4] = e0;
        bad[5] = n > 1 ? e1 : 0u;
    }
}

// n (1 or 2) device words -> out (pinned), through the count schedule. Each
// count sizes launches over a buffer: out[0] <= cap0 and out[1] <= cap1, else
// the frame fails before anything is launched from it (a replayed count that
// does not fit is a broken schedule; a read one, a queue that overran).
static hipError_t counts_fit(const uint32_t* out, int n, uint32_t cap0, uint32_t cap1) {
    if (out[0] <= cap0 && (n < 2 || out[1] <= cap1)) return hipSuccess;
    if (g_cs && g_cs->mode == CountSchedule::REPLAY) g_cs->broken = true;
    RT_STEP("count check (a device count exceeds its buffer's capacity)");
    return hipErrorInvalidValue;
}

static hipError_t read_counts(const uint32_t* dev, int n, uint32_t* out, hipStream_t s, uint32_t cap0,
                              uint32_t cap1 = 0xffffffffu) {
    if (g_cs && g_cs->mode == CountSchedule::REPLAY) {
        if (g_cs->pos + (size_t)n > g_cs->vals.size()) {
            g_cs->broken = true;
            return hipErrorInvalidValue;
        }
        const uint32_t pos = (uint32_t)g_cs->pos | (g_cs->tag << 16);
        for (int i = 0; i < n; i++) out[i] = g_cs->vals[g_cs->pos++];
#ifdef RT580_DIAGNOSTICS
        // DIAGNOSTIC build only, RT580_REPLAY_CORRUPT: 1 makes every device
        // check fail (the launches are still sized by the right counts); 2
        // replays a wrong far-queue segment count itself (its capacity, the
        // queue length), so the launches after it are sized by a count larger
        // than the frame's and would cover stale entries (frame_poisoned, the
        // bound in far_chunk_*_kernel: the call must end as RT_FAILURE, with no
        // device fault)
        static int corrupt = -1;
        if (corrupt < 0) {
            const char* ev = getenv("RT580_REPLAY_CORRUPT");
            corrupt = ev ? atoi(ev) : 0;
        }
        if (corrupt == 2 && n == 1 && !strcmp(g_where, "far queue segments"))
            out[0] = out[0] < cap0 ? cap0 : out[0] - 1u;
#endif
        if (counts_fit(out, n, cap0, cap1) != hipSuccess) return hipErrorInvalidValue;
        uint32_t e0 = out[0];
#ifdef RT580_DIAGNOSTICS
        if (corrupt == 1) e0 ^= 1u;
#endif
        hipLaunchKernelGGL(count_check_kernel, dim3(1), dim3(64), 0, s, dev, e0, n > 1 ? out[1] : 0u, n, g_cs->bad,
                           pos);
        return hipGetLastError();
    }
    hipError_t e = hipMemcpyAsync(out, dev, (size_t)n * 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e == hipSuccess) e = counts_fit(out, n, cap0, cap1);
    if (e == hipSuccess && g_cs && g_cs->mode == CountSchedule::RECORD)
        for (int i = 0; i < n; i++) {
            g_cs->vals.push_back(out[i]);
            g_cs->where.push_back(g_where);
        }
    return e;
}

// Queues of at most kSmallSort rays: one workgroup sorts them in LDS (one
// launch) instead of the device-wide radix sort's chain of ~5-20 launches
// (per pass a histogram, a scan, a scatter, and their fills), which at a
// K-way row share's queue sizes is latency, not work. Stable on the same bits,
// so the same order. Padding keys sort after every real key (all ones).
constexpr int kSmallSortThreads = 512, kSmallSortItems = 8;
constexpr uint32_t kSmallSort = kSmallSortThreads * kSmallSortItems;
__global__ void __launch_bounds__(kSmallSortThreads)
small_sort_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, uint32_t n, int begin_bit,
                  int end_bit, uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out) {
    using Sort = hipcub::BlockRadixSort<uint32_t, kSmallSortThreads, kSmallSortItems, uint32_t>;
    __shared__ typename Sort::TempStorage tmp;
    uint32_t k[kSmallSortItems], v[kSmallSortItems];
#pragma unroll
    for (int q = 0; q < kSmallSortItems; q++) {
        const uint32_t i = threadIdx.x * kSmallSortItems + q;  // blocked arrangement: input order kept per thread
        k[q] = i < n ? keys[i] : 0xffffffffu;
        v[q] = i < n ? vals[i] : 0u;
    }
    Sort(tmp).Sort(k, v, begin_bit, end_bit);
#pragma unroll
    for (int q = 0; q < kSmallSortItems; q++) {
        const uint32_t i = threadIdx.x * kSmallSortItems + q;
        if (i < n) {
            keys_out[i] = k[q];
            vals_out[i] = v[q];
        }
    }
}

// Work items of the cell pass: segment k (W.far_vals[k] rays) is cut into
// ceil(count / 64) chunks; chunk counts first (into far_keys_alt, free after
// the run-length encoding), then, after their scan into far_wofs, one entry
// per chunk naming its segment, and the total.
// nseg is the host's (possibly replayed) count; both kernels also bound it by
// the device's own (far_seg_n[0], written by the run-length encoding), so a
// replayed count larger than the frame's never reads the stale entries beyond
// it (their chunk counts would size work items past far_work's end).
__global__ void far_chunk_count_kernel(DevWork W, uint32_t nseg) {
    if (frame_poisoned(W)) return;
    const uint32_t m = min(nseg, W.far_seg_n[0]);
    for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < nseg; k += gridDim.x * blockDim.x)
        W.far_keys_alt[k] = k < m ? (W.far_vals[k] + 63u) / 64u : 0u;
}
// One descriptor per work item (sorted rays [x, y), the cell list's first
// entry z and length w; w = ~0: a plane-tree segment), so the cell pass reads
// one record per item instead of a chain of lookups. A lane per segment writes
// its first item; the rare segments of more than 64 rays (a directional
// light's shadow rays all share a cell) get their other items from the whole
// wave. (A wave per segment: 265-350 us for the AO queue's ~3M segments.)
__global__ void far_chunk_expand_kernel(DevScene S, DevWork W, uint32_t nseg, uint32_t n) {
    if (frame_poisoned(W)) return;
    const int lane = threadIdx.x & 63;
    const int shift = 24 - 2 * S.bv.grid_log2;
    nseg = min(nseg, W.far_seg_n[0]);  // (see far_chunk_count_kernel)
    for (uint32_t base = (blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)) * 64u; base < nseg;
         base += gridDim.x * blockDim.x) {
        const uint32_t k = base + (uint32_t)lane;
        const bool valid = k < nseg;
        uint32_t b = 0, c = 0, s0 = 0, s1 = 0, lb = 0, lw = 0xffffffffu;
        if (valid) {
            b = W.far_wofs[k];
            c = W.far_keys_alt[k];
            const uint32_t key = W.far_keys[k];
            s0 = W.far_seg_off[k];
            s1 = k + 1 < nseg ? W.far_seg_off[k + 1] : n;
            if (key < RT_KEY_TREE) {
                const uint32_t cell = key >> shift;
                lb = S.bv.grid_start[cell];
                lw = S.bv.grid_start[cell + 1] - lb;
            }
            W.far_work[b] = make_uint4(s0, s1 - s0 < 64u ? s1 : s0 + 64u, lb, lw);
            if (k == nseg - 1) W.far_seg_n[1] = b + c;
        }
        uint64_t big = __ballot(valid && c > 1u);
        while (big) {
            const int src = __ffsll((unsigned long long)big) - 1;
            big &= big - 1;
            const uint32_t bb = (uint32_t)__shfl((int)b, src), cc = (uint32_t)__shfl((int)c, src);
            const uint32_t ss0 = (uint32_t)__shfl((int)s0, src), ss1 = (uint32_t)__shfl((int)s1, src);
            const uint32_t llb = (uint32_t)__shfl((int)lb, src), llw = (uint32_t)__shfl((int)lw, src);
            for (uint32_t j = 1u + (uint32_t)lane; j < cc; j += 64u) {
                const uint32_t r0 = ss0 + 64u * j;
                W.far_work[bb + j] = make_uint4(r0, ss1 - r0 < 64u ? ss1 : r0 + 64u, llb, llw);
            }
        }
    }
}

// launch_far_cells' segments and work items of a queue of n <= kSmallSort
// sorted rays in one workgroup (one launch instead of the run-length encoding,
// the segment-count read, two scans and two kernels): a segment starts where
// the key changes; its chunks of <= 64 rays become work items (sorted rays
// [r0, r1), the cell list's first entry and length, or ~0 for a plane-tree
// key), in segment order; far_seg_n = (segments, work items).
__global__ void __launch_bounds__(kSmallSortThreads) small_cells_kernel(DevScene S, DevWork W, uint32_t n) {
    if (frame_poisoned(W)) return;
    using Scan = hipcub::BlockScan<uint32_t, kSmallSortThreads>;
    __shared__ typename Scan::TempStorage scan_tmp;
    __shared__ uint32_t seg_start[kSmallSort + 1];
    __shared__ uint32_t s_nseg;
    const int shift = 24 - 2 * S.bv.grid_log2;
    uint32_t key[kSmallSortItems], f[kSmallSortItems], idx[kSmallSortItems];
#pragma unroll
    for (int q = 0; q < kSmallSortItems; q++) {
        const uint32_t i = threadIdx.x * kSmallSortItems + q;
        key[q] = i < n ? W.far_keys_alt[i] : 0u;
        f[q] = i < n && (i == 0 || W.far_keys_alt[i - 1] != key[q]) ? 1u : 0u;
    }
    uint32_t nseg = 0;
    Scan(scan_tmp).ExclusiveSum(f, idx, nseg);
#pragma unroll
    for (int q = 0; q < kSmallSortItems; q++)
        if (f[q]) seg_start[idx[q]] = threadIdx.x * kSmallSortItems + q;
    if (threadIdx.x == 0) {
        seg_start[nseg] = n;
        s_nseg = nseg;
    }
    __syncthreads();
    uint32_t cnt[kSmallSortItems], wofs[kSmallSortItems];
#pragma unroll
    for (int q = 0; q < kSmallSortItems; q++) {
        const uint32_t i = threadIdx.x * kSmallSortItems + q;
        cnt[q] = f[q] ? (seg_start[idx[q] + 1] - i + 63u) / 64u : 0u;
    }
    uint32_t nwork = 0;
    __syncthreads();  // scan_tmp reused
    Scan(scan_tmp).ExclusiveSum(cnt, wofs, nwork);
#pragma unroll
    for (int q = 0; q < kSmallSortItems; q++) {
        if (!f[q]) continue;
        const uint32_t s0 = threadIdx.x * kSmallSortItems + q, s1 = seg_start[idx[q] + 1];
        uint32_t lb = 0, lw = 0xffffffffu;
        if (key[q] < RT_KEY_TREE) {
            const uint32_t cell = key[q] >> shift;
            lb = S.bv.grid_start[cell];
            lw = S.bv.grid_start[cell + 1] - lb;
        }
        for (uint32_t j = 0; j < cnt[q]; j++) {
            const uint32_t r0 = s0 + 64u * j;
            W.far_work[wofs[q] + j] = make_uint4(r0, s1 - r0 < 64u ? s1 : r0 + 64u, lb, lw);
        }
    }
    if (threadIdx.x == 0) {
        W.far_seg_n[0] = s_nseg;
        W.far_seg_n[1] = nwork;
    }
}

// The any-hit far pass over the sorted queue [0, n) (far-origin rays
// excluded): segments of one key (run-length encoding of the sorted keys into
// far_keys / far_vals -- the sort's inputs, free now -- and the exclusive scan
// of the run lengths), their chunks of <= 64 rays as work items, then
// far_cell_any_kernel. One host read (the segment count).
static hipError_t launch_far_cells(const DevScene& S, const DevWork& W, uint32_t n, uint8_t* flag, hipStream_t s,
                                   bool closest = false) {
    if (n <= kSmallSort) {  // segments and work items in one workgroup
        RT_STEP("far queue small segments");
        hipLaunchKernelGGL(small_cells_kernel, dim3(1), dim3(kSmallSortThreads), 0, s, S, W, n);
        RT_STEP("far cell pass");
        const dim3 cg(grid_for((uint64_t)n * 64, 16384));  // work items <= rays
        if (closest)
            hipLaunchKernelGGL(far_cell_closest_kernel, cg, dim3(TB), 0, s, S, W);
        else
            hipLaunchKernelGGL(far_cell_any_kernel, cg, dim3(TB), 0, s, S, W, n, flag);
        return hipGetLastError();
    }
    size_t tmp = W.sort_tmp_bytes;
    RT_STEP("far queue segments");
    hipError_t e = hipcub::DeviceRunLengthEncode::Encode(W.sort_tmp, tmp, W.far_keys_alt, W.far_keys, W.far_vals,
                                                         W.far_seg_n, (int)n, s);
    if (e == hipSuccess) e = read_counts(W.far_seg_n, 1, W.far_count_host + 2, s, n);
    if (e != hipSuccess) return e;
    const uint32_t nseg = W.far_count_host[2];
    if (nseg == 0) return hipSuccess;
    tmp = W.sort_tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(W.sort_tmp, tmp, W.far_vals, W.far_seg_off, (int)nseg, s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(far_chunk_count_kernel, dim3(grid_for(nseg, 4096)), dim3(TB), 0, s, W, nseg);
    tmp = W.sort_tmp_bytes;
    if ((e = hipcub::DeviceScan::ExclusiveSum(W.sort_tmp, tmp, W.far_keys_alt, W.far_wofs, (int)nseg, s)) != hipSuccess)
        return e;
    hipLaunchKernelGGL(far_chunk_expand_kernel, dim3(grid_for(nseg, 16384)), dim3(TB), 0, s, S, W, nseg, n);
    RT_STEP("far cell pass");
#ifdef RT580_DIAGNOSTICS
    {
        const char* ev = getenv("RT580_CELL_SKIP");
        const int sk = ev ? atoi(ev) : 0;
        if ((e = hipStreamSynchronize(s)) != hipSuccess ||
            (e = hipMemcpyToSymbol(HIP_SYMBOL(g_cell_skip), &sk, sizeof sk, 0, hipMemcpyHostToDevice)) != hipSuccess)
            return e;
    }
#endif
    const dim3 cgrid(grid_for((uint64_t)(n / 64 + nseg) * 64, 16384));
    if (closest)
        hipLaunchKernelGGL(far_cell_closest_kernel, cgrid, dim3(TB), 0, s, S, W);
    else
        hipLaunchKernelGGL(far_cell_any_kernel, cgrid, dim3(TB), 0, s, S, W, n, flag);
#ifdef RT580_DIAGNOSTICS
    {
        uint32_t nw[2] = {0, 0};
        if (hipMemcpyAsync(nw, W.far_seg_n, 8, hipMemcpyDeviceToHost, s) == hipSuccess && hipStreamSynchronize(s) == hipSuccess)
            progress("far cell pass: rays %u segments %u work items %u", n, nw[0], nw[1]);
    }
#endif
    return hipGetLastError();
}

__constant__ uint8_t c_gamma_lut[256];

__global__ void gamma_u8_kernel(const int16_t* __restrict__ fb, uint64_t n, uint8_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const int v = fb[i];
        out[i] = c_gamma_lut[v < 0 ? 0 : (v > 255 ? 255 : v)];
    }
}

hipError_t upload_gamma_lut(const uint8_t* lut, hipStream_t s) {
    return hipMemcpyToSymbolAsync(HIP_SYMBOL(c_gamma_lut), lut, 256, 0, hipMemcpyHostToDevice, s);
}

hipError_t launch_gamma_u8(const int16_t* fb, uint64_t n, uint8_t* out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(gamma_u8_kernel, dim3(grid_for(n, 8192)), dim3(TB), 0, s, fb, n, out);
    return hipGetLastError();
}

// 16 pixel bytes per lane, one 16-byte store: the form for an `out` in mapped
// host memory (the PPM body written over the host link by the kernel itself,
// no separate copy; whole 16-byte stores keep the link's write combining
// full). The LUT is staged in LDS (per-lane indices).
__device__ __forceinline__ uint32_t gamma4(const uint32_t* lut, uint32_t lo, uint32_t hi) {
    auto one = [&](int v) { return lut[v < 0 ? 0 : (v > 255 ? 255 : v)]; };
    return one((int16_t)(lo & 0xffffu)) | (one((int16_t)(lo >> 16)) << 8) | (one((int16_t)(hi & 0xffffu)) << 16) |
           (one((int16_t)(hi >> 16)) << 24);
}
__global__ void __launch_bounds__(TB) gamma_u8_wide_kernel(const int16_t* __restrict__ fb, uint64_t n16,
                                                           uint8_t* __restrict__ out) {
    __shared__ uint32_t lut[256];
    for (int k = threadIdx.x; k < 256; k += TB) lut[k] = c_gamma_lut[k];
    __syncthreads();
    const uint4* src = reinterpret_cast<const uint4*>(fb);
    uint4* dst = reinterpret_cast<uint4*>(out);
    for (uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * TB) {
        const uint4 a = src[2 * i], b = src[2 * i + 1];
        dst[i] = make_uint4(gamma4(lut, a.x, a.y), gamma4(lut, a.z, a.w), gamma4(lut, b.x, b.y), gamma4(lut, b.z, b.w));
    }
}

// Workgroups of the kernels that write mapped host memory. Their waves wait on
// the host link (~55 GB/s), so a few suffice to keep it busy; a full grid would
// hold most of the chip's wave slots for the whole transfer, away from the other
// frames' kernels (16 to 4096 workgroups: no difference in the step).
constexpr int kD2HBlocks = 64;

hipError_t launch_gamma_u8_wide(const int16_t* fb, uint64_t n, uint8_t* out, hipStream_t s) {
    const uint64_t n16 = n / 16;
    if (n16) hipLaunchKernelGGL(gamma_u8_wide_kernel, dim3(grid_for(n16, kD2HBlocks)), dim3(TB), 0, s, fb, n16, out);
    if (n > n16 * 16)
        hipLaunchKernelGGL(gamma_u8_kernel, dim3(1), dim3(TB), 0, s, fb + n16 * 16, n - n16 * 16, out + n16 * 16);
    return hipGetLastError();
}

// A rank's rows (rows row0, row0 + step, ... of the frame; n_rows int16 rows of
// `width` pixels, packed) mapped to PPM bytes and stored at their places in the
// whole frame's body `out` (mapped host memory shared by the ranks, or any
// frame-sized buffer): each rank writes its own rows over its own host link,
// no gather. 16 bytes per lane when a row is a whole number of them.
__global__ void __launch_bounds__(TB) gamma_rows_u8_wide_kernel(const int16_t* __restrict__ fb, uint32_t row16,
                                                                uint32_t n_rows, uint32_t row0, uint32_t step,
                                                                uint8_t* __restrict__ out) {
    __shared__ uint32_t lut[256];
    for (int k = threadIdx.x; k < 256; k += TB) lut[k] = c_gamma_lut[k];
    __syncthreads();
    const uint4* src = reinterpret_cast<const uint4*>(fb);
    uint4* dst = reinterpret_cast<uint4*>(out);
    const uint64_t total = (uint64_t)row16 * n_rows;
    for (uint64_t i = (uint64_t)blockIdx.x * TB + threadIdx.x; i < total; i += (uint64_t)gridDim.x * TB) {
        const uint64_t y = i / row16, e = i - y * row16;
        const uint4 a = src[2 * i], b = src[2 * i + 1];
        dst[(row0 + y * step) * row16 + e] =
            make_uint4(gamma4(lut, a.x, a.y), gamma4(lut, a.z, a.w), gamma4(lut, b.x, b.y), gamma4(lut, b.z, b.w));
    }
}
__global__ void gamma_rows_u8_kernel(const int16_t* __restrict__ fb, uint32_t row_bytes, uint32_t n_rows,
                                     uint32_t row0, uint32_t step, uint8_t* __restrict__ out) {
    const uint64_t total = (uint64_t)row_bytes * n_rows;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t y = i / row_bytes, e = i - y * row_bytes;
        const int v = fb[i];
        out[(row0 + y * step) * row_bytes + e] = c_gamma_lut[v < 0 ? 0 : (v > 255 ? 255 : v)];
    }
}

hipError_t launch_gamma_rows_u8(const int16_t* fb, int n_rows, int width, int row0, int step, uint8_t* out,
                                hipStream_t s) {
    const uint32_t rb = (uint32_t)width * 3u;
    if (n_rows <= 0 || rb == 0) return hipSuccess;
    if (rb % 16 == 0 && ((uintptr_t)out % 16) == 0 && ((uintptr_t)fb % 32) == 0)
        hipLaunchKernelGGL(gamma_rows_u8_wide_kernel, dim3(grid_for((uint64_t)rb / 16 * n_rows, kD2HBlocks)), dim3(TB),
                           0, s, fb, rb / 16, (uint32_t)n_rows, (uint32_t)row0, (uint32_t)step, out);
    else
        hipLaunchKernelGGL(gamma_rows_u8_kernel, dim3(grid_for((uint64_t)rb * n_rows, 8192)), dim3(TB), 0, s, fb, rb,
                           (uint32_t)n_rows, (uint32_t)row0, (uint32_t)step, out);
    return hipGetLastError();
}

// One read of host memory from the device after this device's writes into it
// (a rank's rows in the shared host frame): a read does not pass the earlier
// posted writes of its requester on the host link, so when it completes every
// byte those writes carried is in host memory -- whatever path the frame's
// "done" signal later takes to the rank that reads the frame (the 4-byte
// all-gather over xGMI). The value lands in a device word.
__global__ void host_flush_read_kernel(const volatile uint32_t* p, uint32_t* sink) {
    if (threadIdx.x == 0) sink[0] = p[0];
}

hipError_t launch_host_flush_read(const void* host_dev, uint32_t* sink, hipStream_t s) {
    hipLaunchKernelGGL(host_flush_read_kernel, dim3(1), dim3(64), 0, s,
                       (const volatile uint32_t*)((uintptr_t)host_dev & ~(uintptr_t)3), sink);
    return hipGetLastError();
}

// ---------------------------------------------------------------- math self-test
// The device-only fast sequences against the plain operations they replace:
//  [0] rt_sqrt_nr vs sqrtf over EVERY float in [2^-96, +inf] and +0
//  [1] rt_div_nr vs '/' for n random pairs (|num| in [2^-60, 4] or +-0, den in [0.5, 2])
//  [2] v3_normalize_unit vs v3_normalize for n random vectors (|v| in ~[0.5, 2])
//  [3] rt_ao_dir_xy vs glibc sincos (rt_glibc_sincos_simd_t) for n random AO samples
__device__ __forceinline__ uint64_t st_mix(uint64_t x) {  // splitmix64
    x += 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ float st_float(uint64_t r, int emin, int emax) {  // random sign/exponent/mantissa
    const int e = emin + (int)((r >> 24) % (uint64_t)(emax - emin + 1));
    const uint32_t bits = ((uint32_t)(e + 127) << 23) | (uint32_t)(r & 0x7fffffu) | ((uint32_t)(r >> 63) << 31);
    return __uint_as_float(bits);
}
__global__ void math_selftest_kernel(uint64_t seed, uint64_t n, unsigned long long* bad) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lo = __float_as_uint(0x1p-96f), hi = 0x7f800000u;  // +inf
    unsigned long long b[4] = {0, 0, 0, 0};
    for (uint64_t u = i0; u <= (uint64_t)(hi - lo) + 1; u += stride) {
        const float x = u == (uint64_t)(hi - lo) + 1 ? 0.0f : __uint_as_float(lo + (uint32_t)u);
        if (__float_as_uint(rt_sqrt_nr(x)) != __float_as_uint(sqrtf(x))) b[0]++;
    }
    for (uint64_t i = i0; i < n; i += stride) {
        const uint64_t r0 = st_mix(seed ^ (i * 4)), r1 = st_mix(seed ^ (i * 4 + 1)), r2 = st_mix(seed ^ (i * 4 + 2));
        const uint64_t r3 = st_mix(seed ^ (i * 4 + 3));
        // [1] division
        float num = st_float(r0, -60, 1);
        if ((r0 & 0xff00000000ull) == 0) num = (r0 & 1) ? -0.0f : 0.0f;
        const float den = fabsf(st_float(r1, -1, 0));
        const float y0 = __builtin_amdgcn_rcpf(den);
        const float y = __builtin_fmaf(__builtin_fmaf(-den, y0, 1.0f), y0, y0);
        if (__float_as_uint(rt_div_nr(num, den, y)) != __float_as_uint(num / den)) b[1]++;
        // [2] normalize: components of a vector of length ~[0.5, 2], some exact zeros
        rv3 v = v3(st_float(r1, -30, 0), st_float(r2, -30, 0), st_float(r3, -30, 0));
        const float sc = 0.5f + (float)(r0 & 0xffff) * (1.5f / 65536.0f);
        v = v3_scale(v3_normalize(v), sc);
        if ((r3 & 0xf) == 0) v.x = 0.0f;
        if ((r3 & 0xf0) == 0) v.y = -0.0f;
        const rv3 a = v3_normalize_unit(v), e = v3_normalize(v);
        if (__float_as_uint(a.x) != __float_as_uint(e.x) || __float_as_uint(a.y) != __float_as_uint(e.y) ||
            __float_as_uint(a.z) != __float_as_uint(e.z)) b[2]++;
        // [3] AO direction from the sampler's canonical floats (Raytracer.cpp:270-278)
        const float u0 = canon_minstd(1u + (uint32_t)(r2 % 2147483646u));
        const float u1 = canon_minstd(1u + (uint32_t)(r3 % 2147483646u));
        const float z = u0 * (1.0f - (-1.0f)) + (-1.0f);
        const float ang = u1 * ((float)(2 * 3.14159265) - 0.0f) + 0.0f;
        const float rr = sqrtf(1 - z * z);
        float fx, fy;
        rt_ao_dir_xy(rt_dev::rt_sincostab, rr, ang, &fx, &fy);
        double sa, ca;
        rt_glibc_sincos_simd_t(rt_dev::rt_sincostab, (double)ang, &sa, &ca);
        if (__float_as_uint(fx) != __float_as_uint((float)((double)rr * ca)) ||
            __float_as_uint(fy) != __float_as_uint((float)((double)rr * sa))) b[3]++;
    }
    for (int k = 0; k < 4; k++)
        if (b[k]) atomicAdd(bad + k, b[k]);
}

// The device restatement of glibc powf (rt_libm.h), as CalculateLocalColor
// calls it (Raytracer.cpp:253), over caller-given inputs: checked against the
// host's glibc by tests/test_gpu_libm.py.
// ---------------------------------------------------------------- mt19937 windows
// The twist of a 624-word window (rt_mt.h: W_n = y_n .. y_{n+623} -> the next
// 624 words, draws n .. n+623), in phases over a workgroup: words [0, 227) read
// only old words, [227, 454) and [454, 623) the new words 227 before them, 623
// also the new word 0 -- then every draw tempered (libstdc++ random.tcc / MSVC).
__device__ __forceinline__ uint32_t mt_twist(uint32_t yn, uint32_t yn1, uint32_t yn397) {
    const uint32_t y = (yn & 0x80000000u) | (yn1 & 0x7fffffffu);
    return yn397 ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

__global__ void __launch_bounds__(TB) mt_generate_kernel(const uint32_t* __restrict__ windows, uint64_t k0,
                                                         uint64_t lo, uint64_t hi, uint32_t* __restrict__ out) {
    __shared__ uint32_t buf[2][624];
    const uint64_t blk = (uint64_t)kMtBlock;
    const uint64_t start = (k0 + blockIdx.x) * blk;  // absolute index of this block's first draw
    const uint32_t* w = windows + (size_t)blockIdx.x * 624;
    for (int i = threadIdx.x; i < 624; i += TB) buf[0][i] = w[i];
    __syncthreads();
    int cur = 0;
    for (uint64_t d0 = start; d0 < start + blk && d0 < hi; d0 += 624) {
        const uint32_t* o = buf[cur];
        uint32_t* n = buf[cur ^ 1];
        const int i = threadIdx.x;
        if (i < 227) n[i] = mt_twist(o[i], o[i + 1], o[i + 397]);
        __syncthreads();
        if (i < 227) n[227 + i] = mt_twist(o[227 + i], o[228 + i], n[i]);
        __syncthreads();
        if (i < 169) n[454 + i] = mt_twist(o[454 + i], o[455 + i], n[227 + i]);
        __syncthreads();
        if (i == 0) n[623] = mt_twist(o[623], n[0], n[396]);
        __syncthreads();
        for (int k = threadIdx.x; k < 624; k += TB) {
            const uint64_t d = d0 + (uint64_t)k;
            if (d >= lo && d < hi) out[d - lo] = mt_temper(n[k]);
        }
        cur ^= 1;
        // (the next twist writes buf[cur ^ 1], which this one read: the barriers above order it)
        __syncthreads();
    }
}

hipError_t launch_mt_generate(const uint32_t* windows, uint64_t k0, uint32_t nblk, uint64_t lo, uint64_t hi,
                              uint32_t* out, hipStream_t s) {
    if (nblk == 0 || hi <= lo) return hipSuccess;
    hipLaunchKernelGGL(mt_generate_kernel, dim3(nblk), dim3(TB), 0, s, windows, k0, lo, hi, out);
    return hipGetLastError();
}

__global__ void powf_eval_kernel(const float* __restrict__ x, float y, float* __restrict__ out, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        out[i] = rt_glibc_powf(x[i], y);
}

hipError_t launch_powf_eval(const float* x, float y, float* out, uint64_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(powf_eval_kernel, dim3(grid_for(n, 16384)), dim3(TB), 0, s, x, y, out, n);
    return hipGetLastError();
}

hipError_t launch_math_selftest(uint64_t seed, uint64_t n, unsigned long long* bad, hipStream_t s) {
    hipLaunchKernelGGL(math_selftest_kernel, dim3(16384), dim3(TB), 0, s, seed, n, bad);
    return hipGetLastError();
}

__global__ void copy_rows_kernel(const int16_t* __restrict__ src, int width, int row_begin, int row_step, int n_rows,
                                 int16_t* __restrict__ dst) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t per_row = (size_t)width * 3;
    if (i >= per_row * (size_t)n_rows) return;
    const size_t k = i / per_row, e = i - k * per_row;
    dst[i] = src[(size_t)(row_begin + k * row_step) * per_row + e];
}

// (T = int16_t: the Pixel framebuffer; uint8_t: the PPM body)
template <typename T>
__global__ void deinterleave_kernel(const T* __restrict__ tiles, int world, int n_max, int width, int height,
                                    T* __restrict__ out) {
    const size_t per_row = (size_t)width * 3;
    const size_t total = per_row * (size_t)height;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t y = i / per_row, e = i - y * per_row;
        const size_t r = y % (size_t)world, j = y / (size_t)world;
        out[i] = tiles[(r * (size_t)n_max + j) * per_row + e];
    }
}

hipError_t launch_deinterleave(const int16_t* tiles, int world, int n_max, int width, int height, int16_t* out,
                               hipStream_t s) {
    const uint64_t n = (uint64_t)width * 3 * height;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(deinterleave_kernel<int16_t>, dim3(grid_for(n, 16384)), dim3(256), 0, s, tiles, world, n_max,
                       width, height, out);
    return hipGetLastError();
}

// 16 bytes per lane when a row is a whole number of them (1920 x 3 is): the
// form for an `out` in mapped host memory, like gamma_u8_wide_kernel
__global__ void deinterleave_u8_wide_kernel(const uint4* __restrict__ tiles, int world, int n_max, int row16,
                                            int height, uint4* __restrict__ out) {
    const size_t total = (size_t)row16 * (size_t)height;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t y = i / (size_t)row16, e = i - y * (size_t)row16;
        const size_t r = y % (size_t)world, j = y / (size_t)world;
        out[i] = tiles[(r * (size_t)n_max + j) * (size_t)row16 + e];
    }
}

hipError_t launch_deinterleave_u8(const uint8_t* tiles, int world, int n_max, int width, int height, uint8_t* out,
                                  hipStream_t s) {
    const uint64_t n = (uint64_t)width * 3 * height;
    if (n == 0) return hipSuccess;
    if ((width * 3) % 16 == 0 && ((uintptr_t)tiles | (uintptr_t)out) % 16 == 0)
        hipLaunchKernelGGL(deinterleave_u8_wide_kernel, dim3(grid_for(n / 16, kD2HBlocks)), dim3(256), 0, s,
                           (const uint4*)tiles, world, n_max, width * 3 / 16, height, (uint4*)out);
    else
        hipLaunchKernelGGL(deinterleave_kernel<uint8_t>, dim3(grid_for(n, 16384)), dim3(256), 0, s, tiles, world,
                           n_max, width, height, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------- launchers

hipError_t upload_minstd_table(hipStream_t s) {
    static uint32_t j1[512];  // async copies read host memory later: keep it alive
    uint64_t x = 16807;  // a^(2s+1)
    for (int i = 0; i < 512; i++) {
        j1[i] = (uint32_t)x;
        x = (x * 16807ull) % 2147483647ull;
        x = (x * 16807ull) % 2147483647ull;
    }
    hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(c_minstd_j1), j1, sizeof j1, 0, hipMemcpyHostToDevice, s);
    return e;
}

// ---------------------------------------------------------------- kernel timer
// HIP events around each launch of the AO ray kernel (the scene query of every
// AO sample: ao_kernel for small scenes, ao_near_kernel for BVH scenes), on the
// stream it runs on, while rt_gpu_profile is on: bench.py's roofline divides
// the kernel's work by these per-launch durations.
namespace {
struct KernelTimer {
    bool on = false;
    std::vector<hipEvent_t> pool;  // begin/end pairs
    size_t used = 0;
    uint64_t units = 0;            // AO samples covered by the timed launches
};
KernelTimer g_kt;
}  // namespace

static void kt_begin(hipStream_t s) {
    if (!g_kt.on) return;
    if (g_kt.pool.size() < g_kt.used + 2) {
        hipEvent_t a, b;
        if (hipEventCreate(&a) != hipSuccess) return;
        if (hipEventCreate(&b) != hipSuccess) { (void)hipEventDestroy(a); return; }
        g_kt.pool.push_back(a);
        g_kt.pool.push_back(b);
    }
    (void)hipEventRecord(g_kt.pool[g_kt.used], s);
}
static void kt_end(hipStream_t s, uint64_t units) {
    if (!g_kt.on || g_kt.pool.size() < g_kt.used + 2) return;
    (void)hipEventRecord(g_kt.pool[g_kt.used + 1], s);
    g_kt.used += 2;
    g_kt.units += units;
}

void kernel_timer_enable(bool on) {
    g_kt.on = on;
    g_kt.used = 0;
    g_kt.units = 0;
}

hipError_t kernel_timer_read(double* ms, int* launches, uint64_t* units) {
    double t = 0;
    for (size_t i = 0; i + 1 < g_kt.used; i += 2) {
        float x = 0;
        const hipError_t e = hipEventElapsedTime(&x, g_kt.pool[i], g_kt.pool[i + 1]);
        if (e != hipSuccess) return e;
        t += x;
    }
    *ms = t;
    *launches = (int)(g_kt.used / 2);
    *units = g_kt.units;
    return hipSuccess;
}

void kernel_timer_release() {
    for (hipEvent_t e : g_kt.pool) (void)hipEventDestroy(e);
    g_kt = KernelTimer();
}


// Sort the far queue (W.far_count entries) by direction key; returns its length.
// Radix-sorted key bits: grid keys are cell << (24 - 2 L), so their low
// 24 - 2 L bits are zero and the sort skips them (3 digit passes instead of
// 4 at L = 10, 11); plane-tree keys then group by their top direction bits
// only -- grouping, never a result (RT580_SORT_BITS=0: every bit, A/B).
static int sort_begin_bit(const DevScene& S) {
    if (S.bv.grid_log2 <= 0) return 0;
    const int b = 24 - 2 * S.bv.grid_log2;
    return b > 0 ? b : 0;
}

// one_dir: every ray of the queue has the same direction (a directional
// light's shadow rays): its keys take at most three values (the light's grid
// cell, RT_KEY_TREE | its direction key, RT_KEY_BRUTE), which differ in bits
// 24-25 -- one digit pass on those bits groups them as the whole sort would
// (stable: within a class the keys are equal, so the order is the same).
static hipError_t sort_far_queue(const DevScene& S, const DevWork& W, hipStream_t s, uint32_t& nq, uint32_t& nb,
                                 bool one_dir = false) {
    RT_STEP("far queue count D2H");
    hipError_t e = read_counts(W.far_count, 2, W.far_count_host, s, W.far_cap, W.far_cap);
    if (e != hipSuccess) return e;
    nq = W.far_count_host[0];
    if (W.far_count_host[1] > nq) return counts_fit(W.far_count_host, 2, W.far_cap, nq);
    nb = W.far_count_host[1];  // far-origin rays: keyed to sort last
    if (nq == 0) return hipSuccess;
    if (one_dir && nb == nq)  // every key RT_KEY_BRUTE: already grouped; the brute pass reads the sorted values
        return hipMemcpyAsync(W.far_vals_alt, W.far_vals, (size_t)nq * 4, hipMemcpyDeviceToDevice, s);
    const int b0 = one_dir ? 24 : sort_begin_bit(S);
    if (nq <= kSmallSort) {
        RT_STEP("far queue small sort");
        hipLaunchKernelGGL(small_sort_kernel, dim3(1), dim3(kSmallSortThreads), 0, s, W.far_keys, W.far_vals, nq, b0,
                           RT_DIR_KEY_BITS, W.far_keys_alt, W.far_vals_alt);
        return hipGetLastError();
    }
    size_t tmp = W.sort_tmp_bytes;
    RT_STEP("far queue radix sort");
    return hipcub::DeviceRadixSort::SortPairs(W.sort_tmp, tmp, W.far_keys, W.far_keys_alt, W.far_vals,
                                              W.far_vals_alt, (int)nq, b0, RT_DIR_KEY_BITS, s);
}

// Per-frame counters, one launch: level counts/bases, the node-capacity probe,
// the AO fix-up queue count.
__global__ void frame_init_kernel(DevWork W) {
    for (int i = threadIdx.x; i < 2 * LVL_BASE; i += blockDim.x) W.lvl[i] = 0;
    if (threadIdx.x == 0) {
        *W.needed = 0;
        *W.aofix_count = 0;
    }
}

hipError_t launch_trace(const DevScene& S, const DevFrame& F, const DevWork& W, hipStream_t s) {
    (void)hipGetLastError();  // launch checks below must not see a stale error
    const uint64_t npix = (uint64_t)F.n_rows * F.width;
    hipLaunchKernelGGL(frame_init_kernel, dim3(1), dim3(64), 0, s, W);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const bool split = S.use_bvh && S.bv.has_far && W.hit4 && W.far_cap;
    for (int level = 0; level <= F.depth; level++) {
        if (split) {
            // near phase, sorted far pass, shading; in chunks of the far queue's capacity
            uint32_t count = (uint32_t)npix;
            if (level > 0) {
                RT_STEP("level count D2H");
                if ((e = read_counts(W.lvl + level, 1, W.far_count_host, s, 0xffffffffu)) != hipSuccess) return e;
                // children beyond the node capacity were never stored (the
                // kernels clamp to it too; the frame is rendered again larger)
                count = *W.far_count_host < W.node_cap ? *W.far_count_host : W.node_cap;
            }
            if (count == 0) {  // still publish the next level's base
                hipLaunchKernelGGL((trace_kernel<true, 2>), dim3(1), dim3(TB), 0, s, S, F, W, level, 0u, 0u);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                continue;
            }
            for (uint32_t c0 = 0; c0 < count; c0 += W.far_cap) {
                const uint32_t c1 = count - c0 > W.far_cap ? c0 + W.far_cap : count;
                const int grid = grid_for(c1 - c0, 1 << 20);
                if ((e = hipMemsetAsync(W.far_count, 0, 8, s)) != hipSuccess) return e;
                RT_STEP("trace near phase");
                hipLaunchKernelGGL((trace_kernel<true, 1>), dim3(grid), dim3(TB), 0, s, S, F, W, level, c0, c1);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                uint32_t nq = 0, nb = 0;
                if ((e = sort_far_queue(S, W, s, nq, nb)) != hipSuccess) return e;
                if (nb) {
                    RT_STEP("trace brute scan");
                    if ((uint64_t)nb * 2 <= W.far_cap) {
                        // the sort's input keys are free now: 64-bit minima per brute ray
                        unsigned long long* best = reinterpret_cast<unsigned long long*>(W.far_keys);
                        if ((e = hipMemsetAsync(best, 0xff, (size_t)nb * 8, s)) != hipSuccess) return e;
                        const uint32_t ng = (nb + (uint32_t)kBruteRays - 1) / (uint32_t)kBruteRays;
                        uint32_t splits = kBruteWaves / ng;
                        splits = splits < 1u ? 1u : (splits > 512u ? 512u : splits);
                        const dim3 grid(grid_for((uint64_t)ng * splits * 64, 16384));
                        hipLaunchKernelGGL(far_brute_split_kernel<kBruteRays>, grid, dim3(TB), 0, s, S, W, nq - nb, nb,
                                           splits, best);
                        if ((e = hipGetLastError()) != hipSuccess) return e;
                        hipLaunchKernelGGL(far_brute_merge_kernel, dim3(grid_for(nb, 4096)), dim3(TB), 0, s, S, W,
                                           nq - nb, nb, (const unsigned long long*)best);
                    } else {  // (no room for the minima in the free keys: one wave per ray over every record)
                        hipLaunchKernelGGL(far_scan_kernel, dim3(grid_for((uint64_t)nb * 64, 16384)), dim3(TB), 0, s,
                                           S, W, nq - nb, nq, 1, (int)S.bv.n_far, 1, (uint8_t*)nullptr);
                    }
                    if ((e = hipGetLastError()) != hipSuccess) return e;
                    nq -= nb;
                }
#ifdef RT580_DIAGNOSTICS
                if (const char* dump = getenv("RT580_DUMP_FAR")) {  // DIAGNOSTIC build: queued rays per level
                    std::vector<float4> host((size_t)nq * 2);
                    if (nq) (void)hipMemcpy(host.data(), W.far_rays, (size_t)nq * 32, hipMemcpyDeviceToHost);
                    if (FILE* f = fopen(dump, "ab")) {
                        const uint32_t m = nq < 100000u ? nq : 100000u;  // a sample per level
                        const int hdr[2] = {level, (int)m};
                        fwrite(hdr, sizeof hdr, 1, f);
                        fwrite(host.data(), 32, m, f);
                        fclose(f);
                    }
                }
#endif
                if (nq) {
                    RT_STEP("trace far pass");
                    if ((e = launch_far_cells(S, W, nq, nullptr, s, /*closest=*/true)) != hipSuccess) return e;
                }
                // shadow rays of the directional lights: near any-hit, then the
                // sorted far pass (brute scan for far-origin rays), like AO rays
                if (W.shadow) {
                    for (int dl = 0; dl < S.n_shadow; dl++) {
                        const int li = S.shadow_light[dl];
                        if ((e = hipMemsetAsync(W.far_count, 0, 8, s)) != hipSuccess) return e;
                        RT_STEP("trace shadow near pass");
                        hipLaunchKernelGGL((trace_kernel<true, 3>), dim3(grid), dim3(TB), 0, s, S, F, W, level, c0, c1,
                                           li, dl);
                        if ((e = hipGetLastError()) != hipSuccess) return e;
                        uint32_t sq = 0, sb = 0;
                        if ((e = sort_far_queue(S, W, s, sq, sb, /*one_dir=*/true)) != hipSuccess) return e;
                        uint8_t* flags = W.shadow + (size_t)dl * W.far_cap;
                        progress("trace level %d shadow light %d: far queue %u (brute %u)", level, dl, sq, sb);
                        if (sb) {
                            RT_STEP("trace shadow brute scan");
                            if ((e = launch_brute_any(S, W, sq - sb, sb, flags, s)) != hipSuccess) return e;
                            sq -= sb;
                        }
                        if (sq) {
                            RT_STEP("trace shadow far pass");
                            if ((e = launch_far_cells(S, W, sq, flags, s)) != hipSuccess) return e;
                        }
                    }
                }
                RT_STEP("trace shade phase");
                hipLaunchKernelGGL((trace_kernel<true, 2>), dim3(grid), dim3(TB), 0, s, S, F, W, level, c0, c1);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                progress("trace level %d: rays [%u, %u) of %u, far queue %u (brute %u)", level, c0, c1, count, nq + nb, nb);
            }
            continue;
        }
        // level 0 has exactly npix rays; deeper levels read their count on the device
        const int grid = level == 0 ? grid_for(npix, 1 << 20) : grid_for(2 * npix, kDeepGrid);
        if (S.use_bvh) hipLaunchKernelGGL((trace_kernel<true, 0>), dim3(grid), dim3(TB), 0, s, S, F, W, level, 0u, ~0u);
        else if (S.n_prims <= TILE)  // small scenes: wave-uniform scalar scene loads
            hipLaunchKernelGGL((trace_kernel<false, 0, true>), dim3(grid), dim3(TB), 0, s, S, F, W, level, 0u, ~0u);
        else hipLaunchKernelGGL((trace_kernel<false, 0>), dim3(grid), dim3(TB), 0, s, S, F, W, level, 0u, ~0u);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_row_counts(const DevScene& S, const DevFrame& F, const DevWork& W, hipStream_t s) {
    if (F.n_rows == 0) return hipSuccess;
    hipLaunchKernelGGL(row_counts_kernel, dim3(F.n_rows), dim3(TB), 0, s, S, F, W);
    hipLaunchKernelGGL(row_scan_kernel, dim3(1), dim3(1024), 0, s, F, W);
    return hipGetLastError();
}

hipError_t launch_rank(const DevScene& S, const DevFrame& F, const DevWork& W, const uint64_t* row_base_global,
                       hipStream_t s) {
    const uint64_t npix = (uint64_t)F.n_rows * F.width;
    if (npix == 0 || !F.ao_enabled || S.n_ambient == 0) return hipSuccess;
    hipLaunchKernelGGL(rank_kernel, dim3((unsigned)((npix + TB - 1) / TB)), dim3(TB), 0, s, S, F, W, row_base_global);
    return hipGetLastError();
}

size_t far_sort_tmp_bytes(uint32_t cap) {
    size_t bytes = 0, rle = 0, scan = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                             (uint32_t*)nullptr, (uint32_t*)nullptr, (int)cap, 0, RT_DIR_KEY_BITS);
    (void)hipcub::DeviceRunLengthEncode::Encode(nullptr, rle, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                                (uint32_t*)nullptr, (uint32_t*)nullptr, (int)cap);
    (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (uint32_t*)nullptr, (uint32_t*)nullptr, (int)cap);
    return std::max(bytes, std::max(rle, scan));
}

hipError_t launch_ao_fix(const DevScene& S, const DevFrame& F, const DevWork& W, uint64_t b, uint64_t e,
                         hipStream_t s, const uint64_t* call_lo = nullptr, const uint64_t* call_hi = nullptr);
hipError_t launch_ao_small(const DevScene& S, const DevFrame& F, const DevWork& W, hipStream_t s,
                           const uint64_t* call_lo = nullptr, const uint64_t* call_hi = nullptr);

hipError_t launch_ao(const DevScene& S, const DevFrame& F, const DevWork& W, hipStream_t s) {
    (void)hipGetLastError();  // launch checks below must not see a stale error
    if (!F.ao_enabled || S.n_ambient == 0 || F.n_rows == 0) return hipSuccess;
#ifdef RT580_DIAGNOSTICS
    const AuditBuf* audit = S.use_bvh ? audit_for(W) : nullptr;
#endif
    if (S.use_bvh) {
        // chunks of the AO items: near pass + queue, sort the misses by
        // direction, wave-cooperative far pass
        RT_STEP("AO-call total D2H");
        hipError_t e = read_counts(reinterpret_cast<const uint32_t*>(W.totals), 2, W.far_count_host + 4, s, W.call_cap, 0u);
        if (e != hipSuccess) return e;
        const uint64_t calls = (uint64_t)W.far_count_host[4] | ((uint64_t)W.far_count_host[5] << 32);
        const uint64_t items = calls * (uint64_t)F.ao_samples;
        if (!W.ao_rays || !S.bv.nodes4) return hipErrorInvalidValue;  // (the shim sizes ao_rays for BVH frames)
        if (W.call_hint && S.bv.has_far && calls &&
            (e = hipMemsetAsync(W.call_hint, 0xff, calls * 4, s)) != hipSuccess)
            return e;
        uint64_t chunk = S.bv.has_far ? (uint64_t)W.far_cap : items;
        if (chunk > (uint64_t)W.ao_cap) chunk = W.ao_cap;
        for (uint64_t b = 0; b < items; b += chunk) {
            const uint64_t e1 = b + chunk < items ? b + chunk : items;
            if (S.bv.has_far && (e = hipMemsetAsync(W.far_count, 0, 8, s)) != hipSuccess) return e;
            if ((e = hipMemsetAsync(W.aofix_count, 0, 4, s)) != hipSuccess) return e;
#ifdef RT580_DIAGNOSTICS
            const uint32_t c_lo = (uint32_t)(b / (uint64_t)F.ao_samples);
            const uint32_t c_n = (uint32_t)((e1 - 1) / (uint64_t)F.ao_samples) + 1u - c_lo;
            if (audit) {
                if ((e = hipMemcpyAsync(audit->before, W.occ + c_lo, (size_t)c_n * 4, hipMemcpyDeviceToDevice, s)) !=
                        hipSuccess ||
                    (e = hipMemsetAsync(audit->exp, 0, (size_t)c_n * 4, s)) != hipSuccess ||
                    (e = hipMemsetAsync(audit->aud, 0, 4 * 8, s)) != hipSuccess)
                    return e;
            }
#endif
            // the samples' rays (32-byte records), then the budgeted near any-hit in
            // speculative form (ao_trace_kernel) and the late pass for the rays
            // out of budget (ao_late_kernel), timed together (kt_*)
            constexpr int V = 512 | 1024 | 2048 | 4096 | 16384;
            hipLaunchKernelGGL((ao_near_kernel_w<8, V>), dim3(grid_for(e1 - b, 8192)), dim3(TB), 0, s, S, F, W, b, e1);
            if ((e = hipGetLastError()) != hipSuccess) return e;
            if ((e = hipMemsetAsync(W.ao_late_count, 0, 8, s)) != hipSuccess) return e;
            kt_begin(s);
            const uint64_t c0 = b / (uint64_t)F.ao_samples;  // the chunk's first call (the records' call base)
            // up to 65536 workgroups: one 2048-sample block each for a full 2^27 chunk
            // (AO trace per 4 north-star frames, cap 4608 / 8192 / 16384 / 32768 /
            // 65536 / 131072: 92.4 / 90.8 / 89.7-89.8 / 88.1 / 88.0-88.2 / 88.0 ms;
            // Cornell 165.3 -> 164.6 ms at 65536)
            hipLaunchKernelGGL((ao_trace_kernel<6, 16, 8, 4, 4>), dim3(grid_for(e1 - b, 65536)), dim3(TB), 0, s, S, W,
                               e1 - b, c0);
            // 12288 workgroups (~2 late rays per lane): late pass per 4 north-star
            // frames 1536 / 3072 / 4096 / 12288 / 24576 / 49152 workgroups:
            // 11.93 / 11.49 / 11.15-11.24 / 10.47-10.55 / 11.04 / 10.82 ms
            hipLaunchKernelGGL((ao_late_kernel<6, 16>), dim3(12288), dim3(TB), 0, s, S, W, c0);
            kt_end(s, e1 - b);
            if ((e = hipGetLastError()) != hipSuccess) return e;
#ifdef RT580_DIAGNOSTICS
            if (audit) {  // (before the fix-up pass adds to the queue and the counts)
                hipLaunchKernelGGL(ao_audit_expect_kernel, dim3(grid_for(e1 - b, 16384)), dim3(TB), 0, s, S, W, e1 - b,
                                   c_lo, audit->exp, audit->aud, g_verify_out);
                hipLaunchKernelGGL(ao_audit_compare_kernel, dim3(4096), dim3(TB), 0, s, S, W, c_lo, c_n,
                                   (uint32_t)F.ao_samples, b, e1 - b, audit->before, audit->exp, audit->aud,
                                   g_verify_out);
                hipLaunchKernelGGL(ao_audit_finish_kernel, dim3(1), dim3(64), 0, s, S, W, audit->aud, g_verify_out);
                if ((e = hipGetLastError()) != hipSuccess) return e;
            }
#endif
            // exact recompute of the fast pass's failing samples; their misses join the far queue
            if ((e = launch_ao_fix(S, F, W, b, e1, s)) != hipSuccess) return e;
            if (!S.bv.has_far) continue;
            uint32_t nq = 0, nb = 0;
            if ((e = sort_far_queue(S, W, s, nq, nb)) != hipSuccess) return e;
            if (nb) {
                if ((e = launch_brute_any(S, W, nq - nb, nb, (uint8_t*)nullptr, s)) != hipSuccess) return e;
                nq -= nb;
            }
            progress("AO items [%llu, %llu) of %llu: far queue %u (brute %u)", (unsigned long long)b,
                     (unsigned long long)e1, (unsigned long long)items, nq, nb);
#ifdef RT580_DIAGNOSTICS
            {
                unsigned long long st[5] = {0, 0, 0, 0, 0};
                if (hipMemcpyFromSymbolAsync(st, HIP_SYMBOL(g_brute_stats), sizeof st, 0, hipMemcpyDeviceToHost, s) ==
                        hipSuccess &&
                    hipStreamSynchronize(s) == hipSuccess)
                    progress("brute any-hit so far: rays %llu, steps %llu, no acceptor %llu (steps %llu), by hint %llu",
                             st[0], st[1], st[2], st[3], st[4]);
            }
#endif
            if (nq == 0) continue;
            if ((e = launch_far_cells(S, W, nq, (uint8_t*)nullptr, s)) != hipSuccess) return e;
#ifdef RT580_DIAGNOSTICS
            {
                unsigned long long st[9];
                if (hipMemcpyFromSymbolAsync(st, HIP_SYMBOL(g_far_stats), sizeof st, 0, hipMemcpyDeviceToHost, s) ==
                        hipSuccess &&
                    hipStreamSynchronize(s) == hipSuccess)
                    progress("far_any so far: rays %llu grid %llu uniform waves %llu lane waves %llu list entries %llu "
                             "lock-step steps %llu tree rays %llu candidates %llu hits %llu",
                             st[0], st[1], st[2], st[3], st[4], st[5], st[6], st[7], st[8]);
                unsigned long long cs[3];
                if (hipMemcpyFromSymbolAsync(cs, HIP_SYMBOL(g_cell_stats), sizeof cs, 0, hipMemcpyDeviceToHost, s) ==
                        hipSuccess &&
                    hipStreamSynchronize(s) == hipSuccess)
                    progress("cell pass so far: rays in empty cells %llu, (ray, candidate) pairs %llu, passing "
                             "far_candidate %llu", cs[0], cs[1], cs[2]);
            }
#endif
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        return hipSuccess;
    }
    kt_begin(s);  // (frame_init_kernel zeroed W.aofix_count)
    const hipError_t e = launch_ao_small(S, F, W, s);
    kt_end(s, 0);  // one launch per frame: its AO rays are the frame's (no host sync here)
    if (e != hipSuccess) return e;
    return launch_ao_fix(S, F, W, 0, ~0ull, s);
}

bool ao_calls_supported(const DevScene& S, const DevFrame& F) {
    return !S.use_bvh && F.ao_enabled && S.n_ambient > 0;
}

hipError_t launch_ao_calls(const DevScene& S, const DevFrame& F, const DevWork& W, const uint64_t* call_lo,
                           const uint64_t* call_hi, hipStream_t s) {
    (void)hipGetLastError();
    if (!ao_calls_supported(S, F)) return hipErrorInvalidValue;
    // a fresh fix-up queue for this range (frame_init_kernel zeroed it for the first)
    hipError_t e = hipMemsetAsync(W.aofix_count, 0, 4, s);
    if (e != hipSuccess) return e;
    if ((e = launch_ao_small(S, F, W, s, call_lo, call_hi)) != hipSuccess) return e;
    return launch_ao_fix(S, F, W, 0, ~0ull, s, call_lo, call_hi);
}

// Exact recompute of the samples the fast pass queued (or, on queue overflow,
// of every failing sample of items [b, e)); exits at once with nothing to do.
hipError_t launch_ao_fix(const DevScene& S, const DevFrame& F, const DevWork& W, uint64_t b, uint64_t e,
                         hipStream_t s, const uint64_t* call_lo, const uint64_t* call_hi) {
    // a few hundred samples per frame at most (the queue; its overflow case
    // re-tests every item of [b, e) grid-stride): a small grid exits at once
    hipLaunchKernelGGL(ao_fix_kernel, dim3(64), dim3(TB), 0, s, S, F, W, b, e, call_lo, call_hi);
    return hipGetLastError();
}

// Small-scene AO (brute force): the wave-uniform scalar scene loop, sign-decided
// rejections, the fast sincos / unit-vector sequences with the exact fix-up
// queue, two samples per lane, 8 waves per SIMD (ao_kernel_occ8; config 2:
// 1.519 / 1.539 vs 1.586 / 1.582 ms per frame for one sample per lane,
// profiles/r05/ab/spl_*.json). 16384 workgroups (64 per CU; 8192 / 32768
// within 1 %).
hipError_t launch_ao_small(const DevScene& S, const DevFrame& F, const DevWork& W, hipStream_t s,
                           const uint64_t* call_lo, const uint64_t* call_hi) {
    constexpr int V = 4 | 8 | 1024 | 2048 | 4096 | 32768;
    hipLaunchKernelGGL(ao_kernel_occ8<V>, dim3(16384), dim3(TB), 0, s, S, F, W, call_lo, call_hi);
    return hipGetLastError();
}

hipError_t launch_resolve(const DevScene& S, const DevFrame& F, const DevWork& W, int16_t* fb, hipStream_t s) {
    const uint64_t npix = (uint64_t)F.n_rows * F.width;
    if (npix == 0) return hipSuccess;
    return launch_resolve_range(S, F, W, fb, 0, (uint32_t)npix, s);
}

hipError_t launch_resolve_range(const DevScene& S, const DevFrame& F, const DevWork& W, int16_t* fb, uint32_t p_lo,
                                uint32_t p_hi, hipStream_t s) {
    const uint64_t npix = (uint64_t)F.n_rows * F.width;
    for (int level = F.depth; level >= 0; level--) {
        const int grid = level == 0 ? grid_for(p_hi - p_lo, 1 << 20) : grid_for(2 * npix, kDeepGrid);
        hipLaunchKernelGGL(resolve_level_kernel, dim3(grid), dim3(TB), 0, s, S, F, W, level, fb, p_lo, p_hi);
    }
    return hipGetLastError();
}

hipError_t launch_copy_rows(const int16_t* src, int width, int row_begin, int row_step, int n_rows, int16_t* dst,
                            hipStream_t s) {
    const uint64_t n = (uint64_t)width * 3 * n_rows;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(copy_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, width, row_begin,
                       row_step, n_rows, dst);
    return hipGetLastError();
}

}  // namespace rt580

#ifdef RT580_DIAGNOSTICS
// DIAGNOSTIC build only: the RT580_AO_VERIFY totals (ao_verify_kernel's out[0..63])
// since the last call, after a device-wide sync; then zeroed. 1: verification off.
extern "C" int rt580_diag_ao_verify(unsigned long long* out64) {
    if (!rt580::g_verify_out) return 1;
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    if (hipMemcpy(out64, rt580::g_verify_out, 64 * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    return hipMemset(rt580::g_verify_out, 0, 64 * 8) == hipSuccess ? 0 : 1;
}
#endif

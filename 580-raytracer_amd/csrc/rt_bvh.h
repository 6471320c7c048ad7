// rt_bvh.h — exact-semantics acceleration structures over the scene's
// triangles, built on the host at upload time.
//
// The reference brute-forces every primitive for every ray
// (IntersectScene, Raytracer.cpp:473-526). Here the structures only decide
// which primitives are *tested*; every test is the unchanged per-primitive
// arithmetic on the same rt_prim record, and the combination rule is the
// reference's: closest hit = lexicographic minimum of (t, primitive index)
// (what "first hit taken, later ones only if strictly closer" yields for
// finite t, :491-516); any-hit = the boolean over all primitives.
//
// The catch is that the reference's float triangle test also ACCEPTS some
// hit points far outside the triangle: for rays nearly parallel to the plane,
// t = num/nd is huge and the signed sub-areas of (Pp, v_i, v_j) are then
// dominated by rounding (measured: ~2.5e-4 of AO rays on a 100k-triangle
// scene get such a "far hit" at t ~ 1e6-1e7). A culling structure must keep
// those. Per triangle j (edges e_min..e_max, smallest angle a_min,
// s = sin(a_min/2)), with u = 2^-24 and kappa = 9.25 (rt_bvh.cpp analyse):
//   |computed 2*sub-area - exact| <= kappa*u*|a||b|  (a, b = v - Pp, |.| <= D + e')
//   exact most negative 2*sub-area of a point at in-plane distance D outside
//     <= -G * D   (G from the edges and angles)
// so an accepted hit point is either within D_lo of the triangle ("near") or
// at distance >= D_hi ("far"), the roots of kappa*u*(D + e')^2 = G*D.
//   near hits: found by a spatial BVH whose triangle boxes are inflated by
//     delta_j >= 2 D_lo and tested with a "fat ray" (box grown by alpha + beta t
//     covering the float error of the hit point and of the slab arithmetic,
//     rt_isect.h), conservative at every t;
//   far hits (t >= T_j = D_hi(j) - |o| - sqrt3*S): candidates are planes the
//     ray crosses beyond T_j. For origins near the scene they come from a
//     direction grid: a far hit needs the ray nearly parallel to the plane AND
//     pointing into the triangle's angle at v0 (the two sub-areas through v0
//     are computed accurately), a thin arc of directions per triangle, listed
//     in every octahedral direction cell it touches (build_dir_grid). Other
//     origins walk a second tree over the triangles' planes (normal boxes + D
//     ranges) with exact interval padding. Candidates get the full reference test.
// Triangles for which the analysis does not give a usable split (degenerate,
// or D_hi below 8 S) and all spheres are tested brute force for every ray.
#pragma once
#include <stdint.h>

#include <vector>

#include "../../include/rt580.h"

namespace rt580 {

// Spatial BVH node: both children's boxes live in the parent, so one 64-byte
// fetch culls both. Child link: n == 0 -> internal node `c`; n > 0 -> leaf of
// the n triangles at slots [c, c + n) of the reordered arrays; n < 0 -> empty.
struct alignas(16) BvhNode {
    float lo0[3], hi0[3];
    float lo1[3], hi1[3];
    int32_t c0, c1, n0, n1;
};
static_assert(sizeof(BvhNode) == 64, "BvhNode is one 64-byte line");

// 4-wide form of the same spatial BVH (collapse_bvh4: a node's children are
// its binary node's children and grandchildren, with the boxes the binary tree
// stores for them): the same boxes and leaves, half the depth. Boxes as
// lo[axis][child] / hi[axis][child]; child link as BvhNode's (n == 0: node
// `c` of this array; n > 0: leaf slots [c, c + n); n < 0: empty). 128 bytes.
struct alignas(16) Bvh4Node {
    float lo[3][4];
    float hi[3][4];
    int32_t c[4];
    int32_t n[4];
};
static_assert(sizeof(Bvh4Node) == 128, "Bvh4Node is two 64-byte lines");

// The 4-wide node as the device reads it: the four child boxes quantized to
// 8 bits per plane against the node's own frame (origin = the children's
// smallest corner, per-axis power-of-two scale), rounded outward so that the
// decoded box fmaf(q, scale, origin) contains the child's float box -- the
// same culling decisions or more conservative ones (more boxes entered, never
// fewer), hence the same answers. Child link as a stack entry: n << 27 | c
// (n == 0: node c; n > 0: leaf slots [c, c + n)); 0xffffffff: empty. 64 bytes:
// half the bytes and registers of Bvh4Node per traversal step.
struct alignas(16) Bvh4QNode {
    float origin[3];
    uint32_t exps;      // biased float exponents of the three scales, bits 0-7, 8-15, 16-23
    uint8_t qlo[3][4];  // [axis][child]
    uint8_t qhi[3][4];
    uint32_t link[4];
    uint32_t pad[2];
};
static_assert(sizeof(Bvh4QNode) == 64, "Bvh4QNode is one 64-byte line");

// Plane-tree node (own bounds): normals in [nlo, nhi], plane offsets D in
// [dlo, dhi], and the subtree minima of D_hi and delta (for its T bound).
// count > 0: leaf of far_tris [first, first + count); else children first, first + 1.
struct alignas(16) FarNode {
    float nlo[3], nhi[3];
    float dlo, dhi;
    float min_dhi, min_delta;
    int32_t first, count;
};
static_assert(sizeof(FarNode) == 48, "FarNode layout");

// A triangle's plane as the far search reads it (same floats as rt_prim).
struct alignas(16) FarTri {
    float n[3];
    float d;
    float dhi;      // D_hi(j)
    float delta;    // delta_j (box inflation)
    uint32_t id;    // scene primitive index
    uint32_t pad;
};
static_assert(sizeof(FarTri) == 32, "FarTri layout");

#define RT_BVH_STACK 64  // device traversal stack; deeper trees are rejected

struct BvhBuild {
    std::vector<BvhNode> nodes;     // node 0 is the root
    std::vector<Bvh4Node> nodes4;   // the same tree 4-wide (collapse_bvh4); node 0 is the root
    std::vector<Bvh4QNode> nodes4q; // nodes4 quantized (collapse_bvh4): what the traversal reads
    std::vector<rt_prim> prims;     // near-set triangles in leaf order (copies of the scene records)
    std::vector<uint32_t> ids;      // scene index of each slot (tie-break + shading lookups)
    std::vector<FarNode> far_nodes; // node 0 is the root (empty when no far-set triangle)
    std::vector<FarTri> far_tris;
    std::vector<uint32_t> brute;    // spheres + unanalysable triangles, ascending scene index
    float scale = 0.0f;             // S: largest |coordinate| of the primitives
    int depth = 0, far_depth = 0;   // deepest levels (stack bounds)
    int max_leaf = 0;
    int n_tri = 0;
    int n_far = 0;                  // far_tris.size() (kept after the host copy is dropped)
    float dhi_median = 0.0f;        // typical D_hi (routing of far-origin rays)
    double inflate = 0.0;           // delta_j / e_min(j)
    double build_ms = 0.0;
    // Direction grid for the far search (build_dir_grid): for rays with |o| <= grid_r,
    // the far_tris entries (indices) that can give a far hit for a direction in
    // each octahedral cell; grid_always: entries to test for every such ray.
    int grid_log2 = 0;              // M = 2^grid_log2 cells per axis; 0: no grid
    float grid_r = 0.0f;
    std::vector<uint32_t> grid_start;   // [M*M + 1]
    std::vector<uint32_t> grid_items;
    std::vector<uint32_t> grid_always;
    double grid_ms = 0.0;
    // The same grid at half the resolution per axis (coarsen_dir_grid): a cell's
    // list is the union of its four children's, for frames of few rays (rows of
    // a K-way split), whose cells would hold few rays each.
    std::vector<uint32_t> grid2_start;  // [(M/2)^2 + 1]
    std::vector<uint32_t> grid2_items;
};

// Build over prims[0..n). Returns false if there are no triangles or a tree
// would exceed the device stack (the caller then keeps brute force).
bool build_bvh(const rt_prim* prims, int n, BvhBuild& out);

// The 4-wide form of out.nodes (after build_bvh), float and quantized.
void collapse_bvh4(BvhBuild& out);

// Build the far-search direction grid over out.far_tris (after build_bvh; the
// query side is rt_isect.h grid_cell / far_any / far_closest).
void build_dir_grid(const rt_prim* prims, BvhBuild& out, int log2_cells);
// The grid's geometry, for its checks (tests/native/octgrid_check.cpp): the unit
// direction at the centre of quadtree node (i, j) of `level` (2^level nodes per
// map axis), and the chord radius the build assumes every direction whose
// cell lies in that node to be within.
void oct_node_centre(int level, int i, int j, double out[3]);
double oct_node_radius(int level);

// out.grid2_* from out.grid_* (after build_dir_grid): coarse cell (i, j) lists
// the sorted union of fine cells (2i + a, 2j + b). grid_cell(d, L - 1) is
// grid_cell(d, L)'s (i >> 1, j >> 1) (power-of-two scalings of one float), and
// a direction of the coarse cell lies in one of its children, whose list is
// conservative: so is the union.
void coarsen_dir_grid(BvhBuild& out);

// Render-time guard for the camera (float ranges only; the bounds hold for any origin).
bool bvh_usable(const BvhBuild& b, const float cam_from[3]);

}  // namespace rt580

// rt_kernels.h — device-side views, per-frame workspace and launchers
// (rt_kernels.hip), used by rt_shim.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/rt580.h"
#include "rt_isect.h"

// Deepest recursion supported (reference default 4; BASELINE config 5 uses 8).
#define RT_MAX_DEPTH 16

namespace rt580 {

struct DevScene {
    const rt_prim* prims;
    const rt_prim_shade* shade;
    const rt_material* mats;
    const rt_light* lights;
    int n_prims;
    int n_lights;
    int n_ambient;
    int use_bvh;   // triangle scenes: exact BVH queries (rt_isect.h) instead of brute force
    // The primitives in a fixed pseudo-random order: the any-hit scan of
    // far-origin rays reads them this way (any order gives the same boolean;
    // accepted primitives come clustered by mesh in scene order, see far_scan_kernel).
    const rt_prim* scan_prims;
    // scene indices of the shadow-casting (directional and point) lights, in
    // JSON order, for the host-side launch loop of the shadow passes; <= 8
    int n_shadow;
    int shadow_light[8];
    BvhView bv;
};

struct DevFrame {
    int width, height, depth, ao_samples, ao_enabled, rng_engine;
    uint32_t rng_seed;
    int row_begin, row_step, n_rows;  // local row k is frame row row_begin + k*row_step
    int view_inverse_ok;
    float view_inv[9];
    float cam_from[3];
    float ao_angle_max;
    double ndc_kx, ndc_ky;
    // minstd_rand0: step = 16807^(2 * ao_samples) mod (2^31 - 1), the state
    // advance of one AO call; step_pow2[i] = step^(2^i)
    uint32_t step_pow2[32];
};

// One node of the reflect/refract recursion tree (a Raycast call). 48 bytes.
struct alignas(16) NodeRec {
    float hp[3];          // hit point (hitInfo.hitPoint)
    float n[3];           // geometric normal (hitInfo.normal)
    int32_t local_rg;     // non-ambient local colour: r | g << 16 (int16 each)
    int32_t local_b_flags;// b | flags << 16
    float kr, kt;         // ComputeFresnel
    int32_t shape;        // material index
    int32_t spare;
};  // 48 bytes; the children and flags are also in DevWork::topo, a hit node's first AO call in node_call0
static_assert(sizeof(NodeRec) == 48, "NodeRec is three 16-byte words");
#define RT_NODE_HIT 1
#define RT_NODE_LEAF 2  // bounces == 0: no combine

// A queued tree ray (child of a node of the previous level). 32 bytes.
struct RayItem {
    float o[3];
    float d[3];
    int32_t pixel;  // local pixel index
    int32_t pad;
};

// Per-frame device workspace (owned by the shim, sized by capacity).
constexpr int kLateSaved = 22;               // stack entries a saved late-ray walk may hold
constexpr int kLateWords = 2 + kLateSaved;  // words per saved walk

struct DevWork {
    NodeRec* nodes;        // [node_cap]
    int4* topo;            // [node_cap] child[0], child[1], flags (rank_kernel's walk reads these 16 bytes, not the record)
    uint32_t* node_call0;  // [node_cap] first AO call of a hit node (rank_kernel -> resolve)
    int2* node_val;        // [node_cap] a node's value (Raycast's return, r | g << 16, b) for its parent's resolve
    RayItem* rays;         // [node_cap] (indexed by node id; level 0 is implicit)
    uint32_t* lvl;         // [2 * (RT_MAX_DEPTH + 2)]: counts then bases
    uint32_t* needed;      // [1] highest node id requested + 1 (overflow check)
    uint32_t* pix_hits;    // [npix]
    uint32_t* pix_nodes;   // [npix]
    uint32_t* pix_prefix;  // [npix] in-row exclusive prefix of AO calls
    uint32_t* row_calls;   // [n_rows]
    uint32_t* row_hits;    // [n_rows]
    uint32_t* row_nodes;   // [n_rows]
    uint64_t* row_base_local;  // [n_rows] exclusive scan of this call's rows
    uint64_t* totals;      // [2]: total local AO calls, spare
    uint32_t* call_node;   // [call_cap]
    uint64_t* call_rng;    // [call_cap] minstd state at the call's first draw / mt19937 global call index
    uint32_t* occ;         // [call_cap] occluded samples
    const uint32_t* mt_stream;  // mt19937 draws [mt_base, ...) of the serial stream, else null
    uint64_t mt_base;      // absolute index (in the serial stream) of mt_stream[0]
    uint32_t node_cap;
    uint32_t call_cap;
    // BVH scenes: AO rays that miss every near triangle, queued for the sorted
    // far-hit pass (rt_bvh.h): (o.xyz, call) and (d.xyz, -) per ray, its
    // direction key, and the radix sort's double buffers + temporary storage.
    float4* far_rays;      // [2 * far_cap]
    uint32_t* far_keys;    // [far_cap] x2 (keys, sorted keys)
    uint32_t* far_keys_alt;
    uint32_t* far_vals;    // [far_cap] x2 (ray index, sorted)
    uint32_t* far_vals_alt;
    uint32_t* far_count;   // [2]: queued rays, of which far-origin (brute scan)
    // the sorted queue in segments of one key (run-length encoding into
    // far_keys / far_vals, then offsets): far_seg_off[k] = first sorted ray of
    // segment k; work items = chunks of <= 64 rays of one segment
    uint32_t* far_seg_off; // [far_cap]
    uint32_t* far_seg_n;   // [2]: segments, work items (chunks of <= 64 rays of one segment)
    uint32_t* far_wofs;    // [far_cap] first work item of each segment
    uint4* far_work;       // [far_cap + far_cap / 64 + 64] work items: sorted rays [x, y), cell list at z, w entries
    uint32_t* far_count_host;  // pinned
    void* sort_tmp;
    size_t sort_tmp_bytes;
    uint32_t far_cap;
    // split AO pass (ao_trace_kernel): (o.xyz, call), (d.xyz, flag) per item of a chunk
    float4* ao_rays;       // [ao_cap] 16-byte AO ray records of a chunk (ao_record) or null
    float4* ao_hp;         // [ao_cap + 2]: the hit point of each call of the chunk (after ao_rays)
    uint32_t ao_cap;
    // AO rays of a chunk whose near traversal ran out of its step budget in
    // ao_trace_kernel (item index in the chunk), finished by ao_late_kernel
    uint32_t* ao_late;       // [ao_cap] or null
    uint32_t* ao_late_count; // [1]
    // the walk state of late rays [0, ao_state_cap) of the late queue, saved by
    // ao_trace_kernel and resumed by ao_late_kernel instead of starting over:
    // per slot kLateWords words -- the entry about to be descended (c), n | sp << 8
    // (~0: not saved, the stack was deeper than kLateSaved), then the stack
    // [0, sp). Rays past ao_state_cap start over.
    uint32_t* ao_state;
    uint32_t ao_state_cap;
    // provisional closest hits of the tree rays (node id) between the near and
    // far phases of a BVH trace level: (t, alpha, beta, gamma), prim (-1: none)
    float4* hit4;          // [node_cap]
    int32_t* hit_prim;     // [node_cap]
    // shadow rays of a BVH trace level, decided before the shading phase:
    // [shadow light k][item - chunk start] occluded flags (near pass + the
    // sorted far pass / brute scan), far_cap entries per light
    uint8_t* shadow;       // [n_shadow * far_cap] or null
    // AO samples whose fast sincos rounding test failed (rt_libm.h), recomputed
    // exactly by ao_fix_kernel: item ids, count (may exceed the capacity)
    uint64_t* aofix_items; // [aofix_cap]
    uint32_t* aofix_count; // [1]
    // brute any-hit scans of far-origin AO rays: per AO call, a record (scan
    // order) that accepted one of its samples, tried first by its other
    // samples (they share the origin; tools/far_origin_study.cpp). 0xffffffff:
    // none yet. [call_cap] or null
    uint32_t* call_hint;
    uint32_t aofix_cap;
    // the slot's replay-check word (count_check_kernel sets it when a replayed
    // count differs from the frame's own): kernels of BVH frames return at
    // entry when it is set (rt_kernels.hip frame_poisoned). Null: never set.
    const uint32_t* poison;
};

// Host reads of device counts during a frame's enqueue (trace-level ray
// counts, far-queue lengths and segment counts, the AO-call total) go through
// the current count schedule. RECORD reads each count (a D2H copy and a sync
// of the frame's stream) and appends it; REPLAY takes the counts from the
// recorded list instead -- the frame then enqueues without a host sync, so
// consecutive frames overlap on the two frame slots -- and enqueues a device
// check per count that sets *bad when the frame's own count differs. The
// counts are a function of (scene, params, rows, chunk size); the shim
// replays only a verified repeat of the frame that recorded them, and fails
// the frame when *bad is set (rt_shim.cpp begin_slot).
struct CountSchedule {
    enum Mode { OFF, RECORD, REPLAY };
    Mode mode = OFF;
    std::vector<uint32_t> vals;
    std::vector<const char*> where;  // the launcher step that read each count (RECORD), for error messages
    uint32_t tag = 0;                // which schedule (the device check reports index | tag << 16)
    size_t pos = 0;
    uint32_t* bad = nullptr;  // device word (REPLAY)
    bool broken = false;      // REPLAY asked for more counts than were recorded
};
void set_count_schedule(CountSchedule* cs);  // null: plain reads

hipError_t upload_minstd_table(hipStream_t s);
// Breadth-first trace of all levels: nodes, shading except AO, per-pixel counters.
hipError_t launch_trace(const DevScene& S, const DevFrame& F, const DevWork& W, hipStream_t s);
// Per-row AO-call totals + in-row prefixes, then the local row scan.
hipError_t launch_row_counts(const DevScene& S, const DevFrame& F, const DevWork& W, hipStream_t s);
// AO-call numbering (RNG positions) from the global row bases (nullptr: local scan).
hipError_t launch_rank(const DevScene& S, const DevFrame& F, const DevWork& W, const uint64_t* row_base_global,
                       hipStream_t s);
hipError_t launch_ao(const DevScene& S, const DevFrame& F, const DevWork& W, hipStream_t s);
// The launcher step that ran last (for error messages).
const char* launch_where();
// Temporary storage of the far-queue radix sort / run-length encoding / scan for `cap` rays.
size_t far_sort_tmp_bytes(uint32_t cap);
hipError_t launch_resolve(const DevScene& S, const DevFrame& F, const DevWork& W, int16_t* fb, hipStream_t s);
// Latency path of small-scene frames (a frame split by rows so that the first
// part's resolve and copy overlap the second part's AO): AO of the calls
// [*call_lo, *call_hi) (device values; null: from the first / to the last),
// and the resolve of the local pixels [p_lo, p_hi).
bool ao_calls_supported(const DevScene& S, const DevFrame& F);
hipError_t launch_ao_calls(const DevScene& S, const DevFrame& F, const DevWork& W, const uint64_t* call_lo,
                           const uint64_t* call_hi, hipStream_t s);
hipError_t launch_resolve_range(const DevScene& S, const DevFrame& F, const DevWork& W, int16_t* fb, uint32_t p_lo,
                                uint32_t p_hi, hipStream_t s);
hipError_t launch_row_bases(const int32_t* gathered, int world, int n_max, int height, int rank, uint64_t* out,
                            hipStream_t s);
hipError_t upload_gamma_lut(const uint8_t* lut, hipStream_t s);
hipError_t launch_gamma_u8(const int16_t* fb, uint64_t n, uint8_t* out, hipStream_t s);
// the same, 16 bytes per lane (out 16-byte aligned; e.g. mapped host memory)
hipError_t launch_gamma_u8_wide(const int16_t* fb, uint64_t n, uint8_t* out, hipStream_t s);
// rows row0, row0 + step, ... (n_rows packed int16 rows) as PPM bytes at their
// places in a whole frame's body (a rank's rows straight into the shared host frame)
hipError_t launch_gamma_rows_u8(const int16_t* fb, int n_rows, int width, int row0, int step, uint8_t* out,
                                hipStream_t s);
// one device read of host memory (a mapped host address) after this device's
// writes into it: those writes are in host memory when it completes
hipError_t launch_host_flush_read(const void* host_dev, uint32_t* sink, hipStream_t s);
// mt19937 draws [lo, hi) of the serial stream into out[0, hi - lo): one
// workgroup per checkpoint block k in [k0, k0 + nblk) (rt_mt.h: windows[j] =
// W_{(k0 + j) kMtBlock}), each running the twist from its window.
hipError_t launch_mt_generate(const uint32_t* windows, uint64_t k0, uint32_t nblk, uint64_t lo, uint64_t hi,
                              uint32_t* out, hipStream_t s);
hipError_t launch_powf_eval(const float* x, float y, float* out, uint64_t n, hipStream_t s);
hipError_t launch_math_selftest(uint64_t seed, uint64_t n, unsigned long long* bad, hipStream_t s);
// Per-launch HIP-event timing of the AO ray kernel (profiling; see rt_kernels.hip).
void kernel_timer_enable(bool on);
hipError_t kernel_timer_read(double* ms, int* launches, uint64_t* units);
void kernel_timer_release();
// Multi-GPU frame: tiles[k] holds rows k, k+world, ... (n_max rows each) -> out
// in raster order.
hipError_t launch_deinterleave(const int16_t* tiles, int world, int n_max, int width, int height, int16_t* out,
                               hipStream_t s);
hipError_t launch_deinterleave_u8(const uint8_t* tiles, int world, int n_max, int width, int height, uint8_t* out,
                                  hipStream_t s);
hipError_t launch_copy_rows(const int16_t* src, int width, int row_begin, int row_step, int n_rows,
                            int16_t* dst, hipStream_t s);

}  // namespace rt580

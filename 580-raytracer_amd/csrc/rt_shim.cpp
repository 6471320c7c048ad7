// rt_shim.cpp — the extern "C" rt_gpu_* boundary (include/rt580.h): device
// buffers resident in HBM, one HIP stream, HIP-event timings, error mapping to
// the reference's status codes (Raytracer.h:8-10). No exception crosses it.
//
// State lives in per-device contexts. The public entry points act on context 0
// (the device of rt_gpu_init); rt_gpu_render_multi drives contexts 0..G-1, one
// per GPU of the node, and exchanges over RCCL (loaded on first use).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <array>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../../include/rt580.h"
#include "rt_bvh.h"
#include "rt_kernels.h"
#include "rt_knobs.h"
#include "rt_mt.h"

using namespace rt580;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

enum { EV_START, EV_TRACE, EV_RANK, EV_AO, EV_RESOLVE, EV_N };

struct Slot {
    hipStream_t stream = nullptr;  // frame stream (non-blocking)
    hipEvent_t done = nullptr;     // end of the slot's last enqueued phase
    hipEvent_t ao_done = nullptr;  // end of the AO kernels of the slot's last frame
    DevBuf nodes, topo, node_call0, node_val, rays, lvl, needed, pix_hits, pix_nodes, pix_prefix, row_calls, row_hits, row_nodes,
        row_base_local, totals, call_node, call_rng, occ, fb, fb_full, mt_stream, aofix_items, aofix_count,
        call_hint, mt_windows, fb8;
    uint64_t mt_base = 0;  // absolute index of mt_stream's first draw
    // BVH frames: the far queue, the AO ray records and the split trace's
    // provisional hits -- per slot, so that consecutive BVH frames overlap
    // like the others (count schedule replay, see trace_rows)
    DevBuf ao_state;  // saved walks of late AO rays (DevWork::ao_state)
    DevBuf ao_rays, ao_late, ao_late_count, far_rays, far_keys, far_keys_alt, far_vals, far_vals_alt, far_count,
        far_seg_off, far_seg_n, far_wofs, far_work, sort_tmp, hit4, hit_prim, shadow;
    uint32_t far_cap = 0, ao_cap = 0;
    // replayed count schedules: the device checks' flag, its host copy (read
    // when the slot is next used), and whether a replayed frame is unchecked
    DevBuf bad;
    uint32_t* bad_host = nullptr;  // pinned
    bool check_pending = false;
};

// Key of a recorded count schedule: the frame it was recorded on.
struct SchedKey {
    rt_render_params p;
    uint64_t gen;
    int rows[3];
    uint32_t far_chunk, ao_chunk;  // the frame's chunk sizes (they set the passes' sequence)
    int32_t accel;                 // the scene query (brute-force frames read no counts)
};

struct State {
    bool inited = false;
    DevBuf ppm_stage;  // rt_gpu_deinterleave_ppm without the host mapping (RT580_D2H_MAPPED=0)
    hipEvent_t ppm_done = nullptr;  // rt_gpu_shade_rows_ppm's frame-done event when frames are not pipelined
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    std::array<hipEvent_t, EV_N> ev_default{};
    hipEvent_t* ev = nullptr;  // events of the frame being enqueued
    bool profiling = false;
    bool kt_keep = false;
    int prof_frames = 0;
    std::vector<std::array<hipEvent_t, EV_N>> prof_pool;
    // scene
    DevBuf prims, shade, mats, lights;
    int n_prims = 0, n_lights = 0, n_ambient = 0, n_nonambient = 0;
    std::vector<int> shadow_lights;  // scene indices of the directional and point lights
    bool have_scene = false;
    // exact BVH (rt_bvh.h), built at upload for triangle scenes beyond one LDS tile
    DevBuf bvh_nodes, bvh_nodes4, bvh_prims, bvh_ids, far_nodes, far_tris, brute, grid_start, grid_items, grid_always, scan_prims;
    DevBuf grid2_start, grid2_items;  // the half-resolution grid (coarsen_dir_grid)
    DevBuf grid_live, grid2_live;     // bitmaps of the grids' non-empty cells (far_live)
    BvhBuild bvh;
    bool bvh_ok = false;
    int grid_log2 = 0, grid_n_always = 0;  // far-search direction grid (uploaded; host copy dropped)
    bool grid2 = false;                    // grid2_* uploaded (log2 = grid_log2 - 1)
    int accel = RT_ACCEL_AUTO;
    bool last_accel = false;
    uint64_t scene_gen = 0;
    // per-frame workspace: two slots, so that consecutive frames overlap on
    // two streams (frame pipelining, see begin_slot)
    static constexpr int kSlots = 4;
    Slot slot[kSlots];
    int nslots = 3;            // slots in use (RT580_SLOTS): frames in flight
    int small_slots = 3;       // the same for whole small-scene frames
    int cur = 0;               // slot of the frame being enqueued
    int last_slot = -1;        // slot of the previous frame call
    uint64_t frames = 0;       // frames begun
    int last_ao_slot = -1;     // slot of the last frame whose AO phase was enqueued (ao_order)
    int64_t slot_last[kSlots] = {-1, -1, -1, -1};  // the frame call that last used each slot
    hipEvent_t user_mark[kSlots] = {};  // the caller's stream at the start of the last frame calls (ring)
    // rt_gpu_render's host copy: pinned staging, filled in chunks (one event each)
    int16_t* stage = nullptr;
    size_t stage_bytes = 0;
    std::array<hipEvent_t, 16> stage_ev{};
    // every other host <-> device copy of pageable memory: two halves of a
    // pinned buffer (copy_h2d / copy_d2h), so the runtime never pins or maps
    // caller memory on the fly
    uint8_t* xfer = nullptr;
    hipEvent_t xfer_ev[2] = {};
    bool pipeline = true;      // RT580_PIPELINE=0: every frame on the caller's stream
    // rt_gpu_render's latency path: a second stream for the first part's
    // resolve + copy, and the hand-off events
    hipStream_t aux = nullptr;
    hipEvent_t aux_go = nullptr, aux_done = nullptr;
    // its split row for a (params, scene): read once, deterministic afterwards
    rt_render_params lat_params{};
    uint64_t lat_gen = ~0ull;
    int lat_row = -1;
    // render_split's frame as a HIP graph per slot: one launch instead of the
    // ~40 enqueue calls. Captured on the second identical call of a slot (the
    // first allocates), replayed while the key holds.
    struct FrameGraph {
        rt_render_params p{};
        uint64_t gen = ~0ull, buf_gen = ~0ull;
        const void* fb = nullptr;
        int seen = 0;
        hipGraphExec_t exec = nullptr;
    };
    std::array<FrameGraph, 4> fgraph{};
    bool graphs_off = false;
    uint32_t* far_count_host = nullptr;  // pinned: counts read on the host (rt_kernels.hip read_counts)
    // count schedules of the trace phase and of the AO phase (rt_kernels.h
    // CountSchedule), each valid for the frame of its key
    CountSchedule sched_trace, sched_ao;
    SchedKey key_trace{}, key_ao{};
    bool trace_valid = false, ao_valid = false;
    bool replayed = false;  // the frame being enqueued replays a schedule (its check is pending)
    uint32_t frame_fc = 0, frame_ac = 0;  // chunk sizes of the frame being enqueued (<= the slot's buffers)
    int chunk_log2 = 27;  // largest far-queue / AO-ray chunk: 2^chunk_log2 rays (RT580_CHUNK_LOG2;
                          // 2^27: the north-star frame's 117M AO samples in one chunk, 41.8 -> 40.8 ms)
    uint32_t node_cap = 0, call_cap = 0;
    double node_factor = 4.0;         // node capacity per pixel (grown on overflow)
    uint32_t* needed_host = nullptr;  // pinned
    // capacity verification: a (params, scene) already rendered without overflow
    rt_render_params verified{};
    uint64_t verified_gen = ~0ull;
    int verified_rows[3] = {0, 0, 0};  // the rows that frame traced: begin, step, count
    int traced_rows[3] = {0, 0, 0};    // the rows the current frame traces
    bool verified_valid = false;
    // stats of the last traced rows
    int last_rows = 0, last_width = 0, last_ao_samples = 0, last_ao_enabled = 0;
    bool last_valid = false;
    int stats_slot = 0;  // the slot those rows' per-row counters are in
    // multi-rank split
    rt_render_params split_params{};
    bool split_ready = false;
};

constexpr int kMaxCtx = 16;
constexpr int kChunkLog2Min = 6, kChunkLog2Max = 27;  // chunk capacities of BVH frames (rays)
State g_ctx[kMaxCtx];
int g_cur = 0;  // context the entry points act on (0 outside rt_gpu_render_multi)
#define g (g_ctx[g_cur])
char g_err[512] = "";
uint64_t g_scene_counter = 0;  // process-wide upload counter (survives rt_gpu_shutdown)

// Fault attribution. A device fault is reported by whichever HIP call next
// looks at the device, so every error names the entry point that saw it
// (g_call) and every device-side error also the last entry point that enqueued
// device work (g_last_work): a fault raised by a frame but first seen by the
// next call's upload is charged to that frame.
const char* g_call = "";
const char* g_last_work = "(no device work yet)";
struct CallScope {
    const char* prev;
    CallScope(const char* name, bool work) : prev(g_call) {
        g_call = name;
        if (work) g_last_work = name;
    }
    ~CallScope() { g_call = prev; }
};
#define RT_ENTRY(name) CallScope rt_call_scope_(name, false)  // entry point that does not enqueue device work
#define RT_WORK(name) CallScope rt_call_scope_(name, true)    // entry point that enqueues device work

#define SL (g.slot[g.cur])

// Stream of the frame being enqueued.
hipStream_t fs() { return g.pipeline ? g.slot[g.cur].stream : g.stream; }


int fail(const char* fmt, ...) {
    char msg[448];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    if (g_call[0]) std::snprintf(g_err, sizeof g_err, "%s: %s", g_call, msg);
    else std::snprintf(g_err, sizeof g_err, "%s", msg);
    std::fprintf(stderr, "rt_gpu: %s\n", g_err);
    return RT_FAILURE;
}

// A checked wait for the whole device (every stream of this process on it).
// An error here was raised by earlier device work: named as such.
int device_sync(const char* what) {
    const hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess)
        return fail("device error seen %s (raised by device work enqueued up to %s): %s", what, g_last_work,
                    hipGetErrorString(e));
    return RT_SUCCESS;
}

#define HIP_TRY(expr)                                                              \
    do {                                                                           \
        hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess) return fail("%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

// Frame pipelining. Consecutive frame calls rotate over three slots (own
// stream and workspace; RT580_SLOTS=2: two), so frame k+1's latency-bound
// trace overlaps frame k's AO kernels, and with three slots two frames' traces
// overlap each other as well. BVH frames too: their host reads (trace-level counts, the AO-call
// total) synchronize their own slot's stream only, and their AO chunks enqueue
// without one (binned far queue), so the host returns while frame k's AO runs
// and frame k+1's trace levels run beside it. Ordering:
//  - a frame on the slot the PREVIOUS call did not use waits on the caller's
//    stream as it was at the start of the previous call (user_mark): that
//    covers whatever the caller queued against this slot's last framebuffer
//    before it made that call;
//  - a frame on the same slot as the previous call (serialize) waits on the
//    caller's stream as it is now, so work the caller queued against the
//    previous frame's framebuffer completes first;
//  - the caller's stream waits for the frame (end_slot), so work the caller
//    queues after the call sees its results ("asynchronous on the shim's stream").
int check_replay(Slot& sl);
int post_replay_check();

// ns: slots this frame rotates over (whole small-scene frames: 2, see below).
int begin_slot(bool serialize, int ns) {
    if (!g.pipeline) {
        g.cur = 0;
        return check_replay(SL);
    }
    const uint64_t call = g.frames;
    const int k = (int)(call % (uint64_t)State::kSlots);
    HIP_TRY(hipEventRecord(g.user_mark[k], g.stream));  // this call's start
    const int slot = serialize ? 0 : (g.last_slot < 0 ? 0 : (g.last_slot + 1) % ns);
    // the caller's stream at the start of the call after this slot's last one
    // (it holds the wait for that frame and the caller's work on its
    // framebuffer queued before that call), or now when that is this call or
    // its mark has left the ring
    hipEvent_t wait = g.user_mark[k];
    if (g.slot_last[slot] >= 0) {
        const uint64_t wc = (uint64_t)g.slot_last[slot] + 1;
        if (wc < call && call - wc < (uint64_t)State::kSlots) wait = g.user_mark[wc % (uint64_t)State::kSlots];
    }
    g.slot_last[slot] = (int64_t)call;
    g.cur = slot;
    g.last_slot = slot;
    if (check_replay(SL)) return RT_FAILURE;
    HIP_TRY(hipStreamWaitEvent(SL.stream, wait, 0));
    g.frames++;
    return RT_SUCCESS;
}

// The caller's stream waits for what the current slot has enqueued.
int end_slot() {
    if (post_replay_check()) return RT_FAILURE;
    if (!g.pipeline) return RT_SUCCESS;
    HIP_TRY(hipEventRecord(SL.done, SL.stream));
    HIP_TRY(hipStreamWaitEvent(g.stream, SL.done, 0));
    return RT_SUCCESS;
}

// The current slot waits for what the caller's stream holds now (inputs the
// caller produced there, e.g. the all-gathered row bases of rt_gpu_shade_rows).
int slot_wait_user() {
    if (!g.pipeline) return RT_SUCCESS;
    const int k = (int)(g.frames % (uint64_t)State::kSlots);  // the mark the next begin_slot overwrites, unused until then
    HIP_TRY(hipEventRecord(g.user_mark[k], g.stream));
    HIP_TRY(hipStreamWaitEvent(SL.stream, g.user_mark[k], 0));
    return RT_SUCCESS;
}

bool frame_uses_bvh(const rt_render_params* p) {
    return g.accel == RT_ACCEL_AUTO && g.bvh_ok && bvh_usable(g.bvh, p->cam_from);
}

// A checked wait for one stream; an error was raised by earlier device work.
int stream_sync(hipStream_t s, const char* what) {
    const hipError_t e = hipStreamSynchronize(s);
    if (e != hipSuccess)
        return fail("device error seen %s (raised by device work enqueued up to %s): %s", what, g_last_work,
                    hipGetErrorString(e));
    return RT_SUCCESS;
}

// Wait for every enqueued frame and the caller's stream -- of every context on
// this context's device (the split rehearsal keeps several contexts on one
// GPU; a scene upload or buffer release must not race any of them).
int sync_all() {
    const int dev = g.device;
    for (int k = 0; k < kMaxCtx; k++) {
        State& c = g_ctx[k];
        if (!c.inited || c.device != dev) continue;
        if (stream_sync(c.stream, "waiting for the caller's stream")) return RT_FAILURE;
        if (c.own_stream != c.stream && stream_sync(c.own_stream, "waiting for the library's stream")) return RT_FAILURE;
        for (auto& sl : c.slot)
            if (sl.stream && stream_sync(sl.stream, "waiting for a frame slot")) return RT_FAILURE;
        if (c.aux && stream_sync(c.aux, "waiting for the latency path's stream")) return RT_FAILURE;
    }
    return RT_SUCCESS;
}

// Bumped by every workspace (re)allocation and release: a captured frame
// graph (render_split) holds the buffer addresses of its capture.
uint64_t g_buf_gen = 0;

int ensure(DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return RT_SUCCESS;
    g_buf_gen++;
    if (b.p) {  // frames in flight may still read the old buffer
        if (device_sync("before a workspace buffer is resized")) return RT_FAILURE;
        HIP_TRY(hipFree(b.p));
        b.p = nullptr;
        b.bytes = 0;
    }
    if (bytes == 0) bytes = 64;
    size_t want = bytes + bytes / 8 + 256;
    HIP_TRY(hipMalloc(&b.p, want));
    b.bytes = want;
    return RT_SUCCESS;
}

void release(DevBuf& b) {
    if (b.p) g_buf_gen++;
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

int n_selected_rows(const rt_render_params* p) {
    if (p->row_step <= 0 || p->row_begin >= p->row_end) return 0;
    return (p->row_end - p->row_begin + p->row_step - 1) / p->row_step;
}

int check_params(const rt_render_params* p) {
    if (!p || p->abi_version != RT580_ABI_VERSION) return fail("bad rt_render_params / ABI version");
    if (p->width <= 0 || p->height <= 0) return fail("bad resolution %dx%d", p->width, p->height);
    if ((int64_t)p->width * p->height > (int64_t)1 << 30) return fail("frame too large");
    if (p->depth < 0 || p->depth > RT_MAX_DEPTH) return fail("depth %d outside [0,%d]", p->depth, RT_MAX_DEPTH);
    if (p->ao_samples <= 0 || p->ao_samples > 512) return fail("ao_samples must be in [1, 512]");
    if (p->rng_engine != RT_RNG_MINSTD_RAND0 && p->rng_engine != RT_RNG_MT19937) return fail("bad rng engine");
    if (p->row_begin < 0 || p->row_end > p->height || p->row_step <= 0) return fail("bad row selection");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (!g.have_scene) return fail("no scene uploaded");
    return RT_SUCCESS;
}

// Frames of fewer pixels than this use the half-resolution direction grid:
// fewer rays per cell there, and a cell's list is read once per chunk of its
// rays. North-star frame's K-way row shares (rank 1), fine -> coarse: K = 2
// 22.45 -> 21.62 ms, 4: 13.40 -> 12.32, 8: 8.66 -> 7.55; the whole frame (2.07M
// pixels) keeps the fine grid (38.8 vs 39.1 ms). RT580_GRID_COARSE_PX (0: never).
long grid_coarse_px() {
    static long v = -1;
    if (v < 0) {
        const char* e = std::getenv("RT580_GRID_COARSE_PX");
        v = e ? std::atol(e) : 1572864L;
    }
    return v;
}

// Bit c set: cell c of a grid (its list offsets `start`) lists a candidate.
std::vector<uint32_t> live_bitmap(const std::vector<uint32_t>& start) {
    std::vector<uint32_t> bits(start.empty() ? 0 : (start.size() - 1 + 31) / 32, 0u);
    for (size_t c = 0; c + 1 < start.size(); c++)
        if (start[c + 1] != start[c]) bits[c >> 5] |= 1u << (c & 31);
    return bits;
}

// n_rows: the frame's rows (selects the direction grid; -1: the fine one).
DevScene dev_scene(const rt_render_params* p, int n_rows) {
    DevScene s;
    std::memset(&s, 0, sizeof s);
    s.prims = (const rt_prim*)g.prims.p;
    s.shade = (const rt_prim_shade*)g.shade.p;
    s.mats = (const rt_material*)g.mats.p;
    s.lights = (const rt_light*)g.lights.p;
    s.n_prims = g.n_prims;
    s.n_lights = g.n_lights;
    s.n_ambient = g.n_ambient;
    s.use_bvh = g.accel == RT_ACCEL_AUTO && g.bvh_ok && bvh_usable(g.bvh, p->cam_from);
    s.scan_prims = g.scan_prims.p ? (const rt_prim*)g.scan_prims.p : s.prims;
    s.n_shadow = 0;
    if ((int)g.shadow_lights.size() <= 8)
        for (int li : g.shadow_lights) s.shadow_light[s.n_shadow++] = li;
    BvhView& v = s.bv;
    v.all = s.prims;
    v.nodes = (const BvhNode*)g.bvh_nodes.p;
    v.nodes4 = g.bvh.nodes4q.empty() ? nullptr : (const Bvh4QNode*)g.bvh_nodes4.p;
    v.prims = (const rt_prim*)g.bvh_prims.p;
    v.ids = (const uint32_t*)g.bvh_ids.p;
    v.far_nodes = (const FarNode*)g.far_nodes.p;
    v.far_tris = (const FarTri*)g.far_tris.p;
    v.brute = (const uint32_t*)g.brute.p;
    v.n_brute = (int)g.bvh.brute.size();
    v.n_far = g.bvh.n_far;
    v.dhi_median = g.bvh.dhi_median;
    v.has_tree = !g.bvh.nodes.empty();
    v.has_far = !g.bvh.far_nodes.empty();
#ifdef RT580_DIAGNOSTICS
    {   // DIAGNOSTIC build only (timing ablation, wrong results): RT580_BVH_DIAG=1 skips the far search
        static int diag = -1;
        if (diag < 0) {
            const char* e = std::getenv("RT580_BVH_DIAG");
            diag = e ? std::atoi(e) : 0;
        }
        if (diag & 1) v.has_far = 0;
    }
#endif
    v.scale = g.bvh.scale;
    const bool coarse = g.grid2 && n_rows >= 0 && (long)n_rows * p->width < grid_coarse_px();
    v.grid_start = (const uint32_t*)(coarse ? g.grid2_start.p : g.grid_start.p);
    v.grid_items = (const uint32_t*)(coarse ? g.grid2_items.p : g.grid_items.p);
    v.grid_always = (const uint32_t*)g.grid_always.p;
    v.grid_live = (const uint32_t*)(coarse ? g.grid2_live.p : g.grid_live.p);
    v.n_always = g.grid_n_always;
    v.grid_log2 = coarse ? g.grid_log2 - 1 : g.grid_log2;
    v.grid_r = g.bvh.grid_r;
    return s;
}

// Scene uploads are synchronous: every copy has completed (and any device
// error it met is reported, naming the array) before the call returns or the
// host array is freed.
int copy_h2d(void* dst, const void* src, size_t n, hipStream_t s, const char* what);
int h2d(void* dst, const void* src, size_t bytes, const char* what) { return copy_h2d(dst, src, bytes, g.stream, what); }

// Host ranges page-locked by rt_gpu_host_register (process-wide).
struct HostRange {
    const char* p;
    size_t bytes;
    // the last frame copy enqueued into the range (rt_gpu_render_async): the
    // next one waits for it, so frames land in call order
    hipEvent_t copied = nullptr;
    int copied_device = -1;
    void* dev = nullptr;  // the range mapped into the devices' address space
};
std::vector<HostRange> g_host_ranges;

bool host_registered(const void* p, size_t bytes) {
    const char* c = (const char*)p;
    for (const HostRange& r : g_host_ranges)
        if (c >= r.p && c + bytes <= r.p + r.bytes) return true;
    return false;
}

// Host <-> device copies of caller or library host memory that is not page
// locked go through the context's pinned transfer buffer (two halves, one
// chunk in flight while the other is filled or drained). The HIP runtime
// otherwise pins pageable memory on the fly for large copies and keeps those
// pins; a later allocation at a reused virtual address could then be read
// through a stale mapping -- the device fault the round-3 GPU suite met in a
// scene upload. Both return once the copy is complete.
constexpr size_t kXferHalf = (size_t)8 << 20;

int xfer_ready() {
    if (g.xfer) return RT_SUCCESS;
    HIP_TRY(hipHostMalloc((void**)&g.xfer, 2 * kXferHalf, hipHostMallocDefault));
    for (auto& e : g.xfer_ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return RT_SUCCESS;
}

int copy_h2d(void* dst, const void* src, size_t n, hipStream_t s, const char* what) {
    if (!n) return RT_SUCCESS;
    char w[128];
    std::snprintf(w, sizeof w, "by the copy of %s to the device", what);
    if (host_registered(src, n)) {
        HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, s));
        return stream_sync(s, w);
    }
    if (xfer_ready()) return RT_FAILURE;
    bool used[2] = {false, false};
    int h = 0;
    for (size_t off = 0; off < n; off += kXferHalf, h ^= 1) {
        const size_t c = n - off < kXferHalf ? n - off : kXferHalf;
        if (used[h]) {  // this half's previous chunk has left
            const hipError_t e = hipEventSynchronize(g.xfer_ev[h]);
            if (e != hipSuccess)
                return fail("device error seen %s (raised by device work enqueued up to %s): %s", w, g_last_work,
                            hipGetErrorString(e));
        }
        uint8_t* b = g.xfer + (size_t)h * kXferHalf;
        std::memcpy(b, (const char*)src + off, c);
        const hipError_t e = hipMemcpyAsync((char*)dst + off, b, c, hipMemcpyHostToDevice, s);
        if (e != hipSuccess)
            return fail("copy of %s (%zu bytes) to the device (device work enqueued up to %s): %s", what, n,
                        g_last_work, hipGetErrorString(e));
        HIP_TRY(hipEventRecord(g.xfer_ev[h], s));
        used[h] = true;
    }
    return stream_sync(s, w);
}

int copy_d2h(void* dst, const void* src, size_t n, hipStream_t s, const char* what) {
    if (!n) return RT_SUCCESS;
    char w[128];
    std::snprintf(w, sizeof w, "by the copy of %s to the host", what);
    if (host_registered(dst, n)) {
        HIP_TRY(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s));
        return stream_sync(s, w);
    }
    if (xfer_ready()) return RT_FAILURE;
    size_t pend_off[2] = {0, 0}, pend_n[2] = {0, 0};
    int h = 0;
    auto drain = [&](int k) -> int {
        if (!pend_n[k]) return RT_SUCCESS;
        const hipError_t e = hipEventSynchronize(g.xfer_ev[k]);
        if (e != hipSuccess)
            return fail("device error seen %s (raised by device work enqueued up to %s): %s", w, g_last_work,
                        hipGetErrorString(e));
        std::memcpy((char*)dst + pend_off[k], g.xfer + (size_t)k * kXferHalf, pend_n[k]);
        pend_n[k] = 0;
        return RT_SUCCESS;
    };
    for (size_t off = 0; off < n; off += kXferHalf, h ^= 1) {
        const size_t c = n - off < kXferHalf ? n - off : kXferHalf;
        if (drain(h)) return RT_FAILURE;
        const hipError_t e = hipMemcpyAsync(g.xfer + (size_t)h * kXferHalf, (const char*)src + off, c,
                                            hipMemcpyDeviceToHost, s);
        if (e != hipSuccess)
            return fail("copy of %s (%zu bytes) to the host (device work enqueued up to %s): %s", what, n, g_last_work,
                        hipGetErrorString(e));
        HIP_TRY(hipEventRecord(g.xfer_ev[h], s));
        pend_off[h] = off;
        pend_n[h] = c;
    }
    if (drain(h) || drain(h ^ 1)) return RT_FAILURE;
    return RT_SUCCESS;
}

template <typename T>
int upload_vec(DevBuf& b, const std::vector<T>& v, const char* what) {
    if (ensure(b, sizeof(T) * v.size() + 64)) return RT_FAILURE;
    return h2d(b.p, v.data(), sizeof(T) * v.size(), what);
}

DevFrame dev_frame(const rt_render_params* p, int row_begin, int row_step, int n_rows) {
    DevFrame f;
    std::memset(&f, 0, sizeof f);
    f.width = p->width;
    f.height = p->height;
    f.depth = p->depth;
    f.ao_samples = p->ao_samples;
    f.ao_enabled = p->ao_enabled;
    f.rng_engine = p->rng_engine;
    f.rng_seed = p->rng_seed;
    f.row_begin = row_begin;
    f.row_step = row_step;
    f.n_rows = n_rows;
    f.view_inverse_ok = p->view_inverse_ok;
    std::memcpy(f.view_inv, p->view_inv, sizeof f.view_inv);
    std::memcpy(f.cam_from, p->cam_from, sizeof f.cam_from);
    f.ao_angle_max = p->ao_angle_max;
    f.ndc_kx = p->ndc_kx;
    f.ndc_ky = p->ndc_ky;
    {   // 16807^(2 N) mod (2^31 - 1), then its repeated squares
        const uint64_t m = 2147483647ull;
        uint64_t b = 16807, st = 1;
        for (uint64_t e = 2ull * (uint64_t)p->ao_samples; e; e >>= 1, b = b * b % m)
            if (e & 1) st = st * b % m;
        for (int i = 0; i < 32; i++, st = st * st % m) f.step_pow2[i] = (uint32_t)st;
    }
    return f;
}

DevWork dev_work() {
    DevWork w;
    w.nodes = (NodeRec*)SL.nodes.p;
    w.topo = (int4*)SL.topo.p;
    w.node_call0 = (uint32_t*)SL.node_call0.p;
    w.node_val = (int2*)SL.node_val.p;
    w.rays = (RayItem*)SL.rays.p;
    w.lvl = (uint32_t*)SL.lvl.p;
    w.needed = (uint32_t*)SL.needed.p;
    w.pix_hits = (uint32_t*)SL.pix_hits.p;
    w.pix_nodes = (uint32_t*)SL.pix_nodes.p;
    w.pix_prefix = (uint32_t*)SL.pix_prefix.p;
    w.row_calls = (uint32_t*)SL.row_calls.p;
    w.row_hits = (uint32_t*)SL.row_hits.p;
    w.row_nodes = (uint32_t*)SL.row_nodes.p;
    w.row_base_local = (uint64_t*)SL.row_base_local.p;
    w.totals = (uint64_t*)SL.totals.p;
    w.call_node = (uint32_t*)SL.call_node.p;
    w.call_rng = (uint64_t*)SL.call_rng.p;
    w.occ = (uint32_t*)SL.occ.p;
    w.mt_stream = (const uint32_t*)SL.mt_stream.p;
    w.mt_base = SL.mt_base;
    w.node_cap = g.node_cap;
    w.call_cap = g.call_cap;
    w.far_rays = (float4*)SL.far_rays.p;
    w.far_keys = (uint32_t*)SL.far_keys.p;
    w.far_keys_alt = (uint32_t*)SL.far_keys_alt.p;
    w.far_vals = (uint32_t*)SL.far_vals.p;
    w.far_vals_alt = (uint32_t*)SL.far_vals_alt.p;
    w.far_count = (uint32_t*)SL.far_count.p;
    w.far_seg_off = (uint32_t*)SL.far_seg_off.p;
    w.far_seg_n = (uint32_t*)SL.far_seg_n.p;
    w.far_wofs = (uint32_t*)SL.far_wofs.p;
    w.far_work = (uint4*)SL.far_work.p;
    w.far_count_host = g.far_count_host;
    w.sort_tmp = SL.sort_tmp.p;
    w.sort_tmp_bytes = SL.sort_tmp.bytes;
    w.far_cap = std::min(SL.far_cap, g.frame_fc);
    w.ao_cap = std::min(SL.ao_cap, g.frame_ac);
    w.ao_rays = w.ao_cap ? (float4*)SL.ao_rays.p : nullptr;
    w.ao_hp = w.ao_cap ? (float4*)SL.ao_rays.p + w.ao_cap : nullptr;  // (the buffer holds 2 ao_cap + 4 float4)
    w.ao_late = w.ao_cap ? (uint32_t*)SL.ao_late.p : nullptr;
    w.ao_late_count = w.ao_cap ? (uint32_t*)SL.ao_late_count.p : nullptr;
    w.ao_state_cap = w.ao_cap ? w.ao_cap / 16 : 0u;
    w.ao_state = w.ao_state_cap ? (uint32_t*)SL.ao_state.p : nullptr;
    const bool split = g.bvh_ok && !g.bvh.far_nodes.empty();
    w.hit4 = split ? (float4*)SL.hit4.p : nullptr;
    w.hit_prim = split ? (int32_t*)SL.hit_prim.p : nullptr;
    // shadow flags of the split trace's lights (more than 8: decided in the shading phase)
    w.shadow = (split && SL.shadow.p && !g.shadow_lights.empty() && g.shadow_lights.size() <= 8) ? (uint8_t*)SL.shadow.p
                                                                                                      : nullptr;
    w.aofix_items = (uint64_t*)SL.aofix_items.p;
    w.aofix_count = (uint32_t*)SL.aofix_count.p;
    w.call_hint = (uint32_t*)SL.call_hint.p;  // per-call acceptor hints of the brute any-hit scans
    w.aofix_cap = (uint32_t)(SL.aofix_items.bytes / 8);
    w.poison = (const uint32_t*)SL.bad.p;
    return w;
}

int begin_frame() {
    if (!g.profiling && g.kt_keep) {  // the first frame after profiling ends its kernel timing
        kernel_timer_enable(false);
        g.kt_keep = false;
    }
    if (!g.profiling) {
        g.ev = g.ev_default.data();
        return RT_SUCCESS;
    }
    if ((int)g.prof_pool.size() <= g.prof_frames) {
        std::array<hipEvent_t, EV_N> q;
        for (auto& e : q) HIP_TRY(hipEventCreate(&e));
        g.prof_pool.push_back(q);
    }
    g.ev = g.prof_pool[g.prof_frames].data();
    g.prof_frames++;
    return RT_SUCCESS;
}

// A new chunk limit: the next frame sizes the chunk buffers again (at most
// 2^log2 rays). The context's streams are idle.
void set_chunk_log2(int log2) {
    if (g.chunk_log2 == log2) return;
    g.chunk_log2 = log2;
    for (Slot& sl : g.slot) {
        for (DevBuf* b : {&sl.far_rays, &sl.far_keys, &sl.far_keys_alt, &sl.far_vals, &sl.far_vals_alt, &sl.sort_tmp,
                          &sl.ao_rays, &sl.far_seg_off, &sl.far_wofs, &sl.far_work, &sl.ao_late, &sl.shadow, &sl.ao_state})
            release(*b);
        sl.far_cap = sl.ao_cap = 0;
    }
}

// Size the workspace for n_rows x width pixels.
int ensure_work(const rt_render_params* p, int n_rows) {
    const uint64_t npix = (uint64_t)n_rows * p->width;
    const uint64_t tree_max = (1ull << (p->depth + 1)) - 1;  // nodes of a full tree
    const double f = g.node_factor < (double)tree_max ? g.node_factor : (double)tree_max;
    uint64_t cap = (uint64_t)((double)npix * f) + 4096;
    if (cap < npix) cap = npix;
    if (cap > 0xffffff00ull) return fail("node capacity exceeds 2^32");
    const uint64_t ccap = cap * (uint64_t)(g.n_ambient > 0 ? g.n_ambient : 1);
    if (ccap > 0xffffff00ull) return fail("AO-call capacity exceeds 2^32");
    if (ensure(SL.nodes, cap * sizeof(NodeRec)) || ensure(SL.topo, cap * 16) || ensure(SL.node_call0, cap * 4) ||
        ensure(SL.node_val, cap * 8) ||
        ensure(SL.rays, cap * sizeof(RayItem)) ||
        ensure(SL.lvl, 4 * (RT_MAX_DEPTH + 2) * sizeof(uint32_t)) || ensure(SL.needed, 64) ||
        ensure(SL.pix_hits, npix * 4) || ensure(SL.pix_nodes, npix * 4) || ensure(SL.pix_prefix, npix * 4) ||
        ensure(SL.row_calls, (size_t)n_rows * 4) || ensure(SL.row_hits, (size_t)n_rows * 4) ||
        ensure(SL.row_nodes, (size_t)n_rows * 4) || ensure(SL.row_base_local, (size_t)n_rows * 8) ||
        ensure(SL.totals, 64) || ensure(SL.call_node, ccap * 4) || ensure(SL.call_rng, ccap * 8) ||
        ensure(SL.occ, ccap * 4) || ensure(SL.aofix_items, (size_t)8 << 20) || ensure(SL.aofix_count, 64))
        return RT_FAILURE;
    // the slot's replay-check word (count_check_kernel sets it; DevWork::poison)
    // and its pinned host copy: zero from the start, and again after a failure
    if (!SL.bad.p) {
        if (ensure(SL.bad, 64)) return RT_FAILURE;
        HIP_TRY(hipMemsetAsync(SL.bad.p, 0, 64, fs()));
    }
    if (!SL.bad_host) {
        HIP_TRY(hipHostMalloc((void**)&SL.bad_host, 64, hipHostMallocDefault));
        std::memset(SL.bad_host, 0, 64);
    }
    if (g.bvh_ok && !g.bvh.far_nodes.empty() && ensure(SL.call_hint, ccap * 4)) return RT_FAILURE;
    g.node_cap = (uint32_t)cap;
    g.call_cap = (uint32_t)ccap;
    // Chunked passes of BVH frames: the far-hit queue (one trace level's rays,
    // or the misses of one AO chunk) and the AO ray records. Sized to what the
    // frame can need, at most 2^chunk_log2 rays, and grown on demand; a larger
    // frame runs in several chunks (same results, checked by the GPU tests with
    // small chunks).
    auto pow2ceil = [](uint64_t v) { uint64_t r = 1024; while (r < v) r <<= 1; return r; };
    const uint64_t chunk_max = 1ull << g.chunk_log2;
    const uint64_t ao_items = p->ao_enabled && g.n_ambient > 0 ? ccap * (uint64_t)p->ao_samples : 0;
    const uint32_t ac = (uint32_t)std::min(chunk_max, pow2ceil(ao_items));
    g.frame_ac = g.bvh_ok ? ac : 0;
    g.frame_fc = 0;
    if (g.bvh_ok && SL.ao_cap < ac) {  // ray records of the split AO pass (ao_trace_kernel)
        // 16-byte records, then one hit point per call (<= ac + 2 calls per chunk)
        if (ensure(SL.ao_rays, (size_t)ac * 32 + 64) || ensure(SL.ao_late, (size_t)ac * 4) ||
            ensure(SL.ao_late_count, 64) ||
            ensure(SL.ao_state, (size_t)(ac / 16) * kLateWords * 4))
            return RT_FAILURE;
        SL.ao_cap = ac;
    }
    if (!g.bvh_ok || g.bvh.far_nodes.empty()) return RT_SUCCESS;
    const uint32_t fc = (uint32_t)std::min(chunk_max, pow2ceil(std::max<uint64_t>(cap, ac)));
    g.frame_fc = fc;
    if (SL.far_cap < fc) {
        if (ensure(SL.far_rays, (size_t)fc * 32) || ensure(SL.far_keys, (size_t)fc * 4) ||
            ensure(SL.far_keys_alt, (size_t)fc * 4) || ensure(SL.far_vals, (size_t)fc * 4) ||
            ensure(SL.far_vals_alt, (size_t)fc * 4) || ensure(SL.far_count, 64) ||
            ensure(SL.far_seg_off, (size_t)fc * 4) || ensure(SL.far_seg_n, 64) || ensure(SL.far_wofs, (size_t)fc * 4) ||
            ensure(SL.far_work, ((size_t)fc + fc / 64 + 64) * 16) ||
            ensure(SL.sort_tmp, far_sort_tmp_bytes(fc) + 256))
            return RT_FAILURE;
        SL.far_cap = fc;
    }
    if (ensure(SL.hit4, (size_t)cap * 16) || ensure(SL.hit_prim, (size_t)cap * 4)) return RT_FAILURE;
    if (!g.shadow_lights.empty() && g.shadow_lights.size() <= 8 &&
        ensure(SL.shadow, g.shadow_lights.size() * (size_t)fc))
        return RT_FAILURE;
    return RT_SUCCESS;
}

// ---------------------------------------------------------------- count schedules
// A BVH frame reads a few device counts on the host while it is enqueued
// (rt_kernels.h CountSchedule). They are a function of the frame's key, so a
// repeat of a verified frame replays the counts recorded on an earlier run of
// it: no host sync, and the next frame's trace overlaps this frame's AO on the
// other slot. Every replayed count is checked on the device; a mismatch fails
// the call that next uses the slot (check_replay), and drops the schedules.
SchedKey sched_key(const rt_render_params* p) {
    SchedKey k;
    std::memset(&k, 0, sizeof k);
    k.p = *p;
    k.gen = g.scene_gen;
    std::memcpy(k.rows, g.traced_rows, sizeof k.rows);
    k.far_chunk = g.frame_fc;
    k.ao_chunk = g.frame_ac;
    k.accel = frame_uses_bvh(p) ? 1 : 0;
    return k;
}

bool same_key(const SchedKey& a, const SchedKey& b) {
    static int on = -1;  // RT580_REPLAY=0 (A/B): every frame reads its counts on the host
    if (on < 0) {
        const char* e = std::getenv("RT580_REPLAY");
        on = e ? std::atoi(e) : 1;
    }
    return on && std::memcmp(&a, &b, sizeof a) == 0;
}

// (params, scene, traced rows) already rendered without node overflow
bool frame_verified(const rt_render_params* p) {
    return g.verified_valid && g.verified_gen == g.scene_gen && std::memcmp(&g.verified, p, sizeof *p) == 0 &&
           std::memcmp(g.verified_rows, g.traced_rows, sizeof g.traced_rows) == 0;
}

int begin_schedule(CountSchedule& cs, bool replay) {
    if (replay) {
        cs.mode = CountSchedule::REPLAY;
        cs.pos = 0;
        cs.broken = false;
        cs.bad = (uint32_t*)SL.bad.p;
        g.replayed = true;
    } else {
        cs.mode = CountSchedule::RECORD;
        cs.vals.clear();
        cs.where.clear();
    }
    cs.tag = &cs == &g.sched_ao ? 1u : 0u;
    set_count_schedule(&cs);
    return RT_SUCCESS;
}

int end_schedule(CountSchedule& cs, const char* what, hipError_t e) {
    set_count_schedule(nullptr);
    if (cs.mode == CountSchedule::REPLAY && (cs.broken || (e == hipSuccess && cs.pos != cs.vals.size()))) {
        g.trace_valid = g.ao_valid = false;
        return fail("replayed %s count schedule does not fit the frame (%zu of %zu counts used)", what, cs.pos,
                    cs.vals.size());
    }
    return RT_SUCCESS;
}

// After a frame that replayed a schedule: its check flag to the host, read
// when the slot is used next (the frame is complete by then).
int post_replay_check() {
    if (!g.replayed) return RT_SUCCESS;
    g.replayed = false;
    HIP_TRY(hipMemcpyAsync(SL.bad_host, SL.bad.p, 24, hipMemcpyDeviceToHost, fs()));
    SL.check_pending = true;
    return RT_SUCCESS;
}

// Which count of which schedule a failed device check names (bad[1] = its
// index + 1, count_check_kernel), with the launcher step that recorded it.
std::string replay_mismatch_detail(const uint32_t* bad) {
    if (bad[1] == 0) return "";
    const size_t pos = (bad[1] - 1) & 0xffffu;
    const CountSchedule& cs = (bad[1] - 1) >> 16 ? g.sched_ao : g.sched_trace;
    const char* sched = &cs == &g.sched_ao ? "AO" : "trace";
    const char* where = pos < cs.where.size() ? cs.where[pos] : "?";
    char buf[256];
    std::snprintf(buf, sizeof buf, "; first mismatch: count #%zu (%s schedule, %s): this frame %u/%u, recorded %u/%u",
                  pos, sched, where, bad[2], bad[3], bad[4], bad[5]);
    return buf;
}

// The replay check of the slot's last frame (waits for that frame).
int check_replay(Slot& sl) {
    if (!sl.check_pending) return RT_SUCCESS;
    if (g.pipeline) HIP_TRY(hipEventSynchronize(sl.done));
    else HIP_TRY(hipStreamSynchronize(g.stream));
    sl.check_pending = false;
    if (*sl.bad_host == 0) return RT_SUCCESS;
    const std::string detail = replay_mismatch_detail(sl.bad_host);
    std::memset(sl.bad_host, 0, 24);
    HIP_TRY(hipMemset(sl.bad.p, 0, 64));
    g.trace_valid = g.ao_valid = false;
    return fail("a replayed count schedule did not match its frame's counts (the last frame enqueued on this "
                "slot, %d frame calls back at most; schedules dropped)%s", g.nslots, detail.c_str());
}

// The host-side record of the frame being enqueued (rt_gpu_last_stats,
// rt_gpu_accel_active): its rows, their slot, the parameters the stats need.
void note_rows(const rt_render_params* p, int n_rows, bool accel) {
    g.last_accel = accel;
    g.last_rows = n_rows;
    g.last_width = p->width;
    g.last_ao_samples = p->ao_samples;
    g.last_ao_enabled = p->ao_enabled;
    g.last_valid = true;
    g.stats_slot = g.cur;
}

// Phase 1: trace every level of the selected rows and count their AO calls.
static hipError_t phase_mark(int e, hipStream_t s);

int trace_rows(const rt_render_params* p, int row_begin, int row_step, int n_rows) {
    if (ensure_work(p, n_rows)) return RT_FAILURE;  // (launch_trace zeroes the per-frame counters)
    DevFrame f = dev_frame(p, row_begin, row_step, n_rows);
    const DevScene sc = dev_scene(p, n_rows);
    g.last_accel = sc.use_bvh != 0;
    g.traced_rows[0] = row_begin;
    g.traced_rows[1] = row_step;
    g.traced_rows[2] = n_rows;
    {
        const SchedKey key = sched_key(p);
        const bool replay = g.trace_valid && same_key(g.key_trace, key);
        if (begin_schedule(g.sched_trace, replay)) return RT_FAILURE;
        if (!replay) {
            g.key_trace = key;
            g.trace_valid = false;
        }
        const hipError_t e = launch_trace(sc, f, dev_work(), fs());
        if (end_schedule(g.sched_trace, "trace", e)) return RT_FAILURE;
        if (e != hipSuccess) return fail("launch_trace (%s): %s", launch_where(), hipGetErrorString(e));
        // a verified frame cannot overflow: its recording is valid at once (else check_capacity decides)
        if (!replay && frame_verified(p)) g.trace_valid = true;
    }
    HIP_TRY(launch_row_counts(sc, f, dev_work(), fs()));
    HIP_TRY(phase_mark(EV_TRACE, fs()));
    note_rows(p, n_rows, sc.use_bvh != 0);
    return RT_SUCCESS;
}

// mt19937: the draws these rows need, [lo, hi) of the reference's serial
// stream (single call: [0, the local total); multi-rank rows: from the lowest
// to the highest draw of their global row bases), generated on the device:
// the host supplies the stream's checkpoint windows at every kMtBlock draws
// (rt_mt.h block jump-ahead, cached per seed for later frames), one workgroup
// per block runs the twist (launch_mt_generate). Draws are addressed by
// absolute index minus the window's base.
constexpr uint64_t kMtMaxWindow = 1ull << 34;  // draws held at once per device (64 GiB of the 288 GB),
                                                // split over its frame slots

int prepare_mt_stream(const rt_render_params* p, const uint64_t* row_base_global, int n_rows) {
    if (p->rng_engine != RT_RNG_MT19937 || !p->ao_enabled || g.n_ambient == 0) return RT_SUCCESS;
    uint64_t lo_call = 0, hi_call = 0;
    if (!row_base_global) {
        if (copy_d2h(&hi_call, SL.totals.p, 8, fs(), "the AO-call total")) return RT_FAILURE;
    } else if (n_rows > 0) {
        std::vector<uint64_t> base((size_t)n_rows);
        std::vector<uint32_t> calls((size_t)n_rows);
        if (copy_d2h(base.data(), row_base_global, (size_t)n_rows * 8, fs(), "the row bases") ||
            copy_d2h(calls.data(), SL.row_calls.p, (size_t)n_rows * 4, fs(), "the per-row AO calls"))
            return RT_FAILURE;
        lo_call = ~0ull;
        for (int i = 0; i < n_rows; i++)
            if (calls[(size_t)i]) {
                lo_call = std::min(lo_call, base[(size_t)i]);
                hi_call = std::max(hi_call, base[(size_t)i] + calls[(size_t)i]);
            }
        if (lo_call > hi_call) lo_call = hi_call;
    }
    const uint64_t per_call = 2ull * (uint64_t)p->ao_samples;
    const uint64_t lo = lo_call * per_call, hi = hi_call * per_call;
    const uint64_t max_window = kMtMaxWindow / (uint64_t)(g.nslots > 0 ? g.nslots : 1);
    if (hi - lo > max_window)
        return fail("mt19937: these rows need draws [%llu, %llu), more than the %llu a frame slot's window holds "
                    "(use minstd_rand0, or fewer rows per call)",
                    (unsigned long long)lo, (unsigned long long)hi, (unsigned long long)max_window);
    SL.mt_base = lo;
    if (hi == lo) return RT_SUCCESS;
    const uint64_t k0 = lo / kMtBlock, k1 = (hi + kMtBlock - 1) / kMtBlock;
    const uint32_t nblk = (uint32_t)(k1 - k0);
    if (ensure(SL.mt_stream, (hi - lo) * 4 + 8) || ensure(SL.mt_windows, (size_t)nblk * sizeof(MtWindow)))
        return RT_FAILURE;
    std::vector<MtWindow> cps;
    if (!mt_checkpoints(p->rng_seed, k0, k1, cps))
        return fail("mt19937: the engine's characteristic polynomial could not be found (jump-ahead unavailable)");
    if (copy_h2d(SL.mt_windows.p, cps.data(), (size_t)nblk * sizeof(MtWindow), fs(), "the mt19937 checkpoint windows"))
        return RT_FAILURE;
    HIP_TRY(launch_mt_generate((const uint32_t*)SL.mt_windows.p, k0, nblk, lo, hi, (uint32_t*)SL.mt_stream.p, fs()));
    return RT_SUCCESS;
}

// The frame's phase boundaries for rt_gpu_last_stats (ms_count, ms_scan,
// ms_render). (Recording only the frame's start and end instead: no difference
// measured, profiles/r05/ab.)
static hipError_t phase_mark(int e, hipStream_t s) {
    return hipEventRecord(g.ev[e], s);
}

// AO phases in frame order (RT580_AO_ORDER=1, rt580_set_ao_order): a frame's
// AO kernels start after the previous frame's, so consecutive frames overlap
// one frame's trace with the other's AO only. Off by default: AO phases that
// run together fill each other's tails (north-star frame 44.9 -> 41.8 ms,
// config 2 1.532 -> 1.497 ms) at the price of longer launches (config 2's AO
// kernel 1.16 -> 2.08 ms per launch). bench.py times the AO kernel once more
// in order, untimed, to report its isolated launch beside the live one.
int g_ao_order = -1;  // process-wide; rt580_set_ao_order overrides
bool ao_order() {
    if (g_ao_order < 0) {
        const char* e = std::getenv("RT580_AO_ORDER");
        g_ao_order = e ? std::atoi(e) : 0;
    }
    return g_ao_order != 0;
}

hipError_t wait_previous_ao() {
    if (!g.pipeline || g.last_ao_slot < 0 || g.last_ao_slot == g.cur) return hipSuccess;
    return hipStreamWaitEvent(fs(), g.slot[g.last_ao_slot].ao_done, 0);
}

// Phase 2: number AO calls (RNG positions), AO, resolve into fb_out.
int shade_rows(const rt_render_params* p, int row_begin, int row_step, int n_rows, const uint64_t* row_base_global,
               int16_t* fb_out) {
    DevFrame f = dev_frame(p, row_begin, row_step, n_rows);
    const DevScene sc = dev_scene(p, n_rows);
    HIP_TRY(launch_rank(sc, f, dev_work(), row_base_global, fs()));
    HIP_TRY(phase_mark(EV_RANK, fs()));
    if (prepare_mt_stream(p, row_base_global, n_rows)) return RT_FAILURE;
    DevWork w = dev_work();
    {
        const SchedKey key = sched_key(p);
        const bool replay = g.ao_valid && same_key(g.key_ao, key);
        if (begin_schedule(g.sched_ao, replay)) return RT_FAILURE;
        if (!replay) {
            g.key_ao = key;
            g.ao_valid = false;
        }
        if (ao_order()) HIP_TRY(wait_previous_ao());
        const hipError_t e = launch_ao(sc, f, w, fs());
        if (end_schedule(g.sched_ao, "AO", e)) return RT_FAILURE;
        HIP_TRY(e);
        if (!replay && frame_verified(p)) g.ao_valid = true;
    }
    HIP_TRY(phase_mark(EV_AO, fs()));
    if (g.pipeline && ao_order()) {  // only the ordered AO phases wait on it
        HIP_TRY(hipEventRecord(SL.ao_done, fs()));
        g.last_ao_slot = g.cur;
    }
    HIP_TRY(launch_resolve(sc, f, w, fb_out, fs()));
    HIP_TRY(hipEventRecord(g.ev[EV_RESOLVE], fs()));
    return RT_SUCCESS;
}

// Node-capacity check. A (params, scene, traced rows) triple that already
// rendered without overflow never overflows again (the frame is deterministic);
// otherwise wait for the frame and read the highest node id it requested. The
// traced rows are part of the key: rt_gpu_count_rows traces the selected rows
// and rt_gpu_render_device the prefix [0, row_end) for the same params.
int check_capacity(const rt_render_params* p, bool& retry) {
    retry = false;
    if (g.verified_valid && g.verified_gen == g.scene_gen && std::memcmp(&g.verified, p, sizeof *p) == 0 &&
        std::memcmp(g.verified_rows, g.traced_rows, sizeof g.traced_rows) == 0)
        return RT_SUCCESS;
    HIP_TRY(hipMemcpyAsync(g.needed_host, SL.needed.p, 4, hipMemcpyDeviceToHost, fs()));
    HIP_TRY(hipStreamSynchronize(fs()));
    const uint32_t need = *g.needed_host;
    if (need > g.node_cap) {
        const uint64_t npix = (uint64_t)g.last_rows * p->width;
        g.node_factor = (double)need / (double)(npix ? npix : 1) * 1.25 + 0.5;
        retry = true;
        return RT_SUCCESS;
    }
    g.verified = *p;
    g.verified_gen = g.scene_gen;
    std::memcpy(g.verified_rows, g.traced_rows, sizeof g.traced_rows);
    g.verified_valid = true;
    // this frame's trace recording (no overflow) is valid for its repeats
    if (g.sched_trace.mode == CountSchedule::RECORD && same_key(g.key_trace, sched_key(p))) g.trace_valid = true;
    return RT_SUCCESS;
}

// Every device buffer of the resident scene (records, shading table, BVH,
// plane tree, direction grid, shuffled scan order).
std::vector<DevBuf State::*> scene_bufs() {
    return {&State::prims, &State::shade, &State::mats, &State::lights, &State::bvh_nodes, &State::bvh_nodes4,
            &State::bvh_prims, &State::bvh_ids, &State::far_nodes, &State::far_tris, &State::brute,
            &State::grid_start, &State::grid_items, &State::grid_always, &State::scan_prims, &State::grid2_start,
            &State::grid2_items, &State::grid_live, &State::grid2_live};
}

// The scene of context `src` into the current context without building
// anything again (the scene is built once and replicated): its
// device buffers by device-to-device copies (xGMI peer copies between GPUs),
// the small host-side description by assignment. Both contexts are idle.
int clone_scene(int src) {
    const State& c = g_ctx[src];
    if (!c.have_scene) return fail("clone_scene: context %d has no scene", src);
    HIP_TRY(hipSetDevice(g.device));
    if (sync_all()) return RT_FAILURE;
    for (DevBuf State::*m : scene_bufs()) {
        const DevBuf& from = c.*m;
        DevBuf& to = g.*m;
        if (!from.p) {
            release(to);
            continue;
        }
        if (ensure(to, from.bytes)) return RT_FAILURE;
        HIP_TRY(hipMemcpyPeerAsync(to.p, g.device, from.p, c.device, from.bytes, g.stream));
    }
    HIP_TRY(hipStreamSynchronize(g.stream));
    g.bvh = c.bvh;  // the host copy keeps only the small arrays (nodes, far nodes, brute list)
    g.bvh_ok = c.bvh_ok;
    g.grid_log2 = c.grid_log2;
    g.grid2 = c.grid2;
    g.grid_n_always = c.grid_n_always;
    g.n_prims = c.n_prims;
    g.n_lights = c.n_lights;
    g.n_ambient = c.n_ambient;
    g.n_nonambient = c.n_nonambient;
    g.shadow_lights = c.shadow_lights;
    g.have_scene = true;
    g.scene_gen = ++g_scene_counter;
    g.verified_valid = false;
    return RT_SUCCESS;
}

}  // namespace

extern "C" {

int rt_gpu_init(int device) {
    RT_WORK("rt_gpu_init");
    if (g.inited) return RT_SUCCESS;
    {   // every RT580_* switch known and valid (rt_knobs.cpp), before anything reads one
        char why[256];
        if (!knobs_check(why, sizeof why)) return fail("%s", why);
    }
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) return fail("no HIP device available (%s)", hipGetErrorString(e));
    if (device < 0) {
        const char* lr = std::getenv("LOCAL_RANK");
        device = lr ? std::atoi(lr) : 0;
    }
    if (device >= n) return fail("device %d out of range (%d devices)", device, n);
    g.device = device;
    HIP_TRY(hipSetDevice(device));
    HIP_TRY(hipStreamCreateWithFlags(&g.own_stream, hipStreamNonBlocking));
    g.stream = g.own_stream;
    for (auto& ev : g.ev_default) HIP_TRY(hipEventCreate(&ev));
    {
        const char* e = std::getenv("RT580_PIPELINE");
        g.pipeline = !(e && std::atoi(e) == 0);
        const char* ns = std::getenv("RT580_SLOTS");  // frames in flight (2-4)
        g.nslots = ns ? std::atoi(ns) : 3;
        g.small_slots = g.nslots;
    }
    if (const char* e = std::getenv("RT580_CHUNK_LOG2")) {
        char* end = nullptr;
        const long v = std::strtol(e, &end, 10);
        if (end == e || *end || v < kChunkLog2Min || v > kChunkLog2Max)
            return fail("RT580_CHUNK_LOG2=%s: not an integer in [%d, %d]", e, kChunkLog2Min, kChunkLog2Max);
        g.chunk_log2 = (int)v;
    }
    for (auto& sl : g.slot) {
        HIP_TRY(hipStreamCreateWithFlags(&sl.stream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&sl.ao_done, hipEventDisableTiming));
    }
    for (auto& ev : g.user_mark) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    HIP_TRY(hipStreamCreateWithFlags(&g.aux, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&g.aux_go, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&g.aux_done, hipEventDisableTiming));
    g.ev = g.ev_default.data();
    HIP_TRY(hipHostMalloc((void**)&g.needed_host, 64, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&g.far_count_host, 64, hipHostMallocDefault));
    HIP_TRY(upload_minstd_table(g.stream));
    {   // FlushFrameBufferToPPM's mapping, with this host's glibc powf (Raytracer.cpp:816-818);
        // called through a volatile pointer so no compiler constant-folds it
        float (*volatile pf)(float, float) = ::powf;
        static uint8_t lut[256];
        for (int c = 0; c < 256; c++) lut[c] = static_cast<unsigned char>(pf(c / 255.0f, 1.0f / 2.2f) * 255.0f);
        HIP_TRY(upload_gamma_lut(lut, g.stream));
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(g.stream));
    g.inited = true;
    return RT_SUCCESS;
}

int rt_gpu_set_stream(void* s) {
    RT_ENTRY("rt_gpu_set_stream");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (sync_all()) return RT_FAILURE;
    g.stream = (hipStream_t)s;  // NULL: the HIP null stream (e.g. PyTorch's default stream)
    return RT_SUCCESS;
}

void* rt_gpu_own_stream(void) { return g.inited ? (void*)g.own_stream : nullptr; }

int rt_gpu_upload_scene(const rt_scene_soa* s) {
    RT_WORK("rt_gpu_upload_scene");
    if (!g.inited && rt_gpu_init(-1) != RT_SUCCESS) return RT_FAILURE;
    if (!s || s->abi_version != RT580_ABI_VERSION) return fail("bad rt_scene_soa / ABI version");
    if (s->n_prims < 0 || s->n_lights < 0 || s->n_materials < 0) return fail("negative scene sizes");
    if (s->n_prims > 0 && (!s->prims || !s->shade)) return fail("null primitive arrays");
    for (int i = 0; i < s->n_prims; i++)
        if (s->prims[i].shape < 0 || s->prims[i].shape >= s->n_materials ||
            (s->prims[i].kind != RT_PRIM_TRIANGLE && s->prims[i].kind != RT_PRIM_SPHERE))
            return fail("primitive %d: bad shape index or kind", i);
    for (int i = 0; i < s->n_lights; i++)
        if (s->lights[i].kind < RT_LIGHT_DIRECTIONAL || s->lights[i].kind > RT_LIGHT_AMBIENT)
            return fail("light %d: bad kind", i);
    HIP_TRY(hipSetDevice(g.device));
    // frames in flight still read the old scene; a fault they raised is
    // reported here, charged to the call that enqueued them
    if (sync_all() || device_sync("before the scene upload")) return RT_FAILURE;
    g.have_scene = false;  // until the new one is complete
    g_last_work = "rt_gpu_upload_scene";
    if (ensure(g.prims, sizeof(rt_prim) * (size_t)s->n_prims + 64) ||
        ensure(g.shade, sizeof(rt_prim_shade) * (size_t)s->n_prims + 64) ||
        ensure(g.mats, sizeof(rt_material) * (size_t)s->n_materials + 64) ||
        ensure(g.lights, sizeof(rt_light) * (size_t)s->n_lights + 64))
        return RT_FAILURE;
    if (h2d(g.prims.p, s->prims, sizeof(rt_prim) * (size_t)s->n_prims, "the primitive records") ||
        h2d(g.shade.p, s->shade, sizeof(rt_prim_shade) * (size_t)s->n_prims, "the shading table") ||
        h2d(g.mats.p, s->materials, sizeof(rt_material) * (size_t)s->n_materials, "the materials") ||
        h2d(g.lights.p, s->lights, sizeof(rt_light) * (size_t)s->n_lights, "the lights"))
        return RT_FAILURE;
    // exact BVH for triangle scenes that do not fit one LDS tile (rt_bvh.h)
    g.bvh = BvhBuild();
    g.bvh_ok = false;
    release(g.scan_prims);
    g.grid_log2 = g.grid_n_always = 0;
    g.grid2 = false;
    if (s->n_prims > 64) {
        g.bvh_ok = build_bvh(s->prims, s->n_prims, g.bvh);
        // far-search direction grid: 2048^2 cells (field100k: 19.4 candidates
        // per far-pass ray against 33.7 at 1024^2; 139M list entries, 5.6 s host
        // build; config 5's 1M triangles: its row sample 1,370 -> 1,227 ms, 12 s
        // build)
        constexpr int glog2 = 11;
        if (g.bvh_ok) build_dir_grid(s->prims, g.bvh, glog2);
        if (g.bvh_ok && grid_coarse_px() > 0) coarsen_dir_grid(g.bvh);
        // the 4-wide form for the near queries (AO, shadows, trace levels)
        if (g.bvh_ok) collapse_bvh4(g.bvh);
        if (g.bvh_ok &&
            (upload_vec(g.bvh_nodes, g.bvh.nodes, "the BVH nodes") ||
             upload_vec(g.bvh_nodes4, g.bvh.nodes4q, "the 4-wide BVH nodes") ||
             upload_vec(g.bvh_prims, g.bvh.prims, "the leaf-ordered primitives") ||
             upload_vec(g.bvh_ids, g.bvh.ids, "the leaf primitive ids") ||
             upload_vec(g.far_nodes, g.bvh.far_nodes, "the plane-tree nodes") ||
             upload_vec(g.far_tris, g.bvh.far_tris, "the plane records") ||
             upload_vec(g.brute, g.bvh.brute, "the brute-force list") ||
             upload_vec(g.grid_start, g.bvh.grid_start, "the direction-grid offsets") ||
             upload_vec(g.grid_live, live_bitmap(g.bvh.grid_start), "the direction-grid cell bitmap") ||
             upload_vec(g.grid2_live, live_bitmap(g.bvh.grid2_start), "the half-resolution cell bitmap") ||
             upload_vec(g.grid_items, g.bvh.grid_items, "the direction-grid lists") ||
             upload_vec(g.grid_always, g.bvh.grid_always, "the direction-grid always-list") ||
             upload_vec(g.grid2_start, g.bvh.grid2_start, "the half-resolution grid offsets") ||
             upload_vec(g.grid2_items, g.bvh.grid2_items, "the half-resolution grid lists")))
            return RT_FAILURE;
        if (g.bvh_ok && !g.bvh.far_nodes.empty()) {
            // The any-hit scan order of far-origin rays (far_scan_kernel): a fixed
            // shuffle of the scene. Such a ray (origin ~1e6 out, from one of the
            // reference's far hits) is accepted by hundreds to thousands of
            // primitives, but often only by one mesh's: in scene order the first
            // acceptor can be ~75k records in (field100k), in shuffled order it
            // is ~N / (acceptors + 1) in. The boolean does not depend on the order.
            std::vector<rt_prim> perm(s->prims, s->prims + s->n_prims);
            std::mt19937 rng(580u);
            std::shuffle(perm.begin(), perm.end(), rng);
            if (upload_vec(g.scan_prims, perm, "the shuffled scan order")) return RT_FAILURE;
        }
        g.grid_log2 = g.bvh.grid_start.empty() ? 0 : g.bvh.grid_log2;
        g.grid2 = g.grid_log2 > 1 && !g.bvh.grid2_start.empty();
        g.grid_n_always = (int)g.bvh.grid_always.size();
        // the device needs only the arrays; keep the host copy small
        g.bvh.prims = std::vector<rt_prim>();
        g.bvh.nodes4 = std::vector<Bvh4Node>();
        g.bvh.ids = std::vector<uint32_t>();
        g.bvh.n_far = (int)g.bvh.far_tris.size();
        g.bvh.far_tris = std::vector<FarTri>();
        g.bvh.grid_start = std::vector<uint32_t>();
        g.bvh.grid_items = std::vector<uint32_t>();
        g.bvh.grid_always = std::vector<uint32_t>();
        g.bvh.grid2_start = std::vector<uint32_t>();
        g.bvh.grid2_items = std::vector<uint32_t>();
    }
    if (device_sync("at the end of the scene upload")) return RT_FAILURE;
    g.n_prims = s->n_prims;
    g.n_lights = s->n_lights;
    g.n_ambient = 0;
    g.n_nonambient = 0;
    g.shadow_lights.clear();
    for (int i = 0; i < s->n_lights; i++) {
        if (s->lights[i].kind == RT_LIGHT_AMBIENT) g.n_ambient++;
        else g.n_nonambient++;
        if (s->lights[i].kind != RT_LIGHT_AMBIENT) g.shadow_lights.push_back(i);
    }
    g.have_scene = true;
    g.scene_gen = ++g_scene_counter;
    return RT_SUCCESS;
}

uint64_t rt_gpu_scene_id(void) { return g.inited && g.have_scene ? g.scene_gen : 0; }

// The frame of rt_gpu_render_device; with fb_host (a registered range of the
// selected rows' bytes) also its D2H copy on the frame's slot stream, before
// the slot's end, so the caller's stream waits for the copy too.
// host: a registered range receiving the selected rows as the int16
// framebuffer (u8 = false) or as the PPM body (u8 = true: FlushFrameBufferToPPM's
// pixel mapping on the device first, rt_gpu_gamma_u8, half the bytes).
static int render_device_frame(const rt_render_params* p, int16_t** fb_device, void* host, bool u8);

int rt_gpu_render_device(const rt_render_params* p, int16_t** fb_device) {
    RT_WORK("rt_gpu_render_device");
    return render_device_frame(p, fb_device, nullptr, false);
}

int rt_gpu_render_async(const rt_render_params* p, int16_t* fb_host) {
    RT_WORK("rt_gpu_render_async");
    if (!fb_host) return fail("rt_gpu_render_async: NULL framebuffer");
    return render_device_frame(p, nullptr, fb_host, false);
}

int rt_gpu_render_async_ppm(const rt_render_params* p, uint8_t* ppm_body_host) {
    RT_WORK("rt_gpu_render_async_ppm");
    if (!ppm_body_host) return fail("rt_gpu_render_async_ppm: NULL buffer");
    return render_device_frame(p, nullptr, ppm_body_host, true);
}

static HostRange* host_range(const void* p, size_t bytes) {
    const char* c = (const char*)p;
    for (HostRange& r : g_host_ranges)
        if (c >= r.p && c + bytes <= r.p + r.bytes) return &r;
    return nullptr;
}

// The registered range of `bytes` at `host` with its copy-ordering event on
// this context's device (created on first use); null when not registered.
static HostRange* host_range_ready(const void* host, size_t bytes) {
    HostRange* hr = host_range(host, bytes);
    if (!hr) return nullptr;
    if (hr->copied && hr->copied_device != g.device) {
        // a copy from the other device may still be in flight: it completes
        // before the range changes hands (frames land in call order)
        if (hipEventSynchronize(hr->copied) != hipSuccess) return nullptr;
        (void)hipEventDestroy(hr->copied);
        hr->copied = nullptr;
    }
    if (!hr->copied) {
        if (hipEventCreateWithFlags(&hr->copied, hipEventDisableTiming) != hipSuccess) return nullptr;
        hr->copied_device = g.device;
        if (hipEventRecord(hr->copied, g.stream) != hipSuccess) return nullptr;
    }
    return hr;
}

// RT580_D2H_MAPPED (default 1): the PPM body is written into the registered
// range by the kernel that produces it (the range mapped into the device's
// address space) instead of a device buffer and a copy (0, A/B)
static bool d2h_mapped() {
    static int v = -1;
    if (v < 0) {
        const char* e = std::getenv("RT580_D2H_MAPPED");
        v = e ? std::atoi(e) : 1;
    }
    return v != 0;
}

// host's address inside the range as the device sees it (null: not mapped)
static void* mapped(const HostRange* hr, const void* host) {
    if (!d2h_mapped() || !hr->dev || ((uintptr_t)host % 16) != 0) return nullptr;
    return (char*)hr->dev + ((const char*)host - hr->p);
}

// src (device) -> host on stream s, after the previous copy into the same range
static int ordered_d2h(HostRange* hr, void* host, const void* src, size_t bytes, hipStream_t s) {
    HIP_TRY(hipStreamWaitEvent(s, hr->copied, 0));
    HIP_TRY(hipMemcpyAsync(host, src, bytes, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipEventRecord(hr->copied, s));
    return RT_SUCCESS;
}

static int render_device_frame(const rt_render_params* p, int16_t** fb_device, void* host, bool u8) {
    if (check_params(p)) return RT_FAILURE;
    HIP_TRY(hipSetDevice(g.device));
    HostRange* hr = nullptr;
    const size_t host_bytes = (size_t)n_selected_rows(p) * p->width * (u8 ? 3 : 6);
    if (host) {
        hr = host_range_ready(host, host_bytes);
        if (!hr)
            return fail("%s: the buffer is not a registered range of %zu bytes (rt_gpu_host_register)", g_call,
                        host_bytes);
    }
    const int n_sel = n_selected_rows(p);
    const bool prefix = p->row_begin == 0 && p->row_step == 1;
    // The RNG offsets need every row before a selected one: render the prefix
    // [0, row_end) and copy the selected rows out when the selection is sparse.
    const int n_rows = prefix ? n_sel : p->row_end;
    // (RT580_SMALL_SLOTS: the slots of whole small-scene frames, A/B; config 2
    // 1.478 ms with two, 1.460 with three)
    if (begin_slot(false, frame_uses_bvh(p) ? g.nslots : g.small_slots)) return RT_FAILURE;
    for (int attempt = 0; attempt < 4; attempt++) {
        if (begin_frame()) return RT_FAILURE;
        HIP_TRY(hipEventRecord(g.ev[EV_START], fs()));
        if (trace_rows(p, 0, 1, n_rows)) return RT_FAILURE;
        int16_t* out;
        if (prefix) {
            if (ensure(SL.fb, (size_t)n_rows * p->width * 6)) return RT_FAILURE;
            out = (int16_t*)SL.fb.p;
        } else {
            if (ensure(SL.fb_full, (size_t)n_rows * p->width * 6)) return RT_FAILURE;
            out = (int16_t*)SL.fb_full.p;
        }
        if (shade_rows(p, 0, 1, n_rows, nullptr, out)) return RT_FAILURE;
        if (!prefix) {
            if (ensure(SL.fb, (size_t)n_sel * p->width * 6)) return RT_FAILURE;
            HIP_TRY(launch_copy_rows(out, p->width, p->row_begin, p->row_step, n_sel, (int16_t*)SL.fb.p, fs()));
        }
        bool retry = false;
        if (check_capacity(p, retry)) return RT_FAILURE;
        if (!retry) {
            if (hr && u8 && mapped(hr, host)) {  // the PPM body straight into the host range
                HIP_TRY(hipStreamWaitEvent(fs(), hr->copied, 0));
                HIP_TRY(launch_gamma_u8_wide((const int16_t*)SL.fb.p, host_bytes, (uint8_t*)mapped(hr, host), fs()));
                HIP_TRY(hipEventRecord(hr->copied, fs()));
            } else if (hr && u8) {  // the PPM body: gamma u8 on the device, then to the host
                if (ensure(SL.fb8, host_bytes)) return RT_FAILURE;
                HIP_TRY(launch_gamma_u8((const int16_t*)SL.fb.p, host_bytes, (uint8_t*)SL.fb8.p, fs()));
                if (ordered_d2h(hr, host, SL.fb8.p, host_bytes, fs())) return RT_FAILURE;
            } else if (hr) {  // the frame to the host, after the previous copy into the same range
                if (ordered_d2h(hr, host, SL.fb.p, host_bytes, fs())) return RT_FAILURE;
            }
            if (end_slot()) return RT_FAILURE;
            if (fb_device) *fb_device = (int16_t*)SL.fb.p;
            return RT_SUCCESS;
        }
        if (g.profiling) g.prof_frames--;
    }
    return fail("node capacity could not be sized");
}


// The framebuffer to the caller's memory: one DMA into a registered range;
// else device -> pinned staging in up to 16 chunks, each chunk's host copy
// overlapping the next chunks' DMA.
static int copy_out(const int16_t* dev, int16_t* fb_out, size_t bytes, hipStream_t stream = nullptr) {
    if (host_registered(fb_out, bytes)) {
        // on the stream that produced the frame when given (no cross-stream hand-off)
        const hipStream_t cs = stream ? stream : g.stream;
        HIP_TRY(hipMemcpyAsync(fb_out, dev, bytes, hipMemcpyDeviceToHost, cs));
        HIP_TRY(hipStreamSynchronize(cs));
        return RT_SUCCESS;
    }
    if (g.stage_bytes < bytes) {
        if (g.stage) (void)hipHostFree(g.stage);
        g.stage = nullptr;
        g.stage_bytes = 0;
        HIP_TRY(hipHostMalloc((void**)&g.stage, bytes, hipHostMallocDefault));
        g.stage_bytes = bytes;
    }
    if (!g.stage_ev[0])
        for (auto& ev : g.stage_ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const size_t nch = g.stage_ev.size();
    size_t chunk = (bytes + nch - 1) / nch;
    if (chunk < ((size_t)1 << 20)) chunk = (size_t)1 << 20;
    const char* src = (const char*)dev;
    char* stg = (char*)g.stage;
    size_t k = 0;
    for (size_t off = 0; off < bytes; off += chunk, k++) {
        const size_t n = bytes - off < chunk ? bytes - off : chunk;
        HIP_TRY(hipMemcpyAsync(stg + off, src + off, n, hipMemcpyDeviceToHost, g.stream));
        HIP_TRY(hipEventRecord(g.stage_ev[k], g.stream));
    }
    k = 0;
    for (size_t off = 0; off < bytes; off += chunk, k++) {
        const size_t n = bytes - off < chunk ? bytes - off : chunk;
        HIP_TRY(hipEventSynchronize(g.stage_ev[k]));
        std::memcpy((char*)fb_out + off, stg + off, n);
    }
    return RT_SUCCESS;
}

// render_split's enqueue on stream s (both halves; the caller ends the slot).
static int enqueue_split(const rt_render_params* p, int16_t* fb_out, hipStream_t s) {
    const int H = p->height, W = p->width;
    const size_t bytes = (size_t)H * W * 6;
    DevFrame f = dev_frame(p, 0, 1, H);
    const DevScene sc = dev_scene(p, H);
    HIP_TRY(hipEventRecord(g.ev[EV_START], s));
    if (trace_rows(p, 0, 1, H)) return RT_FAILURE;
    if (ensure(SL.fb, bytes)) return RT_FAILURE;
    int16_t* out = (int16_t*)SL.fb.p;
    DevWork w = dev_work();
    HIP_TRY(launch_rank(sc, f, w, nullptr, s));
    HIP_TRY(hipEventRecord(g.ev[EV_RANK], s));
    if (prepare_mt_stream(p, nullptr, H)) return RT_FAILURE;
    w = dev_work();
    // The split row: the last part should hold few rows (its resolve and copy
    // are the tail of the call) and enough AO calls that its AO covers the
    // first part's resolve and copy: the largest row r with at least 20 % of
    // the frame's calls in rows [r, H) (config 2's Render(): 10 / 20 / 35 / 50 %
    // 1.911 / 1.894 / 1.916-1.922 / 1.956 ms). Taken from this frame's per-row
    // counts once per (params, scene) -- they do not change between calls.
    if (!(g.lat_gen == g.scene_gen && std::memcmp(&g.lat_params, p, sizeof *p) == 0)) {
        std::vector<uint32_t> rc((size_t)H);
        if (copy_d2h(rc.data(), SL.row_calls.p, (size_t)H * 4, s, "the per-row AO calls")) return RT_FAILURE;
        uint64_t tot = 0, tail = 0;
        for (uint32_t v : rc) tot += v;
        int r = H;
        constexpr uint64_t pct = 20;  // the second part's share of the AO calls
        while (r > 1 && (tail < (tot * pct + 99) / 100 || r > H - 1)) tail += rc[(size_t)--r];
        g.lat_params = *p;
        g.lat_gen = g.scene_gen;
        g.lat_row = r;
    }
    const int h0 = g.lat_row;
    const uint32_t p0 = (uint32_t)h0 * (uint32_t)W, np = (uint32_t)H * (uint32_t)W;
    const uint64_t* split = w.row_base_local + h0;  // calls before row h0
    HIP_TRY(launch_ao_calls(sc, f, w, nullptr, split, s));
    HIP_TRY(hipEventRecord(g.aux_go, s));
    // first half: resolve + copy on the second stream
    HIP_TRY(hipStreamWaitEvent(g.aux, g.aux_go, 0));
    HIP_TRY(launch_resolve_range(sc, f, w, out, 0, p0, g.aux));
    HIP_TRY(hipMemcpyAsync(fb_out, out, (size_t)p0 * 6, hipMemcpyDeviceToHost, g.aux));
    HIP_TRY(hipEventRecord(g.aux_done, g.aux));
    // second half
    HIP_TRY(launch_ao_calls(sc, f, w, split, w.totals, s));
    HIP_TRY(hipEventRecord(g.ev[EV_AO], s));
    HIP_TRY(launch_resolve_range(sc, f, w, out, p0, np, s));
    HIP_TRY(hipEventRecord(g.ev[EV_RESOLVE], s));
    HIP_TRY(hipMemcpyAsync(fb_out + (size_t)p0 * 3, out + (size_t)p0 * 3, (size_t)(np - p0) * 6,
                           hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamWaitEvent(s, g.aux_done, 0));  // the slot is free once both halves are done
    return RT_SUCCESS;
}

// A captured render_split frame. The graph holds the kernels and copies, not
// the host-side bookkeeping of trace_rows and not the frame's timing events
// (events recorded during a capture only order the capture): both are done
// here, the frame's whole time going to its render phase (ms_render).
static int launch_frame_graph(hipGraphExec_t exec, const rt_render_params* p, hipStream_t s) {
    for (int e : {EV_START, EV_TRACE, EV_RANK}) HIP_TRY(hipEventRecord(g.ev[e], s));
    HIP_TRY(hipGraphLaunch(exec, s));
    for (int e : {EV_AO, EV_RESOLVE}) HIP_TRY(hipEventRecord(g.ev[e], s));
    g.traced_rows[0] = 0;
    g.traced_rows[1] = 1;
    g.traced_rows[2] = p->height;
    note_rows(p, p->height, false);
    return RT_SUCCESS;
}

// rt_gpu_render's latency path for small-scene whole frames into a registered
// host framebuffer: after the trace and the AO-call numbering, the frame's
// rows split in two at row r (the calls of rows [0, r) are the first ones of
// the serial RNG stream, so the split needs no other change): AO of the first
// part, then -- on a second stream -- its resolve and copy to the host while
// the second part's AO runs. Same kernels, same bytes. done = false when the
// frame does not qualify (the caller takes the plain path).
static int render_split(const rt_render_params* p, int16_t* fb_out, bool& done) {
    done = false;
    const int H = p->height, W = p->width;
    const size_t bytes = (size_t)H * W * 6;
    if (!g.pipeline || H < 2 || p->row_begin != 0 || p->row_step != 1 || p->row_end != H ||
        !host_registered(fb_out, bytes) || frame_uses_bvh(p))
        return RT_SUCCESS;
    DevFrame f = dev_frame(p, 0, 1, H);
    const DevScene sc = dev_scene(p, H);
    if (!ao_calls_supported(sc, f)) return RT_SUCCESS;
    // only a (params, scene) whose node capacity is verified (no retry here)
    g.traced_rows[0] = 0;
    g.traced_rows[1] = 1;
    g.traced_rows[2] = H;
    if (!(g.verified_valid && g.verified_gen == g.scene_gen && std::memcmp(&g.verified, p, sizeof *p) == 0 &&
          std::memcmp(g.verified_rows, g.traced_rows, sizeof g.traced_rows) == 0))
        return RT_SUCCESS;
    if (begin_slot(false, 2) || begin_frame()) return RT_FAILURE;
    const hipStream_t s = fs();
    // As a graph once the split row is known and the slot has run this exact
    // frame (its buffers exist); not while profiling (per-frame event sets)
    // or for mt19937 (its stream is prepared on the host per call).
    State::FrameGraph& G = g.fgraph[g.cur];
    const bool key = G.gen == g.scene_gen && G.buf_gen == g_buf_gen && G.fb == fb_out &&
                     std::memcmp(&G.p, p, sizeof *p) == 0;
    static int graphs = -1;  // RT580_GRAPH=0: plain enqueue (A/B)
    if (graphs < 0) {
        const char* e = std::getenv("RT580_GRAPH");
        graphs = e ? std::atoi(e) : 1;
    }
    const bool graph_ok = graphs && !g.graphs_off && !g.profiling && p->rng_engine != RT_RNG_MT19937 &&
                          g.lat_gen == g.scene_gen && std::memcmp(&g.lat_params, p, sizeof *p) == 0;
    if (graph_ok && key && G.exec) {
        if (launch_frame_graph(G.exec, p, s)) return RT_FAILURE;
    } else if (graph_ok && key && G.seen) {
        if (G.exec) (void)hipGraphExecDestroy(G.exec);
        G.exec = nullptr;
        HIP_TRY(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
        const int rc = enqueue_split(p, fb_out, s);
        hipGraph_t gr = nullptr;
        const hipError_t ec = hipStreamEndCapture(s, &gr);
        hipError_t ei = hipErrorUnknown;
        if (rc == RT_SUCCESS && ec == hipSuccess && gr) ei = hipGraphInstantiate(&G.exec, gr, nullptr, nullptr, 0);
        if (gr) (void)hipGraphDestroy(gr);
        if (ei != hipSuccess) {  // no graphs on this device/runtime: the plain enqueue from now on
            (void)hipGetLastError();
            G.exec = nullptr;
            g.graphs_off = true;
            if (enqueue_split(p, fb_out, s)) return RT_FAILURE;
        } else {
            if (launch_frame_graph(G.exec, p, s)) return RT_FAILURE;
        }
    } else {
        if (enqueue_split(p, fb_out, s)) return RT_FAILURE;
        G.p = *p;
        G.gen = g.scene_gen;
        G.buf_gen = g_buf_gen;
        G.fb = fb_out;
        G.seen = 1;
        if (G.exec) (void)hipGraphExecDestroy(G.exec);
        G.exec = nullptr;
    }
    if (end_slot()) return RT_FAILURE;
    HIP_TRY(hipStreamSynchronize(s));
    done = true;
    return RT_SUCCESS;
}

int rt_gpu_render(const rt_render_params* p, int16_t* fb_out) {
    RT_WORK("rt_gpu_render");
    if (check_params(p)) return RT_FAILURE;
    HIP_TRY(hipSetDevice(g.device));
    if (fb_out) {
        bool done = false;
        if (render_split(p, fb_out, done)) return RT_FAILURE;
        if (done) {
            HIP_TRY(hipStreamSynchronize(g.stream));
            return RT_SUCCESS;
        }
    }
    int16_t* dev = nullptr;
    if (rt_gpu_render_device(p, &dev)) return RT_FAILURE;
    const size_t bytes = (size_t)n_selected_rows(p) * p->width * 6;
    if (bytes && fb_out && copy_out(dev, fb_out, bytes, fs())) return RT_FAILURE;
    HIP_TRY(hipStreamSynchronize(g.stream));
    return check_replay(SL);  // the frame is complete: its replayed counts are checked now
}

int rt_gpu_host_register(void* host_ptr, uint64_t bytes) {
    RT_ENTRY("rt_gpu_host_register");
    if (!host_ptr || bytes == 0) return fail("rt_gpu_host_register: empty range");
    if (host_registered(host_ptr, bytes)) return RT_SUCCESS;
    if (!g.inited && rt_gpu_init(-1) != RT_SUCCESS) return RT_FAILURE;
    HIP_TRY(hipHostRegister(host_ptr, bytes, hipHostRegisterPortable | hipHostRegisterMapped));
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, host_ptr, 0) != hipSuccess) dev = nullptr;
    (void)hipGetLastError();
    HostRange r;
    r.p = (const char*)host_ptr;
    r.bytes = (size_t)bytes;
    r.dev = dev;
    g_host_ranges.push_back(r);
    return RT_SUCCESS;
}

int rt_gpu_host_unregister(void* host_ptr) {
    RT_ENTRY("rt_gpu_host_unregister");
    for (size_t i = 0; i < g_host_ranges.size(); i++)
        if (g_host_ranges[i].p == (const char*)host_ptr) {
            // the range's last write (possibly on a caller-supplied stream,
            // rt_gpu_deinterleave_ppm), then every context's streams
            if (g_host_ranges[i].copied) (void)hipEventSynchronize(g_host_ranges[i].copied);
            for (int k = 0; k < kMaxCtx; k++)  // no copy into it may still be in flight
                if (g_ctx[k].inited) {
                    const int cur = g_cur;
                    g_cur = k;
                    (void)hipSetDevice(g.device);
                    (void)sync_all();
                    g_cur = cur;
                }
            // frame graphs whose captured copies land in the range go with its registration
            const char* lo = g_host_ranges[i].p;
            const char* hi = lo + g_host_ranges[i].bytes;
            for (int k = 0; k < kMaxCtx; k++)
                for (State::FrameGraph& G : g_ctx[k].fgraph)
                    if (G.fb && (const char*)G.fb >= lo && (const char*)G.fb < hi) {
                        if (G.exec) (void)hipGraphExecDestroy(G.exec);
                        G = State::FrameGraph{};
                    }
            if (g_host_ranges[i].copied) (void)hipEventDestroy(g_host_ranges[i].copied);
            g_host_ranges.erase(g_host_ranges.begin() + (long)i);
            HIP_TRY(hipHostUnregister(host_ptr));
            return RT_SUCCESS;
        }
    return fail("rt_gpu_host_unregister: %p was not registered", host_ptr);
}

int rt_gpu_count_rows(const rt_render_params* p, uint32_t* row_calls_device) {
    RT_WORK("rt_gpu_count_rows");
    if (check_params(p)) return RT_FAILURE;
    if (!row_calls_device) return fail("row_calls_device is NULL");
    HIP_TRY(hipSetDevice(g.device));
    const int n_rows = n_selected_rows(p);
    if (begin_slot(false, g.nslots)) return RT_FAILURE;
    for (int attempt = 0; attempt < 4; attempt++) {
        if (begin_frame()) return RT_FAILURE;
        HIP_TRY(hipEventRecord(g.ev[EV_START], fs()));
        if (trace_rows(p, p->row_begin, p->row_step, n_rows)) return RT_FAILURE;
        bool retry = false;
        if (check_capacity(p, retry)) return RT_FAILURE;
        if (!retry) break;
        if (attempt == 3) return fail("node capacity could not be sized");
        if (g.profiling) g.prof_frames--;
    }
    if (end_slot()) return RT_FAILURE;  // the caller's stream waits for the count pass
    // The counts go into the caller's buffer, which the caller may have just
    // allocated or cleared on its own stream (after the mark begin_slot waited
    // on): the copy is queued on the caller's stream, behind that work and the
    // count pass. The slot's next frame (two calls on) waits for this call's
    // copy through the user mark of the next call's start (begin_slot).
    if (n_rows)
        HIP_TRY(hipMemcpyAsync(row_calls_device, SL.row_calls.p, (size_t)n_rows * 4, hipMemcpyDeviceToDevice,
                               g.stream));
    g.split_params = *p;
    g.split_ready = true;
    return RT_SUCCESS;
}

int rt_gpu_shade_rows(const rt_render_params* p, const uint64_t* row_base_device, int16_t* fb_device) {
    RT_WORK("rt_gpu_shade_rows");
    if (check_params(p)) return RT_FAILURE;
    if (!row_base_device || !fb_device) return fail("row_base_device / fb_device is NULL");
    if (!g.split_ready || std::memcmp(&g.split_params, p, sizeof *p) != 0)
        return fail("rt_gpu_shade_rows must follow rt_gpu_count_rows with the same params");
    HIP_TRY(hipSetDevice(g.device));
    g.split_ready = false;
    if (slot_wait_user()) return RT_FAILURE;  // the row bases were produced on the caller's stream
    if (shade_rows(p, p->row_begin, p->row_step, n_selected_rows(p), row_base_device, fb_device)) return RT_FAILURE;
    return end_slot();
}

int rt_gpu_shade_rows_ppm(const rt_render_params* p, const uint64_t* row_base_device, uint8_t* tile_u8_device,
                          void* done_stream) {
    RT_WORK("rt_gpu_shade_rows_ppm");
    if (check_params(p)) return RT_FAILURE;
    if (!row_base_device || !tile_u8_device) return fail("row_base_device / tile_u8_device is NULL");
    if (!g.split_ready || std::memcmp(&g.split_params, p, sizeof *p) != 0)
        return fail("rt_gpu_shade_rows_ppm must follow rt_gpu_count_rows with the same params");
    HIP_TRY(hipSetDevice(g.device));
    g.split_ready = false;
    if (slot_wait_user()) return RT_FAILURE;  // the row bases were produced on the caller's stream
    const size_t n = (size_t)n_selected_rows(p) * p->width * 3;
    if (ensure(SL.fb, n * 2)) return RT_FAILURE;  // the slot's own int16 rows
    if (shade_rows(p, p->row_begin, p->row_step, n_selected_rows(p), row_base_device, (int16_t*)SL.fb.p))
        return RT_FAILURE;
    HIP_TRY(launch_gamma_u8((const int16_t*)SL.fb.p, n, tile_u8_device, fs()));
    if (!done_stream) return end_slot();
    // end_slot with the wait on done_stream: the caller's stream goes on with
    // the next frame while this one's AO phase runs
    if (post_replay_check()) return RT_FAILURE;
    if (!g.ppm_done) HIP_TRY(hipEventCreateWithFlags(&g.ppm_done, hipEventDisableTiming));
    hipEvent_t ev = g.pipeline ? SL.done : g.ppm_done;
    HIP_TRY(hipEventRecord(ev, fs()));
    HIP_TRY(hipStreamWaitEvent((hipStream_t)done_stream, ev, 0));
    return RT_SUCCESS;
}

int rt_gpu_gamma_u8(const int16_t* fb, uint64_t n, uint8_t* out) {
    RT_WORK("rt_gpu_gamma_u8");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (n && (!fb || !out)) return fail("rt_gpu_gamma_u8: NULL buffer");
    HIP_TRY(hipSetDevice(g.device));
    HIP_TRY(launch_gamma_u8(fb, n, out, g.stream));
    return RT_SUCCESS;
}

int rt_gpu_deinterleave_ppm(const uint8_t* tiles, int world, int n_max, int width, int height,
                            uint8_t* ppm_body_host, void* stream) {
    RT_WORK("rt_gpu_deinterleave_ppm");
    const hipStream_t cs = stream ? (hipStream_t)stream : g.stream;
    if (!g.inited) return fail("rt_gpu_init not called");
    if (!tiles || !ppm_body_host || world < 1 || width < 1 || height < 1 || (int64_t)n_max * world < height)
        return fail("rt_gpu_deinterleave_ppm: bad arguments");
    HIP_TRY(hipSetDevice(g.device));
    const size_t body = (size_t)width * height * 3;
    HostRange* hr = host_range_ready(ppm_body_host, body);
    if (!hr) return fail("rt_gpu_deinterleave_ppm: the buffer is not a registered range of %zu bytes", body);
    HIP_TRY(hipStreamWaitEvent(cs, hr->copied, 0));
    if (uint8_t* dst = (uint8_t*)mapped(hr, ppm_body_host)) {
        HIP_TRY(launch_deinterleave_u8(tiles, world, n_max, width, height, dst, cs));
    } else {
        DevBuf& f8 = g.ppm_stage;
        if (ensure(f8, body)) return RT_FAILURE;
        HIP_TRY(launch_deinterleave_u8(tiles, world, n_max, width, height, (uint8_t*)f8.p, cs));
        HIP_TRY(hipMemcpyAsync(ppm_body_host, f8.p, body, hipMemcpyDeviceToHost, cs));
    }
    HIP_TRY(hipEventRecord(hr->copied, cs));
    return RT_SUCCESS;
}

int rt580_selftest_math(uint64_t seed, uint64_t n, uint64_t* mismatches) {
    RT_WORK("rt580_selftest_math");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (!mismatches) return fail("rt580_selftest_math: NULL output");
    HIP_TRY(hipSetDevice(g.device));
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc(&d, 4 * sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(d, 0, 4 * sizeof(unsigned long long), g.stream);
    if (e == hipSuccess) e = launch_math_selftest(seed, n, d, g.stream);
    const int st = e == hipSuccess ? copy_d2h(mismatches, d, 4 * sizeof(uint64_t), g.stream, "the mismatch counts")
                                   : RT_FAILURE;
    (void)hipFree(d);
    HIP_TRY(e);
    return st;
}

int rt580_eval_powf(const float* x_device, float y, float* out_device, uint64_t n) {
    RT_WORK("rt580_eval_powf");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (n && (!x_device || !out_device)) return fail("rt580_eval_powf: NULL buffer");
    HIP_TRY(hipSetDevice(g.device));
    HIP_TRY(launch_powf_eval(x_device, y, out_device, n, g.stream));
    return RT_SUCCESS;
}

int rt_gpu_row_bases(const int32_t* gathered, int world, int n_max, int height, int rank, uint64_t* row_base) {
    RT_WORK("rt_gpu_row_bases");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (!gathered || !row_base) return fail("rt_gpu_row_bases: NULL buffer");
    if (world <= 0 || rank < 0 || rank >= world || height < 0 || n_max < (height + world - 1) / world)
        return fail("rt_gpu_row_bases: bad world/rank/n_max/height");
    HIP_TRY(hipSetDevice(g.device));
    HIP_TRY(launch_row_bases(gathered, world, n_max, height, rank, row_base, g.stream));
    return RT_SUCCESS;
}

int rt_gpu_set_accel(int mode) {
    RT_ENTRY("rt_gpu_set_accel");
    if (mode != RT_ACCEL_BRUTE && mode != RT_ACCEL_AUTO) return fail("bad accel mode %d", mode);
    g.accel = mode;
    g.verified_valid = false;  // node capacity is re-verified under the new mode
    g.trace_valid = g.ao_valid = false;  // recorded count schedules belong to the old mode
    return RT_SUCCESS;
}

int rt_gpu_accel_active(void) { return g.last_accel ? 1 : 0; }

int rt580_set_ao_order(int on) {
    RT_ENTRY("rt580_set_ao_order");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (on != 0 && on != 1) return fail("rt580_set_ao_order: %d is not 0 or 1", on);
    g_ao_order = on;
    return RT_SUCCESS;
}

int rt580_set_chunk_log2(int log2) {
    RT_ENTRY("rt580_set_chunk_log2");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (log2 < kChunkLog2Min || log2 > kChunkLog2Max)
        return fail("chunk log2 %d outside [%d, %d]", log2, kChunkLog2Min, kChunkLog2Max);
    HIP_TRY(hipSetDevice(g.device));
    if (sync_all()) return RT_FAILURE;
    set_chunk_log2(log2);
    return RT_SUCCESS;
}

int rt_gpu_last_stats(rt_render_stats* st) {
    RT_ENTRY("rt_gpu_last_stats");
    if (!st) return RT_INVALID_ARG;
    std::memset(st, 0, sizeof *st);
    if (!g.last_valid) return fail("no frame rendered yet");
    if (sync_all()) return RT_FAILURE;
    const int n = g.last_rows;
    const Slot& ls = g.slot[g.stats_slot];
    if ((size_t)n * 4 > ls.row_calls.bytes) return fail("rt_gpu_last_stats: the last frame's counters are gone");
    std::vector<uint32_t> rc(n), rh(n), rn(n);
    if (n && (copy_d2h(rc.data(), ls.row_calls.p, (size_t)n * 4, g.stream, "the per-row AO calls") ||
              copy_d2h(rh.data(), ls.row_hits.p, (size_t)n * 4, g.stream, "the per-row hits") ||
              copy_d2h(rn.data(), ls.row_nodes.p, (size_t)n * 4, g.stream, "the per-row tree nodes")))
        return RT_FAILURE;
    uint64_t calls = 0, hits = 0, tree = 0;
    for (int i = 0; i < n; i++) { calls += rc[i]; hits += rh[i]; tree += rn[i]; }
    st->rays_primary = (uint64_t)n * g.last_width;
    st->rays_secondary = tree - st->rays_primary;
    st->rays_shadow = hits * (uint64_t)g.n_nonambient;
    st->ao_calls = calls;
    st->rays_ao = g.last_ao_enabled ? calls * (uint64_t)g.last_ao_samples : 0;
    st->rays_total = tree + st->rays_shadow + st->rays_ao;
    float ms = 0;
    if (hipEventElapsedTime(&ms, g.ev[EV_START], g.ev[EV_TRACE]) == hipSuccess) st->ms_count = ms;
    if (hipEventElapsedTime(&ms, g.ev[EV_TRACE], g.ev[EV_RANK]) == hipSuccess) st->ms_scan = ms;
    if (hipEventElapsedTime(&ms, g.ev[EV_RANK], g.ev[EV_RESOLVE]) == hipSuccess) st->ms_render = ms;
    if (hipEventElapsedTime(&ms, g.ev[EV_START], g.ev[EV_RESOLVE]) == hipSuccess) st->ms_total = ms;
    (void)hipGetLastError();  // an unrecorded event must not leave a sticky error for the next launch
    return RT_SUCCESS;
}

int rt_gpu_profile(int enable) {
    RT_ENTRY("rt_gpu_profile");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (sync_all()) return RT_FAILURE;
    // keep g.ev on the last profiled frame's events so rt_gpu_last_stats stays valid
    if (enable || g.prof_frames == 0) g.ev = g.ev_default.data();
    g.profiling = enable != 0;
    g.prof_frames = 0;
    if (enable) kernel_timer_enable(true);
    else g.kt_keep = true;  // keep the last profiled launches readable
    return RT_SUCCESS;
}

int rt_gpu_profile_ao_kernel(double* ms_total, int* launches, uint64_t* ao_rays) {
    RT_ENTRY("rt_gpu_profile_ao_kernel");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (!ms_total || !launches || !ao_rays) return fail("rt_gpu_profile_ao_kernel: NULL output");
    if (sync_all()) return RT_FAILURE;
    HIP_TRY(kernel_timer_read(ms_total, launches, ao_rays));
    return RT_SUCCESS;
}

int rt_gpu_profile_read(double* ms_trace, double* ms_rank, double* ms_ao, double* ms_resolve, int* frames) {
    RT_ENTRY("rt_gpu_profile_read");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (sync_all()) return RT_FAILURE;
    double t[4] = {0, 0, 0, 0};
    for (int i = 0; i < g.prof_frames; i++) {
        for (int k = 0; k < 4; k++) {
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, g.prof_pool[i][k], g.prof_pool[i][k + 1]));
            t[k] += ms;
        }
    }
    if (ms_trace) *ms_trace = t[0];
    if (ms_rank) *ms_rank = t[1];
    if (ms_ao) *ms_ao = t[2];
    if (ms_resolve) *ms_resolve = t[3];
    if (frames) *frames = g.prof_frames;
    return RT_SUCCESS;
}

const char* rt_gpu_last_error(void) { return g_err; }

int rt_gpu_copy_to_host(void* host_ptr, const void* device_ptr, uint64_t bytes) {
    RT_ENTRY("rt_gpu_copy_to_host");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (bytes && (!host_ptr || !device_ptr)) return fail("NULL buffer");
    HIP_TRY(hipSetDevice(g.device));
    return copy_d2h(host_ptr, device_ptr, (size_t)bytes, g.stream, "a device buffer");
}

int rt_gpu_synchronize(void) {
    RT_ENTRY("rt_gpu_synchronize");
    const int cur = g_cur;
    int st = RT_SUCCESS;
    for (int k = 0; k < kMaxCtx && st == RT_SUCCESS; k++) {
        if (!g_ctx[k].inited) continue;
        g_cur = k;
        if (hipSetDevice(g.device) != hipSuccess) st = fail("hipSetDevice(%d) failed", g.device);
        else if (sync_all() || device_sync("while waiting for every context")) st = RT_FAILURE;
        for (int s = 0; s < State::kSlots && st == RT_SUCCESS; s++)
            if (check_replay(g.slot[s])) st = RT_FAILURE;
    }
    g_cur = cur;
    if (g_ctx[g_cur].inited) (void)hipSetDevice(g_ctx[g_cur].device);
    return st;
}

}  // extern "C"

namespace {
void destroy_comms();
void release_multi();
void release_multi_ctx(int k);
int rank_teardown();

void shutdown_ctx() {
    if (!g.inited) return;
    (void)hipSetDevice(g.device);
    if (sync_all() || device_sync("at shutdown"))
        std::fprintf(stderr, "rt_gpu: shutting down after a device error (%s)\n", g_err);
    for (DevBuf* b : {&g.grid_start, &g.grid_items, &g.grid_always, &g.grid2_start, &g.grid2_items, &g.grid_live,
                      &g.grid2_live})
        release(*b);
    for (DevBuf* b : {&g.bvh_nodes, &g.bvh_nodes4, &g.bvh_prims, &g.bvh_ids, &g.far_nodes, &g.far_tris, &g.brute,
                      &g.prims, &g.shade, &g.mats, &g.lights, &g.scan_prims, &g.ppm_stage})
        release(*b);
    for (Slot& sl : g.slot) {
        for (DevBuf* b : {&sl.nodes, &sl.topo, &sl.node_call0, &sl.node_val, &sl.rays, &sl.lvl, &sl.needed, &sl.pix_hits, &sl.pix_nodes, &sl.pix_prefix,
                          &sl.row_calls, &sl.row_hits, &sl.row_nodes, &sl.row_base_local, &sl.totals, &sl.call_node,
                          &sl.call_rng, &sl.occ, &sl.fb, &sl.fb_full, &sl.fb8, &sl.mt_stream, &sl.mt_windows, &sl.aofix_items, &sl.aofix_count,
                          &sl.call_hint, &sl.ao_rays, &sl.ao_state, &sl.ao_late, &sl.ao_late_count, &sl.far_rays, &sl.far_keys,
                          &sl.far_keys_alt, &sl.far_vals, &sl.far_vals_alt, &sl.far_count, &sl.far_seg_off,
                          &sl.far_seg_n, &sl.far_wofs, &sl.far_work, &sl.sort_tmp, &sl.hit4, &sl.hit_prim, &sl.shadow,
                          &sl.bad})
            release(*b);
        if (sl.bad_host) (void)hipHostFree(sl.bad_host);
        if (sl.stream) (void)hipStreamDestroy(sl.stream);
        if (sl.done) (void)hipEventDestroy(sl.done);
        if (sl.ao_done) (void)hipEventDestroy(sl.ao_done);
    }
    for (auto& ev : g.user_mark)
        if (ev) (void)hipEventDestroy(ev);
    if (g.aux) (void)hipStreamDestroy(g.aux);
    for (auto& fg : g.fgraph)  // the latency path's frame graphs
        if (fg.exec) (void)hipGraphExecDestroy(fg.exec);
    if (g.aux_go) (void)hipEventDestroy(g.aux_go);
    if (g.aux_done) (void)hipEventDestroy(g.aux_done);
    if (g.ppm_done) (void)hipEventDestroy(g.ppm_done);
    for (auto& ev : g.ev_default)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& q : g.prof_pool)
        for (auto& ev : q) (void)hipEventDestroy(ev);
    if (g.needed_host) (void)hipHostFree(g.needed_host);
    if (g.far_count_host) (void)hipHostFree(g.far_count_host);
    if (g.stage) (void)hipHostFree(g.stage);
    if (g.xfer) (void)hipHostFree(g.xfer);
    for (auto& ev : g.xfer_ev)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& ev : g.stage_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (g.own_stream) (void)hipStreamDestroy(g.own_stream);
    g = State();
}
}  // namespace

extern "C" {

void rt_gpu_shutdown(void) {
    RT_ENTRY("rt_gpu_shutdown");
    const int cur = g_cur;
    if (g_ctx[0].inited) (void)hipSetDevice(g_ctx[0].device);
    (void)rank_teardown();
    release_multi();
    for (int k = kMaxCtx - 1; k >= 0; k--) {
        g_cur = k;
        shutdown_ctx();
    }
    g_cur = cur;
    kernel_timer_release();
}

}  // extern "C"

// ---------------------------------------------------------------- multi-GPU Render
namespace {

// RCCL, loaded on the first multi-GPU frame (single-GPU use never needs it;
// under PyTorch the already loaded librccl.so.1 is reused by its SONAME).
struct Rccl {
    bool tried = false;
    void* h = nullptr;
    decltype(&ncclCommInitAll) CommInitAll = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclAllGather) AllGather = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;  // the one-process-per-GPU path (rt_gpu_rank_*)
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
} g_rccl;

bool rccl_load() {
    if (g_rccl.tried) return g_rccl.h != nullptr;
    g_rccl.tried = true;
    for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
        g_rccl.h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
        if (g_rccl.h) break;
    }
    if (!g_rccl.h) return false;
#define RT_RCCL_SYM(f) g_rccl.f = (decltype(g_rccl.f))dlsym(g_rccl.h, "nccl" #f)
    RT_RCCL_SYM(CommInitAll);
    RT_RCCL_SYM(CommDestroy);
    RT_RCCL_SYM(AllGather);
    RT_RCCL_SYM(Send);
    RT_RCCL_SYM(Recv);
    RT_RCCL_SYM(GroupStart);
    RT_RCCL_SYM(GroupEnd);
    RT_RCCL_SYM(GetErrorString);
    RT_RCCL_SYM(GetUniqueId);
    RT_RCCL_SYM(CommInitRank);
#undef RT_RCCL_SYM
    if (!g_rccl.CommInitAll || !g_rccl.CommDestroy || !g_rccl.AllGather || !g_rccl.Send || !g_rccl.Recv ||
        !g_rccl.GroupStart || !g_rccl.GroupEnd || !g_rccl.GetErrorString || !g_rccl.GetUniqueId ||
        !g_rccl.CommInitRank) {
        dlclose(g_rccl.h);
        g_rccl.h = nullptr;
        return false;
    }
    return true;
}

#define RCCL_TRY(expr)                                                                          \
    do {                                                                                        \
        ncclResult_t r_ = (expr);                                                               \
        if (r_ != ncclSuccess) return fail("%s: %s", #expr, g_rccl.GetErrorString(r_));         \
    } while (0)

// One split of the frame over n contexts (devices), with its RCCL communicator.
struct Multi {
    int n = 0;
    int devs[kMaxCtx] = {};
    bool rccl = false;
    ncclComm_t comms[kMaxCtx] = {};
    uint64_t scene_of[kMaxCtx] = {};  // context 0's scene id last uploaded to context k
    DevBuf row_calls[kMaxCtx], gathered[kMaxCtx], base[kMaxCtx], tile[kMaxCtx];  // on device k
    DevBuf root_tiles, frame;                                                     // on device 0
    hipEvent_t ready[kMaxCtx] = {};                                               // local transport
    // rt_gpu_render_multi_async: a ring of per-frame buffer sets. Frame f + kRing
    // reuses frame f's set only after every stream that read it has passed a
    // wait on frame f + 1's exchange (count gather: each context waits on every
    // other's event, or RCCL's own group), so any kRing >= 2 is safe; 3 matches
    // the frames a context keeps in flight
    static constexpr int kRing = 3;
    int ring = 0;
    DevBuf a_rc[kRing][kMaxCtx], a_gat[kRing][kMaxCtx], a_base[kRing][kMaxCtx], a_t16[kRing][kMaxCtx],
        a_t8[kRing][kMaxCtx];                                                    // on device k
    DevBuf a_root8[kRing], a_frame8[kRing];                                      // on device 0
    hipEvent_t a_ready[kRing][kMaxCtx] = {};                                     // local transport
} g_multi;

void destroy_comms() {
    if (g_multi.rccl)
        for (int k = 0; k < g_multi.n; k++)
            if (g_multi.comms[k]) (void)g_rccl.CommDestroy(g_multi.comms[k]);
    for (auto& c : g_multi.comms) c = nullptr;
    g_multi.rccl = false;
    g_multi.n = 0;
}

// Context k's split buffers and event, released on the device they live on
// (before the context moves to another device, or at shutdown). The
// communicator of a device set that included k is destroyed too.
void release_multi_ctx(int k) {
    if (!g_ctx[k].inited) return;
    if (k < g_multi.n) destroy_comms();
    (void)hipSetDevice(g_ctx[k].device);
    (void)hipDeviceSynchronize();
    for (DevBuf* b : {&g_multi.row_calls[k], &g_multi.gathered[k], &g_multi.base[k], &g_multi.tile[k]}) release(*b);
    if (g_multi.ready[k]) (void)hipEventDestroy(g_multi.ready[k]);
    g_multi.ready[k] = nullptr;
    for (int r = 0; r < Multi::kRing; r++) {
        for (DevBuf* b : {&g_multi.a_rc[r][k], &g_multi.a_gat[r][k], &g_multi.a_base[r][k], &g_multi.a_t16[r][k],
                          &g_multi.a_t8[r][k]})
            release(*b);
        if (g_multi.a_ready[r][k]) (void)hipEventDestroy(g_multi.a_ready[r][k]);
        g_multi.a_ready[r][k] = nullptr;
    }
    g_multi.scene_of[k] = 0;
}

void release_multi() {
    destroy_comms();
    for (int k = 0; k < kMaxCtx; k++) release_multi_ctx(k);
    if (g_ctx[0].inited) {
        (void)hipSetDevice(g_ctx[0].device);
        release(g_multi.root_tiles);
        release(g_multi.frame);
        for (int r = 0; r < Multi::kRing; r++) {
            release(g_multi.a_root8[r]);
            release(g_multi.a_frame8[r]);
        }
    }
}

// RT580_MULTI_TRANSPORT: "rccl" (default for distinct devices), "local"
// (device copies; the only choice when a device appears twice, e.g. the
// split rehearsed on one GPU by the tests).
int transport_env() {
    const char* e = std::getenv("RT580_MULTI_TRANSPORT");
    if (!e) return 0;
    if (!std::strcmp(e, "rccl")) return 1;
    if (!std::strcmp(e, "local")) return 2;
    return 0;
}

// The rest of the frame once every context has counted its rows (phase 2 +
// gather + de-interleave + D2H); g_cur is restored by the caller.
int multi_finish(const rt_render_params* p, int n, int n_max, int16_t* fb_out) {
    const int H = p->height, W = p->width;
    const size_t tile_bytes = (size_t)n_max * W * 6;
    // exchange of the per-row AO-call counts (H int32 in all; the one step the
    // serial RNG stream needs, Raytracer.h:592)
    if (g_multi.rccl) {
        RCCL_TRY(g_rccl.GroupStart());
        for (int k = 0; k < n; k++) {
            g_cur = k;
            RCCL_TRY(g_rccl.AllGather(g_multi.row_calls[k].p, g_multi.gathered[k].p, (size_t)n_max, ncclInt32,
                                      g_multi.comms[k], g.stream));
        }
        RCCL_TRY(g_rccl.GroupEnd());
    } else {
        for (int k = 0; k < n; k++) {
            g_cur = k;
            HIP_TRY(hipSetDevice(g.device));
            HIP_TRY(hipEventRecord(g_multi.ready[k], g.stream));
        }
        for (int k = 0; k < n; k++) {
            g_cur = k;
            HIP_TRY(hipSetDevice(g.device));
            for (int j = 0; j < n; j++) {
                HIP_TRY(hipStreamWaitEvent(g.stream, g_multi.ready[j], 0));
                HIP_TRY(hipMemcpyPeerAsync((char*)g_multi.gathered[k].p + (size_t)j * n_max * 4, g.device,
                                           g_multi.row_calls[j].p, g_ctx[j].device, (size_t)n_max * 4, g.stream));
            }
        }
    }
    // phase 2 on every device: its rows' RNG bases, then shading
    for (int k = 0; k < n; k++) {
        g_cur = k;
        HIP_TRY(hipSetDevice(g.device));
        rt_render_params pk = *p;
        pk.row_begin = k;
        pk.row_step = n;
        pk.row_end = H;
        if (rt_gpu_row_bases((const int32_t*)g_multi.gathered[k].p, n, n_max, H, k, (uint64_t*)g_multi.base[k].p) ||
            rt_gpu_shade_rows(&pk, (const uint64_t*)g_multi.base[k].p, (int16_t*)g_multi.tile[k].p))
            return RT_FAILURE;
    }
    // the int16 row tiles to device 0
    g_cur = 0;
    HIP_TRY(hipSetDevice(g.device));
    if (ensure(g_multi.root_tiles, tile_bytes * n) || ensure(g_multi.frame, (size_t)H * W * 6)) return RT_FAILURE;
    HIP_TRY(hipMemcpyAsync(g_multi.root_tiles.p, g_multi.tile[0].p, tile_bytes, hipMemcpyDeviceToDevice, g.stream));
    if (g_multi.rccl) {
        RCCL_TRY(g_rccl.GroupStart());
        for (int k = 1; k < n; k++) {
            RCCL_TRY(g_rccl.Send(g_multi.tile[k].p, tile_bytes, ncclUint8, 0, g_multi.comms[k], g_ctx[k].stream));
            RCCL_TRY(g_rccl.Recv((char*)g_multi.root_tiles.p + (size_t)k * tile_bytes, tile_bytes, ncclUint8, k,
                                 g_multi.comms[0], g_ctx[0].stream));
        }
        RCCL_TRY(g_rccl.GroupEnd());
    } else {
        for (int k = 1; k < n; k++) {
            g_cur = k;
            HIP_TRY(hipSetDevice(g.device));
            HIP_TRY(hipEventRecord(g_multi.ready[k], g.stream));
        }
        g_cur = 0;
        HIP_TRY(hipSetDevice(g.device));
        for (int k = 1; k < n; k++) {
            HIP_TRY(hipStreamWaitEvent(g.stream, g_multi.ready[k], 0));
            HIP_TRY(hipMemcpyPeerAsync((char*)g_multi.root_tiles.p + (size_t)k * tile_bytes, g.device,
                                       g_multi.tile[k].p, g_ctx[k].device, tile_bytes, g.stream));
        }
    }
    HIP_TRY(launch_deinterleave((const int16_t*)g_multi.root_tiles.p, n, n_max, W, H, (int16_t*)g_multi.frame.p,
                                g.stream));
    if (copy_out((const int16_t*)g_multi.frame.p, fb_out, (size_t)H * W * 6)) return RT_FAILURE;
    HIP_TRY(hipStreamSynchronize(g.stream));
    for (int k = 1; k < n; k++) {  // the other devices' streams are idle again before the next frame
        g_cur = k;
        HIP_TRY(hipSetDevice(g.device));
        HIP_TRY(hipStreamSynchronize(g.stream));
    }
    g_cur = 0;
    HIP_TRY(hipSetDevice(g.device));
    return RT_SUCCESS;
}

// Contexts 1..n-1 on their devices with context 0's scene, and the
// communicator of the device set. false: the caller renders on context 0 alone
// (n == 1 without a forced RCCL transport).
int multi_setup(const rt_render_params* p, int n, const int* devices, bool& single) {
    single = false;
    if (check_params(p)) return RT_FAILURE;  // context 0: inited, scene resident
    if (n < 1 || n > kMaxCtx) return fail("rt_gpu_render_multi: %d devices outside [1, %d]", n, kMaxCtx);
    if (p->row_begin != 0 || p->row_step != 1 || p->row_end != p->height)
        return fail("rt_gpu_render_multi renders whole frames (row_begin 0, row_step 1, row_end height)");
    int devs[kMaxCtx];
    int n_dev = 0;
    HIP_TRY(hipGetDeviceCount(&n_dev));
    for (int k = 0; k < n; k++) {
        devs[k] = devices ? devices[k] : (g.device + k) % (n_dev > 0 ? n_dev : 1);
        if (devs[k] < 0 || devs[k] >= n_dev) return fail("rt_gpu_render_multi: device %d out of range", devs[k]);
    }
    if (devs[0] != g.device) return fail("rt_gpu_render_multi: devices[0] must be rt_gpu_init's device");
    const int tr = transport_env();
    bool dup = false;
    for (int a = 0; a < n; a++)
        for (int b = a + 1; b < n; b++) dup = dup || devs[a] == devs[b];
    if (n == 1 && tr != 1) {
        single = true;
        return RT_SUCCESS;
    }
    const bool use_rccl = tr == 1 || (tr == 0 && !dup);
    if (use_rccl && dup) return fail("rt_gpu_render_multi: RCCL needs distinct devices");
    if (use_rccl && !rccl_load()) return fail("rt_gpu_render_multi: librccl.so.1 could not be loaded");
    // contexts 1..n-1: one per device, same scene and acceleration mode as context 0
    const State& c0 = g_ctx[0];
    for (int k = 1; k < n; k++) {
        g_cur = k;
        if (g.inited && g.device != devs[k]) {  // this context moves to another device
            release_multi_ctx(k);
            shutdown_ctx();
        }
        if (!g.inited && rt_gpu_init(devs[k])) return RT_FAILURE;
        g.accel = c0.accel;
        g.pipeline = c0.pipeline;
        if (g.chunk_log2 != c0.chunk_log2) {
            if (sync_all()) return RT_FAILURE;
            set_chunk_log2(c0.chunk_log2);
        }
        if (g_multi.scene_of[k] != c0.scene_gen) {
            if (clone_scene(0)) return RT_FAILURE;
            g_multi.scene_of[k] = c0.scene_gen;
        }
    }
    g_cur = 0;
    // the communicator of this device set
    bool same = g_multi.n == n && g_multi.rccl == use_rccl;
    for (int k = 0; same && k < n; k++) same = g_multi.devs[k] == devs[k];
    if (!same) {
        destroy_comms();
        if (use_rccl) RCCL_TRY(g_rccl.CommInitAll(g_multi.comms, n, devs));
        g_multi.n = n;
        g_multi.rccl = use_rccl;
        for (int k = 0; k < n; k++) g_multi.devs[k] = devs[k];
    }
    return RT_SUCCESS;
}

int multi_render(const rt_render_params* p, int16_t* fb_out, int n, const int* devices) {
    if (!fb_out) return fail("rt_gpu_render_multi: fb_out is NULL");
    bool single = false;
    if (multi_setup(p, n, devices, single)) return RT_FAILURE;
    if (single) return rt_gpu_render(p, fb_out);
    // phase 1 on every device: trace its interleaved rows, count their AO calls
    const int H = p->height, W = p->width;
    const int n_max = (H + n - 1) / n;
    for (int k = 0; k < n; k++) {
        g_cur = k;
        HIP_TRY(hipSetDevice(g.device));
        if (!g_multi.ready[k]) HIP_TRY(hipEventCreateWithFlags(&g_multi.ready[k], hipEventDisableTiming));
        if (ensure(g_multi.row_calls[k], (size_t)n_max * 4) || ensure(g_multi.gathered[k], (size_t)n * n_max * 4) ||
            ensure(g_multi.base[k], (size_t)n_max * 8) || ensure(g_multi.tile[k], (size_t)n_max * W * 6))
            return RT_FAILURE;
        HIP_TRY(hipMemsetAsync(g_multi.row_calls[k].p, 0, (size_t)n_max * 4, g.stream));  // padding rows count 0
        rt_render_params pk = *p;
        pk.row_begin = k;
        pk.row_step = n;
        pk.row_end = H;
        if (rt_gpu_count_rows(&pk, (uint32_t*)g_multi.row_calls[k].p)) return RT_FAILURE;
    }
    return multi_finish(p, n, n_max, fb_out);
}

// One frame of rt_gpu_render_multi_async: the same phases as multi_render on
// the ring's next buffer set, the tiles mapped to PPM bytes on their devices
// before the gather (half the bytes), the de-interleaved body copied into the
// registered host range on context 0's stream -- and no wait anywhere: each
// context keeps its frame slots in flight, the exchange and the copy of frame
// f overlap the kernels of frame f + 1.
int multi_frame_async(const rt_render_params* p, uint8_t* ppm_host, int n, const int* devices) {
    if (!ppm_host) return fail("rt_gpu_render_multi_async: NULL buffer");
    bool single = false;
    if (multi_setup(p, n, devices, single)) return RT_FAILURE;
    if (single) return rt_gpu_render_async_ppm(p, ppm_host);
    const int H = p->height, W = p->width;
    const int n_max = (H + n - 1) / n;
    const size_t t16 = (size_t)n_max * W * 6, t8 = (size_t)n_max * W * 3, body = (size_t)H * W * 3;
    g_cur = 0;
    HostRange* hr = host_range_ready(ppm_host, body);
    if (!hr) return fail("rt_gpu_render_multi_async: the buffer is not a registered range of %zu bytes", body);
    const int r = g_multi.ring;
    g_multi.ring = (r + 1) % Multi::kRing;
    // phase 1
    for (int k = 0; k < n; k++) {
        g_cur = k;
        HIP_TRY(hipSetDevice(g.device));
        if (!g_multi.a_ready[r][k]) HIP_TRY(hipEventCreateWithFlags(&g_multi.a_ready[r][k], hipEventDisableTiming));
        if (ensure(g_multi.a_rc[r][k], (size_t)n_max * 4) || ensure(g_multi.a_gat[r][k], (size_t)n * n_max * 4) ||
            ensure(g_multi.a_base[r][k], (size_t)n_max * 8) || ensure(g_multi.a_t16[r][k], t16) ||
            ensure(g_multi.a_t8[r][k], t8))
            return RT_FAILURE;
        HIP_TRY(hipMemsetAsync(g_multi.a_rc[r][k].p, 0, (size_t)n_max * 4, g.stream));
        rt_render_params pk = *p;
        pk.row_begin = k;
        pk.row_step = n;
        pk.row_end = H;
        if (rt_gpu_count_rows(&pk, (uint32_t*)g_multi.a_rc[r][k].p)) return RT_FAILURE;
    }
    // the per-row AO-call counts, all-gathered
    if (g_multi.rccl) {
        RCCL_TRY(g_rccl.GroupStart());
        for (int k = 0; k < n; k++) {
            g_cur = k;
            RCCL_TRY(g_rccl.AllGather(g_multi.a_rc[r][k].p, g_multi.a_gat[r][k].p, (size_t)n_max, ncclInt32,
                                      g_multi.comms[k], g.stream));
        }
        RCCL_TRY(g_rccl.GroupEnd());
    } else {
        for (int k = 0; k < n; k++) {
            g_cur = k;
            HIP_TRY(hipSetDevice(g.device));
            HIP_TRY(hipEventRecord(g_multi.a_ready[r][k], g.stream));
        }
        for (int k = 0; k < n; k++) {
            g_cur = k;
            HIP_TRY(hipSetDevice(g.device));
            for (int j = 0; j < n; j++) {
                HIP_TRY(hipStreamWaitEvent(g.stream, g_multi.a_ready[r][j], 0));
                HIP_TRY(hipMemcpyPeerAsync((char*)g_multi.a_gat[r][k].p + (size_t)j * n_max * 4, g.device,
                                           g_multi.a_rc[r][j].p, g_ctx[j].device, (size_t)n_max * 4, g.stream));
            }
        }
    }
    // phase 2, then each tile as PPM bytes
    for (int k = 0; k < n; k++) {
        g_cur = k;
        HIP_TRY(hipSetDevice(g.device));
        rt_render_params pk = *p;
        pk.row_begin = k;
        pk.row_step = n;
        pk.row_end = H;
        if (rt_gpu_row_bases((const int32_t*)g_multi.a_gat[r][k].p, n, n_max, H, k,
                             (uint64_t*)g_multi.a_base[r][k].p) ||
            rt_gpu_shade_rows(&pk, (const uint64_t*)g_multi.a_base[r][k].p, (int16_t*)g_multi.a_t16[r][k].p))
            return RT_FAILURE;
        HIP_TRY(launch_gamma_u8((const int16_t*)g_multi.a_t16[r][k].p, t8, (uint8_t*)g_multi.a_t8[r][k].p, g.stream));
    }
    // the tiles to device 0, de-interleaved, to the host
    g_cur = 0;
    HIP_TRY(hipSetDevice(g.device));
    if (ensure(g_multi.a_root8[r], t8 * n) || ensure(g_multi.a_frame8[r], body)) return RT_FAILURE;
    HIP_TRY(hipMemcpyAsync(g_multi.a_root8[r].p, g_multi.a_t8[r][0].p, t8, hipMemcpyDeviceToDevice, g.stream));
    if (g_multi.rccl) {
        RCCL_TRY(g_rccl.GroupStart());
        for (int k = 1; k < n; k++) {
            RCCL_TRY(g_rccl.Send(g_multi.a_t8[r][k].p, t8, ncclUint8, 0, g_multi.comms[k], g_ctx[k].stream));
            RCCL_TRY(g_rccl.Recv((char*)g_multi.a_root8[r].p + (size_t)k * t8, t8, ncclUint8, k, g_multi.comms[0],
                                 g_ctx[0].stream));
        }
        RCCL_TRY(g_rccl.GroupEnd());
    } else {
        for (int k = 1; k < n; k++) {
            g_cur = k;
            HIP_TRY(hipSetDevice(g.device));
            HIP_TRY(hipEventRecord(g_multi.a_ready[r][k], g.stream));
        }
        g_cur = 0;
        HIP_TRY(hipSetDevice(g.device));
        for (int k = 1; k < n; k++) {
            HIP_TRY(hipStreamWaitEvent(g.stream, g_multi.a_ready[r][k], 0));
            HIP_TRY(hipMemcpyPeerAsync((char*)g_multi.a_root8[r].p + (size_t)k * t8, g.device, g_multi.a_t8[r][k].p,
                                       g_ctx[k].device, t8, g.stream));
        }
    }
    if (uint8_t* dst = (uint8_t*)mapped(hr, ppm_host)) {  // de-interleaved straight into the host range
        HIP_TRY(hipStreamWaitEvent(g.stream, hr->copied, 0));
        HIP_TRY(launch_deinterleave_u8((const uint8_t*)g_multi.a_root8[r].p, n, n_max, W, H, dst, g.stream));
        HIP_TRY(hipEventRecord(hr->copied, g.stream));
        return RT_SUCCESS;
    }
    HIP_TRY(launch_deinterleave_u8((const uint8_t*)g_multi.a_root8[r].p, n, n_max, W, H,
                                   (uint8_t*)g_multi.a_frame8[r].p, g.stream));
    return ordered_d2h(hr, ppm_host, g_multi.a_frame8[r].p, body, g.stream);
}

// ---------------------------------------------------------------- one process per GPU
// The rank's side of a world of processes, one GPU each (rt_gpu_rank_*): the
// library owns the world's RCCL communicator and runs the rank's frame loop --
// count, all-gather, shade, gather -- with no host wait and no Python in it.
//
// Ordering. Every collective of the rank runs on one stream (xs), in the order
// the calls enqueue them, and every rank makes the same calls: the
// communicator sees one sequence per rank, the same on all ranks, so no two
// collectives can wait on each other across ranks. A frame's gather is
// enqueued by the NEXT frame call, after that frame's all-gather:
//   xs: allgather(k), bases(k) | wait shaded(k-1), gather(k-1) | allgather(k+1), bases(k+1) | ...
// so frame k+1's shading waits only for frame k-1's (two frames' AO phases run
// together, as frames do on one GPU), never for frame k's. The frame's own
// chain stays off the caller's stream: the slot stream traces and copies the
// counts, xs exchanges them and scans the row bases, the slot stream shades.
// Rank 0 writes each PPM body into host memory on a stream of its own (hs),
// so the ~0.1 ms of the host link per 1080p frame never holds xs.
//
// Shared body (rt_gpu_rank_share_body, what NativeRankFrame sets on one node):
// every rank's buffer is its own mapping of ONE host frame shared by the
// processes; each rank's shading writes its rows' PPM bytes straight to their
// places in it over its own host link (launch_gamma_rows_u8), and the frame's
// "gather" is a 4-byte all-gather on xs after every rank's write: when it
// completes on rank 0, every rank's rows have landed. No tile moves over xGMI
// and rank 0's link carries 1/world of the frame instead of all of it (at
// 8 ranks its whole-frame write, ~0.12 ms per 1080p frame, was the slowest
// rank's extra). With one rank there is no exchange at all: the row bases are
// scanned on the slot stream. Buffers come
// from a ring of three sets, one per frame slot; frame k+3 starts after frame
// k's gather (the caller's stream, which the slot waits on, waits its xs
// event) and receives into root8 after frame k's host write (xs waits hs).
struct RankLoop {
    bool on = false;
    int world = 0, rank = 0, device = -1;
    ncclComm_t comm = nullptr;
    hipStream_t xs = nullptr, hs = nullptr;
    static constexpr int kRing = 3;
    int ring = 0;
    DevBuf rc[kRing], gat[kRing], base[kRing], t8[kRing], root8[kRing], bar[kRing];
    bool shared = false;  // rt_gpu_rank_share_body
    hipEvent_t counted[kRing] = {}, gathered[kRing] = {}, shaded[kRing] = {}, done[kRing] = {}, recvd[kRing] = {},
               written[kRing] = {};
    bool done_valid[kRing] = {}, written_valid[kRing] = {};
    // the frame whose tiles are still to be gathered (enqueued by the next call)
    bool pending = false;
    int pend_r = 0;
    rt_render_params pend_p{};
    uint8_t* pend_host = nullptr;
    // rt580_rank_rehearse: rank `rank` of `world` on one GPU, no communicator --
    // the all-gather copies a precomputed gathered count vector, the gather
    // moves nothing (rank 0 writes its own rows only); for timing one rank's share
    const int32_t* rehearse_gathered = nullptr;
    std::vector<hipEvent_t*> events() {
        std::vector<hipEvent_t*> v;
        for (int r = 0; r < kRing; r++)
            for (hipEvent_t* e : {&counted[r], &gathered[r], &shaded[r], &done[r], &recvd[r], &written[r]}) v.push_back(e);
        return v;
    }
} g_rank;

int rank_teardown() {
    int st = RT_SUCCESS;
    for (hipStream_t s : {g_rank.xs, g_rank.hs})
        if (s && hipStreamSynchronize(s) != hipSuccess) st = RT_FAILURE;
    if (g_rank.comm) (void)g_rccl.CommDestroy(g_rank.comm);
    g_rank.comm = nullptr;
    for (int r = 0; r < RankLoop::kRing; r++) {
        for (DevBuf* b : {&g_rank.rc[r], &g_rank.gat[r], &g_rank.base[r], &g_rank.t8[r], &g_rank.root8[r],
                          &g_rank.bar[r]})
            release(*b);
        g_rank.done_valid[r] = g_rank.written_valid[r] = false;
    }
    for (hipEvent_t* e : g_rank.events()) {
        if (*e) (void)hipEventDestroy(*e);
        *e = nullptr;
    }
    for (hipStream_t* s : {&g_rank.xs, &g_rank.hs}) {
        if (*s) (void)hipStreamDestroy(*s);
        *s = nullptr;
    }
    g_rank.on = false;
    g_rank.pending = false;
    g_rank.shared = false;
    g_rank.rehearse_gathered = nullptr;
    return st;
}

// The streams and events of a rank (rt_gpu_rank_init, rt580_rank_rehearse).
int rank_open(int world, int rank) {
    HIP_TRY(hipStreamCreateWithFlags(&g_rank.xs, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&g_rank.hs, hipStreamNonBlocking));
    for (hipEvent_t* e : g_rank.events()) HIP_TRY(hipEventCreateWithFlags(e, hipEventDisableTiming));
    g_rank.world = world;
    g_rank.rank = rank;
    g_rank.device = g.device;
    g_rank.ring = 0;
    g_rank.on = true;
    return RT_SUCCESS;
}

// The gather of the pending frame's u8 tiles to rank 0 (on xs, after that
// frame's shading) and, on rank 0, its PPM body into the host range (on hs).
int rank_gather_pending() {
    if (!g_rank.pending) return RT_SUCCESS;
    g_rank.pending = false;
    const rt_render_params* p = &g_rank.pend_p;
    const int r = g_rank.pend_r, n = g_rank.world, H = p->height, W = p->width;
    const int n_max = (H + n - 1) / n;
    const size_t t8 = (size_t)n_max * W * 3, body = (size_t)H * W * 3;
    hipStream_t xs = g_rank.xs, hs = g_rank.hs;
    HIP_TRY(hipStreamWaitEvent(xs, g_rank.shaded[r], 0));
    if (g_rank.shared) {
        // every rank's rows are in the shared frame once each rank's shading
        // (and its host write) has ended: a 4-byte all-gather says so to all
        if (n > 1 && g_rank.comm)
            RCCL_TRY(g_rccl.AllGather((int32_t*)g_rank.bar[r].p + g_rank.rank, g_rank.bar[r].p, 1, ncclInt32,
                                      g_rank.comm, xs));
        HIP_TRY(hipEventRecord(g_rank.done[r], xs));
        g_rank.done_valid[r] = true;
        if (g_rank.rank == 0) {
            HIP_TRY(hipEventRecord(g_rank.written[r], xs));
            g_rank.written_valid[r] = true;
        }
        return RT_SUCCESS;
    }
    if (g_rank.rank == 0) {
        if (g_rank.written_valid[r]) HIP_TRY(hipStreamWaitEvent(xs, g_rank.written[r], 0));  // root8[r] read out
        HIP_TRY(hipMemcpyAsync(g_rank.root8[r].p, g_rank.t8[r].p, t8, hipMemcpyDeviceToDevice, xs));
        if (n > 1 && g_rank.comm) {
            RCCL_TRY(g_rccl.GroupStart());
            for (int k = 1; k < n; k++)
                RCCL_TRY(g_rccl.Recv((char*)g_rank.root8[r].p + (size_t)k * t8, t8, ncclUint8, k, g_rank.comm, xs));
            RCCL_TRY(g_rccl.GroupEnd());
        }
        HIP_TRY(hipEventRecord(g_rank.recvd[r], xs));
        HostRange* hr = host_range_ready(g_rank.pend_host, body);
        if (!hr) return fail("rt_gpu_render_rank_async: the buffer is not a registered range of %zu bytes", body);
        HIP_TRY(hipStreamWaitEvent(hs, g_rank.recvd[r], 0));
        HIP_TRY(hipStreamWaitEvent(hs, hr->copied, 0));
        if (uint8_t* dst = (uint8_t*)mapped(hr, g_rank.pend_host)) {  // straight into the host range
            HIP_TRY(launch_deinterleave_u8((const uint8_t*)g_rank.root8[r].p, n, n_max, W, H, dst, hs));
        } else {
            if (ensure(g.ppm_stage, body)) return RT_FAILURE;
            HIP_TRY(launch_deinterleave_u8((const uint8_t*)g_rank.root8[r].p, n, n_max, W, H,
                                           (uint8_t*)g.ppm_stage.p, hs));
            HIP_TRY(hipMemcpyAsync(g_rank.pend_host, g.ppm_stage.p, body, hipMemcpyDeviceToHost, hs));
        }
        HIP_TRY(hipEventRecord(hr->copied, hs));
        HIP_TRY(hipEventRecord(g_rank.written[r], hs));
        g_rank.written_valid[r] = true;
    } else if (g_rank.comm) {
        RCCL_TRY(g_rccl.Send(g_rank.t8[r].p, t8, ncclUint8, 0, g_rank.comm, xs));
    }
    HIP_TRY(hipEventRecord(g_rank.done[r], xs));
    g_rank.done_valid[r] = true;
    return RT_SUCCESS;
}

int rank_frame(const rt_render_params* p, uint8_t* ppm_host) {
    if (!g_rank.on) return fail("rt_gpu_render_rank_async: rt_gpu_rank_init not called");
    if (check_params(p)) return RT_FAILURE;
    if (p->row_begin != 0 || p->row_step != 1 || p->row_end != p->height)
        return fail("rt_gpu_render_rank_async renders whole frames (row_begin 0, row_step 1, row_end height)");
    if (g.device != g_rank.device) return fail("rt_gpu_render_rank_async: the communicator's device changed");
    const int n = g_rank.world, rank = g_rank.rank, H = p->height, W = p->width;
    const int n_max = (H + n - 1) / n;
    const size_t t8 = (size_t)n_max * W * 3, body = (size_t)H * W * 3;
    const bool sh = g_rank.shared;
    if ((rank == 0 || sh) && !host_range(ppm_host, body))
        return fail("rt_gpu_render_rank_async: %s buffer is not a registered range of %zu bytes",
                    sh ? "the shared frame's" : "rank 0's", body);
    HIP_TRY(hipSetDevice(g.device));
    const int r = g_rank.ring;
    g_rank.ring = (r + 1) % RankLoop::kRing;
    // the ring set's last frame has been gathered (every read of the set is
    // before that); the caller's stream waits, and the slot begins after it
    if (g_rank.pending && g_rank.pend_r == r && rank_gather_pending()) return RT_FAILURE;
    if (g_rank.done_valid[r]) HIP_TRY(hipStreamWaitEvent(g.stream, g_rank.done[r], 0));
    if (ensure(g_rank.rc[r], (size_t)n_max * 4) || ensure(g_rank.gat[r], (size_t)n * n_max * 4) ||
        ensure(g_rank.base[r], (size_t)n_max * 8) || ensure(g_rank.t8[r], t8) ||
        (rank == 0 && !sh && ensure(g_rank.root8[r], t8 * n)) || (sh && ensure(g_rank.bar[r], (size_t)n * 4)))
        return RT_FAILURE;
    rt_render_params pk = *p;
    pk.row_begin = rank;
    pk.row_step = n;
    pk.row_end = H;
    const int n_rows = n_selected_rows(&pk);
    // phase 1 on the frame's slot: this rank's rows traced, their AO calls
    // counted (rt_gpu_count_rows' steps, the counts copied on the slot stream)
    if (begin_slot(false, g.nslots)) return RT_FAILURE;
    for (int attempt = 0; attempt < 4; attempt++) {
        if (begin_frame()) return RT_FAILURE;
        HIP_TRY(hipEventRecord(g.ev[EV_START], fs()));
        if (trace_rows(&pk, pk.row_begin, pk.row_step, n_rows)) return RT_FAILURE;
        bool retry = false;
        if (check_capacity(&pk, retry)) return RT_FAILURE;
        if (!retry) break;
        if (attempt == 3) return fail("node capacity could not be sized");
        if (g.profiling) g.prof_frames--;
    }
    HIP_TRY(hipMemsetAsync(g_rank.rc[r].p, 0, (size_t)n_max * 4, fs()));  // padding rows count 0
    if (n_rows)
        HIP_TRY(hipMemcpyAsync(g_rank.rc[r].p, SL.row_calls.p, (size_t)n_rows * 4, hipMemcpyDeviceToDevice, fs()));
    if (n == 1) {  // one rank: its counts are the world's; the bases on the slot
        HIP_TRY(launch_row_bases((const int32_t*)g_rank.rc[r].p, 1, n_max, H, 0, (uint64_t*)g_rank.base[r].p, fs()));
    } else {
        // the exchange and the row bases on xs: every rank's per-row counts (H int32 in all)
        HIP_TRY(hipEventRecord(g_rank.counted[r], fs()));
        HIP_TRY(hipStreamWaitEvent(g_rank.xs, g_rank.counted[r], 0));
        if (g_rank.comm)
            RCCL_TRY(g_rccl.AllGather(g_rank.rc[r].p, g_rank.gat[r].p, (size_t)n_max, ncclInt32, g_rank.comm,
                                      g_rank.xs));
        else  // rehearsal: the world's counts as precomputed, this rank's own rows included
            HIP_TRY(hipMemcpyAsync(g_rank.gat[r].p, g_rank.rehearse_gathered, (size_t)n * n_max * 4,
                                   hipMemcpyDeviceToDevice, g_rank.xs));
        HIP_TRY(launch_row_bases((const int32_t*)g_rank.gat[r].p, n, n_max, H, rank, (uint64_t*)g_rank.base[r].p,
                                 g_rank.xs));
        HIP_TRY(hipEventRecord(g_rank.gathered[r], g_rank.xs));
        HIP_TRY(hipStreamWaitEvent(fs(), g_rank.gathered[r], 0));
    }
    // phase 2 on the slot: shading with those RNG bases, the rows' PPM bytes
    const size_t nv = (size_t)n_rows * W * 3;
    if (ensure(SL.fb, nv * 2)) return RT_FAILURE;  // the slot's own int16 rows
    if (shade_rows(&pk, pk.row_begin, pk.row_step, n_rows, (const uint64_t*)g_rank.base[r].p, (int16_t*)SL.fb.p))
        return RT_FAILURE;
    if (sh) {  // this rank's rows straight to their places in the shared frame
        HostRange* hr = host_range_ready(ppm_host, body);
        if (!hr) return fail("rt_gpu_render_rank_async: the shared frame's buffer is not registered");
        HIP_TRY(hipStreamWaitEvent(fs(), hr->copied, 0));
        uint8_t* dst = (uint8_t*)mapped(hr, ppm_host);
        if (dst) {
            HIP_TRY(launch_gamma_rows_u8((const int16_t*)SL.fb.p, n_rows, W, rank, n, dst, fs()));
        } else {  // (not device-mapped: the rows' bytes on the device, one strided copy)
            HIP_TRY(launch_gamma_u8((const int16_t*)SL.fb.p, nv, (uint8_t*)g_rank.t8[r].p, fs()));
            if (n_rows)
                HIP_TRY(hipMemcpy2DAsync(ppm_host + (size_t)rank * W * 3, (size_t)n * W * 3, g_rank.t8[r].p,
                                         (size_t)W * 3, (size_t)W * 3, (size_t)n_rows, hipMemcpyDeviceToHost, fs()));
        }
        // other ranks read these rows once the frame's 4-byte all-gather is done:
        // the rows must be in host memory before this rank's part of it is sent
        // (a rehearsed rank pays for the read too)
        if (n > 1 && n_rows && hr->dev) {
            const size_t last = ((size_t)rank + (size_t)(n_rows - 1) * n) * W * 3;
            HIP_TRY(launch_host_flush_read((const char*)hr->dev + ((const char*)ppm_host - hr->p) + last,
                                           (uint32_t*)g_rank.bar[r].p + rank, fs()));
        }
        HIP_TRY(hipEventRecord(hr->copied, fs()));
    } else {
        HIP_TRY(launch_gamma_u8((const int16_t*)SL.fb.p, nv, (uint8_t*)g_rank.t8[r].p, fs()));
    }
    // the slot's end without the caller's stream waiting for it: the gather (on
    // xs, next call) waits for `shaded`, the caller's stream goes on
    if (post_replay_check()) return RT_FAILURE;
    if (g.pipeline) HIP_TRY(hipEventRecord(SL.done, fs()));
    HIP_TRY(hipEventRecord(g_rank.shaded[r], fs()));
    // the previous frame's gather, after this frame's all-gather on xs
    if (rank_gather_pending()) return RT_FAILURE;
    g_rank.pending = true;
    g_rank.pend_r = r;
    g_rank.pend_p = *p;
    g_rank.pend_host = ppm_host;
    return RT_SUCCESS;
}

}  // namespace

extern "C" int rt_gpu_render_multi_async(const rt_render_params* p, uint8_t* ppm_body_host, int n_devices,
                                         const int* devices) {
    RT_WORK("rt_gpu_render_multi_async");
    if (g_cur != 0) return fail("re-entered");
    const int st = multi_frame_async(p, ppm_body_host, n_devices, devices);
    g_cur = 0;
    if (g.inited) (void)hipSetDevice(g.device);
    return st;
}

extern "C" int rt_gpu_render_multi(const rt_render_params* p, int16_t* fb_out, int n_devices, const int* devices) {
    RT_WORK("rt_gpu_render_multi");
    if (g_cur != 0) return fail("re-entered");
    const int st = multi_render(p, fb_out, n_devices, devices);
    g_cur = 0;
    if (g.inited) (void)hipSetDevice(g.device);
    return st;
}

extern "C" int rt_gpu_rank_unique_id(void* id_out, uint64_t id_bytes) {
    RT_ENTRY("rt_gpu_rank_unique_id");
    if (!id_out || id_bytes < sizeof(ncclUniqueId)) return fail("rt_gpu_rank_unique_id: need %zu bytes", sizeof(ncclUniqueId));
    if (!rccl_load()) return fail("rt_gpu_rank_unique_id: librccl.so.1 could not be loaded");
    ncclUniqueId id;
    RCCL_TRY(g_rccl.GetUniqueId(&id));
    std::memcpy(id_out, &id, sizeof id);
    return RT_SUCCESS;
}

extern "C" int rt_gpu_rank_init(const void* id, uint64_t id_bytes, int world, int rank) {
    RT_WORK("rt_gpu_rank_init");
    if (g_cur != 0) return fail("re-entered");
    if (!id || id_bytes < sizeof(ncclUniqueId)) return fail("rt_gpu_rank_init: need a %zu-byte id", sizeof(ncclUniqueId));
    if (world < 1 || rank < 0 || rank >= world) return fail("rt_gpu_rank_init: bad world %d / rank %d", world, rank);
    if (!g.inited) return fail("rt_gpu_init not called");
    if (!rccl_load()) return fail("rt_gpu_rank_init: librccl.so.1 could not be loaded");
    if (g_rank.on && rank_teardown()) return fail("rt_gpu_rank_init: the previous communicator's work failed");
    HIP_TRY(hipSetDevice(g.device));
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof uid);
    RCCL_TRY(g_rccl.CommInitRank(&g_rank.comm, world, uid, rank));
    return rank_open(world, rank);
}

extern "C" int rt580_rank_rehearse(int world, int rank, const int32_t* gathered_device) {
    RT_WORK("rt580_rank_rehearse");
    if (g_cur != 0) return fail("re-entered");
    if (world < 1 || rank < 0 || rank >= world || !gathered_device) return fail("rt580_rank_rehearse: bad arguments");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (g_rank.on && rank_teardown()) return fail("rt580_rank_rehearse: the previous communicator's work failed");
    HIP_TRY(hipSetDevice(g.device));
    if (rank_open(world, rank)) return RT_FAILURE;
    g_rank.rehearse_gathered = gathered_device;
    return RT_SUCCESS;
}

extern "C" int rt_gpu_rank_share_body(int on) {
    RT_ENTRY("rt_gpu_rank_share_body");
    if (!g_rank.on) return fail("rt_gpu_rank_share_body: rt_gpu_rank_init not called");
    if (g_rank.pending || g_rank.done_valid[0] || g_rank.done_valid[1] || g_rank.done_valid[2])
        return fail("rt_gpu_rank_share_body: set before the first frame");
    g_rank.shared = on != 0;
    return RT_SUCCESS;
}

extern "C" int rt_gpu_render_rank_async(const rt_render_params* p, uint8_t* ppm_body_host) {
    RT_WORK("rt_gpu_render_rank_async");
    if (g_cur != 0) return fail("re-entered");
    return rank_frame(p, ppm_body_host);
}

extern "C" int rt_gpu_rank_finish(void) {
    RT_WORK("rt_gpu_rank_finish");
    if (!g_rank.on) return fail("rt_gpu_rank_finish: rt_gpu_rank_init not called");
    HIP_TRY(hipSetDevice(g.device));
    if (rank_gather_pending()) return RT_FAILURE;
    // the caller's stream sees the exchange's end and rank 0's last host write
    const int last = (g_rank.ring + RankLoop::kRing - 1) % RankLoop::kRing;
    if (g_rank.done_valid[last]) HIP_TRY(hipStreamWaitEvent(g.stream, g_rank.done[last], 0));
    if (g_rank.written_valid[last]) HIP_TRY(hipStreamWaitEvent(g.stream, g_rank.written[last], 0));
    return RT_SUCCESS;
}

extern "C" int rt_gpu_rank_shutdown(void) {
    RT_ENTRY("rt_gpu_rank_shutdown");
    if (!g_rank.on) return RT_SUCCESS;
    (void)hipSetDevice(g_rank.device);
    if (rank_teardown()) return fail("rt_gpu_rank_shutdown: the exchange stream reported an error");
    return RT_SUCCESS;
}

extern "C" int rt_gpu_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

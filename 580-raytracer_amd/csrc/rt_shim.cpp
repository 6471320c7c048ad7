// rt_shim.cpp — the extern "C" rt_gpu_* boundary (include/rt580.h): device
// buffers resident in HBM, one HIP stream, HIP-event timings, error mapping to
// the reference's status codes (Raytracer.h:8-10). No exception crosses it.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <array>
#include <random>
#include <string>
#include <vector>

#include "../../include/rt580.h"
#include "rt_kernels.h"

using namespace rt580;

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct State {
    bool inited = false;
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev_default[4] = {nullptr, nullptr, nullptr, nullptr};
    hipEvent_t* ev = ev_default;       // events of the frame being enqueued
    // bench profiling: one event quadruple per frame, summed at read time
    bool profiling = false;
    int prof_frames = 0;
    std::vector<std::array<hipEvent_t, 4>> prof_pool;
    // scene
    DevBuf prims, shade, mats, lights;
    int n_prims = 0, n_lights = 0, n_ambient = 0, n_nonambient = 0;
    bool have_scene = false;
    // per-frame workspaces
    DevBuf pix_calls, pix_base, row_calls, row_tree, row_hits, row_base, row_base_all, fb, mt_stream;
    DevBuf cnt_calls_all, cnt_tree_all, cnt_hits_all, cnt_pix_all;
    // last frame bookkeeping for stats
    int last_rows = 0, last_width = 0, last_ao_samples = 0, last_ao_enabled = 0;
    bool last_valid = false;
    rt_render_params split_params;
    bool split_ready = false;
};

State g;
char g_err[512] = "";

int fail(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    std::fprintf(stderr, "rt_gpu: %s\n", g_err);
    return RT_FAILURE;
}

#define HIP_TRY(expr)                                                              \
    do {                                                                           \
        hipError_t e_ = (expr);                                                    \
        if (e_ != hipSuccess) return fail("%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

int ensure(DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return RT_SUCCESS;
    if (b.p) { (void)hipFree(b.p); b.p = nullptr; b.bytes = 0; }
    if (bytes == 0) return RT_SUCCESS;
    size_t want = bytes + bytes / 4;  // headroom for the next frame
    HIP_TRY(hipMalloc(&b.p, want));
    b.bytes = want;
    return RT_SUCCESS;
}

void release(DevBuf& b) {
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
    if (p->depth < 0 || p->depth > RT_MAX_DEPTH) return fail("depth %d outside [0,%d]", p->depth, RT_MAX_DEPTH);
    if (p->ao_samples <= 0) return fail("ao_samples must be > 0");
    if (p->rng_engine != RT_RNG_MINSTD_RAND0 && p->rng_engine != RT_RNG_MT19937) return fail("bad rng engine");
    if (p->row_begin < 0 || p->row_end > p->height || p->row_step <= 0) return fail("bad row selection");
    if (!g.inited) return fail("rt_gpu_init not called");
    if (!g.have_scene) return fail("no scene uploaded");
    return RT_SUCCESS;
}

DevScene dev_scene() {
    DevScene s;
    s.prims = (const rt_prim*)g.prims.p;
    s.shade = (const rt_prim_shade*)g.shade.p;
    s.mats = (const rt_material*)g.mats.p;
    s.lights = (const rt_light*)g.lights.p;
    s.n_prims = g.n_prims;
    s.n_lights = g.n_lights;
    return s;
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
    f.n_ambient = g.n_ambient;
    std::memcpy(f.view_inv, p->view_inv, sizeof f.view_inv);
    std::memcpy(f.cam_from, p->cam_from, sizeof f.cam_from);
    f.ao_angle_max = p->ao_angle_max;
    f.ndc_kx = p->ndc_kx;
    f.ndc_ky = p->ndc_ky;
    f.mt_stream = (const uint32_t*)g.mt_stream.p;
    return f;
}

// Count pass over `n_rows` rows starting at row_begin with row_step, into the
// given per-row / per-pixel buffers.
int run_count(const rt_render_params* p, int row_begin, int row_step, int n_rows, DevBuf& pix, DevBuf& rc,
              DevBuf& rt, DevBuf& rh) {
    size_t npix = (size_t)n_rows * p->width;
    if (ensure(pix, npix * 4) || ensure(rc, (size_t)n_rows * 4 + 4) || ensure(rt, (size_t)n_rows * 4 + 4) ||
        ensure(rh, (size_t)n_rows * 4 + 4))
        return RT_FAILURE;
    HIP_TRY(hipMemsetAsync(rc.p, 0, (size_t)n_rows * 4, g.stream));
    HIP_TRY(hipMemsetAsync(rt.p, 0, (size_t)n_rows * 4, g.stream));
    HIP_TRY(hipMemsetAsync(rh.p, 0, (size_t)n_rows * 4, g.stream));
    DevFrame f = dev_frame(p, row_begin, row_step, n_rows);
    HIP_TRY(launch_count(dev_scene(), f, (uint32_t*)pix.p, (uint32_t*)rc.p, (uint32_t*)rt.p, (uint32_t*)rh.p,
                         g.stream));
    return RT_SUCCESS;
}

// mt19937: the reference's serial stream is generated on the host up to the
// last draw this frame needs (no jump-ahead), then uploaded.
int prepare_mt_stream(const rt_render_params* p, uint64_t total_calls) {
    if (p->rng_engine != RT_RNG_MT19937 || !p->ao_enabled) return RT_SUCCESS;
    uint64_t n = total_calls * 2ull * (uint64_t)p->ao_samples;
    if (ensure(g.mt_stream, n * 4 + 4)) return RT_FAILURE;
    std::vector<uint32_t> host(n);
    std::mt19937 gen(p->rng_seed);
    for (uint64_t i = 0; i < n; i++) host[i] = (uint32_t)gen();
    HIP_TRY(hipMemcpyAsync(g.mt_stream.p, host.data(), n * 4, hipMemcpyHostToDevice, g.stream));
    HIP_TRY(hipStreamSynchronize(g.stream));
    return RT_SUCCESS;
}

int shade(const rt_render_params* p, int n_rows, const uint64_t* row_base_dev, int16_t* fb_out) {
    size_t npix = (size_t)n_rows * p->width;
    if (ensure(g.pix_base, npix * 8 + 8)) return RT_FAILURE;
    HIP_TRY(launch_pixel_base((const uint32_t*)g.pix_calls.p, p->width, n_rows, row_base_dev,
                              (uint64_t*)g.pix_base.p, g.stream));
    HIP_TRY(hipEventRecord(g.ev[2], g.stream));
    DevFrame f = dev_frame(p, p->row_begin, p->row_step, n_rows);
    HIP_TRY(launch_render(dev_scene(), f, (const uint64_t*)g.pix_base.p, fb_out, g.stream));
    HIP_TRY(hipEventRecord(g.ev[3], g.stream));
    g.last_rows = n_rows;
    g.last_width = p->width;
    g.last_ao_samples = p->ao_samples;
    g.last_ao_enabled = p->ao_enabled;
    g.last_valid = true;
    return RT_SUCCESS;
}

// Select the event quadruple for a new frame (profiling: a fresh slot per frame).
int begin_frame() {
    if (!g.profiling) {
        g.ev = g.ev_default;
        return RT_SUCCESS;
    }
    if ((int)g.prof_pool.size() <= g.prof_frames) {
        std::array<hipEvent_t, 4> q;
        for (auto& e : q) HIP_TRY(hipEventCreate(&e));
        g.prof_pool.push_back(q);
    }
    g.ev = g.prof_pool[g.prof_frames].data();
    g.prof_frames++;
    return RT_SUCCESS;
}

}  // namespace

extern "C" {

int rt_gpu_init(int device) {
    if (g.inited) return RT_SUCCESS;
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
    g.ev = g.ev_default;
    upload_minstd_table(g.stream);
    HIP_TRY(hipGetLastError());
    g.inited = true;
    return RT_SUCCESS;
}

int rt_gpu_set_stream(void* s) {
    if (!g.inited) return fail("rt_gpu_init not called");
    g.stream = s ? (hipStream_t)s : g.own_stream;
    upload_minstd_table(g.stream);
    return RT_SUCCESS;
}

int rt_gpu_upload_scene(const rt_scene_soa* s) {
    if (!g.inited && rt_gpu_init(-1) != RT_SUCCESS) return RT_FAILURE;
    if (!s || s->abi_version != RT580_ABI_VERSION) return fail("bad rt_scene_soa / ABI version");
    if (s->n_prims < 0 || s->n_lights < 0 || s->n_materials < 0) return fail("negative scene sizes");
    for (int i = 0; i < s->n_prims; i++)
        if (s->prims[i].shape < 0 || s->prims[i].shape >= s->n_materials ||
            (s->prims[i].kind != RT_PRIM_TRIANGLE && s->prims[i].kind != RT_PRIM_SPHERE))
            return fail("primitive %d: bad shape index or kind", i);
    for (int i = 0; i < s->n_lights; i++)
        if (s->lights[i].kind < RT_LIGHT_DIRECTIONAL || s->lights[i].kind > RT_LIGHT_AMBIENT)
            return fail("light %d: bad kind", i);
    HIP_TRY(hipSetDevice(g.device));
    if (ensure(g.prims, sizeof(rt_prim) * (size_t)s->n_prims + 64) ||
        ensure(g.shade, sizeof(rt_prim_shade) * (size_t)s->n_prims + 64) ||
        ensure(g.mats, sizeof(rt_material) * (size_t)s->n_materials + 64) ||
        ensure(g.lights, sizeof(rt_light) * (size_t)s->n_lights + 64))
        return RT_FAILURE;
    if (s->n_prims) {
        HIP_TRY(hipMemcpyAsync(g.prims.p, s->prims, sizeof(rt_prim) * s->n_prims, hipMemcpyHostToDevice, g.stream));
        HIP_TRY(hipMemcpyAsync(g.shade.p, s->shade, sizeof(rt_prim_shade) * s->n_prims, hipMemcpyHostToDevice, g.stream));
    }
    if (s->n_materials)
        HIP_TRY(hipMemcpyAsync(g.mats.p, s->materials, sizeof(rt_material) * s->n_materials, hipMemcpyHostToDevice, g.stream));
    if (s->n_lights)
        HIP_TRY(hipMemcpyAsync(g.lights.p, s->lights, sizeof(rt_light) * s->n_lights, hipMemcpyHostToDevice, g.stream));
    HIP_TRY(hipStreamSynchronize(g.stream));
    g.n_prims = s->n_prims;
    g.n_lights = s->n_lights;
    g.n_ambient = 0;
    g.n_nonambient = 0;
    for (int i = 0; i < s->n_lights; i++) {
        if (s->lights[i].kind == RT_LIGHT_AMBIENT) g.n_ambient++;
        else g.n_nonambient++;
    }
    g.have_scene = true;
    return RT_SUCCESS;
}

int rt_gpu_count_rows(const rt_render_params* p, uint32_t* row_calls_device) {
    if (check_params(p)) return RT_FAILURE;
    if (!row_calls_device) return fail("row_calls_device is NULL");
    HIP_TRY(hipSetDevice(g.device));
    int n_rows = n_selected_rows(p);
    if (begin_frame()) return RT_FAILURE;
    HIP_TRY(hipEventRecord(g.ev[0], g.stream));
    if (run_count(p, p->row_begin, p->row_step, n_rows, g.pix_calls, g.row_calls, g.row_tree, g.row_hits))
        return RT_FAILURE;
    if (n_rows)
        HIP_TRY(hipMemcpyAsync(row_calls_device, g.row_calls.p, (size_t)n_rows * 4, hipMemcpyDeviceToDevice,
                               g.stream));
    HIP_TRY(hipEventRecord(g.ev[1], g.stream));
    g.split_params = *p;
    g.split_ready = true;
    return RT_SUCCESS;
}

int rt_gpu_shade_rows(const rt_render_params* p, const uint64_t* row_base_device, int16_t* fb_device) {
    if (check_params(p)) return RT_FAILURE;
    if (!row_base_device || !fb_device) return fail("row_base_device / fb_device is NULL");
    if (p->rng_engine == RT_RNG_MT19937 && p->ao_enabled)
        return fail("mt19937 is not supported by the multi-rank split (no jump-ahead)");
    if (!g.split_ready || std::memcmp(&g.split_params, p, sizeof *p) != 0)
        return fail("rt_gpu_shade_rows must follow rt_gpu_count_rows with the same params");
    HIP_TRY(hipSetDevice(g.device));
    g.split_ready = false;
    return shade(p, n_selected_rows(p), row_base_device, fb_device);
}

int rt_gpu_render_device(const rt_render_params* p, int16_t** fb_device) {
    if (check_params(p)) return RT_FAILURE;
    HIP_TRY(hipSetDevice(g.device));
    const int n_rows = n_selected_rows(p);
    const bool prefix = p->row_begin == 0 && p->row_step == 1;
    if (begin_frame()) return RT_FAILURE;
    HIP_TRY(hipEventRecord(g.ev[0], g.stream));
    // RNG offsets: the count pass must cover every row that precedes a selected row.
    if (ensure(g.row_base, (size_t)n_rows * 8 + 8)) return RT_FAILURE;
    uint64_t total_calls = 0;
    if (prefix) {
        if (run_count(p, 0, 1, n_rows, g.pix_calls, g.row_calls, g.row_tree, g.row_hits)) return RT_FAILURE;
        HIP_TRY(launch_row_base((const uint32_t*)g.row_calls.p, n_rows, (uint64_t*)g.row_base.p, g.stream));
        if (p->rng_engine == RT_RNG_MT19937 && p->ao_enabled) {
            std::vector<uint32_t> rc(n_rows);
            HIP_TRY(hipMemcpyAsync(rc.data(), g.row_calls.p, (size_t)n_rows * 4, hipMemcpyDeviceToHost, g.stream));
            HIP_TRY(hipStreamSynchronize(g.stream));
            for (uint32_t c : rc) total_calls += c;
        }
    } else {
        const int all_rows = p->row_end;
        if (run_count(p, 0, 1, all_rows, g.cnt_pix_all, g.cnt_calls_all, g.cnt_tree_all, g.cnt_hits_all))
            return RT_FAILURE;
        if (ensure(g.row_base_all, (size_t)all_rows * 8 + 8)) return RT_FAILURE;
        HIP_TRY(launch_row_base((const uint32_t*)g.cnt_calls_all.p, all_rows, (uint64_t*)g.row_base_all.p, g.stream));
        HIP_TRY(launch_select_rows((const uint64_t*)g.row_base_all.p, p->row_begin, p->row_step, n_rows,
                                   (uint64_t*)g.row_base.p, g.stream));
        if (p->rng_engine == RT_RNG_MT19937 && p->ao_enabled) {
            std::vector<uint32_t> rc(all_rows);
            HIP_TRY(hipMemcpyAsync(rc.data(), g.cnt_calls_all.p, (size_t)all_rows * 4, hipMemcpyDeviceToHost, g.stream));
            HIP_TRY(hipStreamSynchronize(g.stream));
            for (uint32_t c : rc) total_calls += c;
        }
        if (run_count(p, p->row_begin, p->row_step, n_rows, g.pix_calls, g.row_calls, g.row_tree, g.row_hits))
            return RT_FAILURE;
    }
    HIP_TRY(hipEventRecord(g.ev[1], g.stream));
    if (prepare_mt_stream(p, total_calls)) return RT_FAILURE;
    if (ensure(g.fb, (size_t)n_rows * p->width * 6 + 6)) return RT_FAILURE;
    if (shade(p, n_rows, (const uint64_t*)g.row_base.p, (int16_t*)g.fb.p)) return RT_FAILURE;
    if (fb_device) *fb_device = (int16_t*)g.fb.p;
    return RT_SUCCESS;
}

int rt_gpu_render(const rt_render_params* p, int16_t* fb_out) {
    int16_t* dev = nullptr;
    if (rt_gpu_render_device(p, &dev)) return RT_FAILURE;
    size_t bytes = (size_t)n_selected_rows(p) * p->width * 6;
    if (bytes) HIP_TRY(hipMemcpyAsync(fb_out, dev, bytes, hipMemcpyDeviceToHost, g.stream));
    HIP_TRY(hipStreamSynchronize(g.stream));
    return RT_SUCCESS;
}

int rt_gpu_last_stats(rt_render_stats* st) {
    if (!st) return RT_INVALID_ARG;
    std::memset(st, 0, sizeof *st);
    if (!g.last_valid) return fail("no frame rendered yet");
    HIP_TRY(hipStreamSynchronize(g.stream));
    int n = g.last_rows;
    std::vector<uint32_t> rc(n), rt(n), rh(n);
    if (n) {
        HIP_TRY(hipMemcpy(rc.data(), g.row_calls.p, (size_t)n * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(rt.data(), g.row_tree.p, (size_t)n * 4, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(rh.data(), g.row_hits.p, (size_t)n * 4, hipMemcpyDeviceToHost));
    }
    uint64_t calls = 0, tree = 0, hits = 0;
    for (int i = 0; i < n; i++) { calls += rc[i]; tree += rt[i]; hits += rh[i]; }
    st->rays_primary = (uint64_t)n * g.last_width;
    st->rays_secondary = tree - st->rays_primary;
    st->rays_shadow = hits * (uint64_t)g.n_nonambient;
    st->ao_calls = calls;
    st->rays_ao = g.last_ao_enabled ? calls * (uint64_t)g.last_ao_samples : 0;
    st->rays_total = tree + st->rays_shadow + st->rays_ao;
    float ms = 0;
    if (hipEventElapsedTime(&ms, g.ev[0], g.ev[1]) == hipSuccess) st->ms_count = ms;
    if (hipEventElapsedTime(&ms, g.ev[1], g.ev[2]) == hipSuccess) st->ms_scan = ms;
    if (hipEventElapsedTime(&ms, g.ev[2], g.ev[3]) == hipSuccess) st->ms_render = ms;
    if (hipEventElapsedTime(&ms, g.ev[0], g.ev[3]) == hipSuccess) st->ms_total = ms;
    return RT_SUCCESS;
}

int rt_gpu_profile(int enable) {
    if (!g.inited) return fail("rt_gpu_init not called");
    g.profiling = enable != 0;
    g.prof_frames = 0;
    g.ev = g.ev_default;
    return RT_SUCCESS;
}

int rt_gpu_profile_read(double* ms_count, double* ms_scan, double* ms_render, int* frames) {
    if (!g.inited) return fail("rt_gpu_init not called");
    HIP_TRY(hipStreamSynchronize(g.stream));
    double c = 0, s = 0, r = 0;
    for (int i = 0; i < g.prof_frames; i++) {
        float a = 0, b = 0, d = 0;
        HIP_TRY(hipEventElapsedTime(&a, g.prof_pool[i][0], g.prof_pool[i][1]));
        HIP_TRY(hipEventElapsedTime(&b, g.prof_pool[i][1], g.prof_pool[i][2]));
        HIP_TRY(hipEventElapsedTime(&d, g.prof_pool[i][2], g.prof_pool[i][3]));
        c += a; s += b; r += d;
    }
    if (ms_count) *ms_count = c;
    if (ms_scan) *ms_scan = s;
    if (ms_render) *ms_render = r;
    if (frames) *frames = g.prof_frames;
    return RT_SUCCESS;
}

const char* rt_gpu_last_error(void) { return g_err; }

void rt_gpu_shutdown(void) {
    if (!g.inited) return;
    (void)hipSetDevice(g.device);
    (void)hipStreamSynchronize(g.stream);
    for (DevBuf* b : {&g.prims, &g.shade, &g.mats, &g.lights, &g.pix_calls, &g.pix_base, &g.row_calls,
                      &g.row_tree, &g.row_hits, &g.row_base, &g.row_base_all, &g.fb, &g.mt_stream,
                      &g.cnt_calls_all, &g.cnt_tree_all, &g.cnt_hits_all, &g.cnt_pix_all})
        release(*b);
    for (auto& ev : g.ev_default)
        if (ev) (void)hipEventDestroy(ev);
    for (auto& q : g.prof_pool)
        for (auto& ev : q) (void)hipEventDestroy(ev);
    if (g.own_stream) (void)hipStreamDestroy(g.own_stream);
    g = State();
}

}  // extern "C"

/* rt580.h — C-ABI boundary between the reference's host class surface and the
 * MI355X ray-trace kernels (POD types only; no C++ or torch types cross it).
 *
 * The reference (Xena99/580-Raytracer, "580 Raytracer/") renders inside
 *   int Raytracer::Render(const std::string outputName)      Raytracer.cpp:916-935
 * whose per-pixel loop (GenerateRay :832-858 -> Raycast :28-129 -> IntersectScene
 * :473-526 / CalculateLocalColor :213-267 / CalculateAmbientOcclusion :315-330 /
 * ComputeFresnel :131-166 / CalculateRefraction :168-203) is replaced by
 * rt_gpu_render(). The scene that LoadSceneJSON (:645-779) + LoadMesh (:589-643)
 * build is flattened on the host (reference arithmetic, Raytracer.cpp:528-586,
 * :348-409, :895-915) and handed over once by rt_gpu_upload_scene().
 *
 * Status convention is the reference's (Raytracer.h:8-10):
 *   RT_SUCCESS 0, RT_FAILURE 1, RT_INVALID_ARG 2.
 * No function throws or aborts; HIP/RCCL errors map to RT_FAILURE and a message
 * on stderr (also retrievable with rt_gpu_last_error()).
 */
#ifndef RT580_H
#define RT580_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT580_ABI_VERSION 1

#ifndef RT_SUCCESS
#define RT_SUCCESS 0
#define RT_FAILURE 1
#define RT_INVALID_ARG 2
#endif

/* Primitive kinds, in the reference's Mesh::Type order (Raytracer.h:477-480). */
#define RT_PRIM_TRIANGLE 0
#define RT_PRIM_SPHERE 1

/* Light kinds (Raytracer.h:520-524). */
#define RT_LIGHT_DIRECTIONAL 0
#define RT_LIGHT_POINT 1
#define RT_LIGHT_AMBIENT 2

/* RNG engines for the AO sampler (member mGenerator, Raytracer.h:592). */
#define RT_RNG_MINSTD_RAND0 0 /* libstdc++ std::default_random_engine, seed 1 */
#define RT_RNG_MT19937 1      /* MSVC std::default_random_engine, seed 5489  */

/* One primitive in the reference's intersection order (shapes in JSON order,
 * triangles in mesh-file order, Raytracer.cpp:476-521), world space, with the
 * ray-invariant part of IntersectTriangle/IntersectSphere precomputed.
 * 64 bytes; read wave-uniformly by the kernels.
 *   triangle: p0 = v0, p1 = v1, p2 = v2 (TransformPoint, Raytracer.cpp:353-355),
 *             nrm = normalize(cross(v1-v0, v2-v0))            (:362-365),
 *             d = -dot(nrm, v0)                               (:377),
 *             area = CalcTriangleAreaSigned(v0,v1,v2,nrm)     (:389, :937-942)
 *   sphere:   p0 = model-matrix translation (GetTranslation, Raytracer.h:212),
 *             d = radius*radius                               (:423)          */
typedef struct rt_prim {
    float p0[3];
    float d;
    float p1[3];
    float area;
    float p2[3];
    int32_t kind; /* RT_PRIM_* */
    float nrm[3];
    int32_t shape; /* index into the material table (owning shape) */
} rt_prim;

/* Shading side table, read only for the winning hit (one per primitive). */
typedef struct rt_prim_shade {
    float hit_nrm[3]; /* triangle: normalize(nrm) (Raytracer.cpp:402-403); sphere: unused */
    float vn0[3];     /* object-space vertex normals (Raytracer.cpp:227), triangles only */
    float vn1[3];
    float vn2[3];
    float pad[4];
} rt_prim_shade;

/* Material of a shape (Raytracer.h:442-463). refractiveIndex is never read from
 * JSON by the reference and stays 2.5 (Raytracer.h:460). */
typedef struct rt_material {
    float cs[3];
    float ka, kd, ks, kt;
    float spec_exp; /* "n" */
    float ior;      /* 2.5 */
    float pad[3];
} rt_material;

/* A light in JSON order (Raytracer.cpp:744-771). For directional lights the
 * host also stores L = normalize(-direction) (Raytracer.cpp:59,65,220-221) and
 * L2 = normalize(L) (the shadow Ray constructor, Raytracer.h:431-433). */
typedef struct rt_light {
    int32_t kind; /* RT_LIGHT_* */
    float color[3];
    float intensity;
    float position[3];
    float dir[3];    /* normalized to - from */
    float L[3];      /* directional: normalize(-dir) */
    float L2[3];     /* directional: normalize(L)    */
    float pad[1];
} rt_light;

typedef struct rt_scene_soa {
    int32_t abi_version; /* RT580_ABI_VERSION */
    int32_t n_prims;
    const rt_prim* prims;
    const rt_prim_shade* shade;
    int32_t n_materials;
    const rt_material* materials;
    int32_t n_lights;
    const rt_light* lights;
} rt_scene_soa;

/* Per-Render() constants, computed on the host with the reference arithmetic. */
typedef struct rt_render_params {
    int32_t abi_version;
    int32_t width, height;   /* mDisplay->xRes/yRes (Raytracer.cpp:781-786) */
    int32_t depth;           /* Raycast bounces, default 4 (Raytracer.h:563) */
    int32_t ao_samples;      /* numSamples, default 128 (Raytracer.cpp:317) */
    int32_t ao_enabled;      /* 0 => CalculateAmbientOcclusion returns 1.0f */
    int32_t rng_engine;      /* RT_RNG_* */
    uint32_t rng_seed;       /* engine seed: 1 (minstd_rand0) / 5489 (mt19937) */
    int32_t view_inverse_ok; /* Matrix::Inverse(viewMatrix) succeeded (:850) */
    float view_inv[9];       /* rows 0..2, cols 0..2 of inverse(viewMatrix) */
    float cam_from[3];       /* camera.from: ray origin and specular eye */
    double ndc_kx;           /* (double)aspect * tan(ToRadian(fov/2)) (:836-839) */
    double ndc_ky;           /* tan(ToRadian(fov/2))                  (:840)      */
    float ao_angle_max;      /* (float)(2*PI): uniform_real_distribution b (:270) */
    int32_t row_begin;       /* rows row_begin, row_begin+row_step, ... < row_end */
    int32_t row_end;         /* are rendered by this call (full frame: 0, height, 1); */
    int32_t row_step;        /* rank r of G renders row_begin=r, row_step=G        */
} rt_render_params;

typedef struct rt_render_stats {
    uint64_t rays_total;       /* IntersectScene calls of the frame */
    uint64_t rays_primary;     /* camera rays */
    uint64_t rays_secondary;   /* reflection + refraction */
    uint64_t rays_shadow;      /* directional + point shadow rays */
    uint64_t rays_ao;          /* AO rays */
    uint64_t ao_calls;         /* CalculateAmbientOcclusion calls */
    double ms_count;           /* breadth-first trace + per-row AO-call counts (HIP events) */
    double ms_scan;            /* AO-call numbering (RNG positions) */
    double ms_render;          /* AO kernel + resolve kernel */
    double ms_total;           /* first launch -> framebuffer in HBM */
} rt_render_stats;

/* Select the device (device < 0: $LOCAL_RANK or 0) and create streams/events. */
int rt_gpu_init(int device);
/* Upload (replace) the flattened scene; buffers stay resident in HBM. */
int rt_gpu_upload_scene(const rt_scene_soa* scene);
/* Identity of the resident scene: a process-wide counter value assigned by
 * each successful upload (never reused, also across rt_gpu_shutdown); 0 when
 * no scene is resident. The class surface re-uploads when it changed. */
uint64_t rt_gpu_scene_id(void);
/* Queue all further work on this HIP stream (hipStream_t); NULL is the HIP null
 * stream (PyTorch's default stream). Initially: the shim's own non-blocking
 * stream, whose handle rt_gpu_own_stream() returns. */
int rt_gpu_set_stream(void* hip_stream);
void* rt_gpu_own_stream(void);
/* Render the rows selected by params into fb_out (host, Pixel layout: int16
 * r,g,b interleaved; the selected rows packed in order, each `width` pixels).
 * Single-rank: the RNG offsets are scanned on the device. Blocking. */
int rt_gpu_render(const rt_render_params* params, int16_t* fb_out);
/* Same, leaving the framebuffer in HBM (device pointer valid until the next
 * call); asynchronous on the shim's stream. A frame that replayed recorded
 * counts (repeats of a frame, see rt_shim.cpp) is checked on the device; a
 * mismatch is reported by the call that next uses the frame's slot (up to
 * RT580_SLOTS calls later) or by rt_gpu_synchronize. */
int rt_gpu_render_device(const rt_render_params* params, int16_t** fb_device);
/* Throughput form of rt_gpu_render: the frame and its copy into fb_host are
 * queued and the call returns (frames in flight on the shim's slots; each
 * frame's D2H overlaps the next frames' kernels). fb_host must lie in a range
 * registered with rt_gpu_host_register; copies into one range land in call
 * order. The frame is in fb_host once the shim's stream (rt_gpu_set_stream)
 * reaches the point of this call: rt_gpu_synchronize, or a sync of that
 * stream. Replayed-count checks are reported as for rt_gpu_render_device. */
int rt_gpu_render_async(const rt_render_params* params, int16_t* fb_host);
/* The same with the frame delivered as the PPM body (height x width x 3 bytes,
 * FlushFrameBufferToPPM's pixel mapping applied on the device, Raytracer.cpp:
 * 812-818, rt_gpu_gamma_u8): half the bytes over PCIe. */
int rt_gpu_render_async_ppm(const rt_render_params* params, uint8_t* ppm_body_host);
/* Page-lock a host buffer that will receive frames (rt_gpu_render's fb_out):
 * a frame copied into a registered range lands there with one DMA instead of
 * through the shim's pinned staging buffer. The caller keeps the buffer alive
 * until rt_gpu_host_unregister (the class surface registers its framebuffer on
 * its first Render and unregisters it in its destructor). */
int rt_gpu_host_register(void* host_ptr, uint64_t bytes);
int rt_gpu_host_unregister(void* host_ptr);
/* Multi-rank split of rt_gpu_render_device. Buffers are
 * caller-owned device memory (e.g. torch tensors on this device); the work is
 * queued on the shim's stream (see rt_gpu_set_stream).
 *  phase 1: AO calls of each selected row -> row_calls_device (uint32[n_rows]);
 *  caller:  all-gather the per-row counts of every rank, exclusive-scan them in
 *           raster order, keep its own rows' bases (uint64[n_rows]);
 *  phase 2: shade the selected rows with those RNG bases -> fb_device
 *           (int16[n_rows*width*3]). Phase 2 reuses phase 1's per-pixel counts:
 *           call it with the same params, before any other count/render. */
int rt_gpu_count_rows(const rt_render_params* params, uint32_t* row_calls_device);
int rt_gpu_shade_rows(const rt_render_params* params, const uint64_t* row_base_device,
                      int16_t* fb_device);
/* Between the two phases: from the all-gathered per-row counts
 * (gathered_device: int32[world][n_max], rank k's local row j = frame row
 * k + j*world), the exclusive raster-order scan's values at this rank's rows
 * -> row_base_device (uint64[n_max], zero padded). One kernel on the shim's stream. */
int rt_gpu_row_bases(const int32_t* gathered_device, int world, int n_max, int height, int rank,
                     uint64_t* row_base_device);
/* Multi-GPU rt_gpu_render inside the library: one process drives
 * n_devices GPUs (devices: their ids, devices[0] = rt_gpu_init's device; NULL =
 * consecutive ids from it). Device k renders rows k, k+G, ... (interleaved rows
 * balance sky and geometry); the per-row AO-call counts are all-gathered
 * (ncclAllGather), each device scans them into its rows' RNG bases and shades
 * them, the int16 row tiles go to device 0 (ncclSend/ncclRecv) and are
 * de-interleaved there, then copied into fb_out (Pixel[w*h], whole frames only).
 * The scene of context 0 is uploaded to every device on first use. RCCL
 * (librccl.so.1) is loaded on the first call with distinct devices; a device
 * listed twice selects device-to-device copies instead (the split rehearsed on
 * one GPU; RT580_MULTI_TRANSPORT=rccl|local forces either). n_devices == 1 is
 * rt_gpu_render. Blocking. The image is byte-identical for every G. */
int rt_gpu_render_multi(const rt_render_params* params, int16_t* fb_out, int n_devices, const int* devices);
/* Throughput form of rt_gpu_render_multi (rt_gpu_render_async_ppm across
 * devices): the frame's phases are queued on every device and the call
 * returns; the tiles are mapped to PPM bytes before the gather, and the
 * de-interleaved PPM body is copied into ppm_body_host (a registered range of
 * height x width x 3 bytes) on context 0's stream, in call order. Each device
 * keeps its frame slots in flight: the gather and the copy of one frame overlap
 * the next frame's kernels. Complete after rt_gpu_synchronize. */
int rt_gpu_render_multi_async(const rt_render_params* params, uint8_t* ppm_body_host, int n_devices,
                              const int* devices);
/* The PPM body of a frame from the u8 row tiles of its `world` interleaved
 * shares (tile r = rows r, r + world, ... of n_max rows each, contiguous on
 * this device: what rank 0 gathers in the one-process-per-GPU path), written
 * into ppm_body_host (a registered range of height x width x 3 bytes) on the
 * library's stream, after any earlier write into the same range. The
 * per-process driver's last step (rt580_dist.DistFrame). */
int rt_gpu_deinterleave_ppm(const uint8_t* tiles, int world, int n_max, int width, int height,
                            uint8_t* ppm_body_host, void* stream /* hipStream_t; NULL: the library's stream */);
/* rt_gpu_shade_rows with the rows' PPM bytes (FlushFrameBufferToPPM's gamma
 * mapping) written to tile_u8_device, and the wait for the frame placed on
 * done_stream (a hipStream_t) instead of the caller's stream: the caller's
 * stream goes on with the next frame's count and exchange while this frame's
 * AO phase runs, and the consumers of the tile (the gather, on done_stream)
 * wait for it. NULL done_stream: the caller's stream waits, as rt_gpu_shade_rows. */
int rt_gpu_shade_rows_ppm(const rt_render_params* params, const uint64_t* row_base_device, uint8_t* tile_u8_device,
                          void* done_stream);
/* One process per GPU, driven by the library (the reference's row
 * loop, Raytracer.cpp:921-932, split by interleaved rows over `world` ranks).
 * rt_gpu_rank_unique_id: rank 0 makes the communicator's id (id_bytes >= 128,
 * ncclGetUniqueId), which the launcher hands to every rank (e.g. a
 * torch.distributed broadcast); rt_gpu_rank_init then joins this process's
 * device (rt_gpu_init's) to the world's RCCL communicator (ncclCommInitRank),
 * owned by the library. rt_gpu_render_rank_async queues one whole frame
 * (params: row_begin 0, row_step 1, row_end height) on every rank: this rank's
 * rows (rank, rank + world, ...), the count all-gather, the shading and the PPM
 * bytes of its rows, and the previous frame's gather of the u8 row tiles to
 * rank 0, which writes that frame's PPM body into its ppm_body_host (a
 * registered range of height x width x 3 bytes; other ranks pass NULL), in call
 * order. Every collective of the rank runs on one library stream, in the same
 * order on every rank; a frame's gather is queued by the next call (or
 * rt_gpu_rank_finish), so two frames' shading overlap. Every rank makes the same
 * sequence of calls. Complete after rt_gpu_rank_finish + rt_gpu_synchronize.
 * rt_gpu_rank_shutdown destroys the communicator (rt_gpu_shutdown does too). */
int rt_gpu_rank_unique_id(void* id_out, uint64_t id_bytes);
int rt_gpu_rank_init(const void* id, uint64_t id_bytes, int world, int rank);
int rt_gpu_render_rank_async(const rt_render_params* params, uint8_t* ppm_body_host);
/* Shared body (on != 0; after rt_gpu_rank_init / rt580_rank_rehearse, before
 * the first frame): every rank passes ppm_body_host, its own registered mapping
 * of ONE host frame shared by the ranks' processes (e.g. a /dev/shm file), and
 * writes its rows' PPM bytes straight to their places in it; a frame's gather
 * is then a 4-byte all-gather after every rank's write (no tiles to rank 0).
 * With one rank there is no exchange. */
int rt_gpu_rank_share_body(int on);
int rt_gpu_rank_finish(void);
int rt_gpu_rank_shutdown(void);
/* Bench/test hook: rank `rank` of `world` rehearsed on this one GPU without a
 * communicator (the world's per-row counts precomputed in gathered_device,
 * int32[world][n_max]; the gather moves nothing, rank 0 writes its own rows):
 * rt_gpu_render_rank_async then times exactly one rank's share of the loop. */
int rt580_rank_rehearse(int world, int rank, const int32_t* gathered_device);
/* Visible HIP devices (0 without a GPU). */
int rt_gpu_device_count(void);
/* FlushFrameBufferToPPM's pixel mapping on the device (Raytracer.cpp:812-818):
 * (unsigned char)(powf(c / 255.0f, 1.0f / 2.2f) * 255.0f) per int16 channel,
 * through a 256-entry table built with the host's glibc powf (frame values are
 * clamped to [0, 255] by Raycast). n_values int16 -> n_values bytes = the PPM
 * body; used before the multi-GPU gather (half the bytes). */
int rt_gpu_gamma_u8(const int16_t* fb_device, uint64_t n_values, uint8_t* out_device);
/* Self-test of the device's range-restricted math sequences (rt_math.h,
 * rt_libm.h) against the plain operations: mismatches[0] sqrt over every float
 * in [2^-96, +inf], [1] division, [2] unit-vector normalize, [3] AO direction
 * (fast sincos + exact fallback), the last three on n seeded random inputs.
 * Blocking. Test hook; not part of the reference's surface. */
int rt580_selftest_math(uint64_t seed, uint64_t n, uint64_t* mismatches);
/* The device's glibc-powf restatement (specular term, Raytracer.cpp:253) on n
 * device inputs x with exponent y -> out (device), on the shim's stream. Test
 * hook (compared with the host's glibc powf); not part of the reference. */
int rt580_eval_powf(const float* x_device, float y, float* out_device, uint64_t n);
/* Scene-query acceleration. RT_ACCEL_BRUTE tests every primitive per ray, as
 * the reference's IntersectScene does (Raytracer.cpp:473-526); RT_ACCEL_AUTO
 * (default) uses the exact-semantics BVH for triangle scenes larger than one
 * LDS tile (identical results; see 580-raytracer_amd/csrc/rt_bvh.h). Applies
 * to the following renders. rt_gpu_accel_active: 1 if the last frame used it. */
#define RT_ACCEL_BRUTE 0
#define RT_ACCEL_AUTO 1
int rt_gpu_set_accel(int mode);
int rt_gpu_accel_active(void);
/* Largest chunk of the chunked passes of BVH frames (far-hit queue, AO ray
 * records): 2^log2 rays, log2 in [6, 27] (default 27, or $RT580_CHUNK_LOG2 read
 * by rt_gpu_init). Larger frames run in several chunks with identical results;
 * small chunks let the tests reach the multi-chunk paths on small frames.
 * Synchronizes; applies to the following renders. Test hook. */
int rt580_set_chunk_log2(int log2);
/* AO phases of consecutive frames in frame order (1) or free to overlap (0,
 * default; $RT580_AO_ORDER). Applies to the following frames. Bench hook: the
 * isolated launch time of the AO kernel. */
int rt580_set_ao_order(int on);
/* Counters and HIP-event timings of the last render. */
int rt_gpu_last_stats(rt_render_stats* stats);
/* Bench profiling: with enable=1 every following frame records its own HIP
 * events on the shim's stream; profile_read synchronizes and returns the sums
 * over those frames of: the breadth-first trace of the recursion tree (+ per-row
 * AO-call counts), the AO-call numbering (RNG positions), the AO kernel, and the
 * resolve (int16 blend) kernel. */
int rt_gpu_profile(int enable);
int rt_gpu_profile_read(double* ms_trace, double* ms_rank, double* ms_ao, double* ms_resolve, int* frames);
/* While profiling: HIP events around every launch of the AO ray kernel (the
 * scene query of each AO sample: ao_kernel, or ao_near_kernel for BVH scenes),
 * on the stream it runs on. Sum of their durations, number of launches and the
 * AO rays they covered, since rt_gpu_profile(1) (ao_rays counts the chunked BVH
 * launches only; a small-scene frame is one launch over all of its AO rays,
 * rt_gpu_last_stats). Synchronizes. */
int rt_gpu_profile_ao_kernel(double* ms_total, int* launches, uint64_t* ao_rays);
/* Last error message (static storage). Errors name the entry point that saw
 * them; a device fault (reported by whichever call next waits on the device)
 * also names the last entry point that enqueued device work before it. */
const char* rt_gpu_last_error(void);
/* Copy `bytes` from device memory (e.g. rt_gpu_render_device's framebuffer)
 * to host memory, in order after the work queued on the shim's stream.
 * Blocking. Pageable host memory is staged through the library's pinned
 * buffer (the runtime never pins it on the fly). */
int rt_gpu_copy_to_host(void* host_ptr, const void* device_ptr, uint64_t bytes);
/* Wait for all device work of every context (every frame still in flight,
 * rt_gpu_render_device's included) and check the replayed count schedules of
 * those frames. RT_FAILURE names a device fault or a count mismatch and the
 * call whose work raised it. Blocking. */
int rt_gpu_synchronize(void);
void rt_gpu_shutdown(void);

/* ---- Reference class surface as a C ABI (what an FFI/ctypes binding calls) ----
 * Mirrors Raytracer(int,int) / LoadSceneJSON / InitializeRenderer / Render /
 * FlushFrameBufferToPPM (Raytracer.h:572-588, :604). */
typedef struct rt580_raytracer rt580_raytracer;
rt580_raytracer* rt580_create(int width, int height);
void rt580_destroy(rt580_raytracer* rt);
/* assets_root: directory that contains "Assets/" (the reference uses the CWD). */
int rt580_set_assets_root(rt580_raytracer* rt, const char* assets_root);
int rt580_load_scene_json(rt580_raytracer* rt, const char* scene_path);
int rt580_initialize_renderer(rt580_raytracer* rt);
int rt580_render(rt580_raytracer* rt, const char* output_ppm); /* "" / NULL: no file */
int rt580_flush_ppm(rt580_raytracer* rt, const char* output_ppm);
/* Runtime knobs (reference defaults: depth 4, 128 AO samples, AO on, minstd_rand0). */
int rt580_set_depth(rt580_raytracer* rt, int depth);
int rt580_set_ao(rt580_raytracer* rt, int samples, int enabled);
int rt580_set_rng(rt580_raytracer* rt, int engine);
int rt580_set_rows(rt580_raytracer* rt, int row_begin, int row_end);
/* GPUs Render() shards whole frames across (rt_gpu_render_multi); 0 (default):
 * $RT580_GPUS if set (an integer in [1, 16], else Render fails), else 1. */
int rt580_set_gpus(rt580_raytracer* rt, int n);
const int16_t* rt580_framebuffer(rt580_raytracer* rt); /* Pixel[w*h] */
int rt580_get_render_params(rt580_raytracer* rt, rt_render_params* out);
int rt580_get_scene(rt580_raytracer* rt, rt_scene_soa* out); /* views valid until next load */
int rt580_last_stats(rt580_raytracer* rt, rt_render_stats* out);

#ifdef __cplusplus
}
#endif
#endif /* RT580_H */

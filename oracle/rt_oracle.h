// rt_oracle.h — CPU restatement of the reference's per-pixel ray-trace path.
//
// TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load or run this; the product (580-raytracer_amd/) never
// links it. It is the parity checker for the HIP path on configurations larger
// than the committed golden images, and is itself pinned against the reference
// (oracle/_ref builds of /root/reference, golden PPMs in tests/golden/).
//
// Reference: /root/reference/580 Raytracer/Raytracer.{h,cpp} (MSVC C++, single
// threaded). Restated here, function by function (file:line in each definition),
// with two changes that do not alter a single output bit:
//   * by default ("hoisted") the model matrix of each shape (ComputeModelMatrix,
//     Raytracer.cpp:528-586) and the ray-invariant part of each triangle test
//     (world vertices, normal, plane offset, signed area, :353-389) are computed
//     once at load with the same float operations, instead of per IntersectScene
//     call (:480) / per test; the unused Matrix::Inverse per triangle test
//     (:350-351) is skipped. oracle_set_mode(1) ("ref-faithful") restores that
//     per-call work (string meshMap lookup, ComputeModelMatrix per shape per
//     call, Inverse + TransformPoint per test) so the restatement costs what the
//     reference costs -- the CPU baseline of bench.py; results are identical;
//   * rows may be rendered on several threads: the single serial RNG stream
//     (member mGenerator, Raytracer.h:592) is addressed by absolute draw index,
//     found with a count pass + prefix sum over the raster order.
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

// counters[0..5] = rays_total, primary, secondary, shadow, ao, ao_calls
// fb: (row_end-row_begin)*w*3 int16 (Pixel layout), may be NULL (count only).
// rays_per_row: optional (row_end-row_begin) uint64 totals.
// engine: 0 = minstd_rand0 (libstdc++ default_random_engine), 1 = mt19937
// Returns 0 on success, 1 on failure (message on stderr).
int oracle_render(const char* assets_root, const char* scene, int w, int h, int depth,
                  int ao_samples, int ao_enabled, int engine, int threads, int row_begin,
                  int row_end, int16_t* fb, uint64_t* counters, uint64_t* rays_per_row);

// Multi-rank split for the distributed-logic tests: AO calls per
// selected row, then shading of those rows given each row's RNG base (the
// absolute index of its first AO call). Rows: row_begin + k*row_step, k < n_rows.
int oracle_count_rows(const char* assets_root, const char* scene, int w, int h, int depth, int ao_samples,
                      int ao_enabled, int row_begin, int row_step, int n_rows, uint32_t* out);
int oracle_shade_rows(const char* assets_root, const char* scene, int w, int h, int depth, int ao_samples,
                      int ao_enabled, int row_begin, int row_step, int n_rows, const uint64_t* row_base,
                      int16_t* fb);

// CPU baseline: the reference's raster loop over pixels [p0, p0 + n) of the
// full w x h frame with the RNG at AO-call index call_base; threads == 1: one
// serial stream, stopping after max_pixels or budget_s seconds (*n_done);
// threads > 1: exactly max_pixels pixels (count pass, scan, shade). fb:
// n_done * 3 int16; *seconds: render time, load excluded. See rt_oracle.cpp.
int oracle_time_prefix(const char* assets_root, const char* scene, int w, int h, int depth, int ao_samples,
                       int threads, int64_t p0, int64_t max_pixels, double budget_s, uint64_t call_base,
                       int16_t* fb, uint64_t* counters, int64_t* n_done, double* seconds);

// Frame check of a full-resolution GPU frame: segments [seg_x0[k], seg_x0[k] +
// seg_n[k]) of rows seg_y[k], row k's first AO call at row_base[k] (absolute
// index, minstd_rand0). row_calls[k] <- the AO calls of the whole row seg_y[k].
// fb: sum(seg_n) x 3 int16; counters as oracle_render (segment pixels only).
/* RNG engine of oracle_render_segments: 0 minstd_rand0 (default), 1 mt19937 (the draws
 * of the segments' rows generated from the serial stream at their row bases). */
void oracle_set_segments_engine(int engine);
int oracle_render_segments(const char* assets_root, const char* scene, int w, int h, int depth, int ao_samples,
                           int threads, int n_seg, const int32_t* seg_y, const int32_t* seg_x0,
                           const int32_t* seg_n, const uint64_t* row_base, int16_t* fb, uint64_t* row_calls,
                           uint64_t* counters, double* seconds);

// 0 = hoisted (default), 1 = ref-faithful cost model (see above). Process-global.
int oracle_set_mode(int faithful);

// Writes the reference's P6 output (FlushFrameBufferToPPM, Raytracer.cpp:796-830).
int oracle_write_ppm(const char* path, int w, int h, const int16_t* fb);

#ifdef __cplusplus
}
#endif

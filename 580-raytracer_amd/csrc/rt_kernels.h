// rt_kernels.h — device-side views and launchers (rt_kernels.hip), used by rt_shim.cpp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rt580.h"

// Deepest recursion supported by the fixed-size frame stack (reference default 4;
// BASELINE config 5 uses 8).
#define RT_MAX_DEPTH 16

namespace rt580 {

struct DevScene {
    const rt_prim* prims;
    const rt_prim_shade* shade;
    const rt_material* mats;
    const rt_light* lights;
    int n_prims;
    int n_lights;
};

struct DevFrame {
    int width, height, depth, ao_samples, ao_enabled, rng_engine;
    uint32_t rng_seed;
    int row_begin, row_step, n_rows;  // local row k is frame row row_begin + k*row_step
    int view_inverse_ok;
    int n_ambient;
    float view_inv[9];
    float cam_from[3];
    float ao_angle_max;
    double ndc_kx, ndc_ky;
    const uint32_t* mt_stream;  // RT_RNG_MT19937 draws (absolute index), else null
};

void upload_minstd_table(hipStream_t s);
hipError_t launch_count(const DevScene& S, const DevFrame& F, uint32_t* pix_calls, uint32_t* row_calls,
                        uint32_t* row_tree, uint32_t* row_hits, hipStream_t s);
hipError_t launch_row_base(const uint32_t* row_calls, int n_rows, uint64_t* row_base, hipStream_t s);
hipError_t launch_pixel_base(const uint32_t* pix_calls, int width, int n_rows, const uint64_t* row_base,
                             uint64_t* pix_base, hipStream_t s);
hipError_t launch_render(const DevScene& S, const DevFrame& F, const uint64_t* pix_base, int16_t* fb,
                         hipStream_t s);
hipError_t launch_select_rows(const uint64_t* all_base, int row_begin, int row_step, int n_rows,
                              uint64_t* sel_base, hipStream_t s);

}  // namespace rt580

// raytracer.cpp — see raytracer.h. Host side of the drop-in; the per-pixel work
// runs on the GPU (rt_gpu_render). Compiled with -ffp-contract=off.
#include "raytracer.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iostream>

Raytracer::Raytracer(int width, int height) : mWidth(width), mHeight(height) {
    mFrameBuffer.assign((size_t)(width > 0 ? width : 0) * (height > 0 ? height : 0), Pixel{0, 0, 0});
    std::memset(&mParams, 0, sizeof mParams);
}

Raytracer::~Raytracer() {
    if (mFbRegistered) (void)rt_gpu_host_unregister(mFrameBuffer.data());
}

int Raytracer::LoadSceneJSON(const std::string scenePath) {
    std::string err;
    mSceneValid = false;
    mUploadedScene = 0;
    int st = rt580::load_scene_json(mAssetsRoot, scenePath, mScene, err);
    if (st != RT_SUCCESS) {
        std::cerr << err << "\n";
        return st;
    }
    for (const auto& s : mScene.shapes)
        if (s.mesh < 0) return RT_FAILURE;
    rt580::pack_scene(mScene, mPacked);
    mSceneValid = true;
    std::cout << "Scene parsing completed!" << std::endl;  // Raytracer.cpp:772
    return RT_SUCCESS;
}

int Raytracer::SetDepth(int bounces) {
    if (bounces < 0 || bounces > 16) return RT_INVALID_ARG;
    mDepth = bounces;
    return RT_SUCCESS;
}

int Raytracer::SetAmbientOcclusion(int samples, bool on) {
    if (samples <= 0) return RT_INVALID_ARG;
    mAoSamples = samples;
    mAoOn = on ? 1 : 0;
    return RT_SUCCESS;
}

int Raytracer::SetRngEngine(int engine) {
    if (engine != RT_RNG_MINSTD_RAND0 && engine != RT_RNG_MT19937) return RT_INVALID_ARG;
    mEngine = engine;
    return RT_SUCCESS;
}

int Raytracer::SetRows(int row_begin, int row_end, int row_step) {
    if (row_begin < 0 || row_step <= 0 || (row_end >= 0 && (row_end > mHeight || row_end < row_begin)))
        return RT_INVALID_ARG;
    mRowBegin = row_begin;
    mRowEnd = row_end;
    mRowStep = row_step;
    return RT_SUCCESS;
}

int Raytracer::InitializeRenderer() {
    if (!mSceneValid) return RT_FAILURE;
    rt580::make_render_params(mScene, mWidth, mHeight, mFov, mParams);
    mParams.depth = mDepth;
    mParams.ao_samples = mAoSamples;
    mParams.ao_enabled = mAoOn;
    mParams.rng_engine = mEngine;
    mParams.rng_seed = mEngine == RT_RNG_MT19937 ? 5489u : 1u;
    mParams.row_begin = mRowBegin;
    mParams.row_end = mRowEnd < 0 ? mHeight : mRowEnd;
    mParams.row_step = mRowStep;
    if (!mParams.view_inverse_ok) std::cerr << "Failed to compute the inverse of the view matrix.\n";
    return RT_SUCCESS;
}

int Raytracer::Render(const std::string outputName) {
    if (mWidth <= 0 || mHeight <= 0) return RT_INVALID_ARG;
    if (InitializeRenderer() != RT_SUCCESS) return RT_FAILURE;
    // The device scene is process-wide: upload again when another instance (or
    // rt_gpu_shutdown) replaced the one this instance uploaded.
    if (mUploadedScene == 0 || rt_gpu_scene_id() != mUploadedScene) {
        if (rt_gpu_init(-1) != RT_SUCCESS) return RT_FAILURE;
        rt_scene_soa s;
        std::memset(&s, 0, sizeof s);
        s.abi_version = RT580_ABI_VERSION;
        s.n_prims = (int32_t)mPacked.prims.size();
        s.prims = mPacked.prims.data();
        s.shade = mPacked.shade.data();
        s.n_materials = (int32_t)mPacked.materials.size();
        s.materials = mPacked.materials.data();
        s.n_lights = (int32_t)mPacked.lights.size();
        s.lights = mPacked.lights.data();
        if (rt_gpu_upload_scene(&s) != RT_SUCCESS) return RT_FAILURE;
        mUploadedScene = rt_gpu_scene_id();
    }
    // Selected rows land in their frame positions; other rows keep their contents.
    const int nsel = (mParams.row_end - mParams.row_begin + mParams.row_step - 1) / mParams.row_step;
    const bool whole = mParams.row_begin == 0 && mParams.row_step == 1 && mParams.row_end == mHeight;
    static_assert(sizeof(Pixel) == 6, "Pixel is int16 r, g, b");
    // a whole frame lands in mFrameBuffer directly; selected rows through a row buffer
    std::vector<int16_t> rows(whole ? 0 : (size_t)(nsel > 0 ? nsel : 0) * mWidth * 3);
    int16_t* dst = whole ? reinterpret_cast<int16_t*>(mFrameBuffer.data()) : rows.data();
    // The framebuffer lives as long as this instance: page-lock it once, so
    // every frame lands in it with one DMA (no staging copy)
    if (whole && !mFbRegistered && !mFrameBuffer.empty())
        mFbRegistered = rt_gpu_host_register(mFrameBuffer.data(),
                                             (mFrameBuffer.size() * sizeof(Pixel) + 4095) / 4096 * 4096) == RT_SUCCESS;
    // Whole frames can shard across the node's GPUs (interleaved rows, RCCL
    // exchange + gather, rt_gpu_render_multi) when SetGpuCount or $RT580_GPUS
    // asks for more than one; the default is the one device of rt_gpu_init
    // (one process per GPU stays one GPU per process, e.g. under torchrun).
    int gpus = mGpus;
    if (gpus <= 0) {
        gpus = 1;
        if (const char* e = std::getenv("RT580_GPUS")) {
            char* end = nullptr;
            const long v = std::strtol(e, &end, 10);
            if (end == e || *end || v < 1 || v > 16) {
                std::cerr << "RT580_GPUS=" << e << ": not an integer in [1, 16]\n";
                return RT_FAILURE;
            }
            gpus = (int)v;
        }
    }
    const int st = (gpus > 1 && whole) ? rt_gpu_render_multi(&mParams, dst, gpus, nullptr)
                                       : rt_gpu_render(&mParams, dst);
    if (st != RT_SUCCESS) return RT_FAILURE;
    for (int k = 0; !whole && k < nsel; k++) {
        int y = mParams.row_begin + k * mParams.row_step;
        std::memcpy(&mFrameBuffer[(size_t)y * mWidth], &rows[(size_t)k * mWidth * 3], (size_t)mWidth * 6);
    }
    if (!mWriteOutput || outputName.empty()) return RT_SUCCESS;
    return FlushFrameBufferToPPM(outputName);
}

int Raytracer::FlushFrameBufferToPPM(std::string outputName) {
    if (mFrameBuffer.empty()) {
        std::cerr << "Display or frame buffer is null." << std::endl;
        return RT_FAILURE;
    }
    std::ofstream outfile(outputName, std::ios::binary);
    if (!outfile.is_open()) {
        std::cerr << "Failed to create output file: " << outputName << std::endl;
        return RT_FAILURE;
    }
    // Gamma 1/2.2 of c/255 (Raytracer.cpp:816-818). Pixels are clamped to [0,255]
    // (Raycast returns clamp()); a 256-entry table of the same glibc powf
    // expression is the identical mapping.
    // glibc powf at run time (a volatile pointer: no compile-time folding)
    float (*volatile pf)(float, float) = ::powf;
    unsigned char lut[256];
    for (int c = 0; c < 256; c++)
        lut[c] = static_cast<unsigned char>(pf(c / 255.0f, 1.0f / 2.2f) * 255.0f);
    outfile << "P6\n" << mWidth << " " << mHeight << "\n255\n";
    std::vector<unsigned char> row((size_t)mWidth * 3);
    for (int y = 0; y < mHeight; y++) {
        for (int x = 0; x < mWidth; x++) {
            const Pixel& p = mFrameBuffer[(size_t)y * mWidth + x];
            const short c[3] = {p.r, p.g, p.b};
            for (int k = 0; k < 3; k++)
                row[(size_t)x * 3 + k] = (c[k] >= 0 && c[k] <= 255)
                                             ? lut[c[k]]
                                             : static_cast<unsigned char>(pf(c[k] / 255.0f, 1.0f / 2.2f) * 255.0f);
        }
        outfile.write((const char*)row.data(), (std::streamsize)row.size());
    }
    outfile.close();
    return RT_SUCCESS;
}

int Raytracer::LastStats(rt_render_stats& s) const { return rt_gpu_last_stats(&s); }

// ---------------------------------------------------------------- C ABI over the class
struct rt580_raytracer {
    Raytracer rt;
    rt580_raytracer(int w, int h) : rt(w, h) {}
};

extern "C" {

rt580_raytracer* rt580_create(int width, int height) {
    if (width <= 0 || height <= 0) return nullptr;
    try {
        return new rt580_raytracer(width, height);
    } catch (...) {
        return nullptr;
    }
}

void rt580_destroy(rt580_raytracer* h) { delete h; }

int rt580_set_assets_root(rt580_raytracer* h, const char* root) {
    if (!h || !root) return RT_INVALID_ARG;
    h->rt.SetAssetsRoot(root);
    return RT_SUCCESS;
}

int rt580_load_scene_json(rt580_raytracer* h, const char* path) {
    if (!h || !path) return RT_INVALID_ARG;
    try {
        return h->rt.LoadSceneJSON(path);
    } catch (...) {
        return RT_FAILURE;
    }
}

int rt580_initialize_renderer(rt580_raytracer* h) { return h ? h->rt.InitializeRenderer() : RT_INVALID_ARG; }

int rt580_render(rt580_raytracer* h, const char* out) {
    if (!h) return RT_INVALID_ARG;
    try {
        h->rt.SetWriteOutput(out && out[0]);
        return h->rt.Render(out ? out : "");
    } catch (...) {
        return RT_FAILURE;
    }
}

int rt580_flush_ppm(rt580_raytracer* h, const char* out) {
    if (!h || !out) return RT_INVALID_ARG;
    try {
        return h->rt.FlushFrameBufferToPPM(out);
    } catch (...) {
        return RT_FAILURE;
    }
}

int rt580_set_depth(rt580_raytracer* h, int d) { return h ? h->rt.SetDepth(d) : RT_INVALID_ARG; }
int rt580_set_ao(rt580_raytracer* h, int n, int on) { return h ? h->rt.SetAmbientOcclusion(n, on != 0) : RT_INVALID_ARG; }
int rt580_set_rng(rt580_raytracer* h, int e) { return h ? h->rt.SetRngEngine(e) : RT_INVALID_ARG; }
int rt580_set_rows(rt580_raytracer* h, int a, int b) { return h ? h->rt.SetRows(a, b, 1) : RT_INVALID_ARG; }
int rt580_set_gpus(rt580_raytracer* h, int n) { return h ? h->rt.SetGpuCount(n) : RT_INVALID_ARG; }

const int16_t* rt580_framebuffer(rt580_raytracer* h) {
    return h ? reinterpret_cast<const int16_t*>(h->rt.FrameBuffer()) : nullptr;
}

int rt580_get_render_params(rt580_raytracer* h, rt_render_params* out) {
    if (!h || !out) return RT_INVALID_ARG;
    *out = h->rt.Params();
    return RT_SUCCESS;
}

int rt580_get_scene(rt580_raytracer* h, rt_scene_soa* out) {
    if (!h || !out) return RT_INVALID_ARG;
    const rt580::PackedScene& p = h->rt.Packed();
    std::memset(out, 0, sizeof *out);
    out->abi_version = RT580_ABI_VERSION;
    out->n_prims = (int32_t)p.prims.size();
    out->prims = p.prims.data();
    out->shade = p.shade.data();
    out->n_materials = (int32_t)p.materials.size();
    out->materials = p.materials.data();
    out->n_lights = (int32_t)p.lights.size();
    out->lights = p.lights.data();
    return RT_SUCCESS;
}

int rt580_last_stats(rt580_raytracer* h, rt_render_stats* out) {
    if (!h || !out) return RT_INVALID_ARG;
    return h->rt.LastStats(*out);
}

}  // extern "C"

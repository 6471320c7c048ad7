// raytracer.h — the reference's class surface (Raytracer.h:17-609) for the HIP
// path: same constructor, LoadSceneJSON / InitializeRenderer / Render /
// FlushFrameBufferToPPM, same int status codes (Raytracer.h:8-10), same JSON
// scene format and "Assets/" relative paths (Raytracer.h:15). Render() runs the
// per-pixel path on the GPU through the rt_gpu_* C ABI (include/rt580.h).
#pragma once
#include <cstdint>
#include <cstdlib>
#include <new>
#include <string>
#include <vector>

#include "../../include/rt580.h"
#include "rt_scene.h"

// Page-aligned storage rounded up to whole pages: the framebuffer is
// page-locked for DMA (rt_gpu_host_register), and a registration must not
// share a page with other allocations (they would be page-locked with it, and
// a later registration of a neighbour would overlap it).
template <class T>
struct PageAlloc {
    using value_type = T;
    PageAlloc() = default;
    template <class U>
    PageAlloc(const PageAlloc<U>&) {}
    T* allocate(size_t n) {
        const size_t bytes = (n * sizeof(T) + 4095) / 4096 * 4096;
        void* p = nullptr;
        if (posix_memalign(&p, 4096, bytes ? bytes : 4096) != 0) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) { std::free(p); }
    template <class U>
    bool operator==(const PageAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const PageAlloc<U>&) const { return false; }
};

class Raytracer {
  public:
    struct Pixel {  // Raytracer.h:373-418 storage layout (int16 r, g, b)
        short r, g, b;
    };

    Raytracer(int width, int height);  // Raytracer.cpp:781-788
    ~Raytracer();

    int LoadSceneJSON(const std::string scenePath);      // Raytracer.cpp:645-779
    int Render(const std::string outputName);            // Raytracer.cpp:916-935
    int FlushFrameBufferToPPM(std::string outputName);   // Raytracer.cpp:796-830
    int InitializeRenderer();                            // Raytracer.cpp:895-915 (private there)

    // Runtime knobs the reference hard-codes (defaults = the reference's values).
    void SetAssetsRoot(const std::string& root) { mAssetsRoot = root; }
    int SetDepth(int bounces);                       // Raytracer.h:563 (default 4)
    int SetAmbientOcclusion(int samples, bool on);   // Raytracer.cpp:317 (128, on)
    int SetRngEngine(int engine);                    // Raytracer.h:592 (minstd_rand0)
    int SetRows(int row_begin, int row_end, int row_step = 1);
    int SetWriteOutput(bool on) { mWriteOutput = on; return RT_SUCCESS; }
    // GPUs Render() shards a whole frame across (0: $RT580_GPUS if set, else 1 -- the
    // device of rt_gpu_init, so one process per GPU stays one GPU per process).
    int SetGpuCount(int n) {
        if (n < 0 || n > 16) return RT_INVALID_ARG;
        mGpus = n;
        return RT_SUCCESS;
    }

    const Pixel* FrameBuffer() const { return mFrameBuffer.data(); }
    const rt_render_params& Params() const { return mParams; }
    const rt580::PackedScene& Packed() const { return mPacked; }
    int LastStats(rt_render_stats& s) const;

  private:
    int mWidth, mHeight;
    float mFov = 60.0f;  // Raytracer.cpp:786
    std::string mAssetsRoot = ".";
    std::vector<Pixel, PageAlloc<Pixel>> mFrameBuffer;
    rt580::Scene mScene;
    rt580::PackedScene mPacked;
    bool mSceneValid = false;
    uint64_t mUploadedScene = 0;  // rt_gpu_scene_id() of this instance's upload (0: none)
    bool mWriteOutput = true;
    rt_render_params mParams;
    int mDepth = 4, mAoSamples = 128, mAoOn = 1, mEngine = RT_RNG_MINSTD_RAND0;
    int mRowBegin = 0, mRowEnd = -1, mRowStep = 1;
    int mGpus = 0;
    bool mFbRegistered = false;  // mFrameBuffer page-locked for the GPU (rt_gpu_host_register)
};

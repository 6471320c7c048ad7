// Driver for the reference build in oracle/_ref (TEST INFRASTRUCTURE ONLY).
// It links the reference's own Raytracer.cpp (compiled where it lies under
// /root/reference, main renamed to ref_main) and calls its public surface:
//   Raytracer(w,h)          Raytracer.cpp:781
//   LoadSceneJSON(path)     Raytracer.cpp:645   (path relative to "Assets/", Raytracer.h:15)
//   Render(out)             Raytracer.cpp:916   (depth == -1: the reference loop itself)
//   InitializeRenderer()    Raytracer.cpp:895 + GenerateRay :832 + Raycast(ray,depth) :28
//   FlushFrameBufferToPPM   Raytracer.cpp:796
// usage: rt_ref <dir containing Assets/> <scene.json> <w> <h> <depth|-1> <out.ppm> [ao_n] [ao_off]
// depth -1 calls Render() verbatim (default bounces = 4, Raytracer.h:563), with
// its per-pixel progress printing sent to /dev/null.
#include "Raytracer.h"
#include <unistd.h>
#include <climits>
#include <cstring>

#ifdef RT_REF_PARAM
int g_rt_ao_n = 128;
int g_rt_ao_off = 0;
#endif

int main(int argc, char** argv) {
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s <root> <scene> <w> <h> <depth|-1> <out.ppm> [ao_n] [ao_off]\n", argv[0]);
        return 2;
    }
    char outAbs[PATH_MAX];
    if (argv[6][0] == '/') std::snprintf(outAbs, sizeof outAbs, "%s", argv[6]);
    else {
        char cwd[PATH_MAX];
        if (!getcwd(cwd, sizeof cwd)) return 1;
        std::snprintf(outAbs, sizeof outAbs, "%s/%s", cwd, argv[6]);
    }
    int w = std::atoi(argv[3]), h = std::atoi(argv[4]), depth = std::atoi(argv[5]);
#ifdef RT_REF_PARAM
    if (argc > 7) g_rt_ao_n = std::atoi(argv[7]);
    if (argc > 8) g_rt_ao_off = std::atoi(argv[8]);
#else
    if (argc > 7 && std::atoi(argv[7]) != 128) { std::fprintf(stderr, "pristine build has AO=128 only\n"); return 2; }
    if (argc > 8 && std::atoi(argv[8]) != 0) { std::fprintf(stderr, "pristine build has AO on only\n"); return 2; }
#endif
    if (chdir(argv[1]) != 0) { std::perror("chdir"); return 1; }
    std::streambuf* saved = std::cout.rdbuf();
    std::ofstream devnull("/dev/null");
    std::cout.rdbuf(devnull.rdbuf());
    Raytracer rt(w, h);
    int st = rt.LoadSceneJSON(argv[2]);
    if (st != RT_SUCCESS) { std::cout.rdbuf(saved); std::fprintf(stderr, "LoadSceneJSON failed: %d\n", st); return 1; }
    auto t0 = std::chrono::steady_clock::now();
    if (depth < 0) {
        st = rt.Render(outAbs);
    } else {
        rt.InitializeRenderer();
        for (int y = 0; y < h; y++)
            for (int x = 0; x < w; x++) {
                Raytracer::Ray ray;
                rt.GenerateRay(x, y, ray);
                rt.mDisplay->frameBuffer[y * w + x] = rt.Raycast(ray, depth);
            }
        st = rt.FlushFrameBufferToPPM(outAbs);
    }
    auto t1 = std::chrono::steady_clock::now();
    std::cout.rdbuf(saved);
    std::fprintf(stderr, "render_seconds=%.6f status=%d\n",
                 std::chrono::duration<double>(t1 - t0).count(), st);
    return st;
}

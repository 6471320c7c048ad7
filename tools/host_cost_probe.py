#!/usr/bin/env python3
"""Host cost of one frame call on a tiny frame (GPU work negligible): the
plain single-GPU step (rt_gpu_render_async_ppm) vs the per-process
multi-GPU step (rt580_dist.NativeRankFrame, one rank over RCCL). Prints
one JSON line: microseconds of host time per frame for each (mean of N)."""
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    import helpers
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    w, h = 64, 48
    rt580 = helpers.rt580()
    lib = rt580.load()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29582")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    rt580.check(lib.rt_gpu_init(0), "init")
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "stream")
    rt = rt580.Raytracer(w, h, helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON("simpleSphereScene.json") == 0
    rt.set_depth(4)
    rt.set_ao(64, True)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    sc = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(sc)), "upload")
    res = {"frame": "%dx%d simpleSphereScene d4 AO64" % (w, h), "frames": n}
    # plain step
    span = (w * h * 3 + 4095) // 4096 * 4096
    raw = np.zeros(span + 4096, dtype=np.uint8)
    buf = raw[(-raw.ctypes.data) % 4096:][:span]
    rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "register")
    for _ in range(20):
        rt580.check(lib.rt_gpu_render_async_ppm(ctypes.byref(params), buf.ctypes.data), "async")
    torch.cuda.synchronize()
    lib.rt_gpu_synchronize()
    t0, c0 = time.perf_counter(), time.thread_time()
    for _ in range(n):
        rt580.check(lib.rt_gpu_render_async_ppm(ctypes.byref(params), buf.ctypes.data), "async")
    t1, c1 = time.perf_counter(), time.thread_time()
    lib.rt_gpu_synchronize()
    t2 = time.perf_counter()
    res["plain_us_per_frame_enqueue"] = round((t1 - t0) / n * 1e6, 1)
    res["plain_cpu_us_per_frame"] = round((c1 - c0) / n * 1e6, 1)
    res["plain_us_per_frame_total"] = round((t2 - t0) / n * 1e6, 1)
    lib.rt_gpu_host_unregister(buf.ctypes.data)
    dm = helpers.rt580_dist()
    df = dm.NativeRankFrame(rt580, params, dist, torch, h, w, 0, 1, dev)
    for _ in range(20):
        df.render()
    df.finish()
    t0, c0 = time.perf_counter(), time.thread_time()
    for _ in range(n):
        df.render()
    t1, c1 = time.perf_counter(), time.thread_time()
    df.finish()
    t2 = time.perf_counter()
    res["dist_us_per_frame_enqueue"] = round((t1 - t0) / n * 1e6, 1)
    res["dist_cpu_us_per_frame"] = round((c1 - c0) / n * 1e6, 1)
    res["dist_us_per_frame_total"] = round((t2 - t0) / n * 1e6, 1)
    df.close()
    rt.close()
    dist.destroy_process_group()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

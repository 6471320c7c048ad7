#!/usr/bin/env python3
"""Heap-corruption-at-exit probe (scratch): multi-context frames, then
rt_gpu_shutdown + re-init + one frame, then a clean interpreter exit.

    python tools/repro_exit.py <local|rccl|none> [shutdown:0|1]
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402
import helpers  # noqa: E402


def main():
    mode = sys.argv[1]
    do_shutdown = len(sys.argv) < 3 or sys.argv[2] == "1"
    rt580 = helpers.rt580()
    lib = rt580.load()
    root = helpers.synthetic_root("cornell10k")
    w, h = 53, 29
    rt = rt580.Raytracer(w, h, root)
    assert rt.LoadSceneJSON("cornell10k.json") == 0
    rt.set_depth(4)
    rt.set_ao(16, True)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    s = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    if mode != "none":
        G = 3 if mode == "local" else 1
        if mode == "rccl":
            os.environ["RT580_MULTI_TRANSPORT"] = "rccl"
        devs = (ctypes.c_int * G)(*([0] * G))
        span = (w * h * 3 + 4095) // 4096 * 4096
        raw = np.zeros(span + 4096, dtype=np.uint8)
        off = (-raw.ctypes.data) % 4096
        buf = raw[off:off + span]
        rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "register")
        for _ in range(4):
            rt580.check(lib.rt_gpu_render_multi_async(ctypes.byref(params), buf.ctypes.data, G, devs), "multi_async")
        rt580.check(lib.rt_gpu_synchronize(), "sync")
        rt580.check(lib.rt_gpu_host_unregister(buf.ctypes.data), "unregister")
        print("multi frames done", flush=True)
    if do_shutdown:
        lib.rt_gpu_shutdown()
        rt580.check(lib.rt_gpu_init(0), "init")
        print("shutdown + init done", flush=True)
    out = np.zeros(w * h * 3, dtype=np.int16)
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    rt580.check(lib.rt_gpu_render(ctypes.byref(params), out.ctypes.data), "render")
    rt.close()
    print("exiting", flush=True)


if __name__ == "__main__":
    main()

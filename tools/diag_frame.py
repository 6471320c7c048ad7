#!/usr/bin/env python3
"""One frame of a bench workload through the library named by $RT580_LIB (the
diagnostic build prints its pass statistics with RT580_PROGRESS=1).
usage: RT580_LIB=580-raytracer_amd/lib580rt_diag.so RT580_PROGRESS=1 python tools/diag_frame.py <workload>"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import bench  # noqa: E402
import helpers  # noqa: E402

scene, synth, W, H, depth, ao, _ = bench.WORKLOADS[sys.argv[1]]
root = helpers.synthetic_root(scene[:-5]) if synth else helpers.ASSETS_ROOT
rt580 = helpers.rt580()
lib = rt580.load()
rt = rt580.Raytracer(W, H, root)
assert rt.LoadSceneJSON(scene) == 0
rt.set_depth(depth)
rt.set_ao(ao, True)
t0 = time.time()
assert rt.Render("") == 0, lib.rt_gpu_last_error()
print("frame %.3f s stats %s" % (time.time() - t0, rt.stats()), flush=True)

#!/usr/bin/env python3
"""Render a full-size frame on the HIP path and save what a parity hunt needs
(GPU box): the int16 framebuffer (.npy), the per-row AO-call counts (.npy), and
the sha256 of each band of tests/golden/fullframe.json against the oracle's.

    python tools/fullframe_dump.py north_star gpurun_out/ff
"""
import ctypes
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import numpy as np
    import torch
    import helpers
    name, out = sys.argv[1], sys.argv[2]
    os.makedirs(out, exist_ok=True)
    e = json.load(open(os.path.join(REPO, "tests", "golden", "fullframe.json")))[name]
    root = helpers.synthetic_root(e["assets"])
    rt580 = helpers.rt580()
    lib = rt580.load()
    rt = rt580.Raytracer(e["width"], e["height"], root)
    assert rt.LoadSceneJSON(e["scene"]) == 0
    rt.set_depth(e["depth"])
    rt.set_ao(e["ao_samples"], True)
    assert rt.Render("") == 0, lib.rt_gpu_last_error()
    fb = rt.framebuffer()
    st = rt.stats()
    np.save(os.path.join(out, name + "_fb.npy"), fb)
    params = rt.render_params()
    dev = torch.device("cuda", 0)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "stream")
    cnt = helpers.rt580_dist().GpuRows(rt580, params, torch, dev).count(0, 1)[:e["height"]].cpu().numpy()
    np.save(os.path.join(out, name + "_rowcalls.npy"), cnt)
    body = rt580.ppm_bytes(fb)[-e["width"] * e["height"] * 3:]
    row = e["width"] * 3
    bands = [hashlib.sha256(body[r * row:min(e["height"], r + e["band_rows"]) * row]).hexdigest()
             for r in range(0, e["height"], e["band_rows"])]
    res = {"stats": st, "sha256": helpers.sha256(rt580.ppm_bytes(fb)), "want": e["sha256"],
           "bands_differing": [k * e["band_rows"] for k, (a, b) in enumerate(zip(bands, e["band_sha256"])) if a != b]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Determinism and per-ray check of the BVH AO passes (diagnostic library).

Renders one workload K times back to back through rt_gpu_render_device
(frames in flight, replayed count schedules, as bench.py times them), hashes
every frame's gamma-mapped bytes, and -- with RT580_AO_VERIFY=1 in the
diagnostic build -- reads the AO audit's totals (rt_kernels.hip
ao_audit_*): every near-query AO ray answered again by the unbudgeted query,
and the occlusion counts and far queue that implies against what the product's
ao_trace_kernel / ao_late_kernel wrote (their code is untouched by the audit).

    RT580_LIB=580-raytracer_amd/lib580rt_diag.so RT580_AO_VERIFY=1 \\
        python tools/ao_verify.py [workload] [frames] [--small WxH]

Prints one JSON line: frame hashes, whether they agree, replay errors, the
verification totals and the first wrong rays.
"""
import ctypes
import json
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    import bench
    import helpers
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    name = args[0] if args else "field100k_1080p"
    frames = int(args[1]) if len(args) > 1 else 6
    scene, synth, W, H, depth, ao, _ = bench.WORKLOADS[name]
    for a in sys.argv[1:]:
        if a.startswith("--small="):
            W, H = map(int, a.split("=", 1)[1].split("x"))
    root = helpers.synthetic_root(scene[:-5]) if synth else helpers.ASSETS_ROOT
    rt580 = helpers.rt580()
    lib = rt580.load()
    rt580.check(lib.rt_gpu_init(0), "init")
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(stream.cuda_stream)), "stream")
    rt = rt580.Raytracer(W, H, root)
    assert rt.LoadSceneJSON(scene) == 0
    rt.set_depth(depth)
    rt.set_ao(ao, True)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    sc = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(sc)), "upload")
    n = W * H * 3
    outs, errors = [], []
    for i in range(frames):
        fbp = ctypes.c_void_p()
        st = lib.rt_gpu_render_device(ctypes.byref(params), ctypes.byref(fbp))
        if st != 0:
            msg = lib.rt_gpu_last_error()
            errors.append({"frame": i, "error": msg.decode() if isinstance(msg, bytes) else str(msg)})
            outs.append(None)
            continue
        o = torch.empty(n, dtype=torch.uint8, device=dev)
        rt580.check(lib.rt_gpu_gamma_u8(fbp, n, o.data_ptr()), "gamma_u8")
        outs.append(o)
        print("[ao_verify] frame %d enqueued" % i, file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    head = b"P6\n%d %d\n255\n" % (W, H)  # the PPM as FlushFrameBufferToPPM writes it (bench.py frame_check)
    hashes = [helpers.sha256(head + o.cpu().numpy().tobytes()) if o is not None else None for o in outs]
    res = {"workload": name, "width": W, "height": H, "frames": frames,
           "hashes": hashes,
           "frames_agree": len(set(h for h in hashes if h)) <= 1, "replay_errors": errors}
    if hasattr(lib, "rt580_diag_ao_verify"):
        v = np.zeros(64, dtype=np.uint64)
        f = lib.rt580_diag_ao_verify
        f.argtypes = [ctypes.c_void_p]
        if f(v.ctypes.data) == 0:
            res["verify"] = {"rays_checked": int(v[0]), "calls_differing": int(v[1]),
                             "queue_count_differs": int(v[2]), "queue_checksum_differs": int(v[3]),
                             "chunks": int(v[4]), "near_hits": int(v[5]), "queued": int(v[6]),
                             "first_calls_differing": [{"call": int(v[8 + 2 * k]) & 0xffffffff,
                                                        "got": int(v[8 + 2 * k]) >> 32, "want": int(v[9 + 2 * k])}
                                                       for k in range(min(8, int(v[1])))]}
            res["verify"]["entries_unexplained"] = int(v[7])
            res["verify"]["entry_reasons"] = int(v[24])
            bad = []
            for k in range(min(2, int(v[25]))):
                d = [int(x) for x in v[26 + 18 * k: 26 + 18 * k + 18]]
                f = lambda u: struct.unpack("<f", struct.pack("<I", u & 0xffffffff))[0]
                bad.append({"entry": [f(u) for u in d[0:8]], "entry_call": d[3], "ray": [f(u) for u in d[8:16]],
                            "ray_call": d[11], "key": d[16] & 0xffffffff, "why": d[16] >> 32,
                            "slot": d[17] & 0xffffffff, "item": d[17] >> 32})
            res["verify"]["entries"] = bad
            res["verify"]["ok"] = bool(not (v[1] or v[2] or v[3]) and v[4] > 0)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

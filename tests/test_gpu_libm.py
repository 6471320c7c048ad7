"""The device restatement of glibc powf (rt_libm.h rt_glibc_powf, the specular
term of CalculateLocalColor, Raytracer.cpp:253) against this host's glibc powf,
bit for bit, over EVERY float x in [0, 1.0001] (fmax(dot(V, R), 0) of unit
vectors) for every specular exponent of the scenes the path renders (the
reference's Assets/ and the synthetic scenes of configs 3-5)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

NATIVE = os.path.join(helpers.REPO, "tests", "native")


def _host_powf():
    out = os.path.join(NATIVE, "_build", "libpowf_ref.so")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    subprocess.run(["g++", "-O2", "-fPIC", "-shared", "-pthread", "-ffp-contract=off", "-o", out,
                    os.path.join(NATIVE, "powf_ref.cpp")], check=True)
    lib = ctypes.CDLL(out)
    lib.glibc_powf_array.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
    return lib


def test_device_powf_equals_glibc_all_inputs_all_scene_exponents():
    import torch
    rt580 = helpers.rt580()
    lib = rt580.load()
    assert lib.rt_gpu_init(0) == 0
    host = _host_powf()
    dev = torch.device("cuda", 0)
    assert lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) == 0
    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    exps = helpers.scene_exponents()
    hi = int(np.float32(1.0001).view(np.uint32)) + 1
    chunk = 1 << 26
    bad = {}
    try:
        for lo in range(0, hi, chunk):
            n = min(chunk, hi - lo)
            x = np.arange(lo, lo + n, dtype=np.uint32).view(np.float32)
            xd = torch.from_numpy(x).to(dev)
            od = torch.empty(n, dtype=torch.float32, device=dev)
            want = np.empty(n, dtype=np.float32)
            for y in exps:
                assert lib.rt580_eval_powf(xd.data_ptr(), y, od.data_ptr(), n) == 0
                host.glibc_powf_array(x.ctypes.data, y, want.ctypes.data, n, threads)
                got = od.cpu().numpy()
                diff = int(np.count_nonzero(got.view(np.uint32) != want.view(np.uint32)))
                if diff:
                    bad[y] = bad.get(y, 0) + diff
    finally:
        lib.rt_gpu_set_stream(lib.rt_gpu_own_stream())
    assert not bad, "device powf differs from glibc: %s" % bad

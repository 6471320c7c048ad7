#!/usr/bin/env python3
"""Device -> host copy rates of one frame's int16 framebuffer (probe, not product).

Times hipMemcpyAsync of `MB` megabytes from HBM into (a) torch pinned memory,
(b) a page-aligned numpy buffer page-locked with hipHostRegister (what
rt_gpu_render_async writes into), alone and beside a running compute kernel,
and prints GB/s per case (one JSON line).

    python tools/d2h_probe.py [MB]
"""
import ctypes
import json
import sys
import time


def main():
    import numpy as np
    import torch
    mb = float(sys.argv[1]) if len(sys.argv) > 1 else 12.44
    n = int(mb * 1e6) // 2
    dev = torch.device("cuda", 0)
    src = torch.randint(0, 255, (n,), dtype=torch.int16, device=dev)
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    span = (n * 2 + 4095) // 4096 * 4096
    raw = np.zeros(span + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    reg = raw[off:off + span]
    assert hip.hipHostRegister(reg.ctypes.data, span, 0) == 0
    pinned = torch.empty(n, dtype=torch.int16, pin_memory=True)
    stream = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    busy = torch.randn(4096, 4096, device=dev)
    res = {"MB": mb}

    def run(dst_ptr, reps=20, beside=False):
        torch.cuda.synchronize()
        if beside:
            with torch.cuda.stream(side):
                for _ in range(40):
                    busy.mul_(1.0001)
        t0 = time.perf_counter()
        for _ in range(reps):
            assert hip.hipMemcpyAsync(dst_ptr, src.data_ptr(), n * 2, 2, ctypes.c_void_p(stream.cuda_stream)) == 0
        stream.synchronize()
        dt = (time.perf_counter() - t0) / reps
        torch.cuda.synchronize()
        return round(n * 2 / dt / 1e9, 2)

    for name, ptr in (("torch_pinned", pinned.data_ptr()), ("host_registered", reg.ctypes.data)):
        run(ptr, 3)
        res[name + "_GBs"] = run(ptr)
        res[name + "_beside_kernels_GBs"] = run(ptr, beside=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

"""The multi-rank paths on the real device over RCCL, with one rank (SURVEY
§8e; the GPU box has one MI355X): NativeRankFrame (bench.py's step: the
library's own rank loop) and DistFrame = rt_gpu_count_rows, RCCL
all_gather_into_tensor of the per-row AO counts, the row-base kernel,
rt_gpu_shade_rows, u8 gamma on the device, an asynchronous RCCL gather of the
row tiles, de-interleave. Frames are queued back to back, so consecutive frames
run on the library's two pipelined slots while the caller's stream allocates
and fills the count buffers (the ordering rt_shim.cpp rt_gpu_count_rows keeps).
Every frame must be BASELINE config 2's reference PPM (Raytracer.cpp:916-935)."""
import ctypes

import pytest

import helpers

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rccl_one_rank():
    import torch
    import torch.distributed as dist
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1, device_id=device)
    rt580 = helpers.rt580()
    lib = rt580.load()
    rt580.check(lib.rt_gpu_init(0), "rt_gpu_init")
    stream = torch.cuda.current_stream(device)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(stream.cuda_stream)), "rt_gpu_set_stream")
    try:
        yield torch, dist, device, rt580, lib
    finally:
        torch.cuda.synchronize()
        rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(0)), "rt_gpu_set_stream")
        dist.destroy_process_group()


def _setup(rt580, lib, w, h):
    rt = rt580.Raytracer(w, h, helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON("simpleSphereScene.json") == 0
    rt.set_depth(4)
    rt.set_ao(64, True)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    scene = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(scene)), "rt_gpu_upload_scene")
    return rt, params


@pytest.mark.parametrize("u8", [True, False])
def test_dist_frame_rccl_one_rank_matches_reference(rccl_one_rank, u8):
    torch, dist, device, rt580, lib = rccl_one_rank
    w, h = 1920, 1080
    want = next(e for e in helpers.golden_entries(False) if e["name"] == "config2_1080p_d4_ao64")["sha256"]
    rt, params = _setup(rt580, lib, w, h)
    dm = helpers.rt580_dist()
    df = dm.DistFrame(dm.GpuRows(rt580, params, torch, device), dist, torch, h, w, 0, 1, device, u8=u8)

    def sha(frame):
        arr = frame.cpu().numpy()
        ppm = (b"P6\n%d %d\n255\n" % (w, h) + arr.tobytes()) if u8 else rt580.ppm_bytes(arr)
        return helpers.sha256(ppm)

    try:
        # one frame at a time
        for _ in range(2):
            df.render()
            assert sha(df.finish()) == want
        # five frames queued back to back (pipelined slots, async gathers in flight)
        for _ in range(5):
            df.render()
        assert sha(df.finish()) == want
    finally:
        df.close()  # its registered host buffers leave the library's table before numpy frees them
    rt.close()


def test_native_rank_frame_rccl_one_rank_matches_reference(rccl_one_rank):
    """NativeRankFrame (bench.py's multi-rank step): the library's own rank loop
    (rt_gpu_rank_init from a broadcast RCCL id, rt_gpu_render_rank_async:
    count, all-gather, shading, the previous frame's gather and rank 0's PPM
    write, every collective on one library stream) -- frames one at a time, then
    seven queued back to back (two turns of the buffer ring and one more): every
    host buffer of the ring holds the reference's 1080p render."""
    torch, dist, device, rt580, lib = rccl_one_rank
    w, h = 1920, 1080
    want = next(e for e in helpers.golden_entries(False) if e["name"] == "config2_1080p_d4_ao64")["sha256"]
    rt, params = _setup(rt580, lib, w, h)
    dm = helpers.rt580_dist()
    df = dm.NativeRankFrame(rt580, params, dist, torch, h, w, 0, 1, device)

    def sha(frame):
        return helpers.sha256(b"P6\n%d %d\n255\n" % (w, h) + frame.tobytes())

    try:
        for _ in range(2):
            df.render()
            assert sha(df.finish().numpy()) == want
        for _ in range(7):
            df.render()
        df.finish()
        for k in range(df.R):
            assert sha(df.frame(k)) == want, "ring buffer %d" % k
    finally:
        df.close()
    rt.close()


def test_native_rank_frame_bvh_scene_matches_oracle(rccl_one_rank):
    """The rank loop on a BVH scene (replayed count schedules, frames in
    flight): the Cornell box at depth 3, AO 8, against the oracle."""
    import numpy as np
    torch, dist, device, rt580, lib = rccl_one_rank
    w, h = 96, 54
    root = helpers.synthetic_root("cornell10k")
    rt = rt580.Raytracer(w, h, root)
    assert rt.LoadSceneJSON("cornell10k.json") == 0
    rt.set_depth(3)
    rt.set_ao(8, True)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    scene = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(scene)), "rt_gpu_upload_scene")
    ref, _ = helpers.oracle_render("cornell10k.json", w, h, 3, 8, True, root=root)
    want = rt580.gamma_lut()[ref.astype(np.int64)].astype(np.uint8)
    dm = helpers.rt580_dist()
    df = dm.NativeRankFrame(rt580, params, dist, torch, h, w, 0, 1, device)
    try:
        for _ in range(6):
            df.render()
        df.finish()
        for k in range(df.R):
            assert np.array_equal(df.frame(k), want), "ring buffer %d" % k
    finally:
        df.close()
    rt.close()

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


@pytest.mark.parametrize("shared", [True, False])
def test_native_rank_frame_rccl_one_rank_matches_reference(rccl_one_rank, shared):
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
    df = dm.NativeRankFrame(rt580, params, dist, torch, h, w, 0, 1, device, shared=shared)

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


def _gathered_counts(rt580, params, torch, device, h, world):
    """The world's per-row AO-call counts (int32[world][n_max]) from one
    full-frame count pass: what a rehearsed rank's all-gather would receive."""
    dm = helpers.rt580_dist()
    cnt = dm.GpuRows(rt580, params, torch, device).count(0, 1)[:h]
    torch.cuda.synchronize()
    n_max = dm.n_max_rows(h, world)
    gathered = torch.zeros(world * n_max, dtype=torch.int32, device=device)
    for k in range(world):
        part = cnt[k::world]
        gathered[k * n_max:k * n_max + part.numel()] = part
    return gathered


def test_native_rank_frame_shared_body_rehearsed_ranks(rccl_one_rank):
    """The shared body (rt_gpu_rank_share_body): three ranks of a 3-way split,
    rehearsed one after another on this GPU (rt580_rank_rehearse), each writing
    its own rows' PPM bytes straight into the SAME registered host frames
    (launch_gamma_rows_u8 into mapped host memory): once all three have run,
    every frame of the ring is the reference's 1080p render."""
    import numpy as np
    torch, dist, device, rt580, lib = rccl_one_rank
    w, h, world = 1920, 1080, 3
    want = next(e for e in helpers.golden_entries(False) if e["name"] == "config2_1080p_d4_ao64")["sha256"]
    rt, params = _setup(rt580, lib, w, h)
    dm = helpers.rt580_dist()
    gathered = _gathered_counts(rt580, params, torch, device, h, world)
    span = (h * w * 3 + 4095) // 4096 * 4096
    raws = [np.zeros(span + 4096, dtype=np.uint8) for _ in range(dm.NativeRankFrame.R)]
    frames = [r[(-r.ctypes.data) % 4096:][:span] for r in raws]
    for rank in (2, 0, 1):
        df = dm.NativeRankFrame(rt580, params, None, torch, h, w, rank, world, device, rehearse_gathered=gathered,
                                host_frames=frames)
        try:
            for _ in range(dm.NativeRankFrame.R + 1):
                df.render()
            df.finish()
        finally:
            df.close()
    for k, f in enumerate(frames):
        assert helpers.sha256(b"P6\n%d %d\n255\n" % (w, h) + f[:h * w * 3].tobytes()) == want, "ring frame %d" % k
    rt.close()


def _shm_rank_worker(rank, world, port, out_path):
    """One process of test_native_rank_frame_shared_body_two_processes."""
    import os
    import numpy as np
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        device = torch.device("cuda", 0)
        torch.cuda.set_device(device)
        rt580 = helpers.rt580()
        lib = rt580.load()
        rt580.check(lib.rt_gpu_init(0), "rt_gpu_init")
        w, h = 1920, 1080
        rt, params = _setup(rt580, lib, w, h)
        dm = helpers.rt580_dist()
        gathered = _gathered_counts(rt580, params, torch, device, h, world)
        df = dm.NativeRankFrame(rt580, params, dist, torch, h, w, rank, world, device, rehearse_gathered=gathered)
        for _ in range(4):
            df.render()
        df.finish()
        dist.barrier()  # both ranks' rows are in the shared frames
        if rank == 0:
            np.save(out_path, np.stack([df.frame(k).copy() for k in range(df.R)]))
        dist.barrier()
        df.close()
        rt.close()
        lib.rt_gpu_shutdown()
    finally:
        dist.destroy_process_group()


def test_native_rank_frame_shared_body_two_processes(tmp_path):
    """Two processes (rehearsed ranks 0 and 1 of 2 on this GPU, no RCCL: one GPU
    cannot hold two ranks of a communicator) map ONE /dev/shm frame ring
    (SharedHostFrames, its name broadcast over gloo), each registers its own
    mapping and writes its rows into it: rank 0 reads the whole frame."""
    import numpy as np
    import torch.multiprocessing as mp
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    out = str(tmp_path / "frames.npy")
    mp.start_processes(_shm_rank_worker, args=(2, port, out), nprocs=2, join=True, start_method="spawn")
    want = next(e for e in helpers.golden_entries(False) if e["name"] == "config2_1080p_d4_ao64")["sha256"]
    for k, f in enumerate(np.load(out)):
        assert helpers.sha256(b"P6\n%d %d\n255\n" % (1920, 1080) + f.tobytes()) == want, "ring frame %d" % k

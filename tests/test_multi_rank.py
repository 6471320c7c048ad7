"""Multi-rank path on CPU: world_size 2 and 3 over gloo, each rank
counting and shading its interleaved rows with the CPU backend, exchanging
per-row AO-call counts with all_gather and gathering row tiles to rank 0. The
reassembled frame must equal the single-rank render bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import helpers

CASE = ("simpleSphereScene.json", 41, 29, 3, 8)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene, w, h, depth, ao = CASE
        backend = helpers.OracleRows(scene, w, h, depth, ao)
        frame = helpers.rt580_dist().render_frame(backend, dist, torch, h, w, rank, world)
        if rank == 0:
            np.save(out_path, frame.numpy())
    finally:
        dist.destroy_process_group()


def _worker_steady(rank, world, port, out_path, u8):
    """DistFrame (bench.py's steady-state path): three frames back to back with the
    double-buffered asynchronous gather; the last assembled frame must be exact."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene, w, h, depth, ao = CASE
        backend = helpers.OracleRows(scene, w, h, depth, ao)
        df = helpers.rt580_dist().DistFrame(backend, dist, torch, h, w, rank, world, torch.device("cpu"), u8=u8)
        for _ in range(3):
            df.render()
        frame = df.finish()
        if rank == 0:
            np.save(out_path, frame.numpy())
    finally:
        dist.destroy_process_group()


def _worker_shared(rank, world, port, out_path):
    """The shared-body exchange (NativeRankFrame's default): the ranks map ONE
    /dev/shm frame (SharedHostFrames), each writes its own rows' PPM bytes into
    it, three frames over the ring."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dm = helpers.rt580_dist()
    try:
        scene, w, h, depth, ao = CASE
        backend = helpers.OracleRows(scene, w, h, depth, ao)
        frames = dm.SharedHostFrames(dist, rank, h * w * 3, 3)
        lut = helpers.rt580().gamma_lut()
        for k in range(3):
            body = frames.bufs[k][:h * w * 3].reshape(h, w, 3)
            got = dm.render_frame_shared(backend, dist, torch, h, w, rank, world, body, lut)
        if rank == 0:
            np.save(out_path, np.stack([frames.bufs[k][:h * w * 3].copy() for k in range(3)]))
        del body, got
        dist.barrier()
        frames.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_shared_host_frame_rows(world, tmp_path):
    out = str(tmp_path / "frames.npy")
    mp.start_processes(_worker_shared, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    scene, w, h, depth, ao = CASE
    ref, _ = helpers.oracle_render(scene, w, h, depth, ao, True)
    want = helpers.rt580().ppm_bytes(ref).split(b"\n", 3)[3]
    for k, f in enumerate(np.load(out)):
        assert f.tobytes() == want, "ring frame %d" % k
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("rt580-")]  # rank 0 unlinked the file


def _worker_shm_full(rank, world, port, out_path):
    """/dev/shm without room on rank 0 (posix_fallocate fails): every rank
    gets the same OSError (NativeRankFrame then falls back to the gather)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        if rank == 0:
            def full(fd, off, n):
                raise OSError(28, "No space left on device")
            os.posix_fallocate = full
        try:
            helpers.rt580_dist().SharedHostFrames(dist, rank, 1 << 20, 3)
            raised = False
        except OSError:
            raised = True
        flags = [torch.zeros(1, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(flags, torch.tensor([int(raised)], dtype=torch.int32))
        if rank == 0:
            np.save(out_path, torch.cat(flags).numpy())
    finally:
        dist.destroy_process_group()


def test_shared_host_frame_without_room_fails_on_every_rank(tmp_path):
    out = str(tmp_path / "flags.npy")
    mp.start_processes(_worker_shm_full, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    assert np.load(out).tolist() == [1, 1]
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("rt580-")]


@pytest.mark.parametrize("world,u8", [(2, False), (3, False), (2, True), (3, True)])
def test_steady_state_dist_frame(world, u8, tmp_path):
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker_steady, args=(world, _free_port(), out, u8), nprocs=world, join=True,
                       start_method="spawn")
    scene, w, h, depth, ao = CASE
    ref, _ = helpers.oracle_render(scene, w, h, depth, ao, True)
    got = np.load(out)
    if u8:  # the PPM body the reference writes
        assert got.tobytes() == helpers.rt580().ppm_bytes(ref).split(b"\n", 3)[3]
    else:
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("world", [2, 3])
def test_interleaved_rows_match_single_rank(world, tmp_path):
    out = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    frame = np.load(out)
    scene, w, h, depth, ao = CASE
    ref, _ = helpers.oracle_render(scene, w, h, depth, ao, True)
    assert frame.shape == ref.shape
    assert np.array_equal(frame, ref)


def test_row_partition_covers_frame():
    d = helpers.rt580_dist()
    for h in (1, 7, 1080, 2160):
        for g in (1, 2, 3, 8):
            rows = sorted(r for k in range(g) for r in range(k, h, g))
            assert rows == list(range(h))
            assert max(d.n_local_rows(h, k, g) for k in range(g)) == d.n_max_rows(h, g)

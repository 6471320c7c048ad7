"""Multi-GPU Render inside lib580rt.so (rt_gpu_render_multi):
interleaved rows per device, the per-row AO-count exchange, RNG bases, shading,
gather of the row tiles to device 0 and de-interleave. The GPU box has one
MI355X, so the G-way split runs with every context on device 0 and device
copies as the transport (a device listed twice selects it); the RCCL transport
itself runs here with one rank (RT580_MULTI_TRANSPORT=rccl) and on the 8-GPU
node only in the driver's scaling runs. The frame must be byte-identical to the
single-GPU render for every G."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import helpers
from test_gpu_parity import render_gpu
from test_dropin import assets_dir, build_ref_main

pytestmark = pytest.mark.gpu


def _multi(scene, w, h, depth, ao, G, rng=0, root=helpers.ASSETS_ROOT, transport=None):
    rt580 = helpers.rt580()
    lib = rt580.load()
    rt = rt580.Raytracer(w, h, root)
    assert rt.LoadSceneJSON(scene) == 0
    rt.set_depth(depth)
    rt.set_ao(ao, True)
    rt.set_rng(rng)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    s = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    devs = (ctypes.c_int * G)(*([0] * G))
    out = np.zeros(w * h * 3, dtype=np.int16)
    old = os.environ.get("RT580_MULTI_TRANSPORT")
    if transport:
        os.environ["RT580_MULTI_TRANSPORT"] = transport
    try:
        rt580.check(lib.rt_gpu_render_multi(ctypes.byref(params), out.ctypes.data, G, devs), "rt_gpu_render_multi")
    finally:
        if transport:
            if old is None:
                del os.environ["RT580_MULTI_TRANSPORT"]
            else:
                os.environ["RT580_MULTI_TRANSPORT"] = old
    rt.close()
    return out.reshape(h, w, 3)


@pytest.mark.parametrize("G", [2, 3, 8])
def test_render_multi_matches_single(G):
    scene, w, h, depth, ao = "simpleSphereScene.json", 97, 61, 4, 64
    full, _ = render_gpu(scene, w, h, depth, ao, True)
    got = _multi(scene, w, h, depth, ao, G)
    assert np.array_equal(got, full), "%d pixels differ" % int((got != full).any(axis=2).sum())


def test_render_multi_rccl_transport_one_rank():
    """The RCCL code path (ncclCommInitAll, ncclAllGather of the row counts) with
    a single rank on the one GPU of the box."""
    scene, w, h, depth, ao = "simpleSphereScene.json", 64, 40, 3, 16
    full, _ = render_gpu(scene, w, h, depth, ao, True)
    got = _multi(scene, w, h, depth, ao, 1, transport="rccl")
    assert np.array_equal(got, full)


def test_render_multi_bvh_scene():
    root = helpers.synthetic_root("cornell10k")
    scene, w, h, depth, ao = "cornell10k.json", 48, 27, 4, 8
    full, _ = render_gpu(scene, w, h, depth, ao, True, root=root)
    got = _multi(scene, w, h, depth, ao, 3, root=root)
    assert np.array_equal(got, full)


def test_render_multi_mt19937():
    """MSVC's engine across ranks: each rank addresses the serial mt19937 stream
    by absolute draw index (generated up to its rows' last draw)."""
    entry = next(e for e in helpers.golden_entries(True) if e["name"] == "sss_d2_ao16_mt")
    got = _multi(entry["scene"], entry["width"], entry["height"], entry["depth"], entry["ao_samples"], 3, rng=1)
    assert helpers.rt580().ppm_bytes(got) == helpers.golden_ppm(entry)


def test_class_render_shards_across_gpus():
    """Render() of the class surface with set_gpus(4) (four contexts on the
    box's one device) writes the golden image."""
    entry = next(e for e in helpers.golden_entries(True) if e["name"] == "teapots_d2_ao4")
    rt = helpers.rt580().Raytracer(entry["width"], entry["height"], helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON(entry["scene"]) == 0
    rt.set_depth(entry["depth"])
    rt.set_ao(entry["ao_samples"], entry["ao_enabled"])
    rt.set_gpus(4)
    assert rt.Render("") == 0
    assert helpers.rt580().ppm_bytes(rt.framebuffer()) == helpers.golden_ppm(entry)
    rt.close()


def test_reference_main_with_two_gpus(tmp_path):
    """The reference's main() through the drop-in with RT580_GPUS=2."""
    exe = build_ref_main(str(tmp_path))
    cwd = assets_dir(tmp_path)
    env = dict(os.environ, RT580_GPUS="2")
    p = subprocess.run([exe], cwd=cwd, capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr
    want = next(e for e in helpers.golden_entries(False) if e["name"] == "main_500_d4_ao128")["sha256"]
    assert helpers.sha256(open(os.path.join(cwd, "output.ppm"), "rb").read()) == want


def test_render_multi_follows_scene_and_device_set():
    """Consecutive split frames with different device sets (G = 3, 2, 3) and a
    new scene in between: the other contexts are refreshed from context 0 (the
    scene is replicated by device copies, never rebuilt) and every frame equals
    the single-GPU render of its scene."""
    root = helpers.synthetic_root("cornell10k")
    a = ("cornell10k.json", 40, 24, 3, 8, root)
    b = ("scene.json", 40, 30, 2, 8, helpers.ASSETS_ROOT)
    for (scene, w, h, depth, ao, r), G in ((a, 3), (a, 2), (b, 3), (a, 3)):
        full, _ = render_gpu(scene, w, h, depth, ao, True, root=r)
        got = _multi(scene, w, h, depth, ao, G, root=r)
        assert np.array_equal(got, full), (scene, G)


def test_mt19937_rows_past_two_to_the_32_draws():
    """MSVC's engine from far out in the serial stream (the host
    stream stopped at 2^32 draws): rows shaded through the multi-rank split
    with row bases moved 2^32 / 8 + 12,345 AO calls out (8 draws per call at AO
    4), so every draw lies beyond 2^32 -- the device generates them from the
    block jump-ahead's checkpoint windows -- against the oracle, which steps
    std::mt19937 itself to the rows' first draw."""
    import torch
    rt580 = helpers.rt580()
    lib = rt580.load()
    d = helpers.rt580_dist()
    scene, w, h, depth, ao = "simpleSphereScene.json", 48, 32, 2, 4
    rt = rt580.Raytracer(w, h, helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON(scene) == 0
    rt.set_depth(depth)
    rt.set_ao(ao, True)
    rt.set_rng(1)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    s = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    dev = torch.device("cuda", 0)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "stream")
    offset = (1 << 32) // 8 + 12345
    try:
        rows = d.GpuRows(rt580, params, torch, dev)
        cnt = rows.count(0, 1)[:h].to(torch.int64)
        base = torch.cumsum(cnt, 0) - cnt + offset
        fb = rows.shade(0, 1, base).view(h, w, 3).cpu().numpy()
        torch.cuda.synchronize()
    finally:
        lib.rt_gpu_set_stream(lib.rt_gpu_own_stream())
    ys = [y for y in range(h) if int(cnt[y])]
    assert ys and int(base[ys[0]]) * 8 > (1 << 32)
    px, calls, _, _ = helpers.oracle_render_segments(scene, w, h, depth, ao, [(y, 0, w) for y in ys],
                                                     [int(base[y]) for y in ys], engine=1)
    assert calls == [int(cnt[y]) for y in ys]
    for y, p in zip(ys, px):
        assert np.array_equal(fb[y], p), "row %d" % y
    rt.close()


def _registered_u8(n):
    span = (n + 4095) // 4096 * 4096
    raw = np.zeros(span + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    return raw, raw[off:off + span][:n], span


@pytest.mark.parametrize("G,transport", [(1, None), (2, None), (3, None), (1, "rccl")])
def test_render_multi_async_frames_are_the_ppm_bodies(G, transport):
    """rt_gpu_render_multi_async (bench.py's step for every N): frames of two
    configurations queued over a ring of three registered u8 buffers with no
    wait in between -- after a synchronize each buffer holds the PPM body of the
    last frame queued into it, byte-equal to the single-GPU render mapped by the
    reference's gamma LUT; G = 1 is rt_gpu_render_async_ppm; an unregistered
    buffer is refused."""
    rt580 = helpers.rt580()
    lib = rt580.load()
    root = helpers.synthetic_root("cornell10k")
    w, h = 53, 29
    cfg = [(4, 16), (2, 8)]
    lut = rt580.gamma_lut()
    want = []
    for d, a in cfg:
        full, _ = render_gpu("cornell10k.json", w, h, d, a, True, root=root)
        want.append(lut[full.astype(np.int64)].astype(np.uint8).reshape(-1))
    rts = []
    for d, a in cfg:
        rt = rt580.Raytracer(w, h, root)
        assert rt.LoadSceneJSON("cornell10k.json") == 0
        rt.set_depth(d)
        rt.set_ao(a, True)
        assert rt.InitializeRenderer() == 0
        rts.append((rt, rt.render_params()))
    s = rts[0][0].scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    devs = (ctypes.c_int * G)(*([0] * G))
    bufs = [_registered_u8(w * h * 3) for _ in range(3)]
    for _, buf, span in bufs:
        rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "host_register")
    old = os.environ.get("RT580_MULTI_TRANSPORT")
    if transport:
        os.environ["RT580_MULTI_TRANSPORT"] = transport
    try:
        for _, buf, _ in bufs:
            buf[:] = 7
        last = {}
        for i in range(10):
            k, b = i % 2, i % 3
            rt580.check(lib.rt_gpu_render_multi_async(ctypes.byref(rts[k][1]), bufs[b][1].ctypes.data, G, devs),
                        "rt_gpu_render_multi_async")
            last[b] = k
        rt580.check(lib.rt_gpu_synchronize(), "synchronize")
        for b, k in last.items():
            assert np.array_equal(bufs[b][1], want[k]), "buffer %d (config %d, G %d)" % (b, k, G)
        plain = np.zeros(w * h * 3, dtype=np.uint8)
        assert lib.rt_gpu_render_multi_async(ctypes.byref(rts[0][1]), plain.ctypes.data, G, devs) != 0
    finally:
        if transport:
            if old is None:
                del os.environ["RT580_MULTI_TRANSPORT"]
            else:
                os.environ["RT580_MULTI_TRANSPORT"] = old
        for _, buf, _ in bufs:
            lib.rt_gpu_host_unregister(buf.ctypes.data)
    for rt, _ in rts:
        rt.close()


@pytest.mark.parametrize("world,w,h", [(1, 64, 48), (3, 53, 29), (8, 1920, 1080)])
def test_deinterleave_ppm_into_registered_memory(world, w, h):
    """rt_gpu_deinterleave_ppm (rank 0's last step in rt580_dist.DistFrame): the
    u8 tiles of `world` interleaved row shares (tile r = rows r, r + world, ...,
    n_max rows, the last rows padding) land de-interleaved in a registered host
    range -- against numpy's de-interleave of the same random tiles; twice into
    the same range in call order; an unregistered buffer is refused."""
    import torch
    rt580 = helpers.rt580()
    lib = rt580.load()
    rt580.check(lib.rt_gpu_init(0), "init")
    n_max = (h + world - 1) // world
    g = torch.Generator().manual_seed(world * 1000 + w)
    tiles = [torch.randint(0, 256, (world, n_max, w, 3), dtype=torch.uint8, generator=g) for _ in range(2)]
    want = [t.transpose(0, 1).reshape(n_max * world, w, 3)[:h].numpy().reshape(-1) for t in tiles]
    dev = [t.cuda() for t in tiles]
    torch.cuda.synchronize()  # the tiles are on the device before the library's stream reads them
    raw, buf, span = _registered_u8(w * h * 3)
    rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "host_register")
    try:
        for k in (0, 1):
            rt580.check(lib.rt_gpu_deinterleave_ppm(dev[k].data_ptr(), world, n_max, w, h, buf.ctypes.data, None),
                        "rt_gpu_deinterleave_ppm")
        rt580.check(lib.rt_gpu_synchronize(), "synchronize")
        torch.cuda.synchronize()
        assert np.array_equal(buf, want[1])
        plain = np.zeros(w * h * 3, dtype=np.uint8)
        assert lib.rt_gpu_deinterleave_ppm(dev[0].data_ptr(), world, n_max, w, h, plain.ctypes.data, None) != 0
    finally:
        lib.rt_gpu_host_unregister(buf.ctypes.data)

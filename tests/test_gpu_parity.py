"""GPU parity: the HIP path (through the C ABI) against the reference's own
outputs (golden PPMs made by oracle/_ref from /root/reference, the reference's
committed output.ppm) and against the CPU restatement (oracle) on the same
inputs. Bit-exact PPM bytes are required (integer-quantized output; the
north_star's 1e-4 fp32 tolerance is below one 8-bit step)."""
import ctypes

import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu


def render_gpu(scene, w, h, depth, ao_samples, ao_enabled, rng=0, rows=None, root=helpers.ASSETS_ROOT):
    rt580 = helpers.rt580()
    rt = rt580.Raytracer(w, h, root)
    assert rt.LoadSceneJSON(scene) == 0
    rt.set_depth(depth)
    rt.set_ao(ao_samples, ao_enabled)
    rt.set_rng(rng)
    if rows:
        rt.set_rows(*rows)
    st = rt.Render("")
    assert st == 0, rt580.load().rt_gpu_last_error()
    fb, stats = rt.framebuffer(), rt.stats()
    rt.close()
    return fb, stats


@pytest.mark.parametrize("entry", helpers.golden_entries(True), ids=lambda e: e["name"])
def test_golden_small(entry):
    rng = 1 if entry["rng"] == "mt19937" else 0
    fb, _ = render_gpu(entry["scene"], entry["width"], entry["height"], entry["depth"],
                       entry["ao_samples"], entry["ao_enabled"], rng, root=helpers.entry_root(entry))
    got = helpers.rt580().ppm_bytes(fb)
    want = helpers.golden_ppm(entry)
    assert got == want, helpers.diff_summary(got, want)


def test_reference_output_ppm():
    """The reference's committed 580 Raytracer/output.ppm (mt19937, depth 0, AO 128)."""
    ro, want = helpers.reference_output_ppm()
    fb, st = render_gpu(ro["scene"], ro["width"], ro["height"], ro["depth"], ro["ao_samples"],
                        ro["ao_enabled"], rng=1)
    got = helpers.rt580().ppm_bytes(fb)
    assert got == want, helpers.diff_summary(got, want)
    assert st["rays_total"] == 20368711  # oracle count for this configuration


@pytest.mark.parametrize("entry", helpers.golden_entries(False), ids=lambda e: e["name"])
def test_golden_big_sha(entry):
    fb, st = render_gpu(entry["scene"], entry["width"], entry["height"], entry["depth"],
                        entry["ao_samples"], entry["ao_enabled"])
    got = helpers.rt580().ppm_bytes(fb)
    assert helpers.sha256(got) == entry["sha256"]
    if entry["name"].startswith("config2"):
        assert st["rays_total"] == 124827951
    if entry["name"].startswith("config1"):
        assert st["rays_total"] == 601801


@pytest.mark.parametrize("rows", [(0, 1), (5, 17), (30, 47), (46, 47)])
def test_row_subset_matches_full_frame(rows):
    full, _ = render_gpu("simpleSphereScene.json", 61, 47, 3, 8, True)
    part, _ = render_gpu("simpleSphereScene.json", 61, 47, 3, 8, True, rows=rows)
    assert np.array_equal(part[rows[0]:rows[1]], full[rows[0]:rows[1]])


@pytest.mark.parametrize("scene,w,h,depth,ao", [
    ("simpleSphereScene.json", 160, 120, 6, 32),
    ("scene.json", 96, 72, 3, 8),
    ("simpleSphereSceneAO.json", 128, 96, 8, 16),
    ("cornell10k.json", 96, 54, 4, 8),
    ("cornell10k.json", 40, 30, 8, 2),
    ("field100k.json", 32, 18, 4, 4),
])
def test_against_oracle(scene, w, h, depth, ao):
    root = helpers.synthetic_root(scene[:-5]) if scene.startswith(("cornell", "field")) else helpers.ASSETS_ROOT
    fb, st = render_gpu(scene, w, h, depth, ao, True, root=root)
    ref, cnt = helpers.oracle_render(scene, w, h, depth, ao, True, root=root)
    assert np.array_equal(fb, ref), "%d pixels differ" % int((fb != ref).any(axis=2).sum())
    for k in ("rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls"):
        assert st[k] == cnt[k], k


@pytest.mark.parametrize("world", [2, 3, 8])
def test_multi_rank_split_on_one_gpu(world):
    """The C-ABI split used across GPUs (rt_gpu_count_rows -> all-gather/scan ->
    rt_gpu_shade_rows) driven rank by rank on one device; the de-interleaved
    frame must equal the single-call render."""
    import torch
    rt580 = helpers.rt580()
    d = helpers.rt580_dist()
    scene, w, h, depth, ao = "simpleSphereScene.json", 97, 61, 4, 64
    full, _ = render_gpu(scene, w, h, depth, ao, True)
    rt = rt580.Raytracer(w, h, helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON(scene) == 0
    rt.set_depth(depth)
    rt.set_ao(ao, True)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    lib = rt580.load()
    s = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(s)), "upload")
    dev = torch.device("cuda", 0)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), "stream")
    backend = d.GpuRows(rt580, params, torch, dev)
    n_max = d.n_max_rows(h, world)
    counts = [backend.count(r, world).clone() for r in range(world)]
    full_counts = torch.stack(counts, dim=1).reshape(-1)[:h].to(torch.int64)
    base = torch.cumsum(full_counts, 0) - full_counts
    tiles = []
    for r in range(world):
        backend.count(r, world)                     # phase 1 again (phase 2 reuses its per-pixel data)
        lb = torch.zeros(n_max, dtype=torch.int64, device=dev)
        mine = base[r::world]
        lb[:mine.numel()] = mine
        # the one-kernel form used by DistFrame (rt_gpu_row_bases) gives the same bases
        gathered = torch.stack([c.to(torch.int32) for c in counts]).reshape(-1).contiguous()
        lb2 = backend.row_bases(gathered, r, world, torch.empty(n_max, dtype=torch.int64, device=dev))
        assert torch.equal(lb, lb2)
        tiles.append(backend.shade(r, world, lb).view(n_max, w, 3).clone())
    frame = torch.stack(tiles, dim=1).reshape(n_max * world, w, 3)[:h].cpu().numpy()
    rt580.check(lib.rt_gpu_set_stream(lib.rt_gpu_own_stream()), "stream")
    for r in range(world):
        rows = list(range(r, h, world))
        bad = [y for y in rows if not np.array_equal(frame[y], full[y])]
        assert not bad, "rank %d/%d: rows %s differ" % (r, world, bad[:10])
    assert np.array_equal(frame, full)


@pytest.mark.parametrize("scene,w,h,depth,ao", [
    ("cornell10k.json", 160, 90, 4, 16),
    ("field100k.json", 96, 54, 4, 8),
    ("field100k.json", 64, 36, 6, 4),
])
def test_bvh_equals_brute_force(scene, w, h, depth, ao):
    """The exact-semantics BVH path (default for triangle scenes) and the
    reference's brute-force scene loop give identical frames and ray counts."""
    lib = helpers.rt580().load()
    root = helpers.synthetic_root(scene[:-5])
    try:
        assert lib.rt_gpu_set_accel(0) == 0
        fb_b, st_b = render_gpu(scene, w, h, depth, ao, True, root=root)
        assert lib.rt_gpu_accel_active() == 0
    finally:
        assert lib.rt_gpu_set_accel(1) == 0
    fb_v, st_v = render_gpu(scene, w, h, depth, ao, True, root=root)
    assert lib.rt_gpu_accel_active() == 1
    assert np.array_equal(fb_b, fb_v), "%d pixels differ" % int((fb_b != fb_v).any(axis=2).sum())
    assert st_b["rays_total"] == st_v["rays_total"]


def test_gamma_u8_on_device_matches_ppm_writer():
    """rt_gpu_gamma_u8 (FlushFrameBufferToPPM's mapping before the multi-GPU
    gather) == the glibc-powf table of the host writer, over every channel value
    and on a rendered frame."""
    import torch
    rt580 = helpers.rt580()
    lib = rt580.load()
    assert lib.rt_gpu_init(0) == 0
    dev = torch.device("cuda", 0)
    assert lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) == 0
    vals = torch.arange(256, dtype=torch.int16, device=dev)
    out = torch.empty(256, dtype=torch.uint8, device=dev)
    assert lib.rt_gpu_gamma_u8(vals.data_ptr(), 256, out.data_ptr()) == 0
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), rt580.gamma_lut())
    fb, _ = render_gpu("simpleSphereScene.json", 64, 48, 2, 8, True)
    t = torch.from_numpy(np.ascontiguousarray(fb)).to(dev)
    o = torch.empty(t.numel(), dtype=torch.uint8, device=dev)
    assert lib.rt_gpu_set_stream(ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) == 0
    assert lib.rt_gpu_gamma_u8(t.data_ptr(), t.numel(), o.data_ptr()) == 0
    torch.cuda.synchronize()
    assert o.cpu().numpy().tobytes() == rt580.ppm_bytes(fb).split(b"\n", 3)[3]
    lib.rt_gpu_set_stream(lib.rt_gpu_own_stream())


def test_device_math_sequences_match_plain_operations():
    """The AO kernel's range-restricted sqrt/division sequences and its
    polynomial sincos with exact fallback give the same bits as the plain
    correctly rounded operations / glibc sincos (rt580_selftest_math): sqrt over
    every float in [2^-96, +inf], 2^26 random cases of each of the others."""
    rt580 = helpers.rt580()
    lib = rt580.load()
    assert lib.rt_gpu_init(0) == 0
    bad = (ctypes.c_uint64 * 4)()
    assert lib.rt580_selftest_math(580, 1 << 26, bad) == 0, lib.rt_gpu_last_error()
    assert list(bad) == [0, 0, 0, 0], "mismatches sqrt/div/normalize/aodir: %s" % list(bad)

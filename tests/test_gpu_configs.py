"""GPU parity at the defining parameters of BASELINE configs 4 and 5, and the
RNG stream past the minstd period.

* Config 4 (100k-triangle field, depth 6, 256 AO samples) and config 5 (1M
  triangles, depth 8, 256 AO samples) on small frames: the HIP path (exact BVH,
  the default for these scenes) against the CPU restatement (oracle/) on the
  same scene, and against the reference's own renders where one is committed
  (tests/golden/make_golden.py entries field100k_d6_ao256, field1m_d8_ao256).
  256 samples exercise the upper half of the per-sample RNG table
  (c_minstd_j1[128..255], Raytracer.cpp:317 with N = 256).
* The reference draws every AO sample from one minstd_rand0 stream
  (Raytracer.h:592, Raytracer.cpp:269-281). Config 5 needs ~5e10 draws, far
  past the period 2^31 - 2, so the stream wraps. The multi-rank entry points
  take absolute AO-call bases, which lets the test start a frame's rows just
  before the wrap (and many periods later) and compare with the oracle's
  rows at the same bases.
"""
import ctypes

import numpy as np
import pytest

import helpers
from test_gpu_parity import render_gpu

pytestmark = pytest.mark.gpu

PERIOD = 2147483646  # minstd_rand0 period (16807 is a primitive root mod 2^31 - 1)


@pytest.mark.parametrize("scene,w,h,depth,ao", [
    ("field100k.json", 16, 9, 6, 256),    # BASELINE config 4's depth and AO count
    ("field100k.json", 24, 14, 6, 64),
    ("field1m.json", 8, 5, 8, 256),       # BASELINE config 5's depth and AO count
])
def test_triangle_configs_against_oracle(scene, w, h, depth, ao):
    root = helpers.synthetic_root(scene[:-5])
    fb, st = render_gpu(scene, w, h, depth, ao, True, root=root)
    assert helpers.rt580().load().rt_gpu_accel_active() == 1  # the BVH path, as benchmarked
    ref, cnt = helpers.oracle_render(scene, w, h, depth, ao, True, root=root)
    assert np.array_equal(fb, ref), "%d pixels differ" % int((fb != ref).any(axis=2).sum())
    for k in ("rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls"):
        assert st[k] == cnt[k], k


@pytest.mark.parametrize("name", ["field100k_d6_ao256", "field1m_d8_ao256"])
def test_triangle_configs_against_reference_golden(name):
    entry = next((e for e in helpers.golden_entries(True) if e["name"] == name), None)
    if entry is None:
        pytest.skip("golden %s not generated yet (make_golden.py --only %s)" % (name, name))
    fb, _ = render_gpu(entry["scene"], entry["width"], entry["height"], entry["depth"],
                       entry["ao_samples"], entry["ao_enabled"], root=helpers.entry_root(entry))
    got = helpers.rt580().ppm_bytes(fb)
    assert got == helpers.golden_ppm(entry), helpers.diff_summary(got, helpers.golden_ppm(entry))


def _shade_with_bases(scene, w, h, depth, ao, offset_calls, root=helpers.ASSETS_ROOT):
    """Rows of a 1-rank frame whose AO-call numbering starts at offset_calls
    (as if that many AO calls preceded the frame in the serial stream): GPU
    through rt_gpu_count_rows / rt_gpu_shade_rows, and the oracle's rows."""
    import torch
    rt580 = helpers.rt580()
    d = helpers.rt580_dist()
    rt = rt580.Raytracer(w, h, root)
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
    try:
        backend = d.GpuRows(rt580, params, torch, dev)
        counts = backend.count(0, 1).to(torch.int64)
        base = torch.cumsum(counts, 0) - counts + offset_calls
        gpu = backend.shade(0, 1, base.clone()).view(h, w, 3).cpu().numpy()
    finally:
        rt580.check(lib.rt_gpu_set_stream(lib.rt_gpu_own_stream()), "stream")
    ora = helpers.OracleRows(scene, w, h, depth, ao, True, root=root)
    ocounts = ora.count(0, 1).to(torch.int64)
    assert torch.equal(ocounts, counts.cpu())
    obase = torch.cumsum(ocounts, 0) - ocounts + offset_calls
    cpu = ora.shade(0, 1, obase).view(h, w, 3).numpy()
    return gpu, cpu, int(counts.sum())


@pytest.mark.parametrize("ao,periods", [(64, 1), (256, 1), (256, 23)])
def test_rng_stream_wraps_past_the_minstd_period(ao, periods):
    """Draw indices cross k * (2^31 - 2) inside the frame: the device's
    modular skip-ahead (rank_kernel: seed * step^call, step = 16807^(2N)) and per-sample table must agree with the
    oracle's serial-stream semantics on both sides of the wrap. periods=23 puts
    the frame near draw 4.9e10, where BASELINE config 5's last rows are."""
    scene, w, h, depth = "simpleSphereScene.json", 40, 30, 4
    per_call = 2 * ao
    # start the frame so that the wrap falls in its middle
    _, _, calls = _shade_with_bases(scene, w, h, depth, ao, 0)
    wrap_call = (periods * PERIOD) // per_call
    offset = max(wrap_call - calls // 2, 0)
    assert offset * per_call < periods * PERIOD < (offset + calls) * per_call
    gpu, cpu, _ = _shade_with_bases(scene, w, h, depth, ao, offset)
    assert np.array_equal(gpu, cpu), "%d pixels differ" % int((gpu != cpu).any(axis=2).sum())
    # and the shifted stream really changes the image (the offset is not ignored)
    base_gpu, _, _ = _shade_with_bases(scene, w, h, depth, ao, 0)
    assert not np.array_equal(gpu, base_gpu)

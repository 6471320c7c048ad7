"""GPU parity of the chunked passes that only full-resolution triangle frames
reach by default.

BVH frames run the far-hit queue of each trace level, and the AO samples
(CalculateAmbientOcclusion, Raytracer.cpp:315-330: one RNG draw pair and one
IntersectScene per sample), in chunks of at most 2^27 rays. A 1080p-8K frame
crosses those boundaries; the small frames of the other parity tests never do.
rt580_set_chunk_log2 lowers the limit so that small frames run the same code
over many chunks: a level's rays split across chunks (far queue, shadow flags,
brute-scan split), one AO call's samples split across AO chunks (occlusion
counts and per-call acceptor hints accumulate across them). The frame must
stay byte-identical to the CPU restatement (oracle/), and its ray counters
equal.
"""
import functools

import numpy as np
import pytest

import helpers

pytestmark = pytest.mark.gpu

DEFAULT_LOG2 = 27


@functools.lru_cache(None)
def _oracle(scene, w, h, depth, ao):
    root = helpers.synthetic_root(scene[:-5])
    return helpers.oracle_render(scene, w, h, depth, ao, True, root=root)


def _render_chunked(scene, w, h, depth, ao, log2s):
    """Render the frame once per chunk limit in log2s (one scene upload) ->
    [(framebuffer, stats)]."""
    rt580 = helpers.rt580()
    lib = rt580.load()
    assert lib.rt_gpu_init(0) == 0
    rt = rt580.Raytracer(w, h, helpers.synthetic_root(scene[:-5]))
    assert rt.LoadSceneJSON(scene) == 0
    rt.set_depth(depth)
    rt.set_ao(ao, True)
    res = []
    try:
        for log2 in log2s:
            assert lib.rt580_set_chunk_log2(log2) == 0, lib.rt_gpu_last_error()
            assert rt.Render("") == 0, lib.rt_gpu_last_error()
            assert lib.rt_gpu_accel_active() == 1  # the chunked BVH path
            res.append((rt.framebuffer(), rt.stats()))
    finally:
        assert lib.rt580_set_chunk_log2(DEFAULT_LOG2) == 0
        rt.close()
    return res


@pytest.mark.parametrize("scene,w,h,depth,ao,log2", [
    ("field100k.json", 24, 14, 6, 64, 6),     # 336 camera rays -> 6 trace chunks per level
    ("field100k.json", 24, 14, 6, 64, 10),
    ("cornell10k.json", 96, 54, 4, 64, 10),   # config 3's depth and AO count
    ("cornell10k.json", 96, 54, 4, 64, DEFAULT_LOG2),
])
def test_chunked_frames_match_oracle(scene, w, h, depth, ao, log2):
    (fb, st), = _render_chunked(scene, w, h, depth, ao, [log2])
    ref, cnt = _oracle(scene, w, h, depth, ao)
    assert np.array_equal(fb, ref), "%d pixels differ" % int((fb != ref).any(axis=2).sum())
    for k in ("rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls"):
        assert st[k] == cnt[k], k
    if log2 < DEFAULT_LOG2:
        assert st["ao_calls"] * ao > 4 << log2  # many AO chunks
        if log2 == 6:
            assert st["rays_primary"] > 2 << log2  # level 0 spans several trace chunks


@pytest.mark.parametrize("name,log2", [
    ("field100k_d6_ao256", 6),   # config 4's depth and AO count; each call's 256 samples span 4 chunks
    ("field1m_d8_ao256", 6),     # config 5's depth and AO count
    ("field1m_d8_ao256", 10),
])
def test_chunked_frames_match_reference_golden(name, log2):
    """Against the reference's own render (oracle/_ref, made in the build
    container); counters against the same frame in one chunk."""
    e = next(e for e in helpers.golden_entries(True) if e["name"] == name)
    args = (e["scene"], e["width"], e["height"], e["depth"], e["ao_samples"])
    (fb, st), (fb1, st1) = _render_chunked(*args, [log2, DEFAULT_LOG2])
    got = helpers.rt580().ppm_bytes(fb)
    assert got == helpers.golden_ppm(e), helpers.diff_summary(got, helpers.golden_ppm(e))
    assert np.array_equal(fb, fb1)
    for k in ("rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls"):
        assert st[k] == st1[k], k
    assert st["ao_calls"] * e["ao_samples"] > 4 << log2


def test_chunk_limit_is_validated():
    lib = helpers.rt580().load()
    assert lib.rt_gpu_init(0) == 0
    assert lib.rt580_set_chunk_log2(5) != 0
    assert lib.rt580_set_chunk_log2(28) != 0
    assert lib.rt580_set_chunk_log2(DEFAULT_LOG2) == 0

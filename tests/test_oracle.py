"""The CPU restatement (oracle/) pinned against the reference's own outputs:
golden PPMs produced by the reference binary (tests/golden/make_golden.py),
the reference's committed output.ppm, and the BASELINE hashes."""
import filecmp
import os
import subprocess

import numpy as np
import pytest

import helpers


@pytest.mark.parametrize("entry", helpers.golden_entries(True), ids=lambda e: e["name"])
def test_oracle_matches_reference_golden(entry):
    rng = 1 if entry["rng"] == "mt19937" else 0
    fb, _ = helpers.oracle_render(entry["scene"], entry["width"], entry["height"], entry["depth"],
                                  entry["ao_samples"], entry["ao_enabled"], rng, root=helpers.entry_root(entry))
    got = helpers.rt580().ppm_bytes(fb)
    assert got == helpers.golden_ppm(entry), helpers.diff_summary(got, helpers.golden_ppm(entry))


def test_oracle_matches_reference_output_ppm():
    ro, want = helpers.reference_output_ppm()
    fb, cnt = helpers.oracle_render(ro["scene"], ro["width"], ro["height"], ro["depth"],
                                    ro["ao_samples"], ro["ao_enabled"], engine=1)
    assert helpers.rt580().ppm_bytes(fb) == want
    assert cnt["rays_total"] == 20368711


@pytest.mark.parametrize("name", ["config1_500_d1_aooff", "main_500_d4_ao128"])
def test_oracle_big_hashes(name):
    e = next(x for x in helpers.golden_entries(False) if x["name"] == name)
    fb, cnt = helpers.oracle_render(e["scene"], e["width"], e["height"], e["depth"],
                                    e["ao_samples"], e["ao_enabled"])
    assert helpers.sha256(helpers.rt580().ppm_bytes(fb)) == e["sha256"]
    if name.startswith("config1"):
        assert cnt["rays_total"] == 601801


def test_oracle_row_subsets_and_threads_agree():
    full, c1 = helpers.oracle_render("simpleSphereScene.json", 64, 40, 4, 8, True, threads=1)
    full8, c8 = helpers.oracle_render("simpleSphereScene.json", 64, 40, 4, 8, True, threads=8)
    assert np.array_equal(full, full8) and c1 == c8
    part, _ = helpers.oracle_render("simpleSphereScene.json", 64, 40, 4, 8, True, rows=(13, 29))
    assert np.array_equal(part, full[13:29])


@pytest.mark.parametrize("name", ["teapots_d2_ao4", "cornell10k_d4_ao4", "sss_d4_ao16"])
def test_oracle_faithful_mode_matches_golden(name):
    """The ref-faithful cost model (per-call model matrix, unused Inverse and
    TransformPoint per test; the CPU baseline) gives the golden bytes too."""
    e = next(x for x in helpers.golden_entries(True) if x["name"] == name)
    fb, c_f = helpers.oracle_render(e["scene"], e["width"], e["height"], e["depth"], e["ao_samples"],
                                    e["ao_enabled"], root=helpers.entry_root(e), faithful=True)
    assert helpers.rt580().ppm_bytes(fb) == helpers.golden_ppm(e)
    _, c_h = helpers.oracle_render(e["scene"], e["width"], e["height"], e["depth"], e["ao_samples"],
                                   e["ao_enabled"], root=helpers.entry_root(e))
    assert c_f == c_h


@pytest.mark.skipif(not os.path.isdir(helpers.REFERENCE), reason="reference not mounted")
def test_scene_fixtures_are_the_reference_assets():
    ref = os.path.join(helpers.REFERENCE, "Assets")
    for f in os.listdir(ref):
        assert filecmp.cmp(os.path.join(ref, f), os.path.join(helpers.GOLDEN, "Assets", f), shallow=False), f


@pytest.mark.parametrize("p0,n", [(0, 24 * 18), (24 * 5 + 7, 100)])
def test_time_prefix_is_the_frames_pixels(p0, n):
    """bench.py's CPU-baseline timer (oracle_time_prefix: an exact raster range of
    the full frame with the RNG at the range's AO-call base) gives exactly the
    frame's pixels and rays, serially (the reference's loop, ref-faithful cost
    model) and split over threads (count pass, scan, shade)."""
    w, h, d, ao = 24, 18, 4, 8
    full, _ = helpers.oracle_render("simpleSphereScene.json", w, h, d, ao, True)
    calls = []
    for y in range(h):  # AO calls per pixel of the frame (raster order)
        cnt = helpers.oracle_render("simpleSphereScene.json", w, h, d, ao, True, rows=(y, y + 1))[1]
        calls.append(cnt["ao_calls"])
    # the base of p0 from per-row counts + the pixels of p0's row before it
    y0, x0 = divmod(p0, w)
    base = sum(calls[:y0])
    if x0:
        part = helpers.oracle_time_prefix("simpleSphereScene.json", w, h, d, ao, y0 * w, x0, faithful=False)[1]
        base += part["ao_calls"]
    want = full.reshape(-1, 3)[p0:p0 + n]
    for faithful, threads in ((True, 1), (False, 1), (False, 4)):
        fb, cnt, _ = helpers.oracle_time_prefix("simpleSphereScene.json", w, h, d, ao, p0, n, threads=threads,
                                                call_base=base, faithful=faithful)
        assert fb.shape == want.shape and (fb == want).all(), (faithful, threads)
        assert cnt["rays_primary"] == n
    # the serial timer stops at its budget
    fb, cnt, _ = helpers.oracle_time_prefix("simpleSphereScene.json", w, h, d, ao, 0, w * h, budget_s=0.0)
    assert len(fb) == 1 and cnt["rays_primary"] == 1


@pytest.mark.parametrize("scene,root_name,w,h,d,ao", [
    ("simpleSphereScene.json", None, 40, 30, 4, 8),
    ("cornell10k.json", "cornell10k", 24, 14, 3, 4),
])
def test_render_segments_are_the_frames_pixels(scene, root_name, w, h, d, ao):
    """bench.py's frame check (oracle_render_segments: pixel segments of rows of
    the full frame, each row's RNG base given, threaded) gives exactly the
    frame's pixels, and each row's AO-call total."""
    root = helpers.synthetic_root(root_name) if root_name else helpers.ASSETS_ROOT
    full, _ = helpers.oracle_render(scene, w, h, d, ao, True, root=root)
    calls = [helpers.oracle_render(scene, w, h, d, ao, True, rows=(y, y + 1), root=root)[1]["ao_calls"]
             for y in range(h)]
    base = np.concatenate([[0], np.cumsum(calls)[:-1]]).astype(np.uint64)
    segs = [(h // 2, 0, w), (h - 1, 3, w - 5), (h // 3, w // 2, w - w // 2), (h // 2 + 1, 1, 1)]
    got, row_calls, cnt, _ = helpers.oracle_render_segments(scene, w, h, d, ao, segs, [base[y] for y, _, _ in segs],
                                                            threads=4, root=root)
    for (y, x0, n), px in zip(segs, got):
        assert np.array_equal(px, full[y, x0:x0 + n]), (y, x0, n)
    assert row_calls == [calls[y] for y, _, _ in segs]
    assert cnt["rays_primary"] == sum(n for _, _, n in segs)


def test_simd_triangle_scan_matches_scalar_loop():
    """The 16-wide hoisted triangle scan (AVX-512, used when the CPU has it)
    and the scalar loop give the same frame and rays (ORACLE_SCALAR=1 in a
    child process selects the scalar loop)."""
    import json
    import sys
    root = helpers.synthetic_root("cornell10k")
    code = ("import sys, json; sys.path.insert(0, %r); import helpers; "
            "fb, c = helpers.oracle_render('cornell10k.json', 32, 18, 4, 8, True, root=%r); "
            "print(json.dumps([helpers.sha256(fb.tobytes()), c]))" % (os.path.join(helpers.REPO, "tests"), root))
    outs = []
    for scalar in ("0", "1"):
        env = dict(os.environ)
        env.pop("ORACLE_SCALAR", None)
        if scalar == "1":
            env["ORACLE_SCALAR"] = "1"
        p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=600)
        assert p.returncode == 0, p.stderr
        outs.append(json.loads(p.stdout.strip().splitlines()[-1]))
    assert outs[0] == outs[1]


def test_oracle_segments_mt19937_window_equals_full_stream():
    """oracle_render_segments with engine 1 generates only its rows' draws
    (std::mt19937 discard to the first): the rows equal oracle_render's full
    frame from draw 0 (the GPU test past 2^32 draws compares against this mode)."""
    scene, w, h, depth, ao = "simpleSphereScene.json", 40, 30, 2, 4
    full, _ = helpers.oracle_render(scene, w, h, depth, ao, True, engine=1)
    calls = []
    for y in range(h):
        _, c, _, _ = helpers.oracle_render_segments(scene, w, h, depth, ao, [(y, 0, w)], [0])
        calls.append(c[0])
    base = np.concatenate([[0], np.cumsum(calls)[:-1]]).astype(np.uint64)
    rows = [y for y in range(h) if calls[y]][-6:]
    px, c2, _, _ = helpers.oracle_render_segments(scene, w, h, depth, ao, [(y, 0, w) for y in rows],
                                                  [int(base[y]) for y in rows], engine=1)
    assert c2 == [calls[y] for y in rows]
    for y, p in zip(rows, px):
        assert np.array_equal(p, full[y]), y

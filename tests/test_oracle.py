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


def test_time_pixels_counts_the_frames_rays():
    """bench.py's CPU-baseline sampler (oracle_time_pixels: listed pixels of the
    full frame) traces exactly the rays oracle_render traces for those pixels,
    in both cost modes (only the RNG position differs, not the work)."""
    w, h = 24, 18
    _, want = helpers.oracle_render("simpleSphereScene.json", w, h, 4, 8, True)
    pts = [(x, y) for y in range(h) for x in range(w)]
    for faithful in (False, True):
        got = helpers.oracle_time_pixels("simpleSphereScene.json", w, h, 4, 8, pts, threads=4, faithful=faithful)
        assert got == want

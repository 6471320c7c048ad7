"""Full-frame parity at the target sizes: the north-star frame
(the 100k-triangle field, 1920x1080, depth 4, AO 64) and BASELINE config 3 (the
10k Cornell box, 1920x1080, depth 4, AO 64), rendered in full on the HIP path
(Render(): trace levels, AO in 2^27-sample chunks, far passes, resolve) and
compared byte for byte with the oracle's render of the same frame: the sha256
of the whole PPM, and, on a mismatch, which bands of 108 rows differ.

The oracle (oracle/rt_oracle.cpp, pinned to the reference's own renders by
tests/test_oracle.py) rendered these frames once in the build container:
tests/golden/make_fullframe.py -> tests/golden/fullframe.json (the reference
itself would need days of CPU for them). Reference: Raytracer.cpp:916-935."""
import hashlib
import json
import os

import pytest

import helpers
from test_gpu_parity import render_gpu

pytestmark = pytest.mark.gpu

FULLFRAME = os.path.join(helpers.REPO, "tests", "golden", "fullframe.json")


def _entries():
    if not os.path.exists(FULLFRAME):
        return []
    return sorted(json.load(open(FULLFRAME)).items())


@pytest.mark.parametrize("name,entry", _entries(), ids=[n for n, _ in _entries()])
def test_full_frame_matches_oracle(name, entry):
    root = helpers.synthetic_root(entry["assets"])
    fb, st = render_gpu(entry["scene"], entry["width"], entry["height"], entry["depth"], entry["ao_samples"],
                        entry["ao_enabled"], root=root)
    assert helpers.rt580().load().rt_gpu_accel_active() == 1  # the BVH path, as benchmarked
    ppm = helpers.rt580().ppm_bytes(fb)
    body = ppm[len(ppm) - entry["width"] * entry["height"] * 3:]
    row = entry["width"] * 3
    band = entry["band_rows"]
    bad = [r for r, want in zip(range(0, entry["height"], band), entry["band_sha256"])
           if hashlib.sha256(body[r * row:min(entry["height"], r + band) * row]).hexdigest() != want]
    assert not bad, "bands (first row) differing from the oracle: %s" % bad
    assert helpers.sha256(ppm) == entry["sha256"]
    assert st["rays_total"] == entry["rays_total"]
    assert st["rays_ao"] == entry["rays_ao"]
    assert st["ao_calls"] == entry["ao_calls"]


def test_fullframe_fixture_covers_the_target_frames():
    names = [n for n, _ in _entries()]
    assert "north_star" in names and "config3" in names, names

"""Scene ingest edge cases (LoadSceneJSON / LoadMesh, Raytracer.cpp:589-779)
against the reference's own behaviour on the same files
(tests/golden/loader/, made by tests/golden/make_loader_goldens.py with the
reference binary): malformed and unusual numbers, wrong JSON types, the mesh
type read from data[0] only, unsupported mesh types, missing/malformed mesh
files, duplicate keys, BOM, a file without "scene". CPU: the load status;
GPU: the render of every case the reference loads (8x6, depth 1, AO off)."""
import json
import os

import pytest

import helpers

LOADER = os.path.join(helpers.GOLDEN, "loader")
MANIFEST = json.load(open(os.path.join(LOADER, "manifest.json")))
CASES = MANIFEST["cases"]


def _load(case):
    rt = helpers.rt580().Raytracer(8, 6, LOADER)
    st = rt.LoadSceneJSON(case["file"])
    return rt, st


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_load_status_matches_reference(case):
    rt, st = _load(case)
    want = 0 if case["load_ok"] else case["load_status"]
    assert st == want
    rt.close()


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_oracle_loader_matches_reference(case):
    """The CPU restatement's own JSON reader/loader (oracle/ora_json.h, shared
    with nothing in the product) on the same cases: status, and the render."""
    import numpy as np
    lib = helpers.oracle_lib()
    r = MANIFEST["render"]
    fb = np.zeros((r["height"], r["width"], 3), dtype=np.int16)
    cnt = np.zeros(6, dtype=np.uint64)
    st = lib.oracle_render(os.fsencode(LOADER), os.fsencode(case["file"]), r["width"], r["height"], r["depth"], 128,
                           int(r["ao_enabled"]), 0, 1, 0, r["height"], fb.ctypes.data, cnt.ctypes.data, None)
    assert (st == 0) == case["load_ok"]
    if case.get("ppm_sha256"):
        assert helpers.sha256(helpers.rt580().ppm_bytes(fb)) == case["ppm_sha256"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", [c for c in CASES if c.get("ppm_sha256")], ids=lambda c: c["name"])
def test_loaded_case_renders_like_reference(case):
    rt, st = _load(case)
    assert st == 0
    r = MANIFEST["render"]
    rt.set_depth(r["depth"])
    rt.set_ao(128, r["ao_enabled"])
    assert rt.Render("") == 0
    got = helpers.rt580().ppm_bytes(rt.framebuffer())
    assert helpers.sha256(got) == case["ppm_sha256"]
    rt.close()


@pytest.mark.parametrize("what,old,new", [
    ("material field", '"Kd": 0.7, ', ""),
    ("material", '"material": {"Cs": [1, 0.2, 0.2], "Ka": 0.4, "Kd": 0.7, "Ks": 0.3, "Kt": 0, "n": 20}, ', ""),
    ("camera field", '"bounds": [0.1, 100, 1, -1, 1, -1], ', ""),
    ("light field", '"intensity": 0.8, ', ""),
    ("light type", '"type": "directional"', '"type": "spot"'),
    ("vertex normal", None, None),
])
def test_undefined_reference_cases_fail_cleanly(tmp_path, what, old, new):
    """Where the reference's behaviour is undefined (a missing key read from a
    const nlohmann::json; an unknown light type leaves lightType
    uninitialised), the loader returns RT_FAILURE instead."""
    assets = tmp_path / "Assets"
    assets.mkdir()
    for f in os.listdir(os.path.join(LOADER, "Assets")):
        (assets / f).write_bytes(open(os.path.join(LOADER, "Assets", f), "rb").read())
    base = (assets / "case_base.json").read_text()
    if old is None:  # a mesh vertex without "n"
        mesh = (assets / "ltwo.json").read_text().replace('"n": [0, 0, 1], ', "", 1)
        (assets / "ltwo.json").write_text(mesh)
        text = (assets / "case_type_on_first_item_only.json").read_text()
    else:
        assert old in base
        text = base.replace(old, new, 1)
    (assets / "x.json").write_text(text)
    rt = helpers.rt580().Raytracer(8, 6, str(tmp_path))
    assert rt.LoadSceneJSON("x.json") == 1
    rt.close()

"""The drop-in from C++: the reference's own main() (Raytracer.cpp:944-953)
compiled unchanged against include/Raytracer.h and linked with lib580rt.so, and
the product's PPM writer (FlushFrameBufferToPPM, Raytracer.cpp:796-830) checked
on the file it writes. The compile/link leg runs on the CPU; running it needs
the GPU."""
import os
import subprocess

import pytest

import helpers

NATIVE = os.path.join(helpers.REPO, "tests", "native")


def build_ref_main(out_dir):
    exe = os.path.join(out_dir, "ref_main")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(helpers.REPO, "include"),
                    "-o", exe, os.path.join(NATIVE, "ref_main.cpp"),
                    "-L", helpers.PKG, "-l580rt", "-Wl,-rpath," + helpers.PKG], check=True)
    return exe


def assets_dir(tmp_path):
    os.symlink(os.path.join(helpers.GOLDEN, "Assets"), tmp_path / "Assets")
    return tmp_path


def test_reference_main_compiles_and_links_against_dropin(tmp_path):
    exe = build_ref_main(str(tmp_path))
    assert os.path.exists(exe)
    nm = subprocess.run(["nm", "-D", "--defined-only", os.path.join(helpers.PKG, "lib580rt.so")],
                        capture_output=True, text=True, check=True).stdout
    for sym in ("_ZN9Raytracer13LoadSceneJSONENSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEE",
                "_ZN9Raytracer6RenderENSt7__cxx1112basic_stringIcSt11char_traitsIcESaIcEEE"):
        assert sym in nm, sym


@pytest.mark.gpu
def test_reference_main_writes_the_reference_ppm(tmp_path):
    """Raytracer rt(500,500); LoadSceneJSON("simpleSphereScene.json");
    Render("output.ppm") -> output.ppm byte-identical to the reference's own
    run of the same main() (golden main_500_d4_ao128: depth 4, AO 128)."""
    exe = build_ref_main(str(tmp_path))
    cwd = assets_dir(tmp_path)
    p = subprocess.run([exe], cwd=cwd, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert "Scene parsing completed!" in p.stdout  # Raytracer.cpp:772 prints to stdout
    want = next(e for e in helpers.golden_entries(False) if e["name"] == "main_500_d4_ao128")["sha256"]
    data = open(os.path.join(cwd, "output.ppm"), "rb").read()
    assert helpers.sha256(data) == want


@pytest.mark.gpu
def test_c_abi_render_writes_the_golden_file(tmp_path):
    """rt580_render(h, path) -> Render(path) -> FlushFrameBufferToPPM(path)."""
    entry = next(e for e in helpers.golden_entries(True) if e["name"] == "teapots_d2_ao4")
    rt = helpers.rt580().Raytracer(entry["width"], entry["height"], helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON(entry["scene"]) == 0
    rt.set_depth(entry["depth"])
    rt.set_ao(entry["ao_samples"], entry["ao_enabled"])
    out = str(tmp_path / "out.ppm")
    assert rt.Render(out) == 0
    assert open(out, "rb").read() == helpers.golden_ppm(entry)
    out2 = str(tmp_path / "again.ppm")
    assert rt.FlushFrameBufferToPPM(out2) == 0
    assert open(out2, "rb").read() == helpers.golden_ppm(entry)
    assert rt.FlushFrameBufferToPPM(str(tmp_path / "no" / "such" / "dir.ppm")) == 1  # RT_FAILURE (:803-806)
    rt.close()

"""The C-ABI library loads on CPU, exports every symbol include/rt580.h
declares, and its host side (scene ingest / flattening / PPM writer) behaves
like the reference's — no GPU compute is called here."""
import ctypes
import os
import re

import numpy as np
import pytest

import helpers


def declared_symbols():
    text = open(os.path.join(helpers.REPO, "include", "rt580.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_gpu_\w+|rt580_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    rt580 = helpers.rt580()
    lib = rt580.load()
    names = declared_symbols()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert {n for n, _, _ in rt580.SIGNATURES} == set(names)


def test_struct_sizes_match_header(tmp_path):
    """ctypes mirrors == the C layout of include/rt580.h (compiled here with gcc)."""
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text('#include "rt580.h"\n#include <stdio.h>\nint main(){printf("%zu %zu %zu",'
                   'sizeof(rt_render_params),sizeof(rt_prim),sizeof(rt_render_stats));return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(helpers.REPO, "include"), "-o", str(exe), str(src)], check=True)
    sizes = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split()]
    rt580 = helpers.rt580()
    assert sizes == [ctypes.sizeof(rt580.RenderParams), ctypes.sizeof(rt580.Prim), ctypes.sizeof(rt580.RenderStats)]


@pytest.mark.parametrize("scene,n_prims,n_tri,n_lights", [
    ("simpleSphereScene.json", 5, 2, 2),
    ("scene.json", 4 * 1024, 4 * 1024, 2),
    ("simpleScene.json", 1, 1, 2),
])
def test_scene_ingest_and_flattening(scene, n_prims, n_tri, n_lights):
    rt = helpers.rt580().Raytracer(64, 48, helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON(scene) == 0
    s = rt.scene()
    assert s.n_prims == n_prims and s.n_lights == n_lights
    kinds = [s.prims[i].kind for i in range(s.n_prims)]
    assert kinds.count(0) == n_tri
    rt.close()


def test_plane_mesh_is_empty_polygon_and_missing_mesh_fails(tmp_path):
    assets = tmp_path / "Assets"
    assets.mkdir()
    src = os.path.join(helpers.GOLDEN, "Assets")
    for f in ("1plane.json", "1sphere.json"):
        (assets / f).write_bytes(open(os.path.join(src, f), "rb").read())
    shape = '{"id":"%s","geometry":"%s","material":{"Cs":[1,0,0],"Ka":0.5,"Kd":0.5,"Ks":0,"Kt":0,"n":2},' \
            '"transforms":[{"T":[0,0,0]}]}'
    cam = '"camera":{"from":[0,0,5],"to":[0,0,0],"bounds":[1,2,3,4,5,6],"resolution":[8,8]}'
    (assets / "p.json").write_text('{"scene":{"shapes":[%s,%s],"lights":[],%s}}' % (
        shape % ("a", "1plane"), shape % ("b", "1sphere"), cam))
    (assets / "m.json").write_text('{"scene":{"shapes":[%s],"lights":[],%s}}' % (shape % ("a", "nosuch"), cam))
    rt = helpers.rt580().Raytracer(8, 8, str(tmp_path))
    assert rt.LoadSceneJSON("p.json") == 0
    s = rt.scene()
    assert s.n_prims == 1 and s.prims[0].kind == 1  # the plane contributes no primitive
    assert rt.LoadSceneJSON("m.json") == 1           # RT_FAILURE, like LoadMesh (Raytracer.cpp:597-599)
    assert rt.LoadSceneJSON("absent.json") == 1
    rt.close()


def test_camera_constants_match_reference_arithmetic():
    rt = helpers.rt580().Raytracer(1920, 1080, helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON("simpleSphereScene.json") == 0
    assert rt.InitializeRenderer() == 0
    p = rt.render_params()
    assert p.view_inverse_ok == 1
    f32 = np.float32
    aspect = f32(1920) / f32(1080)
    half = f32(np.float64(f32(30.0)) * (3.14159265 / 180))
    tn = np.tan(np.float64(half))
    assert p.ndc_ky == tn and p.ndc_kx == np.float64(aspect) * tn
    assert p.ao_angle_max == f32(2 * 3.14159265)
    assert list(p.cam_from) == [0.0, 2.5, 10.0]


def test_ppm_writer_matches_oracle(tmp_path):
    rng = np.random.default_rng(580)
    fb = rng.integers(0, 256, size=(7, 11, 3)).astype(np.int16)
    lib = helpers.oracle_lib()
    lib.oracle_write_ppm.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    path = str(tmp_path / "o.ppm")
    assert lib.oracle_write_ppm(path.encode(), 11, 7, np.ascontiguousarray(fb).ctypes.data) == 0
    assert helpers.rt580().ppm_bytes(fb) == open(path, "rb").read()


def test_render_without_gpu_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    rt = helpers.rt580().Raytracer(8, 8, helpers.ASSETS_ROOT)
    assert rt.LoadSceneJSON("simpleSphereScene.json") == 0
    assert rt.Render("") == 1  # RT_FAILURE, no abort
    rt.close()


_ONE_RUNTIME_CHILD = r"""
import ctypes, os, sys
sys.path.insert(0, sys.argv[1])
import helpers
helpers.rt580().load()
ctypes.CDLL("librccl.so.1", mode=ctypes.RTLD_GLOBAL)  # what rt_shim.cpp rccl_load() opens
import torch
maps = open("/proc/self/maps").read().splitlines()
libs = sorted({l.split()[-1] for l in maps if "librccl" in l or "libamdhip64" in l})
print("LIBS", libs)
"""


def test_one_hip_runtime_and_one_rccl_per_process(tmp_path):
    """The binding loads lib580rt.so after torch (when installed), so the
    library's libamdhip64.so.7 and its dlopen("librccl.so.1") bind to torch's
    bundled copies and a later `import torch` adds none: two RCCL copies in one
    process (the library's first, torch's after it) ended the GPU suite with
    "double free or corruption" at exit. Runs without a GPU."""
    import subprocess
    import sys
    script = tmp_path / "child.py"
    script.write_text(_ONE_RUNTIME_CHILD)
    r = subprocess.run([sys.executable, str(script), os.path.dirname(os.path.abspath(__file__))],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("LIBS")]
    assert line, r.stdout
    import ast
    libs = ast.literal_eval(line[0][5:])
    assert sum("librccl" in l for l in libs) <= 1 and sum("libamdhip64" in l for l in libs) == 1, libs

"""The library's RT580_* environment switches are validated at rt_gpu_init
(csrc/rt_knobs.cpp): an unknown RT580_* name or a value outside a switch's
set fails with RT_FAILURE and a message, before any GPU call. Runs on CPU:
without a GPU a valid environment gets as far as the device query."""
import os
import subprocess
import sys

import pytest

import helpers

PROBE = r"""
import sys
sys.path.insert(0, %r)
import helpers
lib = helpers.rt580().load()
st = lib.rt_gpu_init(0)
print(st, (lib.rt_gpu_last_error() or b"").decode())
""" % os.path.join(helpers.REPO, "tests")


def _init_with(env):
    e = {k: v for k, v in os.environ.items() if not k.startswith("RT580_")}
    e.update(env)
    p = subprocess.run([sys.executable, "-c", PROBE], capture_output=True, text=True, env=e, timeout=300)
    assert p.returncode == 0, p.stderr
    st, _, msg = p.stdout.strip().splitlines()[-1].partition(" ")
    return int(st), msg


@pytest.mark.parametrize("env,why", [
    ({"RT580_NO_SUCH_SWITCH": "1"}, "unknown environment switch RT580_NO_SUCH_SWITCH"),
    ({"RT580_SLOTS": "5"}, "RT580_SLOTS=5: not one of the supported values"),
    ({"RT580_PIPELINE": "x"}, "not an integer"),
    ({"RT580_CHUNK_LOG2": "28"}, "RT580_CHUNK_LOG2=28: outside [6, 27]"),
    ({"RT580_MULTI_TRANSPORT": "tcp"}, "not one of the supported values"),
    ({"RT580_DUMP_FAR": "/tmp/x"}, "diagnostic builds only"),
    # kernel-form switches of earlier rounds, removed with their forms
    ({"RT580_AO_VARIANT": "39948"}, "unknown environment switch RT580_AO_VARIANT"),
    ({"RT580_LATE_WPE": "8"}, "unknown environment switch RT580_LATE_WPE"),
])
def test_bad_switch_fails_init(env, why):
    st, msg = _init_with(env)
    assert st == 1 and why in msg, msg


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU would initialise")
def test_valid_switches_pass_validation():
    st, msg = _init_with({"RT580_SLOTS": "2", "RT580_CHUNK_LOG2": "10", "RT580_EXHAUSTIVE": "1",
                          "RT580_REPLAY": "0", "RT580_GRID_COARSE_PX": "0"})
    assert st == 1 and "no HIP device" in msg, msg


def test_every_switch_is_documented():
    """INTEGRATION.md's switch table lists every RT580_* name the library
    validates (csrc/rt_knobs.cpp), so no accepted switch is undocumented."""
    import re
    src = open(os.path.join(helpers.PKG, "csrc", "rt_knobs.cpp")).read()
    names = set(re.findall(r'\{"(RT580_[A-Z0-9_]+)"', src))
    doc = open(os.path.join(helpers.REPO, "INTEGRATION.md")).read()
    missing = sorted(n for n in names if "`%s`" % n not in doc)
    assert 10 < len(names) <= 25 and not missing, (len(names), missing)


_SWITCH_CHILD = r"""
import ctypes, sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import helpers
rt580 = helpers.rt580()
lib = rt580.load()
bad = []
for scene, root, w, h, d, a in (("simpleSphereScene.json", helpers.ASSETS_ROOT, 64, 48, 4, 16),
                                ("cornell10k.json", helpers.synthetic_root("cornell10k"), 48, 27, 2, 8)):
    ref, _ = helpers.oracle_render(scene, w, h, d, a, True, root=root)
    rt = rt580.Raytracer(w, h, root)
    assert rt.LoadSceneJSON(scene) == 0
    rt.set_depth(d)
    rt.set_ao(a, True)
    for k in range(3):  # recorded, replayed / graph-captured, replayed
        if rt.Render("") != 0 or not np.array_equal(rt.framebuffer(), ref):
            bad.append("%s Render %d" % (scene, k))
    # the PPM body into registered host memory, three frames in flight
    params = rt.render_params()
    body = rt580.ppm_bytes(ref).split(b"\n", 3)[3]
    bufs = []
    for k in range(3):
        raw = np.zeros(len(body) + 2 * 4096, dtype=np.uint8)
        off = (-raw.ctypes.data) % 4096
        span = (len(body) + 4095) // 4096 * 4096
        buf = raw[off:off + span]
        rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "register")
        bufs.append((raw, buf))
    for k in range(6):
        rt580.check(lib.rt_gpu_render_async_ppm(ctypes.byref(params), bufs[k % 3][1].ctypes.data), "async_ppm")
    rt580.check(lib.rt_gpu_synchronize(), "sync")
    for k, (_, buf) in enumerate(bufs):
        if buf[:len(body)].tobytes() != body:
            bad.append("%s async_ppm %d" % (scene, k))
        rt580.check(lib.rt_gpu_host_unregister(buf.ctypes.data), "unregister")
    rt.close()
print("BAD", bad)
"""


@pytest.mark.gpu
@pytest.mark.parametrize("env", [
    {"RT580_PIPELINE": "0"}, {"RT580_SLOTS": "2"}, {"RT580_SLOTS": "4"}, {"RT580_AO_ORDER": "1"},
    {"RT580_REPLAY": "0"}, {"RT580_GRAPH": "0"}, {"RT580_D2H_MAPPED": "0"}, {"RT580_PROGRESS": "1"},
], ids=lambda e: ",".join("%s=%s" % kv for kv in e.items()))
def test_switch_keeps_the_frame(env, tmp_path):
    """Every product switch changes how frames are scheduled or delivered, not
    their bytes: with each setting, a small-scene and a BVH frame rendered three
    times through Render() (recorded, then replayed / graph-captured) and six
    times into registered host memory (rt_gpu_render_async_ppm, frames in
    flight) equal the oracle's."""
    e = {k: v for k, v in os.environ.items() if not k.startswith("RT580_")}
    e.update(env)
    script = tmp_path / "child.py"
    script.write_text(_SWITCH_CHILD)
    p = subprocess.run([sys.executable, str(script), os.path.join(helpers.REPO, "tests")], capture_output=True,
                       text=True, env=e, timeout=240)
    line = [l for l in p.stdout.splitlines() if l.startswith("BAD")]
    assert p.returncode == 0 and line, p.stdout + p.stderr
    assert line[0] == "BAD []", line[0]

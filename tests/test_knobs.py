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
    ({"RT580_AO_VARIANT": "512"}, "RT580_AO_VARIANT=512: not one of the supported values"),
    ({"RT580_AO_VARIANT": "x"}, "not an integer"),
    ({"RT580_CHUNK_LOG2": "28"}, "RT580_CHUNK_LOG2=28: outside [6, 27]"),
    ({"RT580_MULTI_TRANSPORT": "tcp"}, "not one of the supported values"),
    ({"RT580_GRID_R": "-1"}, "not a finite number > 0"),
    ({"RT580_DUMP_FAR": "/tmp/x"}, "diagnostic builds only"),
])
def test_bad_switch_fails_init(env, why):
    st, msg = _init_with(env)
    assert st == 1 and why in msg, msg


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU would initialise")
def test_valid_switches_pass_validation():
    st, msg = _init_with({"RT580_AO_VARIANT": str(16 | 7180), "RT580_CHUNK_LOG2": "10", "RT580_EXHAUSTIVE": "1",
                          "RT580_FAR_MODE": "4", "RT580_GRID_R": "2.5"})
    assert st == 1 and "no HIP device" in msg, msg


def test_every_switch_is_documented():
    """INTEGRATION.md's switch table lists every RT580_* name the library
    validates (csrc/rt_knobs.cpp), so no accepted switch is undocumented."""
    import re
    src = open(os.path.join(helpers.PKG, "csrc", "rt_knobs.cpp")).read()
    names = set(re.findall(r'\{"(RT580_[A-Z0-9_]+)"', src))
    doc = open(os.path.join(helpers.REPO, "INTEGRATION.md")).read()
    missing = sorted(n for n in names if "`%s`" % n not in doc)
    assert len(names) > 20 and not missing, missing

#!/usr/bin/env python3
"""Calibrate the CPU baseline's cost model against the reference itself.

bench.py times the repository's CPU restatement (oracle/rt_oracle.cpp) in
ref-faithful mode on the GPU box's host, because the reference cannot travel
there. This script runs, in the build container where /root/reference is
present, the reference binary built from its own sources (oracle/_ref,
rt_ref_param: Raytracer.cpp with the AO count as a parameter) and the port on
the same small full frames of every BASELINE scene, single-threaded, and
records render seconds (scene load excluded on both sides) and their ratio.
bench.py reports the ratio beside its CPU figure:
reference-equivalent Mrays/s = port Mrays/s x (port seconds / reference seconds).

    python tools/cpu_calibrate.py [--out profiles/r03/cpu_calibration.json]
"""
import argparse
import json
import os
import platform
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import helpers  # noqa: E402

REF = os.path.join(REPO, "oracle", "_ref", "rt_ref_param")

# scene, synthetic?, w, h, depth, AO: small full frames (both sides render every pixel)
CASES = [
    ("simpleSphereScene.json", False, 96, 54, 4, 64),
    ("cornell10k.json", True, 12, 8, 2, 4),
    ("field100k.json", True, 8, 6, 2, 2),
    ("field1m.json", True, 3, 2, 1, 1),
]


def cpu_model():
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "r03", "cpu_calibration.json"))
    args = ap.parse_args()
    if not os.path.exists(REF):
        sys.exit("reference binary %s missing (make -C oracle ref, build container only)" % REF)
    rows = {}
    for scene, synth, w, h, d, ao in CASES:
        root = helpers.synthetic_root(scene[:-5]) if synth else helpers.ASSETS_ROOT
        out = subprocess.run([REF, root, scene, str(w), str(h), str(d), "/tmp/_cal.ppm", str(ao)],
                             capture_output=True, text=True, check=True)
        ref_s = float(re.search(r"render_seconds=([0-9.]+)", out.stderr).group(1))
        fb, cnt, port_s = helpers.oracle_time_prefix(scene, w, h, d, ao, 0, w * h, root=root, faithful=True)
        ppm = helpers.rt580().ppm_bytes(fb.reshape(h, w, 3))
        same = ppm == open("/tmp/_cal.ppm", "rb").read()
        rows[scene[:-5]] = {"frame": "%dx%d depth=%d AO=%d" % (w, h, d, ao), "rays": cnt["rays_total"],
                            "reference_s": round(ref_s, 4), "port_s": round(port_s, 4),
                            "port_over_reference": round(port_s / ref_s, 4), "same_pixels": same}
        print(scene, rows[scene[:-5]], flush=True)
    res = {"cpu": cpu_model(), "threads": 1, "when": time.strftime("%Y-%m-%d"),
           "reference": "oracle/_ref/rt_ref_param (the reference's Raytracer.cpp, g++ -O2, AO count parameter)",
           "port": "oracle/rt_oracle.cpp, ref-faithful mode (oracle_time_prefix, serial)",
           "scenes": rows}
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()

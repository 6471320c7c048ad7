#!/usr/bin/env python3
"""Full-frame goldens at the target sizes, rendered by the ORACLE (the CPU
restatement, oracle/_build/rt_oracle; pinned to the reference's own renders by
tests/test_oracle.py). The reference itself would need days of CPU for these
frames (~0.33 us per ray-triangle test, O(prims) per ray), so the restatement
renders them once in the build container:

    make -C oracle oracle && python tests/golden/make_fullframe.py [--threads T] [name ...]

Writes tests/golden/fullframe.json: per frame the parameters, the sha256 of the
whole PPM, the sha256 of each band of 108 rows (to localise a mismatch), and
the oracle's ray counters. tests/test_gpu_fullframe.py renders the same frames
on the HIP path and compares. Frames:
  north_star  -- the 100k-triangle field, 1920x1080, depth 4, AO 64 (BASELINE north_star)
  config3     -- the 10k Cornell box, 1920x1080, depth 4, AO 64 (BASELINE config 3)
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
ORACLE = os.path.join(REPO, "oracle", "_build", "rt_oracle")
OUT = os.path.join(HERE, "fullframe.json")
BAND = 108

FRAMES = {
    "north_star": ("field100k", "field100k.json", 1920, 1080, 4, 64),
    "config3": ("cornell10k", "cornell10k.json", 1920, 1080, 4, 64),
}


def ppm_body(data, w, h):
    """The pixel bytes after the P6 header (the header is 'P6\\n<w> <h>\\n255\\n')."""
    body = data[len(data) - w * h * 3:]
    assert len(body) == w * h * 3
    return body


def render(name, threads):
    synth, scene, w, h, depth, ao = FRAMES[name]
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import helpers
    root = helpers.synthetic_root(synth)
    out = "/tmp/fullframe_%s.ppm" % name
    cmd = [ORACLE, root, scene, str(w), str(h), str(depth), out, "--ao", str(ao), "--threads", str(threads)]
    t0 = time.time()
    p = subprocess.run(cmd, capture_output=True, text=True, check=True)
    counters = json.loads(p.stdout.strip().splitlines()[-1])
    data = open(out, "rb").read()
    body = ppm_body(data, w, h)
    row = w * 3
    rec = {
        "scene": scene, "assets": synth, "width": w, "height": h, "depth": depth, "ao_samples": ao,
        "ao_enabled": True, "rng": "minstd",
        "sha256": hashlib.sha256(data).hexdigest(),
        "band_rows": BAND,
        "band_sha256": [hashlib.sha256(body[r * row:min(h, r + BAND) * row]).hexdigest()
                        for r in range(0, h, BAND)],
        "rays_total": counters["rays_total"], "rays_ao": counters["rays_ao"], "ao_calls": counters["ao_calls"],
        "oracle_seconds": round(time.time() - t0, 1), "oracle_threads": threads,
        "made_by": "tests/golden/make_fullframe.py (oracle/_build/rt_oracle, hoisted mode)",
    }
    os.remove(out)
    print(name, rec["sha256"][:16], rec["rays_total"], rec["oracle_seconds"], "s", flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("names", nargs="*", default=sorted(FRAMES))
    a = ap.parse_args()
    have = json.load(open(OUT)) if os.path.exists(OUT) else {}
    for n in a.names:
        have[n] = render(n, a.threads)
        with open(OUT, "w") as f:
            json.dump(have, f, indent=1, sort_keys=True)
            f.write("\n")


if __name__ == "__main__":
    main()

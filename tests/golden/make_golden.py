#!/usr/bin/env python3
"""Generate the golden fixtures from the REFERENCE ITSELF (oracle/_ref builds of
/root/reference/580 Raytracer/Raytracer.cpp; see oracle/Makefile). Run in the
build container only (the reference does not exist on the GPU box):

    make -C oracle ref && python tests/golden/make_golden.py [--big]

Writes tests/golden/ppm/<name>.ppm (small renders, kept verbatim) and
tests/golden/manifest.json (parameters, sha256, ray-free metadata). --big adds
sha256-only entries for the BASELINE configurations (minutes of CPU each).
Every entry records the exact reference binary and command line used.
"""
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.path.join(REPO, "oracle", "_ref")
ROOT = os.path.join(REF, "root")
REF_OUTPUT_PPM = "/root/reference/580 Raytracer/output.ppm"

# name, scene, w, h, depth, ao_n, ao_on, engine
SMALL = []
for scene, tag in [("simpleSphereScene.json", "sss"), ("simpleSphereSceneAO.json", "sssao"),
                   ("simpleScene.json", "tri")]:
    for depth in (0, 1, 4):
        for ao_n, ao_on in ((128, 0), (4, 1), (16, 1), (128, 1)):
            aotag = "aooff" if not ao_on else "ao%d" % ao_n
            SMALL.append(("%s_d%d_%s" % (tag, depth, aotag), scene, 61, 47, depth, ao_n, ao_on, "minstd"))
SMALL += [
    ("sss_d2_ao16_mt", "simpleSphereScene.json", 61, 47, 2, 16, 1, "mt19937"),
    ("sss_d8_ao4", "simpleSphereScene.json", 64, 64, 8, 4, 1, "minstd"),
    ("sss_d4_ao128_pristine", "simpleSphereScene.json", 40, 30, -1, 128, 1, "minstd"),
    ("teapots_d0_aooff", "scene.json", 48, 36, 0, 128, 0, "minstd"),
    ("teapots_d2_ao4", "scene.json", 64, 48, 2, 4, 1, "minstd"),
    ("teapots_d4_ao16_mt", "scene.json", 32, 24, 4, 16, 1, "mt19937"),
    ("teapots_d1_ao128", "scene.json", 24, 18, 1, 128, 1, "minstd"),
    ("sss_wide_d1_ao4", "simpleSphereScene.json", 97, 13, 1, 4, 1, "minstd"),
    ("sss_tall_d1_aooff", "simpleSphereScene.json", 7, 53, 1, 128, 0, "minstd"),
    ("sss_1x1_d4_ao16", "simpleSphereScene.json", 1, 1, 4, 16, 1, "minstd"),
]
# Synthetic scenes for BASELINE configs 3-5 (tools/gen_scenes.py, seed 580). The
# reference is O(prims) per ray (~0.33 us per ray-triangle test as written), so
# these stay tiny; "assets" names the generated set, whose file hashes are pinned.
SYNTH = [
    ("cornell10k_d4_ao4", "cornell10k.json", 32, 18, 4, 4, 1, "minstd"),
    ("cornell10k_d2_ao16_mt", "cornell10k.json", 20, 12, 2, 16, 1, "mt19937"),
    ("cornell10k_d6_aooff", "cornell10k.json", 24, 16, 6, 128, 0, "minstd"),
    ("field100k_d4_ao4", "field100k.json", 16, 9, 4, 4, 1, "minstd"),
    ("field1m_d2_ao2", "field1m.json", 8, 5, 2, 2, 1, "minstd"),
    # configs 4 and 5 at their own depth and AO count (reference: ~30 min / ~1.5 h of CPU)
    ("field100k_d6_ao256", "field100k.json", 16, 9, 6, 256, 1, "minstd"),
    ("field1m_d8_ao256", "field1m.json", 6, 4, 8, 256, 1, "minstd"),
]
SYNTH_ROOT = os.path.join(REF, "synth")

BIG = [
    # BASELINE config 1 and 2, the reference's committed output.ppm configuration,
    # and the reference main() as shipped (500x500, Render(): depth 4, AO 128)
    ("config1_500_d1_aooff", "simpleSphereScene.json", 500, 500, 1, 128, 0, "minstd"),
    ("main_500_d4_ao128", "simpleSphereScene.json", 500, 500, -1, 128, 1, "minstd"),
    ("config2_1080p_d4_ao64", "simpleSphereScene.json", 1920, 1080, 4, 64, 1, "minstd"),
]


def binary(ao_n, ao_on, engine):
    pristine = ao_n == 128 and ao_on
    name = "rt_ref" if pristine else "rt_ref_param"
    if engine == "mt19937":
        name += "_mt"
    return os.path.join(REF, name)


sys.path.insert(0, os.path.join(REPO, "tools"))
from gen_scenes import scene_files  # noqa: E402


def synth_assets(scene):
    """Generate the synthetic scene and return {file: sha256} of everything it reads."""
    stem = scene[:-5]
    subprocess.run([sys.executable, os.path.join(REPO, "tools", "gen_scenes.py"), SYNTH_ROOT, stem], check=True)
    assets = os.path.join(SYNTH_ROOT, "Assets")
    files = sorted(scene_files(stem))
    return {f: hashlib.sha256(open(os.path.join(assets, f), "rb").read()).hexdigest() for f in files}


def run(entry, keep_ppm, root=ROOT, extra=None):
    name, scene, w, h, depth, ao_n, ao_on, engine = entry
    exe = binary(ao_n, ao_on, engine)
    out = os.path.join("/tmp", "golden_%s.ppm" % name)
    cmd = [exe, root, scene, str(w), str(h), str(depth), out, str(ao_n), str(int(not ao_on))]
    t0 = time.time()
    p = subprocess.run(cmd, capture_output=True, text=True)
    if p.returncode != 0:
        raise SystemExit("reference failed: %s\n%s" % (" ".join(cmd), p.stderr))
    data = open(out, "rb").read()
    rec = {
        "name": name, "scene": scene, "width": w, "height": h,
        "depth": 4 if depth < 0 else depth, "via_render": depth < 0,
        "ao_samples": ao_n, "ao_enabled": bool(ao_on), "rng": engine,
        "sha256": hashlib.sha256(data).hexdigest(),
        "reference_binary": os.path.basename(exe),
        "reference_seconds": round(time.time() - t0, 3),
    }
    rec.update(extra or {})
    if keep_ppm:
        dst = os.path.join(HERE, "ppm", name + ".ppm")
        shutil.copyfile(out, dst)
        rec["ppm"] = "ppm/%s.ppm" % name
    os.remove(out)
    print(name, rec["sha256"][:16], rec["reference_seconds"], "s", flush=True)
    return rec


def merge_entry(man_path, rec):
    """Add one record to the manifest under a file lock (several --only runs may
    finish concurrently)."""
    import fcntl
    with open(man_path + ".lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        man = json.load(open(man_path)) if os.path.exists(man_path) else {"entries": []}
        have = {e["name"]: e for e in man["entries"]}
        have[rec["name"]] = rec
        man["entries"] = sorted(have.values(), key=lambda r: r["name"])
        json.dump(man, open(man_path, "w"), indent=1)


def main():
    big = "--big" in sys.argv
    only = sys.argv[sys.argv.index("--only") + 1] if "--only" in sys.argv else None
    os.makedirs(os.path.join(HERE, "ppm"), exist_ok=True)
    man_path = os.path.join(HERE, "manifest.json")
    man = json.load(open(man_path)) if os.path.exists(man_path) else {"entries": []}
    have = {e["name"]: e for e in man["entries"]}
    todo = [(e, True, False) for e in SMALL] + [(e, True, True) for e in SYNTH] + \
        ([(e, False, False) for e in BIG] if big else [])
    for e, keep, synth in todo:
        if only is not None and e[0] != only:
            continue
        if e[0] in have and (not keep or os.path.exists(os.path.join(HERE, have[e[0]].get("ppm", "-")))):
            continue
        if synth:
            files = synth_assets(e[1])
            have[e[0]] = run(e, keep, SYNTH_ROOT, {"assets": "synthetic", "asset_sha256": files})
        else:
            have[e[0]] = run(e, keep)
        merge_entry(man_path, have[e[0]])
    if only is not None:
        return
    man = json.load(open(man_path))
    # The reference's own committed render (mt19937, depth 0, AO 128, 500x500;
    # provenance established in SURVEY.md §4) — kept gzipped as a data fixture.
    if os.path.exists(REF_OUTPUT_PPM):
        data = open(REF_OUTPUT_PPM, "rb").read()
        with gzip.GzipFile(os.path.join(HERE, "reference_output.ppm.gz"), "wb", mtime=0) as f:
            f.write(data)
        man["reference_output_ppm"] = {
            "file": "reference_output.ppm.gz", "sha256": hashlib.sha256(data).hexdigest(),
            "scene": "simpleSphereScene.json", "width": 500, "height": 500, "depth": 0,
            "ao_samples": 128, "ao_enabled": True, "rng": "mt19937",
            "source": "580 Raytracer/output.ppm (committed by the reference authors)"}
    json.dump(man, open(man_path, "w"), indent=1)


if __name__ == "__main__":
    main()

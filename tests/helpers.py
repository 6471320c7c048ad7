"""Shared test utilities: repository paths, golden manifest, the product's
ctypes binding (580-raytracer_amd/rt580.py) and the oracle's (oracle/_build)."""
import ctypes
import functools
import gzip
import hashlib
import importlib.util
import json
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
ASSETS_ROOT = GOLDEN  # contains Assets/ (reference scene fixtures + synthetic scenes)
PKG = os.path.join(REPO, "580-raytracer_amd")
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "_build", "librt_oracle.so")
REFERENCE = "/root/reference/580 Raytracer"
SCENES_ROOT = os.path.join(REPO, "tests", "_scenes")  # generated synthetic scenes (not committed)


@functools.lru_cache(None)
def rt580():
    spec = importlib.util.spec_from_file_location("rt580", os.path.join(PKG, "rt580.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@functools.lru_cache(None)
def manifest():
    return json.load(open(os.path.join(GOLDEN, "manifest.json")))


def golden_entries(with_ppm=True):
    return [e for e in manifest()["entries"] if ("ppm" in e) == with_ppm]


def synthetic_root(*names):
    """Generate the synthetic scenes (tools/gen_scenes.py, seed 580) under
    tests/_scenes/Assets and check every file against the hashes recorded in the
    manifest when the reference rendered its goldens from them (so the generator
    is pinned across machines). Returns the root to pass as assets root."""
    import sys
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import gen_scenes
    want = {}
    for e in manifest()["entries"]:
        want.update(e.get("asset_sha256", {}))
    for n in names:
        gen_scenes.ensure(SCENES_ROOT, n)
        for f in gen_scenes.scene_files(n):
            if f in want:
                got = hashlib.sha256(open(os.path.join(SCENES_ROOT, "Assets", f), "rb").read()).hexdigest()
                assert got == want[f], "generated %s differs from the one the goldens were made from" % f
    return SCENES_ROOT


def scene_exponents():
    """Every specular exponent ("n", the powf exponent of CalculateLocalColor,
    Raytracer.cpp:253) of the scenes the tests and BASELINE configs render: the
    reference's Assets/ and the synthetic scenes of configs 3-5."""
    import glob
    exps = set()
    for root in (ASSETS_ROOT, synthetic_root("cornell10k", "field100k", "field1m")):
        for f in sorted(glob.glob(os.path.join(root, "Assets", "*.json"))):
            with open(f) as fh:
                head = fh.read(64)
            if '"scene"' not in head:
                continue  # meshes
            j = json.load(open(f))
            for sh in j["scene"].get("shapes", []):
                exps.add(float(np.float32(sh["material"]["n"])))
    return sorted(exps)


def entry_root(entry):
    if entry.get("assets") == "synthetic":
        return synthetic_root(entry["scene"][:-5])
    return ASSETS_ROOT


def golden_ppm(entry):
    return open(os.path.join(GOLDEN, entry["ppm"]), "rb").read()


def reference_output_ppm():
    ro = manifest()["reference_output_ppm"]
    with gzip.open(os.path.join(GOLDEN, ro["file"]), "rb") as f:
        data = f.read()
    assert hashlib.sha256(data).hexdigest() == ro["sha256"]
    return ro, data


def sha256(b):
    return hashlib.sha256(b).hexdigest()


def ppm_pixels(data):
    """(h, w, 3) uint8 array from P6 bytes."""
    parts = data.split(b"\n", 3)
    assert parts[0] == b"P6"
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], dtype=np.uint8).reshape(h, w, 3)


def diff_summary(a, b):
    pa, pb = ppm_pixels(a), ppm_pixels(b)
    if pa.shape != pb.shape:
        return "shape %s vs %s" % (pa.shape, pb.shape)
    d = np.abs(pa.astype(int) - pb.astype(int))
    bad = np.argwhere(d.max(axis=2) > 0)
    return "%d/%d pixels differ, max |d|=%d, first at (y,x)=%s" % (
        len(bad), pa.shape[0] * pa.shape[1], d.max(), bad[:5].tolist())


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR, "oracle"], check=True)


@functools.lru_cache(None)
def oracle_lib():
    build_oracle()
    lib = ctypes.CDLL(ORACLE_LIB)
    lib.oracle_render.restype = ctypes.c_int
    lib.oracle_render.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 9 + \
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.oracle_set_mode.argtypes = [ctypes.c_int]
    return lib


def oracle_render(scene, w, h, depth, ao_samples=128, ao_enabled=True, engine=0, threads=0,
                  rows=None, root=ASSETS_ROOT, faithful=False):
    """CPU restatement render -> (int16 (nrows, w, 3) framebuffer, counters dict).
    faithful=True: the ref-faithful cost model (same results, reference's cost)."""
    lib = oracle_lib()
    lib.oracle_set_mode(1 if faithful else 0)
    r0, r1 = rows if rows else (0, h)
    fb = np.zeros((r1 - r0, w, 3), dtype=np.int16)
    cnt = np.zeros(6, dtype=np.uint64)
    st = lib.oracle_render(os.fsencode(root), os.fsencode(scene), w, h, depth, ao_samples,
                           int(ao_enabled), engine, threads, r0, r1,
                           fb.ctypes.data, cnt.ctypes.data, None)
    lib.oracle_set_mode(0)
    assert st == 0, "oracle_render failed"
    keys = ["rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls"]
    return fb, dict(zip(keys, (int(x) for x in cnt)))


def oracle_time_prefix(scene, w, h, depth, ao_samples, p0, max_pixels, budget_s=1e30, threads=1, call_base=0,
                       root=ASSETS_ROOT, faithful=True):
    """CPU baseline: the reference's raster loop over pixels [p0, p0 + n) of the
    full w x h frame, RNG at AO-call index call_base (oracle_time_prefix).
    threads == 1: serial, stops after max_pixels or budget_s seconds;
    threads > 1: exactly max_pixels pixels. -> (int16 (n, 3) pixels, counters, render seconds
    without the scene load)."""
    lib = oracle_lib()
    f = lib.oracle_time_prefix
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 5 + \
        [ctypes.c_int64, ctypes.c_int64, ctypes.c_double, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
         ctypes.c_void_p, ctypes.c_void_p]
    fb = np.zeros((max_pixels, 3), dtype=np.int16)
    cnt = np.zeros(6, dtype=np.uint64)
    done = ctypes.c_int64(0)
    secs = ctypes.c_double(0)
    lib.oracle_set_mode(1 if faithful else 0)
    st = f(os.fsencode(root), os.fsencode(scene), w, h, depth, ao_samples, threads, p0, max_pixels, budget_s,
           call_base, fb.ctypes.data, cnt.ctypes.data, ctypes.byref(done), ctypes.byref(secs))
    lib.oracle_set_mode(0)
    assert st == 0, "oracle_time_prefix failed"
    keys = ["rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls"]
    return fb[:done.value], dict(zip(keys, (int(x) for x in cnt))), secs.value


def oracle_render_segments(scene, w, h, depth, ao_samples, segments, row_base, threads=0, root=ASSETS_ROOT,
                           engine=0):
    """Pixels of a full w x h frame at segments [(y, x0, n), ...] (hoisted mode,
    threaded), row y's first AO call at row_base[k] -> (list of int16 (n, 3)
    arrays, the AO calls of each segment's whole row, counters, seconds).
    engine 1: mt19937, the rows' draws taken from the serial stream at their bases."""
    lib = oracle_lib()
    f = lib.oracle_render_segments
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 6 + [ctypes.c_void_p] * 7 + \
        [ctypes.POINTER(ctypes.c_double)]
    if threads <= 0:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    ys = np.array([s[0] for s in segments], dtype=np.int32)
    x0 = np.array([s[1] for s in segments], dtype=np.int32)
    ns = np.array([s[2] for s in segments], dtype=np.int32)
    base = np.ascontiguousarray(np.asarray(row_base, dtype=np.uint64))
    fb = np.zeros((int(ns.sum()), 3), dtype=np.int16)
    calls = np.zeros(len(segments), dtype=np.uint64)
    cnt = np.zeros(6, dtype=np.uint64)
    secs = ctypes.c_double(0)
    lib.oracle_set_mode(0)
    lib.oracle_set_segments_engine(engine)
    try:
        st = f(os.fsencode(root), os.fsencode(scene), w, h, depth, ao_samples, threads, len(segments), ys.ctypes.data,
               x0.ctypes.data, ns.ctypes.data, base.ctypes.data, fb.ctypes.data, calls.ctypes.data, cnt.ctypes.data,
               ctypes.byref(secs))
    finally:
        lib.oracle_set_segments_engine(0)
    assert st == 0, "oracle_render_segments failed"
    out, o = [], 0
    for n in ns:
        out.append(fb[o:o + n])
        o += n
    keys = ["rays_total", "rays_primary", "rays_secondary", "rays_shadow", "rays_ao", "ao_calls"]
    return out, [int(c) for c in calls], dict(zip(keys, (int(x) for x in cnt))), secs.value


@functools.lru_cache(None)
def rt580_dist():
    spec = importlib.util.spec_from_file_location("rt580_dist", os.path.join(PKG, "rt580_dist.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class OracleRows:
    """CPU backend of rt580_dist.render_frame (count/shade rows with the oracle),
    used to test the multi-rank exchange logic under gloo without a GPU."""

    def __init__(self, scene, w, h, depth, ao_samples, ao_enabled=True, root=ASSETS_ROOT):
        import torch
        self.torch = torch
        self.args = (os.fsencode(root), os.fsencode(scene), w, h, depth, ao_samples, int(ao_enabled))
        self.width, self.height = w, h
        lib = oracle_lib()
        lib.oracle_count_rows.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 8 + [ctypes.c_void_p]
        lib.oracle_shade_rows.argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 8 + \
            [ctypes.c_void_p, ctypes.c_void_p]
        self.lib = lib

    def count(self, rank, world):
        d = rt580_dist()
        n_loc, n_max = d.n_local_rows(self.height, rank, world), d.n_max_rows(self.height, world)
        out = np.zeros(n_max, dtype=np.uint32)
        assert self.lib.oracle_count_rows(*self.args, rank, world, n_loc, out.ctypes.data) == 0
        return self.torch.from_numpy(out.astype(np.int32))

    def shade(self, rank, world, local_base, out=None):
        d = rt580_dist()
        n_loc, n_max = d.n_local_rows(self.height, rank, world), d.n_max_rows(self.height, world)
        base = np.ascontiguousarray(local_base.numpy().astype(np.uint64))
        fb = np.zeros(n_max * self.width * 3, dtype=np.int16)
        assert self.lib.oracle_shade_rows(*self.args, rank, world, n_loc, base.ctypes.data, fb.ctypes.data) == 0
        if out is not None:
            out.copy_(self.torch.from_numpy(fb))
            return out
        return self.torch.from_numpy(fb)

    def gamma_u8(self, fb, out):
        """Same contract as rt_gpu_gamma_u8 (the glibc-powf table on the CPU)."""
        lut = self.torch.from_numpy(rt580().gamma_lut().astype(np.uint8))
        out.copy_(lut[fb.to(self.torch.int64).clamp(0, 255)])
        return out

    def row_bases(self, gathered, rank, world, out):
        """Same contract as rt_gpu_row_bases (torch on the CPU)."""
        t = self.torch
        n_max = rt580_dist().n_max_rows(self.height, world)
        full = gathered.view(world, n_max).t().reshape(-1)[:self.height].to(t.int64)
        base = t.cumsum(full, 0) - full
        out.zero_()
        mine = base[rank::world]
        out[:mine.numel()] = mine
        return out

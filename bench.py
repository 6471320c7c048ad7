#!/usr/bin/env python3
"""Benchmark of the MI355X per-pixel ray-trace path (BASELINE.json metric:
"Mrays/sec + ms/frame at 1920x1080, depth=4, 64 AO samples; 1/2/4/8 GPU").

A step = one frame of BASELINE config 2 (simpleSphereScene.json, 1920x1080,
depth 4, 64 AO samples; the reference's own scene file) rendered from scratch
by the reference's Render() loop (Raytracer.cpp:916-935): trace of the
recursion tree, AO-call count + RNG-offset scan, AO kernel, resolve (+ for
N > 1 the all-gather of per-row AO counts and the gather of the row tiles),
and the frame copied into host memory. The scene is resident in
HBM.

    python bench.py [--gpus N [--rehearse]] [--steps K] [--warmup W]
                    [--workload config2|cornell10k|field100k_1080p|field100k|field1m]
                    [--no-cpu-baseline] [--no-north-star] [--no-check]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

Parallel modes (the row split of SURVEY §8e, byte-identical frames for every N):
  * N = 1: rt_gpu_render_async_ppm into page-locked host buffers (the frame's
    PPM body), up to three frames in flight (each frame's D2H overlaps the next
    frames' kernels); the blocking Render() latency is reported beside it.
  * --gpus N without a launcher: rt_gpu_render_multi_async over devices
    0..N-1 in this process, the same step (single-process RCCL; each device
    keeps its frame slots in flight, the gather and the D2H of one frame
    overlap the next frame's kernels). N above the visible devices is an
    error; --rehearse runs the same split on device 0 N times (device copies
    instead of RCCL) to rehearse it on a one-GPU box.
  * under torch.distributed.run: one process per GPU (rt580_dist.NativeRankFrame:
    the library's rank loop, rt_gpu_render_rank_async -- RCCL all-gather of the
    counts, each rank's rows written into one shared host frame, frames in
    flight; --backend gloo:
    rt580_dist.DistFrame over torch.distributed). --gpus must equal WORLD_SIZE.

Rank 0 prints ONE JSON line on stdout: metric, value = whole-job Mrays/s,
ms_per_step, roofline of the AO ray kernel, cpu_baseline (N = 1), the frame
check of the last timed frame (config 2: the reference's sha256), the
north_star sub-record (the 100k-triangle 1920x1080 depth-4 AO-64 frame that
BASELINE's target names) and the config3 sub-record (BASELINE config 3, the
10k-triangle Cornell box at 1920x1080 depth 4 AO 64), both measured the same
way in the same run.
"""
import argparse
import contextlib
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "tests"))

# MI355X_MICROARCH.md: 256 CUs x 4 SIMDs, one wave64 VALU instruction per SIMD
# every 2 cycles, 2.4 GHz; HBM3E 8.0 TB/s.
VALU_PEAK_GINST = 256 * 4 * 2.4 / 2.0   # 1228.8 G wave-instructions/s
HBM_PEAK_GBS = 8000.0
PROFILE_ROUNDS = ("r06", "r05", "r04", "r03", "r02")  # newest committed counter profiles first

# name -> (scene, synthetic?, width, height, depth, AO samples, label)
WORKLOADS = {
    "config2": ("simpleSphereScene.json", False, 1920, 1080, 4, 64,
                "BASELINE config 2: simpleSphereScene.json 1920x1080 depth=4 AO=64"),
    "cornell10k": ("cornell10k.json", True, 1920, 1080, 4, 64,
                   "BASELINE config 3: 10k-triangle Cornell box 1920x1080 depth=4 AO=64"),
    "field100k_1080p": ("field100k.json", True, 1920, 1080, 4, 64,
                        "north_star target: 100k-triangle field 1920x1080 depth=4 AO=64"),
    "field100k": ("field100k.json", True, 3840, 2160, 6, 256,
                  "BASELINE config 4: 100k-triangle field 3840x2160 depth=6 AO=256"),
    "field1m": ("field1m.json", True, 7680, 4320, 8, 256,
                "BASELINE config 5: 1M-triangle field 7680x4320 depth=8 AO=256"),
}
CPU_BUDGET_S = 15.0  # one core, per workload (the all-cores leg renders the same pixels)
# Frame check of the last timed frame against the oracle: pixels in 16 segments
# spread over the frame's geometry rows (per workload: the oracle's cost per
# pixel grows with triangles, depth and AO samples)
CHECK_PIXELS = {"config2": 10240, "cornell10k": 10240, "field100k_1080p": 10240, "field100k": 4096, "field1m": 256}
CHECK_SEGMENTS = 16
# workloads whose whole frame the oracle rendered once (tests/golden/make_fullframe.py)
FULLFRAME_KEYS = {"field100k_1080p": "north_star", "cornell10k": "config3"}


def env_int(k, d):
    try:
        return int(os.environ.get(k, d))
    except ValueError:
        return d


def log(msg):
    print("[bench %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


@contextlib.contextmanager
def stdout_to_stderr():
    """The reference prints "Scene parsing completed!" on stdout
    (Raytracer.cpp:772) and so does the drop-in; keep bench.py's stdout to the
    one JSON line by pointing fd 1 at stderr around such calls."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        yield
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


class Ctx:
    """What every workload run shares: torch, the library, the parallel mode."""

    def __init__(self, args):
        import torch
        import torch.distributed as dist
        import helpers
        self.torch, self.dist, self.helpers = torch, dist, helpers
        self.args = args
        self.rank, self.world = env_int("RANK", 0), env_int("WORLD_SIZE", 1)
        self.launched = "WORLD_SIZE" in os.environ
        n_dev = torch.cuda.device_count()
        if self.launched and args.gpus != self.world:
            raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, self.world))
        self.dist_on = self.world > 1 or args.dist
        self.multi = 0 if self.dist_on else (args.gpus if args.gpus > 1 else 0)
        if self.multi and not args.rehearse and self.multi > n_dev:
            raise SystemExit("bench.py: --gpus %d but %d visible device(s); --rehearse splits the frame over "
                             "device 0 instead" % (self.multi, n_dev))
        self.devices = ([0] * self.multi if args.rehearse else list(range(self.multi))) if self.multi else None
        # one GPU per rank; on a box with fewer GPUs than ranks (rehearsal of the
        # multi-rank path with --backend gloo) ranks share devices round-robin
        self.local_rank = env_int("LOCAL_RANK", 0) % max(n_dev, 1)
        torch.cuda.set_device(self.local_rank)
        self.device = torch.device("cuda", self.local_rank)
        if self.dist_on:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29581")
            if args.backend == "nccl":
                dist.init_process_group("nccl", rank=self.rank, world_size=self.world, device_id=self.device)
            else:
                dist.init_process_group(args.backend, rank=self.rank, world_size=self.world)
        self.rt580 = helpers.rt580()
        self.lib = self.rt580.load()
        self.rt580.check(self.lib.rt_gpu_init(self.local_rank), "rt_gpu_init")
        self.stream = torch.cuda.current_stream(self.device)
        self.rt580.check(self.lib.rt_gpu_set_stream(ctypes.c_void_p(self.stream.cuda_stream)), "rt_gpu_set_stream")
        self.n_gpus = self.world if self.dist_on else max(self.multi, 1)
        self.row_sample = args.row_sample if self.n_gpus == 1 and not self.dist_on else 1
        self.row_rank = args.row_rank if self.row_sample > 1 else 0

    def barrier(self):
        if self.dist_on:
            self.dist.barrier()

    def parallelism(self):
        if self.dist_on:
            return "interleaved rows x%d, one process per GPU, %s all_gather/gather" % (
                self.world, "RCCL" if self.args.backend == "nccl" else self.args.backend)
        if self.multi:
            if self.args.rehearse:
                return ("interleaved rows x%d on device 0 (rehearsal: device copies instead of RCCL; "
                        "not a multi-GPU measurement)" % self.multi)
            return "interleaved rows x%d, one process (rt_gpu_render_multi, RCCL)" % self.multi
        return "1 GPU"


def run_workload(ctx, name, steps, warmup, cpu_baseline_on, check):
    """Render `name` warmup + steps times in ctx's parallel mode; returns the
    bench record (rank 0) or None."""
    torch, lib, rt580, helpers = ctx.torch, ctx.lib, ctx.rt580, ctx.helpers
    scene, synth, W, H, depth, ao, label = WORKLOADS[name]
    root = helpers.synthetic_root(scene[:-5]) if synth else helpers.ASSETS_ROOT
    rt = rt580.Raytracer(W, H, root)
    with stdout_to_stderr():
        assert rt.LoadSceneJSON(scene) == 0, "LoadSceneJSON failed"
    rt.set_depth(depth)
    rt.set_ao(ao, True)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    sc = rt.scene()
    t_up = time.perf_counter()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(sc)), "rt_gpu_upload_scene")
    upload_s = time.perf_counter() - t_up
    n_tri = sum(1 for i in range(sc.n_prims) if sc.prims[i].kind == 0)
    log("%s: scene uploaded (%d primitives, %.1f s incl. acceleration build)" % (name, sc.n_prims, upload_s))

    dframe = None
    dist_mod = helpers.rt580_dist() if ctx.dist_on else None
    if ctx.dist_on:
        backend = dist_mod.GpuRows(rt580, params, torch, ctx.device)
        if ctx.args.backend == "nccl":
            dframe = dist_mod.NativeRankFrame(rt580, params, ctx.dist, torch, H, W, ctx.rank, ctx.world, ctx.device)
    import numpy as np
    if ctx.multi:
        devs = (ctypes.c_int * ctx.multi)(*ctx.devices)
    # one process (N = 1, or N devices of rt_gpu_render_multi_async): each
    # step's frame lands in host memory as the PPM body the reference writes
    # (SURVEY 8d's ms/frame ends with the frame on the host): a ring of
    # page-locked u8 buffers, one per frame in flight; the call queues the
    # frame, its gamma/PPM mapping and its D2H copy, which overlaps the next
    # frames' kernels
    ring = []
    step_kind = ctx.args.step if not ctx.multi else "ppm"
    if not ctx.dist_on and ctx.row_sample == 1 and step_kind != "device":
        for _ in range(RING):
            raw, buf, span = registered_buffer(W * H * 3, np.int16 if step_kind == "host16" else np.uint8)
            rt580.check(lib.rt_gpu_host_register(buf.ctypes.data, span), "rt_gpu_host_register")
            ring.append((raw, buf))
    step_i = [0]

    def step():
        if K > 1 or ctx.dist_on:
            if dframe is not None:
                dframe.render()
                return None
            return dist_mod.render_frame(backend, ctx.dist, torch, H, W, ctx.rank, ctx.world)
        if step_kind == "device":
            dev = ctypes.c_void_p()
            rt580.check(lib.rt_gpu_render_device(ctypes.byref(params), ctypes.byref(dev)), "rt_gpu_render_device")
            return None
        buf = ring[step_i[0] % RING][1]
        step_i[0] += 1
        if step_kind == "host16":
            rt580.check(lib.rt_gpu_render_async(ctypes.byref(params), buf.ctypes.data), "rt_gpu_render_async")
        elif ctx.multi:
            rt580.check(lib.rt_gpu_render_multi_async(ctypes.byref(params), buf.ctypes.data, ctx.multi, devs),
                        "rt_gpu_render_multi_async")
        else:
            rt580.check(lib.rt_gpu_render_async_ppm(ctypes.byref(params), buf.ctypes.data),
                        "rt_gpu_render_async_ppm")
        return buf

    def finish():
        return dframe.finish() if dframe is not None else None

    # rank r's exact share of a K-way interleaved split (--row-sample K
    # --row-rank r, one GPU): the rank loop of the multi-rank step
    # (rt_gpu_render_rank_async) rehearsed as rank r of K without a
    # communicator -- the world's per-row counts from an untimed full-frame
    # count pass, no gather traffic (rt580_rank_rehearse)
    K, R = ctx.row_sample, ctx.row_rank
    if K > 1:
        dm = helpers.rt580_dist()
        rows = dm.GpuRows(rt580, params, torch, ctx.device)
        log("%s: row sample %d/%d: full-frame count pass" % (name, R, K))
        cnt = rows.count(0, 1)[:H]
        torch.cuda.synchronize()
        n_max = dm.n_max_rows(H, K)
        gathered = torch.zeros(K * n_max, dtype=torch.int32, device=ctx.device)
        for k in range(K):
            part = cnt[k::K]
            gathered[k * n_max:k * n_max + part.numel()] = part
        dframe = dm.NativeRankFrame(rt580, params, None, torch, H, W, R, K, ctx.device, rehearse_gathered=gathered)

    # a split frame (N > 1 in this process): the frame's rays, and the frame to
    # compare with, from one untimed single-device render (rt_gpu_last_stats
    # of a split frame covers context 0's rows only)
    single = None
    if ctx.multi:
        single = np.zeros(W * H * 3, dtype=np.int16)
        rt580.check(lib.rt_gpu_render(ctypes.byref(params), single.ctypes.data), "rt_gpu_render")
        st = rt580.RenderStats()
        rt580.check(lib.rt_gpu_last_stats(ctypes.byref(st)), "rt_gpu_last_stats")
        rays_single = int(st.rays_total)

    for i in range(warmup):
        step()
        finish()
        if synth and W * H > 1920 * 1080:
            torch.cuda.synchronize()
            log("%s: warmup step %d done" % (name, i))
    torch.cuda.synchronize()
    if not ctx.args.no_live_timing:
        rt580.check(lib.rt_gpu_profile(1), "rt_gpu_profile")
    ctx.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_s = 0.0  # host time inside step(): the enqueue cost of a frame (its kernels run asynchronously)
    last = None
    for i in range(steps):
        th = time.perf_counter()
        r = step()
        host_s += time.perf_counter() - th
        if i == steps - 1:
            # the last frame's gather + de-interleave belong to the timed region
            last = finish() if dframe is not None else r
        if synth and W * H > 1920 * 1080 and ctx.rank == 0:  # 4K/8K frames: a progress line per enqueued step
            log("%s: step %d enqueued" % (name, i))
    ctx.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0

    ms = [ctypes.c_double() for _ in range(4)]
    frames = ctypes.c_int()
    rt580.check(lib.rt_gpu_profile_read(*[ctypes.byref(m) for m in ms], ctypes.byref(frames)), "rt_gpu_profile_read")
    per_frame = [m.value / max(frames.value, 1) for m in ms]  # trace, rank, ao, resolve
    rt580.check(lib.rt_gpu_profile(0), "rt_gpu_profile")
    k_ms, k_launches, k_rays = ctypes.c_double(), ctypes.c_int(), ctypes.c_uint64()
    rt580.check(lib.rt_gpu_profile_ao_kernel(ctypes.byref(k_ms), ctypes.byref(k_launches), ctypes.byref(k_rays)),
                "rt_gpu_profile_ao_kernel")
    st = rt580.RenderStats()
    rt580.check(lib.rt_gpu_last_stats(ctypes.byref(st)), "rt_gpu_last_stats")
    local = st.as_dict()

    # the last timed frame, on rank 0's host (int16 Pixel frame, or the u8 PPM body of DistFrame)
    frame_np = None
    if ctx.rank == 0 and K == 1:
        if ctx.dist_on:
            frame_np = last.cpu().numpy() if last is not None else None
        elif last is not None:
            rt580.check(lib.rt_gpu_synchronize(), "rt_gpu_synchronize")
            frame_np = last.copy().reshape(H, W, 3)

    if ctx.dist_on:
        t = torch.tensor([dt], dtype=torch.float64, device=ctx.device)
        ctx.dist.all_reduce(t, op=ctx.dist.ReduceOp.MAX)
        dt = float(t.item())
        r = torch.tensor([int(local["rays_total"])], dtype=torch.int64, device=ctx.device)
        ctx.dist.all_reduce(r, op=ctx.dist.ReduceOp.SUM)
        rays_frame = int(r.item())
    elif ctx.multi:
        rays_frame = rays_single
    else:
        rays_frame = int(local["rays_total"])  # this call's rows (all of them, or the row sample)
    if ctx.rank != 0:
        return None

    value = rays_frame * steps / dt / 1e6
    out = {
        "metric": "Mrays/sec (+ ms/frame) at %dx%d, depth=%d, %d AO samples" % (W, H, depth, ao),
        "value": round(value, 3),
        "unit": "Mrays/s",
        "n_gpus": ctx.n_gpus,
        "steps": steps,
        "warmup": warmup,
        "ms_per_step": round(dt / steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("synthetic scene (tools/gen_scenes.py, seed 580, %d triangles)" % n_tri) if synth else
                "reference scene file Assets/%s (no dataset needed)" % scene,
        "config": {
            "workload": label,
            "scene": scene, "width": W, "height": H, "depth": depth, "ao_samples": ao,
            "rng": "minstd_rand0 (libstdc++ default_random_engine)",
            "rays_per_frame": rays_frame,
            "parallelism": ctx.parallelism(),
            "row_sample": ("rows r = %d mod %d only (the exact pixels of rank %d in a %d-way interleaved split; "
                           "RNG bases from a full-frame count outside the timed region); value and "
                           "rays_per_frame refer to the sample" % (R, K, R, K)) if K > 1 else None,
            "scene_query": "exact BVH + plane tree (rt_bvh.h)" if lib.rt_gpu_accel_active() else
                           "brute force (every primitive per ray, as the reference)",
        },
        "step": ("one frame into host memory as its PPM body: %s, a ring of %d page-locked host buffers, up to "
                 "three frames in flight (each frame's gather and D2H overlap the next frames' kernels)"
                 % ("rt_gpu_render_multi_async (tiles mapped to bytes on their devices, gathered and de-interleaved "
                    "on device 0)" if ctx.multi else "rt_gpu_render_async_ppm", RING) if not ctx.dist_on else
                 "one frame on every rank; %s (rt580_dist.NativeRankFrame: the library's own rank loop, "
                 "rt_gpu_render_rank_async -- count, RCCL all-gather, shading, the frame's end, on one "
                 "communicator)" % ("every rank writes its rows' PPM bytes into one page-locked host frame shared "
                                    "by the processes (/dev/shm), a 4-byte all-gather ends the frame"
                                    if dframe is not None and dframe.shared else
                                    "rank 0 gathers the u8 tiles and writes the PPM body into page-locked host "
                                    "memory")),
        "step_kind": step_kind,
        "scene_upload_s": round(upload_s, 3),
        "host_enqueue_ms_per_step": round(host_s / steps * 1e3, 4),
        "kernel_ms_per_frame" + ("" if not (ctx.dist_on or ctx.multi) else "_rank0"): {
            "trace": round(per_frame[0], 4), "rank": round(per_frame[1], 4),
            "ao": round(per_frame[2], 4), "resolve": round(per_frame[3], 4)},
    }
    # AO rays per timed launch: the chunked BVH launches report theirs; a
    # small-scene frame is one launch over all of its (this context's) AO rays
    k_units = k_rays.value if k_rays.value else int(local["rays_ao"]) * max(frames.value, 1)
    iso = None
    if not ctx.dist_on and not ctx.multi and K == 1:
        # after the timed region (and after the last frame was copied out): the
        # same frames with AO phases in frame order, so no other frame's AO
        # kernels run beside the timed launch -- its isolated duration
        iso = isolated_ao_launch(lib, rt580, step, torch, int(local["rays_ao"]))
    out["roofline"] = roofline(name, k_ms.value, k_launches.value, k_units, iso)
    # per-row AO-call counts of the frame from one untimed GPU count pass: the
    # RNG bases of the oracle's frame-check rows and of the CPU baseline's range
    row_counts = None
    if frame_np is not None and not ctx.multi and not ctx.dist_on and \
            ((check and ctx.args.check_pixels != 0) or cpu_baseline_on):
        row_counts = helpers.rt580_dist().GpuRows(rt580, params, torch, ctx.device).count(0, 1)[:H].cpu().numpy()
    if frame_np is not None:
        out["frame_check"] = frame_check(ctx, name, frame_np, single, W, H, check)
        if check and row_counts is not None:
            n_px = ctx.args.check_pixels if ctx.args.check_pixels > 0 else CHECK_PIXELS[name]
            if n_px:
                out["frame_check"].update(oracle_rows_check(ctx, name, root, frame_np, row_counts, n_px))
    if not ctx.dist_on and not ctx.multi and K == 1 and not ctx.args.no_render_call:
        out["render_call_ms"] = render_latency(lib, rt580, params, torch)
    for _, buf in ring:
        rt580.check(lib.rt_gpu_host_unregister(buf.ctypes.data), "rt_gpu_host_unregister")
    if cpu_baseline_on and ctx.n_gpus == 1 and not ctx.dist_on:
        gpu_px = frame_np.reshape(-1, 3) if frame_np is not None else None
        out["cpu_baseline"] = cpu_baseline(ctx, name, root, params, gpu_px, row_counts)
    if dframe is not None:
        dframe.close()
    return out


def oracle_rows_check(ctx, name, root, frame_np, row_counts, n_px):
    """The last timed frame against the CPU restatement (oracle/, hoisted mode,
    threaded) on CHECK_SEGMENTS pixel segments spread over the frame's rows
    with geometry (stratified rows, staggered columns), n_px pixels in all.
    Each segment row's RNG base is the GPU's exclusive scan of its per-row AO
    calls; the oracle's own AO-call total of each of those rows must equal the
    GPU's count. Covers the full-size launches (2^27-record AO chunks) that no
    test reaches."""
    import numpy as np
    helpers = ctx.helpers
    scene, _, W, H, depth, ao, _ = WORKLOADS[name]
    counts = np.asarray(row_counts, dtype=np.int64)
    base = np.cumsum(counts) - counts
    nz = counts.nonzero()[0]
    lo, hi = (int(nz[0]), int(nz[-1])) if len(nz) else (0, H - 1)
    ns = min(CHECK_SEGMENTS, hi - lo + 1)
    seg_n = min(W, -(-n_px // ns))
    segs = []
    for k in range(ns):
        y = lo + (k * (hi - lo)) // max(ns - 1, 1)
        x0 = (((k * 7) % ns) * (W - seg_n)) // max(ns - 1, 1)
        segs.append((y, x0, seg_n))
    t0 = time.perf_counter()
    px, calls, cnt, secs = helpers.oracle_render_segments(scene, W, H, depth, ao, segs, [int(base[y]) for y, _, _ in segs],
                                                          root=root)
    lut = ctx.rt580.gamma_lut()
    # the oracle's Pixel values as the frame holds them (u8: the PPM bytes)
    as_frame = (lambda p: lut[np.asarray(p, dtype=np.int64)]) if frame_np.dtype == np.uint8 else (lambda p: p)
    bad_rows = [y for (y, x0, n), p in zip(segs, px) if not np.array_equal(as_frame(p), frame_np[y, x0:x0 + n])]
    bad_counts = [y for (y, _, _), c in zip(segs, calls) if c != int(counts[y])]
    log("%s: frame check: %d pixels in %d segments against the oracle in %.1f s: %d rows differ, %d counts differ"
        % (name, sum(n for _, _, n in segs), len(segs), time.perf_counter() - t0, len(bad_rows), len(bad_counts)))
    return {"pixels_checked": int(sum(n for _, _, n in segs)), "segments": [list(s) for s in segs],
            "matches_oracle_rows": not bad_rows and not bad_counts, "rows_differing": bad_rows,
            "row_ao_calls_differing": bad_counts, "oracle_rays": cnt["rays_total"], "oracle_seconds": round(secs, 2),
            "oracle": "oracle/rt_oracle.cpp oracle_render_segments (hoisted, %s threads); RNG base of each row "
                      "from the GPU's exclusive scan of its per-row AO-call counts" % os.environ.get(
                          "OMP_NUM_THREADS", os.cpu_count())}


def frame_check(ctx, name, frame_np, single, W, H, check):
    """The last timed frame against the reference's hash (config 2: the sha256 of
    the reference's own 1080p render, tests/golden/manifest.json) and, for a
    split frame, against the single-device render of the same frame."""
    import numpy as np
    rt580, helpers = ctx.rt580, ctx.helpers
    res = {"frame": "last timed step"}
    if frame_np.dtype == np.uint8:  # DistFrame(u8=True): already the PPM body
        ppm = b"P6\n%d %d\n255\n" % (W, H) + frame_np.tobytes()
    else:
        ppm = rt580.ppm_bytes(frame_np)
    res["sha256"] = helpers.sha256(ppm)
    if check and name == "config2":
        want = next(e for e in helpers.golden_entries(False) if e["name"] == "config2_1080p_d4_ao64")["sha256"]
        res["reference_sha256"] = want
        res["matches_reference"] = res["sha256"] == want
    # the whole frame against the oracle's full render (tests/golden/fullframe.json)
    ff = os.path.join(REPO, "tests", "golden", "fullframe.json")
    key = FULLFRAME_KEYS.get(name)
    if check and key and os.path.exists(ff):
        want = json.load(open(ff)).get(key, {}).get("sha256")
        if want:
            res["oracle_full_frame_sha256"] = want
            res["matches_oracle_full_frame"] = res["sha256"] == want
    if single is not None and (ctx.multi or ctx.dist_on):
        ref = rt580.gamma_lut()[single.astype(np.int64)] if frame_np.dtype == np.uint8 else single
        res["matches_single_gpu"] = bool(np.array_equal(frame_np.reshape(-1), ref.reshape(-1)))
    return res


def isolated_ao_launch(lib, rt580, step, torch, rays_ao_frame, frames=3):
    """Mean AO-kernel launch (ms) and AO rays per launch over `frames` frames
    rendered one at a time (each step's frame complete before the next is
    queued, AO phases in frame order): the AO kernel runs with no other frame's
    kernels beside it -- its own rate, comparable with the rocprofv3 mean of the
    committed profile. Untimed; restores the default order."""
    rt580.check(lib.rt580_set_ao_order(1), "rt580_set_ao_order")
    try:
        step()
        rt580.check(lib.rt_gpu_synchronize(), "rt_gpu_synchronize")
        torch.cuda.synchronize()
        rt580.check(lib.rt_gpu_profile(1), "rt_gpu_profile")
        for _ in range(frames):
            step()
            rt580.check(lib.rt_gpu_synchronize(), "rt_gpu_synchronize")
        torch.cuda.synchronize()
        ms = [ctypes.c_double() for _ in range(4)]
        nf = ctypes.c_int()
        rt580.check(lib.rt_gpu_profile_read(*[ctypes.byref(m) for m in ms], ctypes.byref(nf)), "rt_gpu_profile_read")
        rt580.check(lib.rt_gpu_profile(0), "rt_gpu_profile")
        k_ms, k_launches, k_rays = ctypes.c_double(), ctypes.c_int(), ctypes.c_uint64()
        rt580.check(lib.rt_gpu_profile_ao_kernel(ctypes.byref(k_ms), ctypes.byref(k_launches), ctypes.byref(k_rays)),
                    "rt_gpu_profile_ao_kernel")
    finally:
        rt580.check(lib.rt580_set_ao_order(0), "rt580_set_ao_order")
    if k_launches.value <= 0:
        return None
    units = k_rays.value if k_rays.value else rays_ao_frame * max(nf.value, 1)
    return {"launch_ms": k_ms.value / k_launches.value, "rays_per_launch": units / k_launches.value,
            "frames": frames}


def roofline(workload, k_ms, k_launches, k_rays, iso=None):
    """Roofline of the AO ray kernel (the scene query of every AO sample; 95 %
    of the frame's rays). Neither MFMA nor HBM bounds it (no dense
    contraction; the scene is re-read from L2/MALL, see `traffic`): it is
    bound by VALU instruction issue; peak = 1024 SIMDs x one wave64 VALU
    instruction per 2 cycles x 2.4 GHz.

    frac / achieved: the committed rocprofv3 profile's own figure
    (profiles/<round>/roofline_<workload>.json: SQ_INSTS_VALU per AO ray x AO
    rays per launch / the kernel trace's mean launch duration), so the headline
    is reproducible from profiles/. Beside it, this run's measurements of the
    same launch with HIP events on its own stream (rt_gpu_profile_ao_kernel):
    `isolated` (frames rendered one at a time: the kernel's own rate, which must
    agree with the profile's mean -- `isolated_over_rocprof`) and `live_frac`
    (the timed frames, whose AO phases overlap and stretch each other's
    launches: a share of a shared chip, not the kernel's cost)."""
    res = {"kernel": "ao_kernel (AO ray scene query)", "bound": "valu", "unit": "Ginst/s",
           "peak": VALU_PEAK_GINST, "achieved": None, "frac": None, "traffic": None}
    prof, path = None, None
    for rnd in PROFILE_ROUNDS:
        p = os.path.join(REPO, "profiles", rnd, "roofline_%s.json" % workload)
        if os.path.exists(p):
            try:
                prof, path = json.load(open(p)), p
                break
            except (ValueError, OSError):
                pass
    if not prof or not prof.get("valu_per_ao_ray"):
        res["note"] = "no committed counter profile for this workload (profiles/*/roofline_%s.json)" % workload
        return res
    vpr = prof["valu_per_ao_ray"]
    res["kernel"] = prof["kernel"]
    if prof.get("avg_ms") and prof.get("ao_rays_per_launch"):
        a = vpr * prof["ao_rays_per_launch"] / (prof["avg_ms"] * 1e-3) / 1e9
        res["achieved"] = round(a, 2)
        res["frac"] = round(a / VALU_PEAK_GINST, 4)
        res["launch_ms"] = prof["avg_ms"]
        res["ao_rays_per_launch"] = int(prof["ao_rays_per_launch"])
        if prof.get("hbm_bytes_per_ao_ray") is not None:
            traffic = prof["hbm_bytes_per_ao_ray"] * prof["ao_rays_per_launch"]
            res["traffic"] = round(traffic)
            res["hbm_frac"] = round(traffic / (prof["avg_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    res["per_ray"] = {"valu_wave_insts": round(vpr, 3), "hbm_bytes": prof.get("hbm_bytes_per_ao_ray")}
    res["profile"] = os.path.relpath(path, REPO)
    if k_launches > 0 and k_ms > 0:
        launch_s = k_ms / k_launches * 1e-3
        res["live_frac"] = round(vpr * (k_rays / k_launches) / launch_s / 1e9 / VALU_PEAK_GINST, 4)
        res["live_launch_ms"] = round(launch_s * 1e3, 4)
    if iso:
        a_iso = vpr * iso["rays_per_launch"] / (iso["launch_ms"] * 1e-3) / 1e9
        res["isolated"] = {"launch_ms": round(iso["launch_ms"], 4), "ao_rays_per_launch": int(iso["rays_per_launch"]),
                           "frac": round(a_iso / VALU_PEAK_GINST, 4)}
        if prof.get("avg_ms"):
            res["isolated_over_rocprof"] = round(iso["launch_ms"] / prof["avg_ms"], 4)
    return res


RING = 3  # host frames of the one-process step (one per frame slot in flight)


def registered_buffer(n_val, dtype):
    """A page-aligned, page-rounded host buffer of n_val values of dtype (a
    registration must not share pages with other allocations) -> (owner, view, span)."""
    import numpy as np
    item = np.dtype(dtype).itemsize
    span = (n_val * item + 4095) // 4096 * 4096
    raw = np.zeros(span + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    return raw, raw[off:off + span].view(dtype)[:n_val], span


def render_latency(lib, rt580, params, torch, n=5, warm=4):
    """Blocking rt_gpu_render (what Render() calls): first launch -> int16
    framebuffer on the host (SURVEY §8d ms/frame), excluding scene load/upload
    and the PPM write. The host framebuffer is page-locked once
    (rt_gpu_host_register), as the class surface does with its own, so the
    frame lands in it with one DMA. Mean of n calls after the timed region,
    after `warm` untimed calls (a small-scene frame is captured as a HIP graph
    on each slot's second call, rt_shim.cpp render_split: the steady state of
    repeated renders)."""
    # page-aligned and page-rounded, like the class surface's own framebuffer
    import numpy as np
    raw, host, span = registered_buffer(params.width * params.height * 3, np.int16)
    rt580.check(lib.rt_gpu_host_register(host.ctypes.data, span), "rt_gpu_host_register")
    try:
        for _ in range(warm):
            rt580.check(lib.rt_gpu_render(ctypes.byref(params), host.ctypes.data), "rt_gpu_render")
        times = []
        for _ in range(n):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rt580.check(lib.rt_gpu_render(ctypes.byref(params), host.ctypes.data), "rt_gpu_render")
            times.append((time.perf_counter() - t0) * 1e3)
    finally:
        rt580.check(lib.rt_gpu_host_unregister(host.ctypes.data), "rt_gpu_host_unregister")
    return round(sum(times) / len(times), 4)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline(ctx, name, root, params, gpu_px, row_counts=None):
    """The repository's CPU restatement (oracle/) in ref-faithful mode (the
    reference's per-call work: string mesh lookup and ComputeModelMatrix per
    shape per IntersectScene call, the unused Matrix::Inverse + TransformPoint
    per triangle test) running the reference's own raster loop
    (Raytracer.cpp:921-932) over an exact range of the workload's full frame:
    from the first row with geometry (the rows above are sky, with no AO call,
    so the RNG starts at draw 0 exactly as in the full frame), one serial
    stream on one core for ~CPU_BUDGET_S seconds; then the same pixels on all
    of this host's cores (count pass, scan, pixels as work items). Both are
    compared with the GPU's last timed frame (parity). The reference itself
    does not travel to this box: profiles/r03/cpu_calibration.json holds the
    port-to-reference cost ratio measured in the build container."""
    helpers, torch = ctx.helpers, ctx.torch
    scene, _, W, H, depth, ao, _ = WORKLOADS[name]
    # first row with an AO call, from the GPU's count pass (untimed)
    if row_counts is None:
        row_counts = ctx.helpers.rt580_dist().GpuRows(ctx.rt580, params, torch, ctx.device).count(0, 1)[:H].cpu().numpy()
    counts = row_counts
    nz = counts.nonzero()[0]
    y0 = int(nz[0]) if len(nz) else 0
    p0 = y0 * W
    threads = env_int("OMP_NUM_THREADS", os.cpu_count() or 1)
    fb1, cnt, secs1 = helpers.oracle_time_prefix(scene, W, H, depth, ao, p0, W * H - p0, budget_s=CPU_BUDGET_S,
                                                 threads=1, root=root, faithful=True)
    n = len(fb1)
    res = {
        "value": float("%.4g" % (cnt["rays_total"] / secs1 / 1e6)),
        "unit": "Mrays/s",
        "cores": 1,
        "kind": "port",
        "seconds": round(secs1, 3),
        "rays": cnt["rays_total"],
        "cpu": cpu_model(),
        "sample": ("%s %dx%d depth=%d AO=%d: exact raster range of the full frame, %d pixel(s) from (0, %d) "
                   "(rows 0-%d are sky: no AO call precedes, the RNG starts at draw 0 as in the frame); "
                   "oracle/rt_oracle.cpp in ref-faithful mode (the reference's arithmetic and per-call work)"
                   % (scene, W, H, depth, ao, n, y0, max(y0 - 1, 0))),
    }
    import numpy as np
    if gpu_px is not None and gpu_px.dtype == np.uint8:  # the PPM body: the oracle's pixels through the same LUT
        fb1_frame = ctx.rt580.gamma_lut()[np.asarray(fb1, dtype=np.int64)]
    else:
        fb1_frame = fb1
    parity = None if gpu_px is None else bool((fb1_frame == gpu_px[p0:p0 + n]).all())
    if threads > 1 and n > 1:
        fbn, cntn, secsn = helpers.oracle_time_prefix(scene, W, H, depth, ao, p0, n, threads=threads, root=root,
                                                      faithful=True)
        res["all_cores"] = {"value": float("%.4g" % (cntn["rays_total"] / secsn / 1e6)), "cores": threads,
                            "host_cpus": os.cpu_count(), "seconds": round(secsn, 3),
                            "note": "same pixels on $OMP_NUM_THREADS threads (the GPU pool's per-GPU CPU share; "
                                    "host_cpus is the whole machine); includes the count pass that splitting the "
                                    "serial RNG stream needs"}
        res["all_cores"]["matches_one_core"] = bool((fbn == fb1).all())
    res["matches_gpu_frame"] = parity
    cal = os.path.join(REPO, "profiles", "r03", "cpu_calibration.json")
    if os.path.exists(cal):
        c = json.load(open(cal))
        row = c["scenes"].get(scene[:-5])
        if row:
            res["calibration"] = {"port_over_reference": row["port_over_reference"], "cpu": c["cpu"],
                                  "frame": row["frame"], "file": os.path.relpath(cal, REPO),
                                  "reference_equiv_value": float("%.4g" % (res["value"] * row["port_over_reference"]))}
    return res


def compact(rec):
    """A sub-record's numbers in a few hundred bytes (the driver keeps the
    tail of stdout: the whole line must stay short)."""
    fc, rf, cb = rec.get("frame_check", {}), rec.get("roofline", {}), rec.get("cpu_baseline") or {}
    return {"value": rec["value"], "unit": rec["unit"], "ms_per_step": rec["ms_per_step"], "steps": rec["steps"],
            "rays_per_frame": rec["config"]["rays_per_frame"], "workload": rec["config"]["workload"],
            "frame_check": {k: fc[k] for k in ("matches_reference", "matches_oracle_full_frame", "matches_oracle_rows",
                                               "pixels_checked", "matches_single_gpu") if k in fc},
            "roofline": {k: rf.get(k) for k in ("kernel", "frac", "achieved", "launch_ms", "live_frac",
                                                "isolated_over_rocprof", "profile")},
            "render_call_ms": rec.get("render_call_ms"),
            "cpu_baseline": {k: cb[k] for k in ("value", "cores", "kind", "matches_gpu_frame") if k in cb}}


def headline(out):
    """The printed line: the contract's keys first, the north-star and config-3
    summaries right after the headline numbers, then the rest (sub-records
    compact; --detail writes them in full)."""
    first = ("metric", "value", "unit", "ms_per_step")
    res = {k: out[k] for k in first}
    for sub in ("north_star", "config3"):
        if out.get(sub):
            res[sub] = compact(out[sub])
    for k, v in out.items():
        if k not in res:
            res[k] = v
    rf = res.get("roofline")
    if rf:
        res["roofline"] = {k: v for k, v in rf.items()}
    if res.get("cpu_baseline", {}).get("calibration"):
        res["cpu_baseline"] = dict(res["cpu_baseline"])
        res["cpu_baseline"].pop("calibration")
    fc = res.get("frame_check")
    if fc:
        res["frame_check"] = {k: v for k, v in fc.items() if k not in ("segments", "oracle")}
    return res


def main():
    # a Python stack dump to stderr every $BENCH_WATCHDOG_S seconds (where a
    # GPU run is when it stops making progress)
    if os.environ.get("BENCH_WATCHDOG_S"):
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["BENCH_WATCHDOG_S"]), repeat=True, file=sys.stderr)
    # stdout carries exactly one JSON line: everything else written to fd 1 (the
    # drop-in's "Scene parsing completed!", RCCL's version banner at communicator
    # init) goes to stderr; the JSON line goes to the saved original stdout
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--rehearse", action="store_true",
                    help="--gpus N on a box with fewer GPUs: split the frame N ways on device 0 (device copies)")
    ap.add_argument("--steps", type=int, default=None,
                    help="default 20 (config2), 10 (synthetic 1080p), 3 (synthetic 4K / 8K)")
    ap.add_argument("--warmup", type=int, default=None, help="default 3")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-north-star", action="store_true", help="skip the north_star sub-record (config2)")
    ap.add_argument("--no-config3", action="store_true", help="skip the config3 sub-record (config2)")
    ap.add_argument("--no-check", action="store_true", help="skip the reference-hash check of the last frame")
    ap.add_argument("--detail", default=None,
                    help="also write the full record (every sub-record in full) to this file; stdout keeps the "
                         "compact line")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    ap.add_argument("--dist", action="store_true",
                    help="the multi-rank path (torch.distributed + DistFrame) even with one rank: rehearses the "
                         "RCCL all-gather/gather and the per-frame host overhead of N>1 on one GPU")
    ap.add_argument("--workload", default="config2", choices=sorted(WORKLOADS))
    ap.add_argument("--check-pixels", type=int, default=-1,
                    help="pixels of the last timed frame checked against the oracle (16 segments over the "
                         "geometry rows; -1: the workload's default, 0: none)")
    ap.add_argument("--row-sample", type=int, default=1,
                    help="N=1 only: time rows r = R mod K of the frame (rank R's exact share of a K-way "
                         "interleaved split; RNG bases from an untimed full-frame count), for huge frames and "
                         "the per-rank shares of a split")
    ap.add_argument("--row-rank", type=int, default=0, help="R of --row-sample")
    ap.add_argument("--no-render-call", action="store_true",
                    help="skip the blocking Render() latency frames (render_call_ms): counter profiles of the step's "
                         "kernels only (small-scene Render() frames run their AO in two launches)")
    ap.add_argument("--no-live-timing", action="store_true",
                    help="no HIP-event timing of the frames' phases and AO launches inside the timed region (A/B of "
                         "its cost; the roofline then has only the isolated timing)")
    ap.add_argument("--step", default="ppm", choices=["ppm", "host16", "device"],
                    help="one process, N = 1 (A/B of the step's end; the default is the contract's): ppm = the PPM "
                         "body in host memory (rt_gpu_render_async_ppm), host16 = the int16 framebuffer in host "
                         "memory (rt_gpu_render_async), device = the framebuffer left in HBM (rt_gpu_render_device)")
    args = ap.parse_args()
    if args.row_sample < 1 or not 0 <= args.row_rank < args.row_sample:
        raise SystemExit("bench.py: need --row-sample K >= 1 and 0 <= --row-rank < K")
    if args.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    synth = WORKLOADS[args.workload][1]
    # 3 warmup frames: the first verifies the node capacity and records the
    # trace phase's host reads, the second the AO phase's; from the third on a
    # frame replays them and enqueues without a host sync (rt_shim.cpp
    # count schedules), so consecutive frames overlap on the two slots
    big = WORKLOADS[args.workload][2] * WORKLOADS[args.workload][3] > 1920 * 1080
    steps = args.steps if args.steps is not None else (20 if not synth else (3 if big else 10))
    warmup = args.warmup if args.warmup is not None else 3

    ctx = Ctx(args)
    out = run_workload(ctx, args.workload, steps, warmup, not args.no_cpu_baseline, not args.no_check)
    if args.workload == "config2" and not args.no_north_star:
        ns = run_workload(ctx, "field100k_1080p", 10, 3, not args.no_cpu_baseline, not args.no_check)
        if out is not None:
            out["north_star"] = ns
    if args.workload == "config2" and not args.no_config3:
        # BASELINE config 3, the other 1 x MI355X configuration, measured the same way
        c3 = run_workload(ctx, "cornell10k", 10, 3, not args.no_cpu_baseline, not args.no_check)
        if out is not None:
            out["config3"] = c3
    if out is not None:
        if args.detail:
            with open(args.detail, "w") as f:
                json.dump(out, f, indent=1)
        print(json.dumps(headline(out)), file=json_out, flush=True)
    if ctx.dist_on:
        ctx.dist.barrier()
        ctx.dist.destroy_process_group()


if __name__ == "__main__":
    main()

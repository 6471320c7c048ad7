#!/usr/bin/env python3
"""Benchmark of the MI355X per-pixel ray-trace path (BASELINE.json metric:
"Mrays/sec + ms/frame at 1920x1080, depth=4, 64 AO samples; 1/2/4/8 GPU").

A step = one frame of BASELINE config 2 (simpleSphereScene.json, 1920x1080,
depth 4, 64 AO samples; the reference's own scene file) rendered from scratch:
trace of the recursion tree, AO-call count + RNG-offset scan, AO kernel,
resolve (+ for N > 1 the all-gather of per-row AO counts and the RCCL gather of
the row tiles to rank 0). The scene is resident in HBM; the framebuffer stays
in HBM (device throughput, frames pipelined on two streams). The blocking
Render() latency (framebuffer copied to the host) is reported beside it.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline]
                    [--workload config2|cornell10k|field100k_1080p|field100k|field1m]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

--workload selects another BASELINE configuration (synthetic scenes from
tools/gen_scenes.py, generated on first use under tests/_scenes); config2 is
the headline. Synthetic workloads default to 2 steps after 1 warm-up.

Rank 0 prints ONE JSON line on stdout (metric, value = whole-job Mrays/s,
ms_per_step, roofline of the AO ray kernel, cpu_baseline = the repository's
CPU restatement in ref-faithful mode on this host, 1 core and all cores).
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

# name -> (scene, synthetic?, width, height, depth, AO samples,
#          CPU-baseline sample, label)
# CPU sample (~10-30 s for the ref-faithful restatement on one core):
#   (w, h, depth, ao)  a downscaled frame of the same scene (config 2: exact bytes);
#   ("pixels", P[, A]) P pixels of the workload's own full-resolution frame on a
#                      stratified grid, at its depth and AO count (A: a smaller AO
#                      count, config 5 only: one 1M-triangle pixel at AO 256 is
#                      minutes of CPU; the reference's IntersectScene loops over every
#                      primitive for every ray, Raytracer.cpp:476-521, so its cost
#                      per ray does not depend on the ray's kind).
WORKLOADS = {
    "config2": ("simpleSphereScene.json", False, 1920, 1080, 4, 64, (640, 360, 4, 64),
                "BASELINE config 2: simpleSphereScene.json 1920x1080 depth=4 AO=64"),
    "cornell10k": ("cornell10k.json", True, 1920, 1080, 4, 64, ("pixels", 64),
                   "BASELINE config 3: 10k-triangle Cornell box 1920x1080 depth=4 AO=64"),
    "field100k_1080p": ("field100k.json", True, 1920, 1080, 4, 64, ("pixels", 32),
                        "north_star target: 100k-triangle field 1920x1080 depth=4 AO=64"),
    "field100k": ("field100k.json", True, 3840, 2160, 6, 256, ("pixels", 2),
                  "BASELINE config 4: 100k-triangle field 3840x2160 depth=6 AO=256"),
    "field1m": ("field1m.json", True, 7680, 4320, 8, 256, ("pixels", 1, 8),
                "BASELINE config 5: 1M-triangle field 7680x4320 depth=8 AO=256"),
}


def stratified_pixels(n, w, h):
    """n pixel centres of a gx x gy (>= n cells) grid over the w x h frame (raster order)."""
    gx = max(1, int(round((n * w / h) ** 0.5)))
    gy = (n + gx - 1) // gx
    pts = [(int((i + 0.5) * w / gx), int((j + 0.5) * h / gy)) for j in range(gy) for i in range(gx)]
    return [pts[k * len(pts) // n] for k in range(n)]  # n cells spread over the whole grid


def env_int(k, d):
    try:
        return int(os.environ.get(k, d))
    except ValueError:
        return d


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


def main():
    # stdout carries exactly one JSON line: everything else written to fd 1 (the
    # drop-in's "Scene parsing completed!", RCCL's version banner at communicator
    # init) goes to stderr; the JSON line goes to the saved original stdout
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="default 20 (config2), 2 (synthetic)")
    ap.add_argument("--warmup", type=int, default=None, help="default 3 (config2), 1 (synthetic)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N>1 (nccl = RCCL)")
    ap.add_argument("--dist", action="store_true",
                    help="the multi-rank path (torch.distributed + DistFrame) even with one rank: rehearses the "
                         "RCCL all-gather/gather and the per-frame host overhead of N>1 on one GPU")
    ap.add_argument("--check", action="store_true", help="verify the frame against the golden sha256 (config2)")
    ap.add_argument("--workload", default="config2", choices=sorted(WORKLOADS))
    ap.add_argument("--row-sample", type=int, default=1,
                    help="N=1 only: time rows r = 0 mod K of the frame (rank 0's exact share of a K-way "
                         "interleaved split; RNG bases from an untimed full-frame count), for huge frames")
    args = ap.parse_args()
    global SCENE, WIDTH, HEIGHT, DEPTH, AO, CPU_SAMPLE, LABEL, SYNTH
    SCENE, SYNTH, WIDTH, HEIGHT, DEPTH, AO, CPU_SAMPLE, LABEL = WORKLOADS[args.workload]
    if args.steps is None:
        args.steps = 2 if SYNTH else 20
    if args.warmup is None:
        args.warmup = 1 if SYNTH else 3

    import torch
    import torch.distributed as dist
    import helpers

    rank, world = env_int("RANK", 0), env_int("WORLD_SIZE", 1)
    # one GPU per rank; on a box with fewer GPUs than ranks (rehearsal of the
    # multi-rank path with --backend gloo) ranks share devices round-robin
    local_rank = env_int("LOCAL_RANK", 0) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    dist_on = world > 1 or args.dist
    if dist_on:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29581")
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
        else:
            dist.init_process_group(args.backend, rank=rank, world_size=world)

    rt580 = helpers.rt580()
    lib = rt580.load()
    rt580.check(lib.rt_gpu_init(local_rank), "rt_gpu_init")
    stream = torch.cuda.current_stream(device)
    rt580.check(lib.rt_gpu_set_stream(ctypes.c_void_p(stream.cuda_stream)), "rt_gpu_set_stream")

    root = helpers.synthetic_root(SCENE[:-5]) if SYNTH else helpers.ASSETS_ROOT
    rt = rt580.Raytracer(WIDTH, HEIGHT, root)
    with stdout_to_stderr():
        assert rt.LoadSceneJSON(SCENE) == 0, "LoadSceneJSON failed"
    rt.set_depth(DEPTH)
    rt.set_ao(AO, True)
    assert rt.InitializeRenderer() == 0
    params = rt.render_params()
    scene = rt.scene()
    rt580.check(lib.rt_gpu_upload_scene(ctypes.byref(scene)), "rt_gpu_upload_scene")
    prims = [scene.prims[i] for i in range(scene.n_prims)]
    n_tri = sum(1 for p in prims if p.kind == 0)

    fbp = ctypes.c_void_p()
    K = max(args.row_sample, 1) if not dist_on else 1
    dist_mod = helpers.rt580_dist() if (dist_on or K > 1) else None
    backend = dist_mod.GpuRows(rt580, params, torch, device) if (dist_on or K > 1) else None
    sample_base = None
    if K > 1:
        # exact global RNG bases: every row's AO-call count, once, outside the timed region
        log("row sample 1/%d: full-frame count pass" % K)
        cnt = backend.count(0, 1)[:HEIGHT].to(torch.int64)
        base = torch.cumsum(cnt, 0) - cnt
        n_loc = dist_mod.n_local_rows(HEIGHT, 0, K)
        sample_base = torch.zeros(dist_mod.n_max_rows(HEIGHT, K), dtype=torch.int64, device=device)
        sample_base[:n_loc] = base[0::K][:n_loc]

    # steady-state multi-rank frames (RCCL): persistent buffers, async gather
    # overlapped with the next frame; gloo (rehearsal) uses the plain form
    dframe = dist_mod.DistFrame(backend, dist, torch, HEIGHT, WIDTH, rank, world, device) \
        if (dist_on and args.backend == "nccl") else None

    def step():
        if K > 1:
            backend.count(0, K)
            return backend.shade(0, K, sample_base)
        if not dist_on:
            rt580.check(lib.rt_gpu_render_device(ctypes.byref(params), ctypes.byref(fbp)), "rt_gpu_render_device")
            return None
        if dframe is not None:
            dframe.render()
            return None
        return dist_mod.render_frame(backend, dist, torch, HEIGHT, WIDTH, rank, world)

    def finish():
        return dframe.finish() if dframe is not None else None

    def barrier():
        if dist_on:
            dist.barrier()

    frame = None
    for i in range(max(args.warmup, 1 if args.check else 0)):
        frame = step()
        if dframe is not None:
            frame = finish()
        if SYNTH:
            torch.cuda.synchronize()
            log("warmup step %d done" % i)
    torch.cuda.synchronize()
    check_ok = None
    if args.check and rank == 0:
        # the frame of the (last warm-up) step vs the reference's config-2 hash
        import numpy as np
        if not dist_on:
            host = np.zeros(WIDTH * HEIGHT * 3, dtype=np.int16)
            rt580.check(lib.rt_gpu_render(ctypes.byref(params), host.ctypes.data), "rt_gpu_render")
            frame_np = host.reshape(HEIGHT, WIDTH, 3)
        else:
            frame_np = frame.cpu().numpy()
        want = next(e for e in helpers.golden_entries(False) if e["name"] == "config2_1080p_d4_ao64")["sha256"]
        if frame_np.dtype == np.uint8:  # DistFrame(u8=True): already the PPM body
            ppm = b"P6\n%d %d\n255\n" % (WIDTH, HEIGHT) + frame_np.tobytes()
        else:
            ppm = rt580.ppm_bytes(frame_np)
        check_ok = helpers.sha256(ppm) == want
    rt580.check(lib.rt_gpu_profile(1), "rt_gpu_profile")
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    host_s = 0.0  # host time inside step(): the enqueue cost of a frame (its kernels run asynchronously)
    for i in range(args.steps):
        th = time.perf_counter()
        step()
        host_s += time.perf_counter() - th
        if i == args.steps - 1:
            finish()  # the last frame's gather + de-interleave belong to the timed region
        if SYNTH:  # long frames: keep a progress line per step (sync costs microseconds)
            torch.cuda.synchronize()
            if rank == 0:
                log("step %d done" % i)
    barrier()
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
    # rays of one frame (this rank's rows), from the count pass of the last frame
    st = rt580.RenderStats()
    rt580.check(lib.rt_gpu_last_stats(ctypes.byref(st)), "rt_gpu_last_stats")
    local = st.as_dict()

    rays_local = int(local["rays_total"])
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        r = torch.tensor([rays_local], dtype=torch.int64, device=device)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays_frame = int(r.item())
    else:
        rays_frame = rays_local

    if rank == 0:
        value = rays_frame * args.steps / dt / 1e6
        out = {
            "metric": "Mrays/sec (+ ms/frame) at %dx%d, depth=%d, %d AO samples" % (WIDTH, HEIGHT, DEPTH, AO),
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic scene (tools/gen_scenes.py, seed 580, %d triangles)" % n_tri) if SYNTH else
                    "reference scene file Assets/%s (no dataset needed)" % SCENE,
            "config": {
                "workload": LABEL,
                "scene": SCENE, "width": WIDTH, "height": HEIGHT, "depth": DEPTH, "ao_samples": AO,
                "rng": "minstd_rand0 (libstdc++ default_random_engine)",
                "rays_per_frame": rays_frame,
                "parallelism": ("interleaved rows x%d + %s all_gather/gather" % (world, "RCCL" if args.backend == "nccl"
                                else args.backend)) if dist_on else "1 GPU",
                "row_sample": ("rows r = 0 mod %d only (the exact pixels of rank 0 in a %d-way interleaved split; "
                               "RNG bases from a full-frame count outside the timed region); value and "
                               "rays_per_frame refer to the sample" % (K, K)) if K > 1 else None,
                "scene_query": "exact BVH + plane tree (rt_bvh.h)" if lib.rt_gpu_accel_active() else
                               "brute force (every primitive per ray, as the reference)",
            },
            "host_enqueue_ms_per_step": round(host_s / args.steps * 1e3, 4),
            "kernel_ms_per_frame": {
                "trace": round(per_frame[0], 4),
                "rank": round(per_frame[1], 4),
                "ao": round(per_frame[2], 4),
                "resolve": round(per_frame[3], 4),
            },
        }
        if check_ok is not None:
            out["frame_matches_reference"] = check_ok
        # AO rays per timed launch: the chunked BVH launches report theirs; a
        # small-scene frame is one launch over all of its AO rays
        k_units = k_rays.value if k_rays.value else int(local["rays_ao"]) * max(frames.value, 1)
        out["roofline"] = roofline(args.workload, k_ms.value, k_launches.value, k_units, int(local["rays_ao"]))
        if not dist_on and K == 1:
            out["render_call_ms"] = render_latency(lib, rt580, params, torch)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(lib, rt580, helpers, root)
        print(json.dumps(out), file=json_out, flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()


def log(msg):
    print("[bench %s] %s" % (time.strftime("%H:%M:%S"), msg), file=sys.stderr, flush=True)


def roofline(workload, k_ms, k_launches, k_rays, rays_ao_frame):
    """Roofline of the AO ray kernel (the scene query of every AO sample; 95 %
    of the frame's rays). Neither MFMA nor HBM bounds it (no dense
    contraction; the scene is re-read from L2/MALL, see `traffic`): it is
    bound by VALU instruction issue. achieved = VALU wave-instructions per AO
    ray (rocprofv3 SQ_INSTS_VALU per dispatch / AO rays per dispatch, from the
    committed profile summary profiles/r02/roofline_<workload>.json) x the AO
    rays of one launch / that launch's mean duration, measured here with HIP
    events around every launch on its own stream (rt_gpu_profile_ao_kernel).
    peak = 1024 SIMDs x one wave64 VALU instruction per 2 cycles x 2.4 GHz."""
    res = {"kernel": "ao_kernel (AO ray scene query)", "bound": "valu", "unit": "Ginst/s",
           "peak": VALU_PEAK_GINST, "achieved": None, "frac": None, "traffic": None}
    if k_launches <= 0 or k_ms <= 0:
        res["note"] = "no AO kernel launch was timed"
        return res
    launch_s = k_ms / k_launches * 1e-3
    rays_launch = k_rays / k_launches
    res["launch_ms"] = round(launch_s * 1e3, 4)
    res["ao_rays_per_launch"] = int(rays_launch)
    path = os.path.join(REPO, "profiles", "r02", "roofline_%s.json" % workload)
    prof = None
    if os.path.exists(path):
        try:
            prof = json.load(open(path))
        except (ValueError, OSError):
            prof = None
    if not prof or not prof.get("valu_per_ao_ray"):
        res["note"] = "no committed counter profile for this workload (%s)" % os.path.relpath(path, REPO)
        return res
    res["kernel"] = prof["kernel"]
    achieved = prof["valu_per_ao_ray"] * rays_launch / launch_s / 1e9
    res["achieved"] = round(achieved, 2)
    res["frac"] = round(achieved / VALU_PEAK_GINST, 4)
    if prof.get("hbm_bytes_per_ao_ray") is not None:
        traffic = prof["hbm_bytes_per_ao_ray"] * rays_launch
        res["traffic"] = round(traffic)
        res["hbm"] = {"achieved": round(traffic / launch_s / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(traffic / launch_s / 1e9 / HBM_PEAK_GBS, 4)}
    res["per_ray"] = {"valu_wave_insts": round(prof["valu_per_ao_ray"], 4),
                      "hbm_bytes": prof.get("hbm_bytes_per_ao_ray")}
    res["profile"] = {"file": os.path.relpath(path, REPO), "launch_ms_rocprof": prof.get("avg_ms"),
                      "valu_issue_frac_rocprof": prof.get("valu_issue_frac"),
                      "frame_share_rocprof": prof.get("frame_share"), "top_kernels": prof.get("top_kernels")}
    res["note"] = ("VALU-issue roofline: counter-measured VALU wave-instructions per AO ray x AO rays per launch "
                   "/ live launch time; traffic = FETCH_SIZE+WRITE_SIZE (x1 KiB) per AO ray x rays per launch "
                   "(HBM is not the bound: see hbm.frac)")
    return res


def render_latency(lib, rt580, params, torch, n=3):
    """Blocking rt_gpu_render (what Render() calls): first launch -> int16
    framebuffer on the host (SURVEY §8d ms/frame), excluding scene load/upload
    and the PPM write. Mean of n calls after the timed region, after one untimed
    call (the first sizes the pinned staging buffer of the host copy)."""
    import numpy as np
    host = np.zeros(params.width * params.height * 3, dtype=np.int16)
    rt580.check(lib.rt_gpu_render(ctypes.byref(params), host.ctypes.data), "rt_gpu_render")
    times = []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rt580.check(lib.rt_gpu_render(ctypes.byref(params), host.ctypes.data), "rt_gpu_render")
        times.append((time.perf_counter() - t0) * 1e3)
    return round(sum(times) / len(times), 4)


def cpu_baseline(lib, rt580, helpers, root):
    """The repository's CPU restatement (oracle/) in ref-faithful mode (the
    reference's per-call work: string mesh lookup and ComputeModelMatrix per
    shape per IntersectScene call, the unused Matrix::Inverse + TransformPoint
    per triangle test; oracle_set_mode(1)) on a bounded sample of the same
    workload (CPU_SAMPLE), on 1 core and on all of this host's cores (threads).
    The reference itself does not travel to this box."""
    threads = env_int("OMP_NUM_THREADS", os.cpu_count() or 1)
    if CPU_SAMPLE[0] == "pixels":
        pts = stratified_pixels(CPU_SAMPLE[1], WIDTH, HEIGHT)
        ao = CPU_SAMPLE[2] if len(CPU_SAMPLE) > 2 else AO
        threads = min(threads, len(pts))

        def run(nt):
            return helpers.oracle_time_pixels(SCENE, WIDTH, HEIGHT, DEPTH, ao, pts, threads=nt, root=root,
                                              faithful=True)
        sample = ("%s %dx%d depth=%d AO=%d: %d pixel(s) of the full-resolution frame on a stratified grid "
                  "(RNG at an estimated draw offset: same work per pixel, not the frame's exact bytes)%s"
                  % (SCENE, WIDTH, HEIGHT, DEPTH, ao, len(pts),
                     "" if ao == AO else "; AO %d instead of %d (CPU cost per ray is independent of the ray's "
                     "kind: the reference tests every primitive per ray)" % (ao, AO)))
    else:
        w, h, depth, ao = CPU_SAMPLE

        def run(nt):
            return helpers.oracle_render(SCENE, w, h, depth, ao, True, threads=nt, root=root, faithful=True)[1]
        sample = ("%s %dx%d depth=%d AO=%d (a downscaled frame of the workload, %.4g%% of its pixels)"
                  % (SCENE, w, h, depth, ao, 100.0 * w * h / (WIDTH * HEIGHT)))
    t0 = time.perf_counter()
    cnt = run(1)
    secs1 = time.perf_counter() - t0
    rays = cnt["rays_total"]
    secsn = secs1
    if threads > 1:
        t0 = time.perf_counter()
        run(threads)
        secsn = time.perf_counter() - t0
    cpu = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {
        "value": float("%.4g" % (rays / secs1 / 1e6)),
        "unit": "Mrays/s",
        "cores": 1,
        "kind": "port",
        "seconds": round(secs1, 3),
        "rays": rays,
        "all_cores": {"value": float("%.4g" % (rays / secsn / 1e6)), "cores": threads, "seconds": round(secsn, 3)},
        "cpu": cpu,
        "sample": sample + ", oracle/rt_oracle.cpp in ref-faithful mode (the reference's arithmetic and "
                  "per-call work; its cost model checked against the reference binary in the build container, "
                  "DESIGN.md)",
    }


if __name__ == "__main__":
    main()

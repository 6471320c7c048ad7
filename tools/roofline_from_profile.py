#!/usr/bin/env python3
"""Per-AO-ray counter figures of the AO ray kernel from a tools/profile.sh
directory, for bench.py's roofline block.

Reads the kernel stats + PMC passes (summarize_profile.summarize) and the bench
JSON line of the trace pass (trace.log: AO rays per launch, measured live in
that run), and writes profiles/$PROFILE_ROUND/roofline_<workload>.json
(default r04) and prints it:
  kernel, avg_ms               the AO ray kernel (ao_kernel* / ao_near_kernel* / ao_trace_kernel*)
  valu_per_ao_ray              SQ_INSTS_VALU per dispatch / AO rays per dispatch
  hbm_bytes_per_ao_ray         (FETCH_SIZE + WRITE_SIZE) x 1 KiB per dispatch / AO rays
  valu_issue_frac              SQ_INSTS_VALU / (avg duration x VALU issue peak)
  frame_share, top_kernels     shares of the profiled GPU time

usage: roofline_from_profile.py <prof_dir> <workload>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import summarize_profile  # noqa: E402

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_line(path):
    for line in open(path):
        line = line.strip()
        if line.startswith("{") and '"metric"' in line:
            return json.loads(line)
    raise SystemExit("no bench JSON line in %s" % path)


def main():
    d, workload = sys.argv[1], sys.argv[2]
    summ = summarize_profile.summarize(d)
    b = bench_line(os.path.join(d, "trace.log"))
    rays_launch = b["roofline"]["ao_rays_per_launch"]
    ks = summ["kernels"]
    name = max((k for k in ks if k.startswith(("ao_kernel", "ao_near_kernel", "ao_trace_kernel"))), key=lambda k: ks[k]["total_ns"])
    k = dict(ks[name])
    c = dict(k["counters"])
    # a step-budgeted AO trace pass (ao_trace_kernel<..., BUDGET>) is followed by
    # ao_late_kernel for the rays it left (one launch each per chunk; the live
    # HIP-event timer spans both): the AO ray kernel is the pair
    late = [n for n in ks if n.startswith("ao_late_kernel")]
    if name.startswith("ao_trace_kernel") and late:
        lk = ks[late[0]]
        assert lk["calls"] == k["calls"], (lk["calls"], k["calls"])
        name = "%s + %s" % (name, late[0])
        for key in ("SQ_INSTS_VALU", "SQ_INSTS_SALU"):
            c[key] = c.get(key, 0) + lk["counters"].get(key, 0)
        if "hbm_bytes" in k and "hbm_bytes" in lk:
            k["hbm_bytes"] = k["hbm_bytes"] + lk["hbm_bytes"]
        k["avg_ns"] = k["avg_ns"] + lk["avg_ns"]
        k["total_ns"] = k["total_ns"] + lk["total_ns"]
        pk = summ["peaks"]
        k["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (k["avg_ns"] * 1e-9) / pk["valu_wave_insts_per_s"]
        k["hbm_frac"] = (k["hbm_bytes"] / (k["avg_ns"] * 1e-9) / pk["hbm_bytes_per_s"]) if "hbm_bytes" in k else 0
    total = sum(v["total_ns"] for v in ks.values())
    top = sorted(ks.items(), key=lambda kv: -kv[1]["total_ns"])[:6]
    out = {
        "workload": workload,
        "source": os.path.relpath(os.path.abspath(d), REPO),
        "kernel": name,
        "avg_ms": round(k["avg_ns"] / 1e6, 4),
        "calls": k["calls"],
        "ao_rays_per_launch": rays_launch,
        "valu_per_ao_ray": c["SQ_INSTS_VALU"] / rays_launch,
        "salu_per_ao_ray": c.get("SQ_INSTS_SALU", 0) / rays_launch,
        "hbm_bytes_per_ao_ray": k["hbm_bytes"] / rays_launch if "hbm_bytes" in k else None,
        "valu_issue_frac": round(k.get("valu_issue_frac", 0), 4),
        "hbm_frac": round(k.get("hbm_frac", 0), 4),
        "l2_hit": round(k.get("l2_hit", 0), 4),
        "clock_ghz": round(k.get("clock_ghz", 0), 3),
        "wait_any_frac": round(k.get("sq_wait_any_frac", 0), 4),
        "frame_share": round(k["total_ns"] / total, 4),
        "top_kernels": [[n, round(v["total_ns"] / total, 4)] for n, v in top],
        "peaks": summ["peaks"],
    }
    dst = os.path.join(REPO, "profiles", os.environ.get("PROFILE_ROUND", "r04"), "roofline_%s.json" % workload)
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

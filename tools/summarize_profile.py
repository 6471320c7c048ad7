#!/usr/bin/env python3
"""Summarize a tools/profile.sh directory (rocprofv3 kernel trace + PMC passes)
into per-kernel figures the bench's roofline block is computed from.

Per kernel (template instantiations kept apart):
  calls, avg_ns, pct                      kernel trace (trace_kernel_stats.csv)
  counters                                mean per dispatch over the PMC passes
  valu_issue_frac                         SQ_INSTS_VALU / (avg_ns * VALU issue peak)
  salu_per_valu, vmem/smem per wave ...
  hbm_bytes                               FETCH_SIZE*1024 + WRITE_SIZE*1024 (per dispatch)
  hbm_bytes_hi                            the same with MI355X_MICROARCH.md's gfx950 x2 read
                                          correction (exact for 16-B/lane streaming reads;
                                          other widths are uncalibrated -> a range)
  clock_ghz                               GRBM_GUI_ACTIVE / 8 XCDs / avg_ns
  l2_hit                                  TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)

Peaks (MI355X_MICROARCH.md): 256 CUs x 4 SIMDs, one wave64 VALU instruction
per SIMD every 2 cycles at 2.4 GHz = 1.2288e12 wave-instructions/s; HBM 8 TB/s.

With PROFILE_AFTER=<kernel> (e.g. row_scan_kernel): only the dispatches
after the first dispatch of that kernel -- bench.py --row-sample's untimed
full-frame count pass comes first, so the summary is the timed frames'. The
kernel statistics then come from the per-dispatch trace (trace_kernel_trace.csv)
and the counters from the PMC rows past the marker in each pass.

usage: summarize_profile.py <prof_dir> <out.json>"""
import collections
import csv
import glob
import json
import os
import re
import sys

CUS, SIMDS, CLOCK_HZ = 256, 4, 2.4e9
VALU_PEAK = CUS * SIMDS * CLOCK_HZ / 2.0   # wave-instructions per second
HBM_PEAK = 8.0e12                          # bytes per second


def short(name):
    n = name.strip()
    if n.startswith("void "):
        n = n[5:]
    depth, cut = 0, len(n)
    for i, ch in enumerate(n):  # drop the parameter list, keep template arguments
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    n = n[:cut].replace("rt580::", "")
    if n.startswith("rocprim::"):
        m = re.search(r"detail::(\w+)<", n)
        n = "rocprim::" + (m.group(1) if m else "kernel")
    return n


def after_marker(rows, name_key, order_key, marker):
    """rows past the first row whose kernel name contains marker (by order_key)"""
    rows = sorted(rows, key=lambda r: int(r[order_key]))
    for i, r in enumerate(rows):
        if marker in r[name_key]:
            return rows[i + 1:]
    return rows


def summarize(d):
    marker = os.environ.get("PROFILE_AFTER", "")
    stats = collections.defaultdict(lambda: {"calls": 0, "total_ns": 0.0, "pct": 0.0})
    if marker:
        tr = after_marker(list(csv.DictReader(open(os.path.join(d, "trace_kernel_trace.csv")))), "Kernel_Name",
                          "Start_Timestamp", marker)
        tot = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr) or 1
        for r in tr:
            s = stats[short(r["Kernel_Name"])]
            dt = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            s["calls"] += 1
            s["total_ns"] += dt
            s["pct"] += 100.0 * dt / tot
    else:
        for r in csv.DictReader(open(os.path.join(d, "trace_kernel_stats.csv"))):
            s = stats[short(r["Name"])]
            s["calls"] += int(r["Calls"])
            s["total_ns"] += float(r["TotalDurationNs"])
            s["pct"] += float(r["Percentage"])
    for s in stats.values():
        s["avg_ns"] = s["total_ns"] / max(s["calls"], 1)
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pmc*_counter_collection.csv"))):
        rows = list(csv.DictReader(open(f)))
        if marker:
            rows = after_marker(rows, "Kernel_Name", "Dispatch_Id", marker)
        for r in rows:
            pmc[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, s in stats.items():
        c = {n: sum(v) / len(v) for n, v in pmc.get(k, {}).items()}
        rec = dict(s, counters=c)
        ns = s["avg_ns"]
        if "SQ_INSTS_VALU" in c and ns > 0:
            rec["valu_insts"] = c["SQ_INSTS_VALU"]
            rec["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (ns * 1e-9 * VALU_PEAK)
        if "SQ_INSTS_SALU" in c and c.get("SQ_INSTS_VALU"):
            rec["salu_per_valu"] = c["SQ_INSTS_SALU"] / c["SQ_INSTS_VALU"]
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rec["hbm_bytes"] = (c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            rec["hbm_bytes_hi"] = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024.0
            if ns > 0:
                rec["hbm_frac"] = rec["hbm_bytes"] / (ns * 1e-9) / HBM_PEAK
                rec["hbm_frac_hi"] = rec["hbm_bytes_hi"] / (ns * 1e-9) / HBM_PEAK
        if "GRBM_GUI_ACTIVE" in c and ns > 0:
            rec["clock_ghz"] = c["GRBM_GUI_ACTIVE"] / 8.0 / ns
        if "TCC_HIT_sum" in c and (c["TCC_HIT_sum"] + c.get("TCC_MISS_sum", 0)) > 0:
            rec["l2_hit"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c.get("TCC_MISS_sum", 0))
        if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"] > 0:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if n in c:
                    rec[n.lower() + "_frac"] = c[n] / c["SQ_WAVE_CYCLES"]
        kernels[k] = rec
    return {"source": os.path.basename(os.path.normpath(d)),
            "peaks": {"valu_wave_insts_per_s": VALU_PEAK, "hbm_bytes_per_s": HBM_PEAK,
                      "note": "MI355X_MICROARCH.md: 256 CUs x 4 SIMDs, wave64 VALU issue every 2 cycles, "
                              "2.4 GHz; HBM3E 8 TB/s"},
            "kernels": kernels}


def main():
    d, out = sys.argv[1], sys.argv[2]
    res = summarize(d)
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    rows = sorted(res["kernels"].items(), key=lambda kv: -kv[1]["total_ns"])
    print("%-34s %5s %11s %6s %6s %6s %9s %6s" % ("kernel", "calls", "avg_us", "pct", "valu", "hbm", "hbm_B", "l2hit"))
    for k, v in rows[:16]:
        print("%-34s %5d %11.1f %5.1f%% %6s %6s %9s %6s" % (
            k[:34], v["calls"], v["avg_ns"] / 1e3, v["pct"],
            "%.3f" % v["valu_issue_frac"] if "valu_issue_frac" in v else "-",
            "%.3f" % v["hbm_frac"] if "hbm_frac" in v else "-",
            "%.3g" % v["hbm_bytes"] if "hbm_bytes" in v else "-",
            "%.3f" % v["l2_hit"] if "l2_hit" in v else "-"))


if __name__ == "__main__":
    main()

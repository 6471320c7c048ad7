#!/usr/bin/env python3
"""Per-kernel GPU time of a rocprofv3 kernel trace, split at the end of the
first row_scan_kernel dispatch (bench.py --row-sample: the untimed full-frame
count pass comes first) -- what the timed frames spend, kernel by kernel.

usage: split_trace.py <kernel_trace.csv>"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    cut = None
    for r in rows:
        if r["Kernel_Name"].startswith("rt580::row_scan_kernel") or "row_scan_kernel" in r["Kernel_Name"]:
            cut = int(r["End_Timestamp"])
            break
    parts = {"count_pass": collections.Counter(), "frames": collections.Counter()}
    calls = {"count_pass": collections.Counter(), "frames": collections.Counter()}
    for r in rows:
        name = r["Kernel_Name"].split("(")[0]
        dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        key = "count_pass" if cut is not None and int(r["End_Timestamp"]) <= cut else "frames"
        parts[key][name] += dur
        calls[key][name] += 1
    for key in ("count_pass", "frames"):
        tot = sum(parts[key].values())
        print("%s: %.1f ms" % (key, tot / 1e6))
        for name, ns in parts[key].most_common(12):
            print("  %-60s %6d calls %10.1f ms %5.1f%%" % (name[:60], calls[key][name], ns / 1e6, 100.0 * ns / max(tot, 1)))


if __name__ == "__main__":
    main()

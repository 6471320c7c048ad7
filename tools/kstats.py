#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --stats kernel_stats.csv, per frame.
usage: kstats.py <kernel_stats.csv> <frames> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
frames = float(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 12
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total %.2f ms/frame" % (tot / frames / 1e6))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
    print("  %-55s %5d calls %8.3f ms/frame %5.1f%%" % (r["Name"][:55], int(r["Calls"]), float(r["TotalDurationNs"]) / frames / 1e6,
                                                      100 * float(r["TotalDurationNs"]) / tot))

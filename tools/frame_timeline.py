#!/usr/bin/env python3
"""Timeline of the last N frames of a rocprofv3 kernel (+ memory copy) trace:
gaps and durations in order, relative to the frame's first kernel.
usage: frame_timeline.py <kernel_trace.csv> [memory_copy_trace.csv] [--frames N] [--marker frame_init_kernel]"""
import argparse
import csv

ap = argparse.ArgumentParser()
ap.add_argument("kernels")
ap.add_argument("copies", nargs="?")
ap.add_argument("--frames", type=int, default=1)
ap.add_argument("--marker", default="frame_init_kernel")
a = ap.parse_args()
ev = []
for r in csv.DictReader(open(a.kernels)):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-60:]))
if a.copies:
    for r in csv.DictReader(open(a.copies)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY %s %s B" % (r.get("Direction", ""), r.get("Size", ""))))
ev.sort()
starts = [i for i, e in enumerate(ev) if a.marker in e[2]]
i0 = starts[-a.frames]
t0 = ev[i0][0]
prev_end = t0
for s, e, n in ev[i0:]:
    print("%9.1f us  +gap %7.1f  dur %8.1f  %s" % ((s - t0) / 1e3, (s - prev_end) / 1e3, (e - s) / 1e3, n))
    prev_end = max(prev_end, e)
print("frame span %.1f us" % ((prev_end - t0) / 1e3))

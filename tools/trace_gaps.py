#!/usr/bin/env python3
"""GPU busy vs idle over the last timed steps of a rocprofv3 kernel trace:
splits the trace at the given marker kernel's occurrences (one per frame) and
reports, for the last N frames, the wall span, the summed kernel time and the
idle gaps (time no kernel ran), plus the top kernels.
usage: trace_gaps.py <kernel_trace.csv> [frames] [marker]"""
import collections
import csv
import sys

path = sys.argv[1]
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 3
marker = sys.argv[3] if len(sys.argv) > 3 else "frame_init_kernel"
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-50:])
            for r in csv.DictReader(open(path)))
starts = [i for i, e in enumerate(ev) if marker in e[2]]
i0 = starts[-frames] if len(starts) >= frames else 0
sel = ev[i0:]
t0, t1 = sel[0][0], max(e for _, e, _ in sel)
busy, cur_s, cur_e = 0, None, None
for s, e, _ in sel:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
tot = collections.Counter()
cnt = collections.Counter()
for s, e, n in sel:
    tot[n] += e - s
    cnt[n] += 1
print("last %d frames: span %.3f ms, GPU busy %.3f ms (%.1f%%), idle %.3f ms, launches %d" % (
    frames, (t1 - t0) / 1e6, busy / 1e6, 100.0 * busy / (t1 - t0), (t1 - t0 - busy) / 1e6, len(sel)))
for n, v in tot.most_common(12):
    print("  %-50s %5d calls %8.3f ms" % (n, cnt[n], v / 1e6))

#!/bin/bash
# GPU box: kernel traces of the north-star frame's 8-way share (rank 1) and of
# the full frame, 6 timed steps each: GPU busy/idle and per-kernel time of the
# timed frames (tools/trace_gaps.py), the raw traces kept for the timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for K in 8 1; do
  R=$(( K > 1 ? 1 : 0 ))
  OUT=gpurun_out/kt_f100k_K$K
  mkdir -p $OUT
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT -o trace -- python3 bench.py --workload field100k_1080p --no-cpu-baseline --no-check --steps 6 --warmup 3 --row-sample $K --row-rank $R > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
  f=$(ls $OUT/*kernel_trace.csv | head -1)
  python3 tools/trace_gaps.py $f 6 > $OUT/gaps.txt && cat $OUT/gaps.txt
  python3 tools/frame_timeline.py $f --frames 2 > $OUT/timeline.txt
  gzip -f $f
done

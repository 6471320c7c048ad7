#!/bin/bash
# GPU box: rocprofv3 trace + PMC passes (short runs) for the triangle workloads,
# roofline summaries, then the bench lines with CPU baseline.
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for W in "$@"; do
  ARGS="--workload $W --steps 2 --warmup 1"
  [ "$W" = field1m ] && ARGS="$ARGS --row-sample 16"
  tools/profile.sh ${TAG}_$W $ARGS || exit 1
  # a row sample's untimed full-frame count pass comes first: summarize the timed frames only
  AFTER=""; [ "$W" = field1m ] && AFTER=row_scan_kernel
  RT580_PROFILE_AFTER=$AFTER python tools/roofline_from_profile.py gpurun_out/prof_${TAG}_$W $W > gpurun_out/roofline_$W.json || exit 1
  RT580_PROFILE_AFTER=$AFTER python tools/summarize_profile.py gpurun_out/prof_${TAG}_$W gpurun_out/prof_${TAG}_$W/summary.json || exit 1
  # the raw per-dispatch CSVs are large (gpurun copies back <= 64 MiB): keep the summaries
  rm -f gpurun_out/prof_${TAG}_$W/pmc*_counter_collection.csv gpurun_out/prof_${TAG}_$W/trace_kernel_trace.csv
done
for W in "$@"; do
  ARGS="--workload $W"
  [ "$W" = field1m ] && ARGS="$ARGS --row-sample 16"
  timeout -k 10 1000 python bench.py $ARGS > gpurun_out/bench_${TAG}_$W.json 2> gpurun_out/bench_${TAG}_$W.err || { tail -5 gpurun_out/bench_${TAG}_$W.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$W.json')); print('$W', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
done

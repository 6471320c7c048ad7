#!/bin/bash
# GPU box: rocprofv3 kernel trace + PMC passes for the roofline workloads, then
# the bench lines (with CPU baseline) of the same workloads.
# usage: tools/gpu_profiles.sh <tag> <workload>...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for W in "$@"; do
  tools/profile.sh ${TAG}_$W --workload $W || exit 1
  python tools/roofline_from_profile.py gpurun_out/prof_${TAG}_$W $W > gpurun_out/roofline_$W.json || exit 1
  python tools/summarize_profile.py gpurun_out/prof_${TAG}_$W gpurun_out/prof_${TAG}_$W/summary.json || exit 1
  # the raw per-dispatch CSVs are large (gpurun copies back <= 64 MiB): keep the summaries
  rm -f gpurun_out/prof_${TAG}_$W/pmc*_counter_collection.csv gpurun_out/prof_${TAG}_$W/trace_kernel_trace.csv
done
for W in "$@"; do
  timeout -k 10 900 python bench.py --workload $W > gpurun_out/bench_${TAG}_$W.json 2> gpurun_out/bench_${TAG}_$W.err || { tail -5 gpurun_out/bench_${TAG}_$W.err; exit 1; }
  cat gpurun_out/bench_${TAG}_$W.json
done

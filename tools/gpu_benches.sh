#!/bin/bash
# GPU box: bench lines of the BASELINE workloads (with CPU baseline).
# usage: tools/gpu_benches.sh <tag> "<workload> [args]" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
i=0
for W in "$@"; do
  i=$((i+1))
  timeout -k 10 1000 python bench.py --workload $W > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err || { tail -5 gpurun_out/bench_${TAG}_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$i.json')); print('$W', d['value'], d['ms_per_step'], d['kernel_ms_per_frame'], d['roofline'].get('frac'), d.get('cpu_baseline',{}).get('value'))"
done

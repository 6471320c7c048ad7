#!/bin/bash
# GPU box: per-kernel A/B of environment settings on one workload.
# usage: tools/gpu_kab.sh <workload> "ENV=a" "ENV=b" ...   (each: bench line + rocprofv3 kernel stats)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W=$1; shift
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --no-north-star > gpurun_out/kab_$i.json 2> gpurun_out/kab_$i.err || { tail -5 gpurun_out/kab_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/kab_$i.json')); print('== $E:', d['value'], 'Mrays/s', d['ms_per_step'], 'ms', d['kernel_ms_per_frame'])"
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kab_prof_$i -o k -- python3 bench.py --workload $W --no-cpu-baseline --no-north-star --steps 3 --warmup 1 > gpurun_out/kab_prof_$i.log 2>&1 || { tail -5 gpurun_out/kab_prof_$i.log; exit 1; }
  python tools/kstats.py $(ls gpurun_out/kab_prof_$i/*/k_kernel_stats.csv gpurun_out/kab_prof_$i/k_kernel_stats.csv 2>/dev/null | head -1) 8 14
  rm -f gpurun_out/kab_prof_$i/*/k_kernel_trace.csv gpurun_out/kab_prof_$i/k_kernel_trace.csv
done

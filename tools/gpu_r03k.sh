#!/bin/bash
# GPU box: XCD-aware block order A/B on the north-star frame (RT580_XCD_ORDER
# 0/1), then the per-level queue sizes (RT580_PROGRESS=1) of the full frame and
# of rank 1's 8-way share.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RT580_XCD_ORDER=0 RT580_XCD_ORDER=1; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['kernel_ms_per_frame'], d['roofline']['launch_ms'])"
done
RT580_PROGRESS=1 timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --steps 1 --warmup 0 > gpurun_out/prog_K1.json 2> gpurun_out/prog_K1.err || { tail -5 gpurun_out/prog_K1.err; exit 1; }
RT580_PROGRESS=1 timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --steps 1 --warmup 0 --row-sample 8 --row-rank 1 > gpurun_out/prog_K8.json 2> gpurun_out/prog_K8.err || { tail -5 gpurun_out/prog_K8.err; exit 1; }
grep -c rt580 gpurun_out/prog_K1.err gpurun_out/prog_K8.err

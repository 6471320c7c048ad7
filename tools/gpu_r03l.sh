#!/bin/bash
# GPU box: the GPU suite with the multi-ray brute scans, then their A/B on the
# north-star frame (RT580_BRUTE_RAYS 1/4/8) and the 8-way share of rank 1.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for E in RT580_BRUTE_RAYS=1 RT580_BRUTE_RAYS=4 RT580_BRUTE_RAYS=8; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['kernel_ms_per_frame'], d['roofline']['launch_ms'])"
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --row-sample 8 --row-rank 1 --steps 5 > gpurun_out/s_$E.json 2> gpurun_out/s_$E.err || { tail -5 gpurun_out/s_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s_$E.json')); print('$E K8 r1', d['ms_per_step'])"
done

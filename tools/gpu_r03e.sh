#!/bin/bash
# GPU box: GPU tests, then the north-star frame's bench line + kernel stats,
# and the rank-0 share of an 8-way row split (--row-sample 8).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
tools/gpu_kab.sh field100k_1080p "RT580_PROGRESS=0" || exit 1
for K in 8; do
  timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-north-star --row-sample $K > gpurun_out/rs$K.json 2> gpurun_out/rs$K.err || { tail -5 gpurun_out/rs$K.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rs$K.json')); print('row-sample $K', d['value'], d['ms_per_step'])"
done

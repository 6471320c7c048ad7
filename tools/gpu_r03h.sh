#!/bin/bash
# GPU box: the GPU suite, then the split any-hit brute scans A/B on the
# north-star frame (RT580_BRUTE_SPLIT 1 = closest only, 3 = both) and the
# north-star frame's K = 1 and 8 rank shares.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for E in RT580_BRUTE_SPLIT=1 RT580_BRUTE_SPLIT=3; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['kernel_ms_per_frame'], d['render_call_ms'])"
done
tools/gpu_rank_shares.sh field100k_1080p 4 "1 8" > gpurun_out/shares_f100k.log 2>&1 || { tail -5 gpurun_out/shares_f100k.log; exit 1; }
tail -2 gpurun_out/shares_f100k.log

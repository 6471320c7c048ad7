#!/bin/bash
# GPU box: the GPU suite with the multi-ray brute scans and the two-stream
# slots, then A/Bs on the north-star frame and its 8-way share of rank 1:
# default (RT580_BRUTE_RAYS=8, RT580_TRACE_PRIORITY=1), brute rays 1, trace
# priority 0, grid lists without inline planes, all sort bits; config 2 with and without the
# trace priority.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
for E in RT580_BRUTE_RAYS=8 RT580_BRUTE_RAYS=1 RT580_TRACE_PRIORITY=0 RT580_GRID_INLINE=0 RT580_SORT_BITS=0; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['kernel_ms_per_frame'], d['roofline']['launch_ms'], d['render_call_ms'])"
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --row-sample 8 --row-rank 1 --steps 5 > gpurun_out/s_$E.json 2> gpurun_out/s_$E.err || { tail -5 gpurun_out/s_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s_$E.json')); print('$E K8 r1', d['ms_per_step'])"
done
for E in RT580_TRACE_PRIORITY=1 RT580_TRACE_PRIORITY=0; do
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star > gpurun_out/c_$E.json 2> gpurun_out/c_$E.err || { tail -5 gpurun_out/c_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c_$E.json')); print('$E config2', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'])"
done

#!/bin/bash
# GPU box: AO phases in frame order (RT580_AO_ORDER) and the slots of
# small-scene frames (RT580_SMALL_SLOTS) on config 2; AO order on the
# north-star frame and its 8-way share of rank 1; pipelining tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in "RT580_AO_ORDER=1" "RT580_AO_ORDER=0" "RT580_AO_ORDER=1 RT580_SMALL_SLOTS=3"; do
  T=$(echo $E | tr ' =' '__')
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star > gpurun_out/c_$T.json 2> gpurun_out/c_$T.err || { tail -5 gpurun_out/c_$T.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c_$T.json')); print('$E config2', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'], d['roofline']['launch_ms'], d['roofline']['frac'])"
done
for E in RT580_AO_ORDER=1 RT580_AO_ORDER=0; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['roofline']['launch_ms'], d['roofline']['frac'])"
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --row-sample 8 --row-rank 1 --steps 5 > gpurun_out/s_$E.json 2> gpurun_out/s_$E.err || { tail -5 gpurun_out/s_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s_$E.json')); print('$E K8 r1', d['ms_per_step'])"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_state.py tests/test_gpu_dist.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_state.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_state.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_state.log

#!/bin/bash
# GPU box: list entries in flight per lane in the closest-hit far pass
# (RT580_FAR_CLOSEST_U 4/1) and three frame slots (RT580_SLOTS=3) on the
# north-star frame and its 8-way share of rank 1 (bounded brute slices in all
# of them); then the GPU suite, and the pipelining tests with three slots.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RT580_FAR_CLOSEST_U=4 RT580_FAR_CLOSEST_U=1 RT580_SLOTS=3; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['kernel_ms_per_frame'], d['roofline']['launch_ms'], d['render_call_ms'])"
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --row-sample 8 --row-rank 1 --steps 5 > gpurun_out/s_$E.json 2> gpurun_out/s_$E.err || { tail -5 gpurun_out/s_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s_$E.json')); print('$E K8 r1', d['ms_per_step'])"
done
RT580_SLOTS=3 timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star > gpurun_out/c_slots3.json 2> gpurun_out/c_slots3.err || { tail -5 gpurun_out/c_slots3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/c_slots3.json')); print('slots3 config2', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'])"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
RT580_SLOTS=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_state.py tests/test_gpu_dist.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_slots3.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_slots3.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_slots3.log

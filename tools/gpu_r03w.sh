#!/bin/bash
# GPU box: chunks of 2^27 rays (one AO chunk per north-star frame instead of
# two) vs 2^26 on the north-star frame and config 4; the chunk tests.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RT580_CHUNK_LOG2=26 RT580_CHUNK_LOG2=27; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16])"
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --row-sample 8 --row-rank 1 --steps 5 > gpurun_out/s_$E.json 2> gpurun_out/s_$E.err || { tail -5 gpurun_out/s_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s_$E.json')); print('$E K8 r1', d['ms_per_step'])"
  env $E timeout -k 10 400 python bench.py --workload field100k --no-cpu-baseline > gpurun_out/h_$E.json 2> gpurun_out/h_$E.err || { tail -5 gpurun_out/h_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/h_$E.json')); print('$E field100k 4K', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_chunks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_chunks.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_chunks.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_chunks.log

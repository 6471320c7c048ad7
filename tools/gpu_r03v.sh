#!/bin/bash
# GPU box: inline cell lists on config 5 (RT580_GRID_INLINE 1 = default above
# 300k triangles, 0), then the GPU tests that render the 1M-triangle scene.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RT580_GRID_INLINE=1 RT580_GRID_INLINE=0; do
  env $E timeout -k 10 600 python bench.py --workload field1m --row-sample 16 --no-cpu-baseline > gpurun_out/g_$E.json 2> gpurun_out/g_$E.err || { tail -5 gpurun_out/g_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/g_$E.json')); print('$E field1m', d['value'], d['ms_per_step'], d['scene_upload_s'], d['kernel_ms_per_frame'])"
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_chunks.py -x -q -rs -k field1m --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_field1m.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_field1m.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_field1m.log

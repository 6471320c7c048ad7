#!/bin/bash
# GPU box: direction-grid size on config 5 (1M triangles): 1024^2 (the default
# above 300k triangles) against 2048^2 (RT580_GRID_LOG2=11).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RT580_GRID_LOG2=10 RT580_GRID_LOG2=11; do
  env $E timeout -k 10 500 python bench.py --workload field1m --row-sample 16 --no-cpu-baseline > gpurun_out/g_$E.json 2> gpurun_out/g_$E.err || { tail -5 gpurun_out/g_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/g_$E.json')); print('$E field1m', d['value'], d['ms_per_step'], d['scene_upload_s'], d['kernel_ms_per_frame'], d['roofline']['profile']['top_kernels'][:1] if 'profile' in d['roofline'] else '')"
done

#!/bin/bash
# GPU box: environment-only A/Bs on the north-star frame at HEAD: a 4096^2
# direction grid (RT580_GRID_LOG2=12), AO step budgets 3 and 6.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RT580_GRID_LOG2=11 RT580_GRID_LOG2=12 RT580_AO_BUDGET=3 RT580_AO_BUDGET=6; do
  env $E timeout -k 10 400 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['scene_upload_s'])"
done

#!/bin/bash
# GPU box: frame pipelining of BVH frames (count-schedule replay) A/B on the
# north-star frame, its 8-way rank share, and the default bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RT580_REPLAY=1 RT580_REPLAY=0; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E ns', d['value'], d['ms_per_step'], d['frame_check'], d['kernel_ms_per_frame'])"
done
for K in 2 4 8; do
  timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --row-sample $K > gpurun_out/rs$K.json 2> gpurun_out/rs$K.err || { tail -5 gpurun_out/rs$K.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/rs$K.json')); print('row-sample $K', d['value'], d['ms_per_step'])"
done
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('default', d['value'], d['ms_per_step'], d['frame_check'], 'ns', d['north_star']['value'], d['north_star']['ms_per_step'], d['north_star']['frame_check'], d['north_star'].get('cpu_baseline'))"

#!/bin/bash
# GPU box: the default bench line (config 2 + north_star with isolated AO
# timing and CPU baselines), then config 5's counter profile over its timed
# frames and its bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); n=d['north_star']; print('default', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'], d['roofline']['frac'], d['roofline'].get('isolated'), '| ns', n['value'], n['ms_per_step'], n['render_call_ms'], n['roofline']['frac'], n['roofline'].get('isolated'))"
for E in RT580_SLOTS=3 RT580_SLOTS=4; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16])"
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --row-sample 8 --row-rank 1 --steps 5 > gpurun_out/s_$E.json 2> gpurun_out/s_$E.err || { tail -5 gpurun_out/s_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s_$E.json')); print('$E K8 r1', d['ms_per_step'])"
done
tools/gpu_profiles2.sh r03 field1m

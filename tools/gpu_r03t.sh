#!/bin/bash
# GPU box: the default bench line (config 2 + north_star with isolated AO
# timing and CPU baselines), frame slots 3 vs 4 and the late-pass sort on the
# north-star frame and its 8-way share of rank 1.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); n=d['north_star']; print('default', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'], d['roofline']['frac'], d['roofline'].get('isolated'), '| ns', n['value'], n['ms_per_step'], n['render_call_ms'], n['roofline']['frac'], n['roofline'].get('isolated'))"
for E in RT580_SLOTS=3 RT580_SLOTS=4 RT580_LATE_SORT=0; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16])"
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline --no-check --row-sample 8 --row-rank 1 --steps 5 > gpurun_out/s_$E.json 2> gpurun_out/s_$E.err || { tail -5 gpurun_out/s_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/s_$E.json')); print('$E K8 r1', d['ms_per_step'])"
done


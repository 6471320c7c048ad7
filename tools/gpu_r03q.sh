#!/bin/bash
# GPU box: frame slots 2 vs 3 on config 2 (bench line with Render() latency,
# 8-way share of rank 0), and the 32 x 32-cell AO sort variant on the
# north-star frame.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for E in RT580_SLOTS=2 RT580_SLOTS=3; do
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star > gpurun_out/c_$E.json 2> gpurun_out/c_$E.err || { tail -5 gpurun_out/c_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/c_$E.json')); print('$E config2', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'])"
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --no-check --row-sample 8 --row-rank 0 --steps 10 > gpurun_out/cs_$E.json 2> gpurun_out/cs_$E.err || { tail -5 gpurun_out/cs_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cs_$E.json')); print('$E config2 K8 r0', d['ms_per_step'])"
  env $E timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star --no-check --row-sample 1 --steps 10 --dist > gpurun_out/cd_$E.json 2> gpurun_out/cd_$E.err || { tail -5 gpurun_out/cd_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cd_$E.json')); print('$E config2 dist1', d['ms_per_step'])"
done
for E in RT580_AO_SORT=3 RT580_AO_SORT=4; do
  env $E timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f_$E.json 2> gpurun_out/f_$E.err || { tail -5 gpurun_out/f_$E.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/f_$E.json')); print('$E', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['roofline']['launch_ms'])"
done

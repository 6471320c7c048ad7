#!/bin/bash
# GPU box: pipelining tests and the default bench line (config 2 + north_star,
# CPU baselines) with two slots for small-scene whole frames, then config 5's
# bench line (1M triangles, 7680x4320 d8 AO256, rows 0 mod 16).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_state.py tests/test_gpu_dist.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_state.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_state.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_state.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); n=d['north_star']; print('default', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], '| ns', n['value'], n['ms_per_step'], n['render_call_ms'], n['roofline']['frac'], n['cpu_baseline']['value'], n['cpu_baseline']['matches_gpu_frame'])"
RT580_PROGRESS=1 timeout -k 10 900 python bench.py --workload field1m --row-sample 16 > gpurun_out/bench_field1m.json 2> gpurun_out/bench_field1m.err || { tail -5 gpurun_out/bench_field1m.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_field1m.json')); print('field1m', d['value'], d['ms_per_step'], d['kernel_ms_per_frame'], d['roofline'].get('frac'), d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('matches_gpu_frame'))"

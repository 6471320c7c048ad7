#!/bin/bash
# GPU box: the 2048^2 grid as config 5's default. Config 5 bench (CPU baseline
# and parity flag), the GPU tests that render the 1M-triangle scene, and the
# north-star frame (its default is unchanged: 2048^2).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp RT580_GRID_LOG2=11
timeout -k 10 600 python bench.py --workload field1m --row-sample 16 > gpurun_out/bench_field1m_g11.json 2> gpurun_out/bench_field1m_g11.err || { tail -5 gpurun_out/bench_field1m_g11.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_field1m_g11.json')); print('field1m', d['value'], d['ms_per_step'], d['scene_upload_s'], d['kernel_ms_per_frame'], d['roofline'].get('frac'), d.get('cpu_baseline',{}).get('value'), d.get('cpu_baseline',{}).get('matches_gpu_frame'))"
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_chunks.py -x -q -rs -k field1m --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_field1m_g11.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_field1m_g11.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_field1m_g11.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_ns_g11.json 2> gpurun_out/bench_ns_g11.err || { tail -5 gpurun_out/bench_ns_g11.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_ns_g11.json')); print('north-star', d['value'], d['ms_per_step'], d.get('frame_hash'))"

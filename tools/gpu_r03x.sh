#!/bin/bash
# GPU box: the GPU suite on HEAD (2^27-ray chunks), the default bench line and
# the bench lines of configs 3 and 4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 600 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_final.log
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -5 gpurun_out/bench_final.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_final.json')); n=d['north_star']; print('final', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'], d['roofline']['frac'], d['roofline'].get('isolated',{}).get('frac'), '| ns', n['value'], n['ms_per_step'], n['render_call_ms'], n['roofline']['frac'], n['roofline'].get('isolated',{}).get('frac'), n['cpu_baseline']['matches_gpu_frame'])"
for W in cornell10k field100k; do
  timeout -k 10 600 python bench.py --workload $W > gpurun_out/bench_final_$W.json 2> gpurun_out/bench_final_$W.err || { tail -5 gpurun_out/bench_final_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/bench_final_$W.json')); print('$W', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('isolated',{}).get('frac'), d['cpu_baseline']['value'], d['cpu_baseline']['matches_gpu_frame'])"
done

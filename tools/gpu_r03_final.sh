#!/bin/bash
# GPU box: the default bench line (config 2 + north_star, CPU baselines), the
# in-process 2-way split rehearsal, and every rank's share of K = 2, 4, 8
# splits of the north-star frame and config 2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { tail -5 gpurun_out/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_default.json')); n=d['north_star']; print('default', d['value'], d['ms_per_step'], d['frame_check']['matches_reference'], d['render_call_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], '| ns', n['value'], n['ms_per_step'], n['render_call_ms'], n['roofline']['frac'], n['cpu_baseline']['value'], n['cpu_baseline']['matches_gpu_frame'])"
timeout -k 10 300 python bench.py --gpus 2 --rehearse --no-cpu-baseline --no-north-star > gpurun_out/bench_rehearse2.json 2> gpurun_out/bench_rehearse2.err || { tail -5 gpurun_out/bench_rehearse2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_rehearse2.json')); print('rehearse2', d['n_gpus'], d['value'], d['ms_per_step'], d['frame_check'])"
tools/gpu_rank_shares.sh field100k_1080p 4 > gpurun_out/shares_f100k.log 2>&1 || { tail -5 gpurun_out/shares_f100k.log; exit 1; }
tail -3 gpurun_out/shares_f100k.log
tools/gpu_rank_shares.sh config2 10 > gpurun_out/shares_config2.log 2>&1 || { tail -5 gpurun_out/shares_config2.log; exit 1; }
tail -3 gpurun_out/shares_config2.log

set -o pipefail
tools/gpu.sh ab rm "RT580_AO_REFILL=0" "RT580_AO_REFILL=1 RT580_AO_REFILL_MIN=1" "RT580_AO_REFILL=1 RT580_AO_REFILL_MIN=32" "RT580_AO_REFILL=1 RT580_AO_REFILL_MIN=48" "RT580_AO_REFILL=3 RT580_AO_REFILL_MIN=32" -- --workload field100k_1080p --no-cpu-baseline --no-config3 --no-north-star || exit 1
tools/gpu.sh ab rmc "RT580_AO_REFILL=0" "RT580_AO_REFILL=1 RT580_AO_REFILL_MIN=32" "RT580_AO_REFILL=3 RT580_AO_REFILL_MIN=32" -- --workload cornell10k --no-cpu-baseline --no-config3 --no-north-star || exit 1
timeout -k 10 400 python bench.py --dist --no-cpu-baseline --no-config3 > gpurun_out/bdist.json 2> gpurun_out/bdist.err || { tail -5 gpurun_out/bdist.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bdist.json')); print('dist1', d['value'], d['ms_per_step'], d['frame_check'].get('matches_reference'), d['north_star']['ms_per_step'], d['north_star']['frame_check'])" | cut -c1-400

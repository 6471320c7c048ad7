set -o pipefail
mkdir -p gpurun_out
for W in cornell10k field100k_1080p; do
  for B in 0 1 0 1; do
    RT580_AO_BUDGET2=$B timeout -k 10 300 python bench.py --workload $W --steps 3 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/b.json')); print('$W budget2 $B', d['value'], d['ms_per_step'], d['kernel_ms_per_frame']['ao'])"
  done
done

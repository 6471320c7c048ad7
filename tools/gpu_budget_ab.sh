set -o pipefail
mkdir -p gpurun_out
RT580_AO_BUDGET=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -k "configs or bvh or oracle" -v --timeout 300 --timeout-method thread > gpurun_out/pytest_budget.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_budget.log | tail -1; grep FAILED gpurun_out/pytest_budget.log | head
[ $rc -eq 0 ] || exit $rc
for W in field100k_1080p cornell10k; do
  for B in 0 2 4 8 0; do
    RT580_AO_BUDGET=$B timeout -k 10 300 python bench.py --workload $W --steps 3 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err || { tail -5 gpurun_out/b.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/b.json')); print('$W budget $B', d['value'], d['ms_per_step'], d['kernel_ms_per_frame']['ao'])"
  done
done

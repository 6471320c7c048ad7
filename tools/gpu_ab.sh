#!/bin/bash
# GPU box: a pytest subset, then bench lines for A/B environment settings.
# usage: tools/gpu_ab.sh "<pytest -k expr>" "<bench args>" "ENV=a ENV2=b" "ENV=c" ...
set -o pipefail
mkdir -p gpurun_out
K=$1; B=$2; shift 2
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -k "$K" \
    > gpurun_out/pytest_ab.log 2>&1
  rc=$?
  grep -E "passed|failed|error" gpurun_out/pytest_ab.log | tail -2
  grep -E "FAILED|ERROR" gpurun_out/pytest_ab.log | head -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
i=0
for E in "$@"; do
  i=$((i+1))
  env $E timeout -k 10 600 python bench.py $B > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { tail -5 gpurun_out/ab_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$i.json')); print('$E', d['value'], d['ms_per_step'], d['kernel_ms_per_frame'])"
done

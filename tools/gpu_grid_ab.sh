#!/bin/bash
# GPU box: deeper-level grid A/B (RT580_DEEP_GRID) on the full config-2 frame and
# on rank 0's share of an 8-way split, plus the one-rank RCCL multi-rank path.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_state.py -m gpu -v --timeout 200 \
  --timeout-method thread > gpurun_out/pytest_grid.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest_grid.log | tail -1
[ $rc -eq 0 ] || exit $rc
for G in ${GRIDS:-4096 1024 512}; do
  for A in "--check" "--row-sample 8"; do
    n=$(echo "$G $A" | tr -c 'a-z0-9' _)
    RT580_DEEP_GRID=$G timeout -k 10 300 python bench.py $A --steps 50 --no-cpu-baseline > gpurun_out/g_$n.json \
      2> gpurun_out/g_$n.err || { tail -5 gpurun_out/g_$n.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/g_$n.json')); print('grid $G $A', d['value'], d['ms_per_step'], d.get('frame_matches_reference'))"
  done
done
timeout -k 10 300 python bench.py --dist --check --steps 50 --no-cpu-baseline > gpurun_out/dist1.json 2> gpurun_out/dist1.err \
  || { tail -20 gpurun_out/dist1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/dist1.json')); print('dist x1', d['value'], d['ms_per_step'], d.get('frame_matches_reference'))"

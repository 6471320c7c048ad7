#!/bin/bash
# GPU box, round 3: the chunked-pass parity tests, then the bench line (config 2
# + north_star sub-record + CPU baselines) and the in-process split modes.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${1:-chunk}" \
  > gpurun_out/pytest_r03a.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_r03a.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_r03a.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/bench_r03a.json 2> gpurun_out/bench_r03a.err || { tail -20 gpurun_out/bench_r03a.err; exit 1; }
cat gpurun_out/bench_r03a.json
timeout -k 10 300 python bench.py --gpus 2 --rehearse --no-cpu-baseline > gpurun_out/bench_r03a_reh2.json 2> gpurun_out/bench_r03a_reh2.err || { tail -20 gpurun_out/bench_r03a_reh2.err; exit 1; }
cat gpurun_out/bench_r03a_reh2.json
timeout -k 10 120 python bench.py --gpus 2 --no-cpu-baseline > gpurun_out/bench_r03a_n2.json 2> gpurun_out/bench_r03a_n2.err
echo "bench --gpus 2 on one GPU: exit $?"; tail -2 gpurun_out/bench_r03a_n2.err

#!/bin/bash
# GPU box: the -m gpu suite, the smoke test and the default bench line.
# usage: tools/gpu_check.sh [pytest -k expression]
set -o pipefail
mkdir -p gpurun_out
K=${1:-}
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread ${K:+-k "$K"} \
  > gpurun_out/pytest.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest.log | tail -3
grep -E "FAILED|ERROR" gpurun_out/pytest.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = test failures (read the log); anything else: stop here
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_config2.json 2> gpurun_out/bench_config2.err || { tail -5 gpurun_out/bench_config2.err; exit 1; }
cat gpurun_out/bench_config2.json
exit $rc

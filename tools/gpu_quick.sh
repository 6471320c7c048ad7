#!/bin/bash
# GPU box: a subset of the -m gpu suite (pytest -k expression) and one bench line.
# usage: tools/gpu_quick.sh "<pytest -k expr>" "<bench args>" [tag]
set -o pipefail
mkdir -p gpurun_out
TAG=${3:-quick}
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -k "$1" \
    > gpurun_out/pytest_$TAG.log 2>&1
  rc=$?
  grep -E "passed|failed|error" gpurun_out/pytest_$TAG.log | tail -2
  grep -E "FAILED|ERROR" gpurun_out/pytest_$TAG.log | head -20
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ -n "$2" ]; then
  timeout -k 10 600 python bench.py $2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -5 gpurun_out/bench_$TAG.err; exit 1; }
  cat gpurun_out/bench_$TAG.json
fi

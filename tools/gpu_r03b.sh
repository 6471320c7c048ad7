#!/bin/bash
# GPU box: BVH-scene parity subset, then per-kernel A/B on the north-star frame.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  -k "${PYK:-chunk or triangle or bvh or cornell or field or multi_bvh}" > gpurun_out/pytest_r03b.log 2>&1
rc=$?
grep -E "passed|failed|error" gpurun_out/pytest_r03b.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_r03b.log | head -20; exit $rc; }
[ $# -gt 0 ] && tools/gpu_kab.sh "$@"

#!/bin/bash
# GPU box: a pytest subset, the one-frame timeline of a blocking Render() on
# config 2, and the bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$PYK" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$PYK" > gpurun_out/pytest_r03c.log 2>&1
  rc=$?
  grep -E "passed|failed|error" gpurun_out/pytest_r03c.log | tail -2
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/pytest_r03c.log | head -20; exit $rc; }
fi
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/tl -o tl -- python3 bench.py --no-cpu-baseline --no-north-star --steps 3 --warmup 1 > gpurun_out/tl.log 2>&1 || { tail -5 gpurun_out/tl.log; exit 1; }
K=$(ls gpurun_out/tl/*/tl_kernel_trace.csv gpurun_out/tl/tl_kernel_trace.csv 2>/dev/null | head -1)
C=$(ls gpurun_out/tl/*/tl_memory_copy_trace.csv gpurun_out/tl/tl_memory_copy_trace.csv 2>/dev/null | head -1)
python3 tools/frame_timeline.py $K $C --frames 1 > gpurun_out/tl_last.txt
rm -rf gpurun_out/tl
tail -12 gpurun_out/tl_last.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star > gpurun_out/bench_r03c.json 2> gpurun_out/bench_r03c.err || { tail -5 gpurun_out/bench_r03c.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r03c.json')); print('bench', d['value'], d['ms_per_step'], 'render_call_ms', d.get('render_call_ms'), d['frame_check'])"

#!/bin/bash
# GPU box: the GPU suite on the folded quantized-node slab, the north-star
# bench line, then tools/gpu_r03i.sh (kernel traces of the 8-way share and the
# full frame).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rs --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -4 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --workload field100k_1080p --no-cpu-baseline > gpurun_out/f.json 2> gpurun_out/f.err || { tail -5 gpurun_out/f.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/f.json')); print('f100k', d['value'], d['ms_per_step'], d['frame_check']['sha256'][:16], d['kernel_ms_per_frame'], d['render_call_ms'], d['roofline']['launch_ms'])"
tools/gpu_r03i.sh

#!/bin/bash
# GPU box: GPU idle time per north-star frame (K = 1 and rank 0 of K = 8), then
# bench.py through the one-process-per-GPU path: one rank over RCCL (--dist)
# and two ranks over gloo on the one device (rehearsal of N > 1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for K in 1 8; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tg$K -o tg -- python3 bench.py --workload field100k_1080p --no-cpu-baseline --no-north-star --no-check --steps 3 --warmup 1 --row-sample $K > gpurun_out/tg$K.log 2>&1 || exit 1
  F=$(ls gpurun_out/tg$K/*/tg_kernel_trace.csv gpurun_out/tg$K/tg_kernel_trace.csv 2>/dev/null | head -1)
  echo "== K=$K"
  python3 tools/trace_gaps.py $F 3
  rm -rf gpurun_out/tg$K
done
timeout -k 10 400 python bench.py --dist --no-cpu-baseline > gpurun_out/dist1.json 2> gpurun_out/dist1.err || { tail -5 gpurun_out/dist1.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/dist1.json')); print('dist1', d['value'], d['ms_per_step'], d['frame_check'], 'ns', d['north_star']['value'], d['north_star']['ms_per_step'], d['north_star']['frame_check'])"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --backend gloo --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/gloo2.json 2> gpurun_out/gloo2.err || { tail -5 gpurun_out/gloo2.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/gloo2.json')); print('gloo2', d['n_gpus'], d['value'], d['frame_check'], 'ns', d['north_star']['value'], d['north_star']['frame_check'])"

#!/bin/bash
# GPU box (one MI355X): the multi-rank path of bench.py rehearsed with one rank
# (torch.distributed over RCCL, DistFrame: all-gather of the row counts, row-base
# kernel, u8 gamma, async gather, de-interleave), then rank 0's exact share of a
# K-way interleaved split (--row-sample K): the per-rank compute of N = K GPUs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --dist --check --steps 50 --no-cpu-baseline > gpurun_out/dist1.json 2> gpurun_out/dist1.err \
  || { tail -20 gpurun_out/dist1.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/dist1.json')); print('dist x1', d['value'], d['ms_per_step'], d['config']['parallelism'], d.get('frame_matches_reference'))"
for K in 1 2 4 8; do
  timeout -k 10 300 python bench.py --row-sample $K --steps 50 --no-cpu-baseline > gpurun_out/rows$K.json 2> gpurun_out/rows$K.err \
    || { tail -5 gpurun_out/rows$K.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/rows$K.json')); print('row-sample $K', d['value'], d['ms_per_step'], d['config']['rays_per_frame'])"
done

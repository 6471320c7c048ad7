#!/bin/bash
# GPU box: every rank's exact share of a K-way interleaved row split, timed on
# one GPU (bench.py --row-sample K --row-rank r), for K = 1, 2, 4, 8.
# usage: tools/gpu_rank_shares.sh <workload> [steps] [K list, default "1 2 4 8"]
set -o pipefail
mkdir -p gpurun_out
W=$1; S=${2:-5}; KS=${3:-1 2 4 8}
OUT=gpurun_out/shares_$W.jsonl
: > $OUT
for K in $KS; do
  for ((r = 0; r < K; r++)); do
    timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --no-north-star --no-check --steps $S --warmup 2 \
      --row-sample $K --row-rank $r > gpurun_out/share.json 2> gpurun_out/share.err || { tail -5 gpurun_out/share.err; exit 1; }
    python3 -c "import json; d=json.load(open('gpurun_out/share.json')); print(json.dumps({'K': $K, 'r': $r, 'ms': d['ms_per_step'], 'rays': d['config']['rays_per_frame']}))" >> $OUT
    tail -1 $OUT
  done
done
python3 - $OUT <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
t1s = [x["ms"] for x in rows if x["K"] == 1]
t1 = t1s[0] if t1s else float("nan")
for K in sorted({x["K"] for x in rows} - {1}):
    ms = [x["ms"] for x in rows if x["K"] == K]
    print("K=%d: rank ms %s  max %.3f  speed-up t1/max %.2f  (rank 0: %.2f)" % (K, [round(m, 3) for m in ms], max(ms), t1 / max(ms), t1 / ms[0]))
PY

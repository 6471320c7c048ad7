#!/bin/bash
# A/B environment settings with the bench (GPU box only). Usage:
#   REPS=2 tools/ab_env.sh "RT580_TRACE_SCALAR=0" "RT580_TRACE_SCALAR=1" ...
# Prints the per-kernel ms/frame and the frame time per run.
BENCH_ARGS=${BENCH_ARGS:-"--steps 20 --warmup 3 --no-cpu-baseline"}
for rep in $(seq ${REPS:-1}); do
  for setting in "$@"; do
    env $setting timeout -k 10 200 python bench.py $BENCH_ARGS 2>/dev/null \
      | python -c "import sys,json; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$setting', d['kernel_ms_per_frame'], 'frame_ms', d['ms_per_step'], 'Mrays/s', d['value'])" || exit 1
  done
done

#!/bin/bash
# A/B the AO-kernel variants (RT580_AO_VARIANT bits) with the bench, twice,
# interleaved. Prints "variant ao_ms total_ms" per run. GPU box only.
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-0 1 2 3 4 5 6 7}; do
    RT580_AO_VARIANT=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null \
      | python -c "import sys,json; d=json.loads(sys.stdin.read()); print('variant', $v, 'ao_ms', d['kernel_ms_per_frame']['ao'], 'frame_ms', d['ms_per_step'])" || exit 1
  done
done

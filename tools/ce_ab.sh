#!/bin/bash
# config2 bench lines under runtime copy-engine settings
for E in "X=0" "GPU_FORCE_BLIT_COPY_SIZE=0" "GPU_BLIT_ENGINE_TYPE=2" "GPU_BLIT_ENGINE_TYPE=1"; do
  env $E timeout -k 10 120 python3 bench.py --no-cpu-baseline --no-north-star --no-config3 --no-check > gpurun_out/ce.json 2> gpurun_out/ce.err || { echo "$E failed"; tail -3 gpurun_out/ce.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ce.json')); print('$E', d['value'], d['ms_per_step'], d.get('render_call_ms'))"
done

set -o pipefail
B="python bench.py --no-cpu-baseline --no-north-star --no-config3"
for v in "X=0:device" "RT580_D2H_BLOCKS=16:ppm" "RT580_D2H_BLOCKS=64:ppm" "RT580_D2H_BLOCKS=256:ppm" "RT580_D2H_BLOCKS=4096:ppm" "X=0:device" "RT580_D2H_BLOCKS=16:ppm" "RT580_D2H_BLOCKS=64:ppm"; do
  E=${v%%:*}; K=${v##*:}
  env $E timeout -k 10 200 $B --step $K > gpurun_out/st.json 2> gpurun_out/st.err || { tail -3 gpurun_out/st.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/st.json')); print('$E $K', d['value'], d['ms_per_step'], d.get('render_call_ms'), d.get('frame_check',{}).get('matches_reference'))"
done

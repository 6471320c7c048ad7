set -o pipefail
for v in "none 1" "local 0" "local 1" "rccl 1"; do
  timeout -k 10 120 python -u tools/repro_exit.py $v > gpurun_out/rx.log 2>&1; rc=$?
  echo "$v rc=$rc: $(tail -2 gpurun_out/rx.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || exit $rc
done
B="python bench.py --no-cpu-baseline --no-north-star --no-config3"
for v in "X=0:device" "X=0:host16" "X=0:ppm" "GPU_FORCE_BLIT_COPY_SIZE=0:ppm" "X=0:device" "X=0:ppm"; do
  E=${v%%:*}; K=${v##*:}
  env $E timeout -k 10 200 $B --step $K > gpurun_out/st.json 2> gpurun_out/st.err || { tail -3 gpurun_out/st.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/st.json')); print('$E $K', d['value'], d['ms_per_step'], d.get('render_call_ms'), d.get('frame_check',{}).get('matches_reference'))"
done

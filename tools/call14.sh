set -o pipefail
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_multi.py tests/test_gpu_state.py -k "async or replay" > gpurun_out/t14.log 2>&1; rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/t14.log)"; [ $rc -le 1 ] || exit $rc
B="python bench.py --no-cpu-baseline --no-north-star --no-config3"
for v in "X=0:device" "RT580_D2H_MAPPED=0:ppm" "X=0:ppm" "X=0:device" "RT580_D2H_MAPPED=0:ppm" "X=0:ppm"; do
  E=${v%%:*}; K=${v##*:}
  env $E timeout -k 10 200 $B --step $K > gpurun_out/st.json 2> gpurun_out/st.err || { tail -3 gpurun_out/st.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/st.json')); print('$E $K', d['value'], d['ms_per_step'], d.get('render_call_ms'), d.get('frame_check',{}).get('matches_reference'))"
done
timeout -k 10 300 python bench.py --gpus 3 --rehearse --no-cpu-baseline --no-north-star --no-config3 > gpurun_out/b14r.json 2> gpurun_out/b14r.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/b14r.json')); print('rehearse3', d['value'], d['ms_per_step'], d['frame_check'])"
bash tools/call13.sh

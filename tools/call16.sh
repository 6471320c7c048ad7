set -o pipefail
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
B="python bench.py --no-cpu-baseline --no-north-star --no-config3"
for v in "X=0:device" "RT580_D2H_MAPPED=0:ppm" "X=0:ppm" "X=0:device" "RT580_D2H_MAPPED=0:ppm" "X=0:ppm"; do
  E=${v%%:*}; K=${v##*:}
  env $E timeout -k 10 200 $B --step $K > gpurun_out/st.json 2> gpurun_out/st.err || { tail -3 gpurun_out/st.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/st.json')); print('$E $K', d['value'], d['ms_per_step'], d.get('render_call_ms'), d.get('frame_check',{}).get('matches_reference'))"
done
timeout -k 10 300 python bench.py --gpus 3 --rehearse --no-cpu-baseline --no-north-star --no-config3 > gpurun_out/b16r.json 2> gpurun_out/b16r.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/b16r.json')); print('rehearse3', d['value'], d['ms_per_step'], d['frame_check'])"
bash tools/call13.sh || exit 1
cat gpurun_out/blk.txt
bash tools/call15.sh

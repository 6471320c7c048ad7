set -o pipefail
export DL=$PWD/580-raytracer_amd/lib580rt_diag.so
timeout -k 10 500 env RT580_AO_REFILL=1 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_chunks.py tests/test_gpu_configs.py tests/test_gpu_state.py -k "not audit and not ao_audit" > gpurun_out/t19.log 2>&1; rc=$?; echo "refill tests rc=$rc $(tail -1 gpurun_out/t19.log)"; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 env RT580_LIB=$DL RT580_AO_VERIFY=1 RT580_AO_REFILL=1 python -u tools/ao_verify.py field100k_1080p 2 > gpurun_out/arefill.json 2> gpurun_out/arefill.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/arefill.json')); print('audit', {k: d[k] for k in d if k != 'verify'} if isinstance(d, dict) else d)" | cut -c1-600
tools/gpu.sh ab refill "RT580_AO_REFILL=0" "RT580_AO_REFILL=1" "RT580_AO_REFILL=0" "RT580_AO_REFILL=1" -- --workload field100k_1080p --no-cpu-baseline --no-config3 || exit 1
tools/gpu.sh ab refillc3 "RT580_AO_REFILL=0" "RT580_AO_REFILL=1" -- --workload cornell10k --no-cpu-baseline --no-config3 --no-north-star

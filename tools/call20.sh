set -o pipefail
export DL=$PWD/580-raytracer_amd/lib580rt_diag.so
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 500 $PT tests/test_gpu_chunks.py tests/test_gpu_configs.py tests/test_gpu_state.py tests/test_gpu_parity.py -k "not ao_audit" > gpurun_out/t20a.log 2>&1; rc=$?; echo "default tests rc=$rc $(tail -1 gpurun_out/t20a.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 env RT580_AO_REFILL=1 $PT tests/test_gpu_chunks.py tests/test_gpu_configs.py tests/test_gpu_state.py -k "not ao_audit" > gpurun_out/t20b.log 2>&1; rc=$?; echo "refill tests rc=$rc $(tail -1 gpurun_out/t20b.log)"; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 env RT580_LIB=$DL RT580_AO_VERIFY=1 RT580_AO_REFILL=1 python -u tools/ao_verify.py field100k_1080p 2 > gpurun_out/arefill.json 2> gpurun_out/arefill.err; echo "audit rc=$?"; cut -c1-700 gpurun_out/arefill.json
tools/gpu.sh ab refill "RT580_AO_REFILL=0" "RT580_AO_REFILL=1" "RT580_AO_REFILL=0" "RT580_AO_REFILL=1" -- --workload field100k_1080p --no-cpu-baseline --no-config3 || exit 1
tools/gpu.sh shares field100k_1080p 5 "1 8"

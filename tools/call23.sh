set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 env RT580_AO_VARIANT=39964 $PT tests/test_gpu_parity.py > gpurun_out/t23.log 2>&1; rc=$?; echo "2spl tests rc=$rc $(tail -1 gpurun_out/t23.log)"; [ $rc -eq 0 ] || exit 1
tools/gpu.sh ab spl "RT580_AO_VARIANT=7196" "RT580_AO_VARIANT=39964" "RT580_AO_VARIANT=39948" "RT580_AO_VARIANT=7196" "RT580_AO_VARIANT=39964" "RT580_AO_VARIANT=39948" -- --no-cpu-baseline --no-config3 --no-north-star || exit 1

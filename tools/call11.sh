set -o pipefail
PT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
run() { local tag=$1; shift; timeout -k 10 500 $PT "$@" > gpurun_out/t11_$tag.log 2>&1; local rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/t11_$tag.log)"; [ $rc -le 1 ] || exit $rc; }
run multi tests/test_gpu_multi.py -k async
run state tests/test_gpu_state.py -k "async or replay"
run chunks tests/test_gpu_chunks.py tests/test_gpu_configs.py
timeout -k 10 600 python bench.py > gpurun_out/b1.json 2> gpurun_out/b1.err || exit 1
timeout -k 10 300 python bench.py --gpus 3 --rehearse --no-cpu-baseline --no-north-star --no-config3 > gpurun_out/b1r.json 2> gpurun_out/b1r.err || exit 1

set -o pipefail
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_dist.py tests/test_gpu_multi.py -k "dist or deinterleave" > gpurun_out/t30.log 2>&1; rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/t30.log)"; [ $rc -eq 0 ] || { tail -30 gpurun_out/t30.log; exit 1; }
timeout -k 10 400 python bench.py --dist --no-cpu-baseline --no-config3 > gpurun_out/bdist.json 2> gpurun_out/bdist.err || { tail -5 gpurun_out/bdist.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bdist.json')); print('dist1', d['value'], d['ms_per_step'], d['host_enqueue_ms_per_step'], d['frame_check'].get('matches_reference'), d['north_star']['ms_per_step'], d['north_star']['frame_check'].get('sha256'))"

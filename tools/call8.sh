set -o pipefail
export DL=$PWD/580-raytracer_amd/lib580rt_diag.so
timeout -k 10 300 env RT580_LIB=$DL RT580_AO_VERIFY=1 RT580_LATE_WPE=8 RT580_LATE_REREAD=0 python -u tools/ao_verify.py field100k_1080p 2 > gpurun_out/a8r2.json 2> gpurun_out/a8r2.err || exit 1
tools/gpu.sh ab cr "RT580_CELL_RAYS=0" "RT580_CELL_RAYS=16" "RT580_CELL_RAYS=32" "RT580_CELL_RAYS=0" "RT580_CELL_RAYS=16" "RT580_CELL_RAYS=32" -- --workload field100k_1080p --no-cpu-baseline > gpurun_out/cr.txt 2>&1

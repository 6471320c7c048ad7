set -o pipefail
export DL=$PWD/580-raytracer_amd/lib580rt_diag.so
timeout -k 10 300 env RT580_LIB=$DL RT580_AO_VERIFY=1 RT580_AO_BLOCK=15 python -u tools/ao_verify.py field100k_1080p 2 > gpurun_out/ablk.json 2> gpurun_out/ablk.err || exit 1
tools/gpu.sh ab blk "RT580_AO_BLOCK=0" "RT580_AO_BLOCK=13" "RT580_AO_BLOCK=15" "RT580_AO_BLOCK=17" "RT580_AO_BLOCK=0" "RT580_AO_BLOCK=15" -- --workload field100k_1080p --no-cpu-baseline --no-config3 > gpurun_out/blk.txt 2>&1 || exit 1

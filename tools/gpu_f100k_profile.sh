set -o pipefail
mkdir -p gpurun_out
RT580_PROGRESS=1 timeout -k 10 300 python bench.py --workload field100k_1080p --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/f100k_progress.json 2> gpurun_out/f100k_progress.err || { tail -5 gpurun_out/f100k_progress.err; exit 1; }
cat gpurun_out/f100k_progress.json
tools/profile.sh r02_f100k --workload field100k_1080p

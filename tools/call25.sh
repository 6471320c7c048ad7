set -o pipefail
tools/gpu.sh ab res "RT580_RESOLVE=1" "RT580_RESOLVE=0" "RT580_RESOLVE=1" "RT580_RESOLVE=0" -- --no-cpu-baseline --no-config3 --no-north-star || exit 1
tools/gpu.sh ab resk8 "RT580_RESOLVE=1" "RT580_RESOLVE=0" "RT580_RESOLVE=1" "RT580_RESOLVE=0" -- --no-cpu-baseline --no-config3 --no-north-star --no-check --row-sample 8 --row-rank 3 --steps 20 || exit 1
tools/gpu.sh ab resns "RT580_RESOLVE=1" "RT580_RESOLVE=0" -- --workload field100k_1080p --no-cpu-baseline --no-config3 --no-north-star || exit 1

set -o pipefail
tools/gpu.sh ab rf "RT580_AO_REFILL=0" "RT580_AO_REFILL=1" "RT580_AO_REFILL=2" "RT580_AO_REFILL=3" -- --workload field100k_1080p --no-cpu-baseline --no-config3 --no-north-star || exit 1
tools/gpu.sh ab rfc "RT580_AO_REFILL=0" "RT580_AO_REFILL=1" "RT580_AO_REFILL=2" "RT580_AO_REFILL=3" -- --workload cornell10k --no-cpu-baseline --no-config3 --no-north-star || exit 1

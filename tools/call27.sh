set -o pipefail
tools/gpu.sh ab rm "RT580_AO_REFILL=0" "RT580_AO_REFILL=1 RT580_AO_REFILL_MIN=1" "RT580_AO_REFILL=1 RT580_AO_REFILL_MIN=32" "RT580_AO_REFILL=1 RT580_AO_REFILL_MIN=48" "RT580_AO_REFILL=3 RT580_AO_REFILL_MIN=32" -- --workload field100k_1080p --no-cpu-baseline --no-config3 --no-north-star || exit 1
tools/gpu.sh ab rmc "RT580_AO_REFILL=0" "RT580_AO_REFILL=1 RT580_AO_REFILL_MIN=32" "RT580_AO_REFILL=3 RT580_AO_REFILL_MIN=32" -- --workload cornell10k --no-cpu-baseline --no-config3 --no-north-star || exit 1

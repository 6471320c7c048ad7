#!/bin/bash
# GPU box: counter profiles + bench lines (with CPU baselines) of the given
# workloads on HEAD (tools/gpu_profiles2.sh), round-3 tag.
# usage: tools/gpu_r03_prof.sh <workload>...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_profiles2.sh r03 "$@"

#!/bin/bash
# GPU box: config 5's counter profile over its timed frames and its bench line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_profiles2.sh r03 field1m

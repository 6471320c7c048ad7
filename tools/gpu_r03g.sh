#!/bin/bash
# GPU box: counter profile of the north-star frame on HEAD (trace + PMC passes,
# roofline summary), then every rank's exact share of a K-way split for the
# north-star frame and config 2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tools/gpu_profiles2.sh r03 field100k_1080p || exit 1
tools/gpu_rank_shares.sh field100k_1080p 4 > gpurun_out/shares_f100k.log 2>&1 || { tail -5 gpurun_out/shares_f100k.log; exit 1; }
tail -3 gpurun_out/shares_f100k.log
tools/gpu_rank_shares.sh config2 10 > gpurun_out/shares_config2.log 2>&1 || { tail -5 gpurun_out/shares_config2.log; exit 1; }
tail -3 gpurun_out/shares_config2.log

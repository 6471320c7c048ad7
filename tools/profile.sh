#!/bin/bash
# rocprofv3 passes over a short bench run (GPU box).
# usage: tools/profile.sh <tag> [bench args...]   e.g. tools/profile.sh r02_f100k --workload field100k_1080p
# Writes gpurun_out/prof_<tag>/: kernel trace + stats, then one PMC pass per
# counter group (PMC passes carry no other tracing, per the pool's rules).
set -o pipefail
TAG=${1:-run}
shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python3 bench.py --no-cpu-baseline --no-north-star $*"
case "$*" in *--steps*) ;; *) BENCH="$BENCH --steps 3 --warmup 1";; esac
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- $BENCH > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -s KILL 600 rocprofv3 --pmc $GROUP --output-format csv -d $OUT -o pmc$i -- $BENCH > $OUT/pmc$i.log 2>&1 || { echo "pmc group $i failed: $GROUP"; tail -5 $OUT/pmc$i.log; exit 1; }
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F32
GROUPS
ls $OUT | head -50

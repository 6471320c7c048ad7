#!/bin/bash
# rocprofv3 passes over a short bench run (GPU box). Usage: tools/profile.sh <tag>
# Writes gpurun_out/prof_<tag>/: kernel trace + stats, then one PMC pass per
# counter group (PMC passes carry no other tracing, per the pool's rules).
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="python bench.py --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- $BENCH > $OUT/trace.log 2>&1 || exit 1
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $GROUP --output-format csv -d $OUT -o pmc$i -- $BENCH > $OUT/pmc$i.log 2>&1 || { echo "pmc group $i failed: $GROUP"; tail -5 $OUT/pmc$i.log; }
done <<GROUPS
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F32
GROUPS
ls $OUT

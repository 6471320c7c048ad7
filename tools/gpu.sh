#!/bin/bash
# The one GPU-box runner (run from the repo root inside gpurun). Every step
# has its own time limit, writes under gpurun_out/, and a failing step ends
# the script (no retries). Steps chain with && on the gpurun command line, e.g.
#   gpurun -- 'tools/gpu.sh suite && tools/gpu.sh bench r04_default'
#
#   suite [-k EXPR]                 the -m gpu suite (+ smoke), log gpurun_out/pytest_gpu[_k].log
#   bench TAG [bench.py args]       one bench line -> gpurun_out/bench_TAG.json (+ .err)
#   ab TAG "ENV=a ENV2=b" "ENV=c" ... [-- bench.py args]
#                                   one bench line per environment setting -> gpurun_out/ab/TAG_<i>.json
#   shares WORKLOAD [STEPS] [KS]    every rank's exact share of K-way interleaved row splits (bench.py
#                                   --row-sample K --row-rank r), K in KS (default "1 2 4 8")
#   profile TAG [bench.py args]     rocprofv3 kernel trace + one PMC pass per counter group,
#                                   roofline + per-kernel summaries -> gpurun_out/prof_TAG/
#   trace TAG [bench.py args]       kernel trace only (per-dispatch CSV kept): GPU busy/idle and
#                                   per-kernel time of the last frames -> gpurun_out/trace_TAG/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cmd=${1:-}; shift || true

summary() {  # one line per bench JSON: value, ms, frame check, roofline
  python3 - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    fc = d.get("frame_check", {})
    rf = d.get("roofline", {})
    out = [f, d.get("value"), d.get("ms_per_step"), "render_call_ms=%s" % d.get("render_call_ms"),
           "match=%s" % fc.get("matches_reference", fc.get("matches_oracle_rows")), "frac=%s" % rf.get("frac")]
    ns = d.get("north_star")
    if ns:
        nfc = ns.get("frame_check", {})
        out += ["| ns", ns.get("value"), ns.get("ms_per_step"), "frac=%s" % ns.get("roofline", {}).get("frac"),
                "rows_ok=%s px=%s full=%s" % (nfc.get("matches_oracle_rows"), nfc.get("pixels_checked"),
                                              nfc.get("matches_oracle_full_frame"))]
    c3 = d.get("config3")
    if c3:
        out += ["| c3", c3.get("value"), c3.get("ms_per_step"),
                "full=%s" % c3.get("frame_check", {}).get("matches_oracle_full_frame")]
    print(*out)
PY
}

case "$cmd" in
suite)
  K=""; [ "${1:-}" = "-k" ] && K=$2
  LOG=gpurun_out/pytest_gpu${K:+_k}.log
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v -rs --timeout 300 --timeout-method thread ${K:+-k "$K"} \
    > $LOG 2>&1
  rc=$?
  grep -E "passed|failed|error" $LOG | tail -2
  grep -E "FAILED|ERROR|SKIPPED" $LOG | head -20
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
  ;;
bench)
  TAG=$1; shift
  timeout -k 10 1000 python -u bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -8 gpurun_out/bench_$TAG.err; exit 1; }
  summary gpurun_out/bench_$TAG.json
  ;;
ab)
  TAG=$1; shift
  SETS=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do SETS+=("$1"); shift; done
  [ "${1:-}" = "--" ] && shift
  mkdir -p gpurun_out/ab
  i=0
  for E in "${SETS[@]}"; do
    i=$((i+1))
    env $E timeout -k 10 600 python bench.py "$@" > gpurun_out/ab/${TAG}_$i.json 2> gpurun_out/ab/${TAG}_$i.err || { tail -5 gpurun_out/ab/${TAG}_$i.err; exit 1; }
    echo "$E: $(summary gpurun_out/ab/${TAG}_$i.json)"
  done
  ;;
shares)
  W=$1; S=${2:-5}; KS=${3:-1 2 4 8}
  OUT=gpurun_out/shares_$W.jsonl
  : > $OUT
  for K in $KS; do
    for ((r = 0; r < K; r++)); do
      timeout -k 10 300 python bench.py --workload $W --no-cpu-baseline --no-north-star --no-config3 --no-check --steps $S --warmup 2 \
        --row-sample $K --row-rank $r > gpurun_out/share.json 2> gpurun_out/share.err || { tail -5 gpurun_out/share.err; exit 1; }
      python3 -c "import json; d=json.load(open('gpurun_out/share.json')); print(json.dumps({'K': $K, 'r': $r, 'ms': d['ms_per_step'], 'rays': d['config']['rays_per_frame']}))" >> $OUT
      tail -1 $OUT
    done
  done
  python3 - $OUT <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])]
t1s = [x["ms"] for x in rows if x["K"] == 1]
t1 = t1s[0] if t1s else float("nan")
for K in sorted({x["K"] for x in rows} - {1}):
    ms = [x["ms"] for x in rows if x["K"] == K]
    print("K=%d: rank ms %s  max %.3f  speed-up t1/max %.2f" % (K, [round(m, 3) for m in ms], max(ms), t1 / max(ms)))
PY
  ;;
profile)
  TAG=$1; shift
  OUT=gpurun_out/prof_$TAG
  mkdir -p $OUT
  # the step's frames only: no Render() latency frames (their AO runs in two launches,
  # which would mix half launches into the per-dispatch averages)
  BENCH="python3 bench.py --no-cpu-baseline --no-north-star --no-config3 --no-check --no-render-call $*"
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
  W=$(python3 -c "import sys; a=sys.argv[1:]; print(a[a.index('--workload')+1] if '--workload' in a else 'config2')" "$@")
  python tools/roofline_from_profile.py $OUT $W > $OUT/roofline.json || exit 1
  python tools/summarize_profile.py $OUT $OUT/summary.json || exit 1
  # the raw per-dispatch CSVs are large (gpurun copies back <= 64 MiB): keep the summaries
  rm -f $OUT/pmc*_counter_collection.csv $OUT/trace_kernel_trace.csv
  ls $OUT
  ;;
trace)
  TAG=$1; shift
  OUT=gpurun_out/trace_$TAG
  mkdir -p $OUT
  BENCH="python3 bench.py --no-cpu-baseline --no-north-star --no-config3 --no-check $*"
  case "$*" in *--steps*) ;; *) BENCH="$BENCH --steps 6 --warmup 3";; esac
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o trace -- $BENCH > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
  python3 tools/trace_gaps.py $OUT/trace_kernel_trace.csv 4 > $OUT/gaps.txt && head -25 $OUT/gaps.txt
  python3 tools/frame_timeline.py $OUT/trace_kernel_trace.csv --frames 1 > $OUT/timeline.txt
  gzip -f $OUT/trace_kernel_trace.csv
  ;;
*)
  sed -n '2,18p' "$0"
  exit 2
  ;;
esac

#!/bin/bash
# GPU sessions (run on the box through gpurun, from the repository root).  One script, one
# subcommand per kind of session; every GPU step has its own time limit and the steps of a
# session are chained so that the first failure ends it.  Output goes to gpurun_out/.
#
#   tools/gpu.sh round TAG            the round's evidence: -m gpu suite, smoke, default bench,
#                                     simulated 8/4/2-GPU shards (C3, C5), plan probe, per-column
#                                     C5 (tools/c5_columns.py), then `prof`
#   tools/gpu.sh tests TAG [EXPR]     -m gpu tests (optionally -k EXPR)
#   tools/gpu.sh bench TAG WL [RUNS]  bench over workloads WL (e.g. c4,c5), RUNS times (default 2);
#                                     prints each config's kernel time and roofline fraction
#   tools/gpu.sh sweep TAG WL VAR V1,V2,..   the same bench with VAR set to each value in turn
#   tools/gpu.sh ab TAG OLD_LIB WL    same-box A/B: the in-tree library vs VXG_GPU_LIB=OLD_LIB,
#                                     alternating, 3 runs each
#   tools/gpu.sh sim TAG [WL]         bench of rank 0's shard at 8, 4 and 2 GPUs (default c3,c5)
#   tools/gpu.sh prof TAG             rocprofv3 kernel trace + stats of the default bench, then
#                                     separate PMC passes (FETCH_SIZE, WRITE_SIZE, two SQ sets)
#   tools/gpu.sh pmc TAG WL COUNTERS...   one PMC pass (<= 8 SQ, <= 4 TCC counters per pass)
#   tools/gpu.sh sq TAG WL            the two SQ passes only, over WL
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="$ROOTDIR/bench.py"
CMD="$1"; TAG="${2:-run}"
SQA="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
SQB="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM"

summary() {  # summary FILE LABEL: one line per config of a bench JSON line
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d["encodings"].items():
    print(sys.argv[2], k, v["kernel_ms_mean"], v["hbm_frac_algorithmic"], v.get("verified"))
PY
}

tests() {
  local k=()
  [ -n "$1" ] && k=(-k "$1")
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q "${k[@]}" --timeout 300 --timeout-method thread \
      -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
  local rc=$?; echo "pytest exit $rc"; tail -3 "$O/pytest_$TAG.log"; return $rc
}

pmc() {  # pmc NAME WL COUNTERS...
  local name="$1" wl="$2"; shift 2
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 200 rocprofv3 --pmc "$@" --output-format csv -d "$O/pmc_${name}_$TAG" -o run -- \
      python "$B" --workloads "$wl" --steps 3 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_${name}_$TAG.err")
}

prof() {
  (cd /tmp && export TMPDIR=/tmp && \
   timeout -k 10 60 rocprofv3 -L > "$O/counters_$TAG.txt" 2>&1 && \
   timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- \
       python "$B" --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_bench_$TAG.json" 2> "$O/prof_bench_$TAG.err") && \
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_$TAG" -o run -- \
       python "$B" --steps 5 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_fetch_$TAG.err") && \
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_$TAG" -o run -- \
       python "$B" --steps 5 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_write_$TAG.err") && \
  pmc sqa c1,c2,c4,c5 $SQA && pmc sqb c1,c2,c4,c5 $SQB
}

sim() {
  local wl="${1:-c3,c5}"
  for n in 8 4 2; do
    timeout -k 10 300 python -u "$B" --workloads "$wl" --simulate-world $n --no-cpu-baseline \
        > "$O/bench_sim${n}_$TAG.json" 2> "$O/bench_sim${n}_$TAG.err" || return 1
    summary "$O/bench_sim${n}_$TAG.json" "sim$n"
  done
}

case "$CMD" in
round)
  tests && \
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.log" 2>&1 && \
  timeout -k 10 400 python -u "$B" > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" && cat "$O/bench_$TAG.json" && \
  sim c3,c5 && \
  timeout -k 10 200 python -u tools/plan_probe.py 1 > "$O/plan_probe_$TAG.txt" 2>&1 && \
  timeout -k 10 200 python -u tools/plan_probe.py 8 >> "$O/plan_probe_$TAG.txt" 2>&1 && \
  timeout -k 10 300 python -u tools/c5_columns.py --rotate 4 > "$O/c5_columns_$TAG.jsonl" 2> "$O/c5_columns_$TAG.err" && \
  prof
  ;;
tests) tests "$3" ;;
bench)
  WL="$3"; RUNS="${4:-2}"
  for r in $(seq 1 "$RUNS"); do
    timeout -k 10 300 python -u "$B" --workloads "$WL" --no-cpu-baseline > "$O/qb_${TAG}_$r.json" 2> "$O/qb_${TAG}_$r.err" || exit 4
    summary "$O/qb_${TAG}_$r.json" "run$r"
  done
  ;;
sweep)
  WL="$3"; VAR="$4"; IFS=, read -ra VALS <<< "$5"
  for v in "${VALS[@]}"; do
    env "$VAR=$v" timeout -k 10 300 python -u "$B" --workloads "$WL" --no-cpu-baseline \
        > "$O/sw_${TAG}_$v.json" 2> "$O/sw_${TAG}_$v.err" || exit 4
    summary "$O/sw_${TAG}_$v.json" "$VAR=$v"
  done
  ;;
ab)
  OLD="$3"; WL="${4:-c4,c5}"
  for i in 1 2 3; do
    timeout -k 10 300 python -u "$B" --workloads "$WL" --no-cpu-baseline > "$O/new_${i}_$TAG.json" 2> "$O/new_${i}_$TAG.err" || exit 4
    VXG_GPU_LIB="$ROOTDIR/$OLD" timeout -k 10 300 python -u "$B" --workloads "$WL" --no-cpu-baseline \
        > "$O/old_${i}_$TAG.json" 2> "$O/old_${i}_$TAG.err" || exit 5
    summary "$O/new_${i}_$TAG.json" "new$i" && summary "$O/old_${i}_$TAG.json" "old$i"
  done
  ;;
sim) sim "$3" ;;
prof) prof ;;
pmc) WL="$3"; shift 3; pmc custom "$WL" "$@" ;;
sq) pmc sqa "$3" $SQA && pmc sqb "$3" $SQB ;;
*) echo "usage: tools/gpu.sh round|tests|bench|sweep|ab|sim|prof|pmc|sq TAG ..."; exit 2 ;;
esac
rc=$?
echo "gpu.sh $CMD exit $rc"
exit $rc

#!/bin/bash
# Iteration on the GPU box: the -m gpu suite, bench of the given workloads, then a rocprofv3
# kernel trace + SQ counter pass of the same workloads.   tools/gpu_quick2.sh TAG WORKLOADS
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-q}"; WL="${2:-c4,c5}"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u bench.py --workloads "$WL" --no-cpu-baseline > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" || { tail -5 "$O/bench_$TAG.err"; exit 4; }
python - "$O/bench_$TAG.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k, v in d["encodings"].items():
    print(k, "ms/step", v["ms_per_step"], "kernel", v["kernel_ms_mean"], "frac", v["hbm_frac_algorithmic"])
PY
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads "$WL" --steps 10 --warmup 3 --no-cpu-baseline > /dev/null 2> "$O/prof_$TAG.err" && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$O/pmc_sq_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads "$WL" --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$O/pmc_sq_$TAG.err"
echo "profiling exit $?"
cd "$ROOTDIR" && python tools/prof_summary.py --trace "$O/prof_$TAG" --skip 3 --pmc "$O/pmc_sq_$TAG" > "$O/summary_$TAG.txt" 2>&1; head -12 "$O/summary_$TAG.txt" | cut -c1-160

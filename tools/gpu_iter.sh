#!/bin/bash
# One iteration on the GPU box: the -m gpu suite, then bench workloads ($2, default c5) and the
# per-column C5 isolation.  Usage: tools/gpu_iter.sh TAG [workloads]
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-iter}"; WL="${2:-c5}"
cd "$ROOTDIR" && \
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > "$O/${TAG}_gpu.log" 2>&1; rc=$?
echo "gpu suite exit $rc"; tail -3 "$O/${TAG}_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workloads "$WL" --no-cpu-baseline > "$O/${TAG}_bench.jsonl" 2> "$O/${TAG}_bench.err" || { echo "bench failed"; tail -5 "$O/${TAG}_bench.err"; exit 1; }
timeout -k 10 300 python -u tools/c5_columns.py --reps 20 > "$O/${TAG}_cols.jsonl" 2> "$O/${TAG}_cols.err" || { echo "cols failed"; exit 1; }
python - "$O/${TAG}_bench.jsonl" "$O/${TAG}_cols.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    try: d = json.loads(l)
    except Exception: continue
    for k, v in (d.get("encodings") or {}).items():
        print("bench", k, v.get("ms_per_step"), v.get("kernel_ms_median"), v.get("hbm_frac_algorithmic"))
for l in open(sys.argv[2]):
    d = json.loads(l); print(d["column"], d.get("ms"), d.get("plan_ms"), d.get("plan_hbm_frac"))
PY

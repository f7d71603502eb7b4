#!/bin/bash
# C5 plan step time vs the number of parallel graph branches (VXG_PLAN_BRANCHES).
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-br}"; WL="${2:-c5}"; SIM="${3:-0}"
cd "$ROOTDIR" || exit 1
for nb in ${NBS:-1 2 3 4 6 8}; do
  VXG_PLAN_BRANCHES=$nb timeout -k 10 200 python -u bench.py --workloads "$WL" --no-cpu-baseline --simulate-world "$SIM" --steps ${STEPS:-20} > "$O/${TAG}_b$nb.jsonl" 2> "$O/${TAG}_b$nb.err" || { echo "bench nb=$nb failed"; exit 1; }
  python -c "
import json,sys
for l in open('$O/${TAG}_b$nb.jsonl'):
    try: d=json.loads(l)
    except Exception: continue
    for k,v in (d.get('encodings') or {}).items(): print('branches $nb', k, v.get('ms_per_step'), v.get('kernel_ms_median'), v.get('hbm_frac_algorithmic'))
"
done

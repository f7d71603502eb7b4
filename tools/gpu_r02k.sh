#!/bin/bash
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > "$O/r02k_gpu.log" 2>&1; rc=$?
echo "gpu suite exit $rc"; tail -3 "$O/r02k_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workloads c4,c5 --no-cpu-baseline > "$O/r02k_bench.jsonl" 2> "$O/r02k_bench.err"; echo "bench exit $?"
python - <<'PY'
import json
for l in open("gpurun_out/r02k_bench.jsonl"):
    try: d=json.loads(l)
    except Exception: continue
    for k,v in (d.get("encodings") or {}).items(): print(k, v.get("ms_per_step"), v.get("hbm_frac_algorithmic"))
PY

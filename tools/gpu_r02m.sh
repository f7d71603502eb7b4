#!/bin/bash
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > "$O/r02m_gpu.log" 2>&1; rc=$?
echo "gpu suite exit $rc"; tail -3 "$O/r02m_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline > "$O/r02m_bench.jsonl" 2> "$O/r02m_bench.err"; echo "bench exit $?"
timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --simulate-world 8 > "$O/r02m_sim8.jsonl" 2> "$O/r02m_sim8.err"; echo "sim8 exit $?"
timeout -k 10 300 python -u tools/c5_columns.py --reps 20 > "$O/r02m_cols.jsonl" 2> "$O/r02m_cols.err"; echo "cols exit $?"
python - <<'PY'
import json
for f in ("gpurun_out/r02m_bench.jsonl", "gpurun_out/r02m_sim8.jsonl"):
    for l in open(f):
        try: d=json.loads(l)
        except Exception: continue
        for k,v in (d.get("encodings") or {}).items():
            print(f[-12:], k, v.get("ms_per_step"), v.get("hbm_frac_algorithmic"))
for l in open("gpurun_out/r02m_cols.jsonl"):
    d=json.loads(l); print(d["column"], d.get("ms"), d.get("plan_ms"), d.get("plan_hbm_frac"))
PY

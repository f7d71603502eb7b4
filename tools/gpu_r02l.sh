#!/bin/bash
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu -k "fsst or FSST or string or lineitem or file" > "$O/r02l_gpu.log" 2>&1; rc=$?
echo "gpu fsst tests exit $rc"; tail -2 "$O/r02l_gpu.log"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --workloads c4,c5 --no-cpu-baseline > "$O/r02l_bench.jsonl" 2> "$O/r02l_bench.err"; echo "bench exit $?"
timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --simulate-world 8 > "$O/r02l_sim8.jsonl" 2> "$O/r02l_sim8.err"; echo "sim8 exit $?"
python - <<'PY'
import json
for f in ("gpurun_out/r02l_bench.jsonl", "gpurun_out/r02l_sim8.jsonl"):
    for l in open(f):
        try: d=json.loads(l)
        except Exception: continue
        for k,v in (d.get("encodings") or {}).items():
            print(f[-12:], k, {kk: v.get(kk) for kk in ("ms_per_step","hbm_frac_algorithmic","graph_launch_us","projected_speedup","sim_world","host_launch_us")})
PY

#!/bin/bash
# K1g blocks per workgroup (VXG_K1G_BPW) after the VarBin-bytes staging: C5 and per-column.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
for b in 1 2 4; do
  VXG_K1G_BPW=$b timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --no-verify > "$O/bpw${b}_$TAG.json" 2> "$O/bpw${b}_$TAG.err" || exit 4
  VXG_K1G_BPW=$b timeout -k 10 300 python tools/c5_columns.py --reps 10 --rotate 4 > "$O/cols_bpw${b}_$TAG.jsonl" 2> "$O/cols_bpw${b}_$TAG.err" || exit 5
done
python - "$O" "$TAG" <<'PY'
import json, sys
o, tag = sys.argv[1], sys.argv[2]
for b in (1, 2, 4):
    d = json.loads(open(f"{o}/bpw{b}_{tag}.json").read().strip().splitlines()[-1])
    c5 = d['encodings']['C5']
    cols = {}
    for l in open(f"{o}/cols_bpw{b}_{tag}.jsonl"):
        x = json.loads(l); cols[x['column']] = x.get('plan_ms')
    print(b, c5['kernel_ms_mean'], c5['hbm_frac_algorithmic'], {k: cols[k] for k in ('l_orderkey', 'l_returnflag', 'l_shipmode', 'SUM (sequential)')})
PY
echo "bpw2 done"

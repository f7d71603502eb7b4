#!/bin/bash
# FSST decode occupancy sensitivity: VXG_FSST_PAD_LDS adds unused LDS per workgroup
# (0 -> 8 workgroups per CU, 2048 -> 7, 4096 -> 6, 8192 -> 5, 16384 -> 4), C4 twice each.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
for i in 1 2; do
  for p in 0 2048 4096 8192 16384; do
    VXG_FSST_PAD_LDS=$p timeout -k 10 300 python -u bench.py --workloads c4 --no-cpu-baseline > "$O/occ${p}_${i}_$TAG.json" 2> "$O/occ${p}_${i}_$TAG.err" || exit 4
  done
done
python - "$O" "$TAG" <<'PY'
import json, sys
o, tag = sys.argv[1], sys.argv[2]
for p in (0, 2048, 4096, 8192, 16384):
    r = []
    for i in (1, 2):
        d = json.loads(open(f"{o}/occ{p}_{i}_{tag}.json").read().strip().splitlines()[-1])
        v = d['encodings']['C4']; r.append((v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified']))
    print(p, r)
PY
echo "occ done"

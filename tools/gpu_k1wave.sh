#!/bin/bash
# C5 with K1w for every K1 launch (VXG_K1_WAVE=force) vs the default (row-split K1 for launches
# under 512 workgroups): alternating, 3 runs each.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline > "$O/kdef_${i}_$TAG.json" 2> "$O/kdef_${i}_$TAG.err" || exit 4
  VXG_K1_WAVE=force timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline > "$O/kw_${i}_$TAG.json" 2> "$O/kw_${i}_$TAG.err" || exit 5
done
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for pat in ("kdef", "kw"):
    for f in sorted(glob.glob(f"{o}/{pat}_*_{tag}.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified']) for k, v in d['encodings'].items()})
PY
echo "k1wave done"

#!/bin/bash
# Same-box A/B of two builds of the library: the in-tree libvortex_gpu.so (new) against
# VXG_GPU_LIB=$2 (old); workloads $3 (default c4,c5) alternating, 3 runs each.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"; OLD="$2"; WL="${3:-c4,c5}"
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workloads "$WL" --no-cpu-baseline > "$O/new_${i}_$TAG.json" 2> "$O/new_${i}_$TAG.err" || exit 4
  VXG_GPU_LIB="$ROOTDIR/$OLD" timeout -k 10 300 python -u bench.py --workloads "$WL" --no-cpu-baseline > "$O/old_${i}_$TAG.json" 2> "$O/old_${i}_$TAG.err" || exit 5
done
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/new_*_{tag}.json") + glob.glob(f"{o}/old_*_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified']) for k, v in d['encodings'].items()})
PY
echo "lib ab done"

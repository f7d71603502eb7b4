#!/bin/bash
# C5 plan shapes: default (unbatched, 2 branches) vs batched plans whose K1 jobs are launched per
# kernel key (VXG_K1G_MAX_BYTES=0: specialized K1 per (T, W, epilogue) group across columns; the
# VarBin-dictionary and RunEnd jobs in one K1g launch), on 1 or 2+1 branches.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
run() {  # name, env...
  local n="$1"; shift
  env "$@" timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline > "$O/g${n}_$TAG.json" 2> "$O/g${n}_$TAG.err" || exit 4
}
for i in 1 2; do
  run def$i VXG_PLAN_DEBUG=
  run b1k$i VXG_PLAN_BATCH=1 VXG_K1G_MAX_BYTES=0
  run b2k$i VXG_PLAN_BATCH=1 VXG_K1G_MAX_BYTES=0 VXG_PLAN_BRANCHES=2
  run b2g$i VXG_PLAN_BATCH=1 VXG_PLAN_BRANCHES=2
done
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/g*_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    v = d['encodings']['C5']
    print(f.split('/')[-1], v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified'], v.get('plan_mode'))
PY
echo "grp done"

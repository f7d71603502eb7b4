#!/bin/bash
# Full -m gpu suite, then the default bench (all configs, no CPU baseline) twice.
#   tools/gpu_full_ab.sh TAG
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"; O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; tail -1 "$O/pytest_$TAG.log"; [ $rc -eq 0 ] || exit 3
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$O/qb_${TAG}_$r.json" 2> "$O/qb_${TAG}_$r.err" || exit 4
  python -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k,v in d['encodings'].items(): print(sys.argv[2], k, v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified'])" "$O/qb_${TAG}_$r.json" "run$r"
done

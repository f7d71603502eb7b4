#!/bin/bash
# C2 A/B of the fused ALP patches (VXG_FUSED_PATCHES=1/0, interleaved twice), then the round's
# evidence session (tools/gpu_round.sh).  Each GPU step has its own time limit; && chains them.
#   tools/gpu_final.sh TAG
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"; O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"
for r in 1 2; do
  for f in 1 0; do
    VXG_FUSED_PATCHES=$f timeout -k 10 200 python -u bench.py --workloads c2 --no-cpu-baseline > "$O/c2ab_${TAG}_${f}_$r.json" 2> "$O/c2ab_${TAG}_${f}_$r.err" || exit 4
    python -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
v=d['encodings']['C2']; print('fused=' + sys.argv[2], 'run' + sys.argv[3], v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified'])" "$O/c2ab_${TAG}_${f}_$r.json" $f $r
  done
done
bash tools/gpu_round.sh "$TAG"

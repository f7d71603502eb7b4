#!/bin/bash
# C5 shard step at simulated world 2 and 4 under plan-batching thresholds (VXG_PLAN_BATCH_MAX_BYTES).
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"; O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in 2 4; do
  for t in 16777216 67108864 0; do
    VXG_PLAN_BATCH_MAX_BYTES=$t timeout -k 10 200 python -u bench.py --workloads c5 --simulate-world $w --no-cpu-baseline > "$O/th_${w}_$t.json" 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('$O/th_${w}_$t.json').read().strip().splitlines()[-1]); v=d['encodings']['C5']; print('world $w thresh $t', v['ms_per_step'])"
  done
done

#!/bin/bash
# C5 plan-recording A/B: bench C5 at 1 GPU and the 8-GPU shard with the plan candidates printed.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"; O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"
for w in 1 8; do
  extra=""; [ $w -gt 1 ] && extra="--simulate-world $w"
  VXG_PLAN_DEBUG=1 timeout -k 10 200 python -u bench.py --workloads c5 --no-cpu-baseline $extra > "$O/c5plan_${TAG}_w$w.json" 2> "$O/c5plan_${TAG}_w$w.err" || exit 3
  grep "plan candidate" "$O/c5plan_${TAG}_w$w.err"
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); v=d['encodings']['C5']; print('w$w', v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified'])" "$O/c5plan_${TAG}_w$w.json"
done

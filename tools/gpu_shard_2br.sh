#!/bin/bash
# Kernel trace of the simulated 8-GPU C5 shard with the batched plan forced onto 2 graph branches
# (FSST pre-pass + decode on one, the K1g batch on the other): do they overlap?
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && \
VXG_PLAN_BATCH=1 VXG_PLAN_BRANCHES=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_2br" -o run -- python "$ROOTDIR/bench.py" --workloads c5 --simulate-world 8 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > "$O/prof_2br.json" 2> "$O/prof_2br.err"
echo "exit $?"

#!/bin/bash
# rocprofv3 kernel trace of the simulated 8-GPU C5 shard (plan replays), for tools/timeline.py.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-sim8}"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c5 --simulate-world 8 --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_$TAG.json" 2> "$O/prof_$TAG.err"
echo "exit $?"

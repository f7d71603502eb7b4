#!/bin/bash
# rocprofv3 kernel trace of the C5 plan replays (bench), for the timeline analysis in tools/timeline.py
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r02n}"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5b_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c5 --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_c5b_$TAG.json" 2> "$O/prof_c5b_$TAG.err"
echo "exit $?"

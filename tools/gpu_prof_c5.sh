#!/bin/bash
# rocprofv3 kernel trace of tools/c5_columns.py (direct and plan-mode canonicalize per column).
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
mkdir -p "$ROOTDIR/gpurun_out"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r02e}"
O="$ROOTDIR/gpurun_out"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5_$TAG" -o run -- python "$ROOTDIR/tools/c5_columns.py" --reps 10 > "$O/prof_c5_$TAG.jsonl" 2> "$O/prof_c5_$TAG.err"
echo "exit $?"

#!/bin/bash
# GPU session: parity tests; C5 per-column isolation (N=1 and the 8-GPU shard) + its rocprof trace.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r02c}"
O="$ROOTDIR/gpurun_out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu_$TAG.log; tail -3 $O/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python tools/c5_columns.py > $O/c5_columns_$TAG.jsonl 2> $O/c5_columns_$TAG.err && \
timeout -k 10 300 python tools/c5_columns.py --world 8 > $O/c5_columns_w8_$TAG.jsonl 2> $O/c5_columns_w8_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5_$TAG" -o run -- python "$ROOTDIR/tools/c5_columns.py" --reps 10 > "$O/prof_c5_$TAG.jsonl" 2> "$O/prof_c5_$TAG.err"
echo "exit $?"

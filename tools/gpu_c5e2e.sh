#!/bin/bash
# C5 N=1 plan timeline (rocprofv3 kernel trace of the bench's C5 replays), per-column isolation,
# and the host->host (--e2e) rates of every config.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
timeout -k 10 600 python -u bench.py --e2e --workloads c1,c2,c3,c4,c5 --no-cpu-baseline > "$O/bench_e2e_$TAG.json" 2> "$O/bench_e2e_$TAG.err" || exit 3
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c5 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > "$O/prof_c5_bench_$TAG.json" 2> "$O/prof_c5_$TAG.err" || exit 4
timeout -k 10 300 python "$ROOTDIR/tools/c5_columns.py" --reps 10 > "$O/c5_columns_$TAG.jsonl" 2> "$O/c5_columns_$TAG.err" || exit 5
echo "c5e2e done"

#!/bin/bash
# GPU session: parity tests, default bench, C5 isolated + e2e from file bytes.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r02b}"
O="$ROOTDIR/gpurun_out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu_$TAG.log; tail -3 $O/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 python bench.py --e2e --workloads c5 --no-cpu-baseline > $O/bench_c5_$TAG.json 2> $O/bench_c5_$TAG.err && cat $O/bench_c5_$TAG.json && \
timeout -k 10 600 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err && cat $O/bench_$TAG.json
echo "bench exit $?"

#!/bin/bash
# Quick GPU session: parity tests, the default bench line, and a rocprofv3 kernel trace of the
# bench (per-kernel stats).  Every GPU step has its own time limit; steps chained with &&.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r02}"
O="$ROOTDIR/gpurun_out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu_$TAG.log; tail -3 $O/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err && cat $O/bench_$TAG.json && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_bench_$TAG.json" 2> "$O/prof_bench_$TAG.err"
echo "profiling exit $?"

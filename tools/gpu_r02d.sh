#!/bin/bash
# GPU session: parity tests (K14 dict rows on), C5 per-column A/B (K14 vs K1 Dict), C3/C5 bench A/B.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r02d}"
O="$ROOTDIR/gpurun_out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu_$TAG.log; tail -3 $O/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python tools/c5_columns.py > $O/c5_columns_$TAG.jsonl 2> $O/c5_columns_$TAG.err && \
VXG_DICT_ROWS=0 timeout -k 10 300 python tools/c5_columns.py > $O/c5_columns_k1dict_$TAG.jsonl 2> $O/c5_columns_k1dict_$TAG.err && \
timeout -k 10 300 python bench.py --workloads c3,c5 --no-cpu-baseline > $O/bench_c35_$TAG.json 2> $O/bench_c35_$TAG.err && \
VXG_DICT_ROWS=0 timeout -k 10 300 python bench.py --workloads c3,c5 --no-cpu-baseline > $O/bench_c35_k1dict_$TAG.json 2> $O/bench_c35_k1dict_$TAG.err
echo "exit $?"

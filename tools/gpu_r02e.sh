#!/bin/bash
# Round-2 GPU pass e: GPU encoder parity, the full gpu suite, then the per-column C5 kernel trace.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"
mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_encode.py -x -v --timeout 120 --timeout-method thread -m gpu > "$O/r02e_encode.log" 2>&1; rc=$?
echo "encode tests exit $rc"; tail -5 "$O/r02e_encode.log"
[ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu --ignore=tests/test_gpu_encode.py > "$O/r02e_gpu.log" 2>&1; rc2=$?
echo "gpu suite exit $rc2"; tail -5 "$O/r02e_gpu.log"
[ $rc2 -le 1 ] || exit $rc2
bash "$ROOTDIR/tools/gpu_prof_c5.sh" r02e

#!/bin/bash
# Round-2 GPU pass f: encoder parity + RoaringBool (K16) parity.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"
mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
timeout -k 10 500 python -u -m pytest tests/test_gpu_encode.py tests/test_roaring.py -v --timeout 120 --timeout-method thread -m gpu > "$O/r02f.log" 2>&1; rc=$?
echo "exit $rc"; grep -E "FAILED|ERROR|passed|failed" "$O/r02f.log" | tail -15
exit $rc

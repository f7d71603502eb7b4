#!/bin/bash
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_encode.py -q --timeout 120 --timeout-method thread -m gpu > "$O/r02g_enc.log" 2>&1; rc=$?
echo "enc exit $rc"; tail -3 "$O/r02g_enc.log"
[ $rc -le 1 ] || exit $rc
bash "$ROOTDIR/tools/gpu_pmc_fsst.sh" r02g c4

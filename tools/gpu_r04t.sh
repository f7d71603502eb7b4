#!/bin/bash
# New round-4 GPU tests (reference KAT replays, Arrow validation), then tools/gpu_c5e2e.sh.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_kats.py tests/test_gpu_arrow.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_new_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -15 "$O/pytest_new_$TAG.log"
[ $rc -eq 0 ] || exit 3
bash tools/gpu_c5e2e.sh "$TAG"

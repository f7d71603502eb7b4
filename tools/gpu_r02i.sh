#!/bin/bash
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
timeout -k 10 300 python -u -m pytest tests/test_capi.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "runend or RunEnd or capi" > "$O/r02i_gpu.log" 2>&1; rc=$?
echo "gpu runend tests exit $rc"; tail -2 "$O/r02i_gpu.log"
[ $rc -eq 0 ] || exit $rc
VXG_GPU_LIB="$ROOTDIR/vortex_amd/libvortex_gpu_stamps.so" timeout -k 10 200 python -u tools/fsst_stamps.py --workload c4 > "$O/r02i_stamps.jsonl" 2>&1 && \
VXG_GPU_LIB="$ROOTDIR/vortex_amd/libvortex_gpu_stamps.so" timeout -k 10 200 python -u tools/fsst_stamps.py --workload l_comment >> "$O/r02i_stamps.jsonl" 2>&1; echo "stamps exit $?"; grep workload "$O/r02i_stamps.jsonl"
bash "$ROOTDIR/tools/gpu_prof_c5.sh" r02i

#!/bin/bash
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
VXG_GPU_LIB="$ROOTDIR/vortex_amd/libvortex_gpu_stamps.so" timeout -k 10 300 python -u tools/fsst_stamps.py --workload c4 --reps 20 --ablate 0,1,2,3,4,8,16,7,15,31 > "$O/r02j_abl.jsonl" 2>&1; echo "abl exit $?"; grep workload "$O/r02j_abl.jsonl"

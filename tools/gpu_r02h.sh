#!/bin/bash
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd "$ROOTDIR" && \
timeout -k 10 400 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu > "$O/r02h_gpu.log" 2>&1; rc=$?
echo "gpu suite exit $rc"; tail -3 "$O/r02h_gpu.log"
[ $rc -eq 0 ] || exit $rc
VXG_GPU_LIB="$ROOTDIR/vortex_amd/libvortex_gpu_stamps.so" timeout -k 10 200 python -u tools/fsst_stamps.py --workload c4 > "$O/r02h_stamps.jsonl" 2>&1 && \
VXG_GPU_LIB="$ROOTDIR/vortex_amd/libvortex_gpu_stamps.so" timeout -k 10 200 python -u tools/fsst_stamps.py --workload l_comment >> "$O/r02h_stamps.jsonl" 2>&1; echo "stamps exit $?"; cat "$O/r02h_stamps.jsonl" | tail -4
timeout -k 10 300 python -u bench.py --workloads c4,c5 --no-cpu-baseline > "$O/r02h_bench.jsonl" 2> "$O/r02h_bench.err"; echo "bench exit $?"

#!/bin/bash
# Same-box A/B of a K8r change (round 6): -m gpu RunEnd tests on the in-tree library, then the
# per-column C5 isolation (tools/c5_columns.py) and the C5 bench, new vs VXG_GPU_LIB=OLD,
# alternating.  Usage: tools/ab_k8r.sh TAG OLD_LIB
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"; OLD="$ROOTDIR/$2"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "runend" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1 || { tail -20 "$O/pytest_$TAG.log"; exit 3; }
tail -2 "$O/pytest_$TAG.log"
for i in 1 2; do
  timeout -k 10 200 python -u tools/c5_columns.py --rotate 4 > "$O/cols_new_${i}_$TAG.jsonl" 2> "$O/cols_new_${i}_$TAG.err" || exit 4
  VXG_GPU_LIB="$OLD" timeout -k 10 200 python -u tools/c5_columns.py --rotate 4 > "$O/cols_old_${i}_$TAG.jsonl" 2> "$O/cols_old_${i}_$TAG.err" || exit 5
  grep -h l_orderkey "$O/cols_new_${i}_$TAG.jsonl" "$O/cols_old_${i}_$TAG.jsonl"
done
bash tools/gpu.sh ab "$TAG" "$2" c5

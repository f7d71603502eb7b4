#!/bin/bash
# (1) parity of table-driven paths with the direct chunk lookup; (2) K1 output stores NT (in-tree
# build) vs plain (VXG_GPU_LIB=$2) on C1/C2 with rotated outputs; (3) direct chunk lookup on/off
# (VXG_EXT_GPE=0) on C3/C5.  Alternating runs, 3 each.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"; PLAIN="$2"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "plan or file or lineitem or chunk or Chunk or dict or Dict or kat" --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -1 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workloads c1,c2 --no-cpu-baseline > "$O/nt_${i}_$TAG.json" 2> "$O/nt_${i}_$TAG.err" || exit 4
  VXG_GPU_LIB="$ROOTDIR/$PLAIN" timeout -k 10 300 python -u bench.py --workloads c1,c2 --no-cpu-baseline > "$O/pl_${i}_$TAG.json" 2> "$O/pl_${i}_$TAG.err" || exit 5
done
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workloads c3,c5 --no-cpu-baseline > "$O/gpe_${i}_$TAG.json" 2> "$O/gpe_${i}_$TAG.err" || exit 6
  VXG_EXT_GPE=0 timeout -k 10 300 python -u bench.py --workloads c3,c5 --no-cpu-baseline > "$O/nogpe_${i}_$TAG.json" 2> "$O/nogpe_${i}_$TAG.err" || exit 7
done
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for pat in ("nt", "pl", "gpe", "nogpe"):
    for f in sorted(glob.glob(f"{o}/{pat}_*_{tag}.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified']) for k, v in d['encodings'].items()})
PY
echo "ab2 done"

#!/bin/bash
# K1g direct job lookup on/off (VXG_EXT_GPE=0): parity subset, then C3/C5 alternating, 3 runs each.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "plan or file or lineitem or chunk or Chunk or dict or Dict or kat or runend or RunEnd" --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -1 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workloads c3,c5 --no-cpu-baseline > "$O/gpe_${i}_$TAG.json" 2> "$O/gpe_${i}_$TAG.err" || exit 6
  VXG_EXT_GPE=0 timeout -k 10 300 python -u bench.py --workloads c3,c5 --no-cpu-baseline > "$O/nogpe_${i}_$TAG.json" 2> "$O/nogpe_${i}_$TAG.err" || exit 7
done
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for pat in ("gpe", "nogpe"):
    for f in sorted(glob.glob(f"{o}/{pat}_*_{tag}.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified']) for k, v in d['encodings'].items()})
PY
echo "gpe done"

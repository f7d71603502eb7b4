#!/bin/bash
# Same-box A/B of an FSST decode variant selected by VXG_FSST_ABL=$2 (outputs correct), against 0:
# FSST parity subset in both modes, then C4+C5 alternating, 3 runs each.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"; B="${2:-16}"
for m in 0 $B; do
  VXG_FSST_ABL=$m timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "fsst or FSST or full_size_c4 or lineitem" --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_${m}_$TAG.log" 2>&1
  rc=$?; echo "pytest $m exit $rc"; tail -1 "$O/pytest_${m}_$TAG.log"
  [ $rc -eq 0 ] || exit 3
done
for i in 1 2 3; do
  for m in 0 $B; do
    VXG_FSST_ABL=$m timeout -k 10 300 python -u bench.py --workloads c4,c5 --no-cpu-baseline > "$O/ab${m}_${i}_$TAG.json" 2> "$O/ab${m}_${i}_$TAG.err" || exit 4
  done
done
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/ab*_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified']) for k, v in d['encodings'].items()})
PY
echo "ab done"

#!/bin/bash
# K1g blocks-per-workgroup sweep (C5 at N=1 and the simulated 8-GPU shard) + C4 (FSST views
# stored non-temporally) + the FSST/string parity subset.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "fsst or FSST or string or dict or plan or file" --timeout 200 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u bench.py --workloads c4 --no-cpu-baseline > "$O/c4_$TAG.json" 2> "$O/c4_$TAG.err" || exit 4
for b in 1 2 4 8; do
  VXG_K1G_BPW=$b timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --no-verify > "$O/bpw${b}_$TAG.json" 2> "$O/bpw${b}_$TAG.err" || exit 5
  VXG_K1G_BPW=$b timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --no-verify --simulate-world 8 > "$O/bpw${b}_sim8_$TAG.json" 2> "$O/bpw${b}_sim8_$TAG.err" || exit 6
done
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/bpw*_{tag}.json") + glob.glob(f"{o}/c4_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic']) for k, v in d['encodings'].items()})
PY

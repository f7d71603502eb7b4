#!/bin/bash
# Global-address-space accesses (no flat instructions in the table-driven kernels): full GPU
# parity suite, the default bench, C5 per-column isolation (rotated) and a C5 kernel trace.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
timeout -k 10 400 python -u bench.py --no-cpu-baseline > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" || exit 4
timeout -k 10 300 python -u bench.py --workloads c4,c5 --no-cpu-baseline > "$O/bench2_$TAG.json" 2> "$O/bench2_$TAG.err" || exit 4
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/bench*_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified']) for k, v in d['encodings'].items()})
PY
timeout -k 10 300 python tools/c5_columns.py --reps 10 --rotate 4 > "$O/c5_columns_$TAG.jsonl" 2> "$O/c5_columns_$TAG.err" || exit 5
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c5 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > /dev/null 2> "$O/prof_$TAG.err" || exit 8
echo "gmem done"

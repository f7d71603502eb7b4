#!/bin/bash
# FSST decode: 1 vs 2 tiles per workgroup (VXG_FSST_TILES), parity subset first.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "fsst or FSST or string or full_size_c4 or file or arrow or filter" --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
VXG_FSST_TILES=1 timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -k "fsst or FSST or full_size_c4" --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest1_$TAG.log" 2>&1 || exit 4
for i in 1 2; do
for t in 1 2; do
  VXG_FSST_TILES=$t timeout -k 10 300 python -u bench.py --workloads c4,c5 --no-cpu-baseline > "$O/t${t}_${i}_$TAG.json" 2> "$O/t${t}_${i}_$TAG.err" || exit 5
done
done
for t in 1 2; do
  VXG_FSST_TILES=$t timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --simulate-world 8 > "$O/t${t}_sim8_$TAG.json" 2> "$O/t${t}_sim8_$TAG.err" || exit 6
done
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/t[12]_*_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified']) for k, v in d['encodings'].items()})
PY
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$O/pmc_sq_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c4 --steps 3 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_sq_$TAG.err" || exit 7
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c4 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > /dev/null 2> "$O/prof_$TAG.err" || exit 8
echo "fsst2 done"

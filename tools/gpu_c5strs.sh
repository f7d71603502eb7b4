#!/bin/bash
# C5 plan A/B: unbatched (2 branches) vs only the string-dictionary columns batched into one K1g
# launch on a third branch (VXG_PLAN_BATCH=s); parity of plans in that mode first.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
VXG_PLAN_BATCH=s timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "(plan or file or lineitem) and not measure_flag" --timeout 200 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
for i in 1 2; do
  for m in 0 s; do
    VXG_PLAN_BATCH=$m timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline > "$O/m${m}_${i}_$TAG.json" 2> "$O/m${m}_${i}_$TAG.err" || exit 5
  done
done
VXG_PLAN_BATCH=s timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --simulate-world 2 > "$O/ms_sim2_$TAG.json" 2> "$O/ms_sim2_$TAG.err" || exit 6
timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --simulate-world 2 > "$O/md_sim2_$TAG.json" 2> "$O/md_sim2_$TAG.err" || exit 6
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/m*_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic'], v['verified'], v.get('plan_mode')) for k, v in d['encodings'].items()})
PY
cd /tmp && export TMPDIR=/tmp
VXG_PLAN_BATCH=s timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c5 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > /dev/null 2> "$O/prof_$TAG.err" || exit 8
echo "c5strs done"

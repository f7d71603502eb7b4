#!/bin/bash
# C5 plan-shape experiments (env knobs read at plan creation) + SQ counters of the C5 kernels.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
run() { name=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --no-verify > "$O/c5m_${name}_$TAG.json" 2> "$O/c5m_${name}_$TAG.err"; }
run default || exit 3
run mixed100 VXG_PLAN_BATCH=mixed VXG_PLAN_BATCH_MAX_BYTES=100000000 || exit 4
run br3 VXG_PLAN_BATCH=0 VXG_PLAN_BRANCHES=3 || exit 5
run br4 VXG_PLAN_BATCH=0 VXG_PLAN_BRANCHES=4 || exit 6
run batched VXG_PLAN_BATCH=1 || exit 7
run default2 || exit 8
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/c5m_*_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    e = d['encodings']['C5']
    print(f.split('/')[-1], e['kernel_ms_mean'], e['hbm_frac_algorithmic'], e.get('plan_candidates'))
PY
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$O/pmc_sq_c5_$TAG" -o run -- python "$ROOTDIR/tools/c5_columns.py" --reps 3 > /dev/null 2> "$O/pmc_sq_c5_$TAG.err" || exit 9
echo "c5modes done"

#!/bin/bash
# FSST decode ablation (VXG_FSST_ABL: 1 segments, 2 copy-out, 4 views, 8 all after the prologue;
# outputs are wrong, --no-verify): C4 kernel time and SQ counters per mask.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04}"
for m in 0 1 2 4 6 7 8; do
  VXG_FSST_ABL=$m timeout -k 10 200 python -u bench.py --workloads c4 --no-cpu-baseline --no-verify > "$O/abl${m}_$TAG.json" 2> "$O/abl${m}_$TAG.err" || exit 3
done
python - "$O" "$TAG" <<'PY'
import json, sys
o, tag = sys.argv[1], sys.argv[2]
for m in (0, 1, 2, 4, 6, 7, 8):
    d = json.loads(open(f"{o}/abl{m}_{tag}.json").read().strip().splitlines()[-1])
    e = d['encodings']['C4']
    print("abl", m, e['kernel_ms_mean'], e['hbm_frac_algorithmic'])
PY
cd /tmp && export TMPDIR=/tmp
for m in 0 1 7; do
  VXG_FSST_ABL=$m timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$O/pmc_abl${m}_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c4 --steps 3 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_abl${m}_$TAG.err" || exit 4
done
echo "abl done"

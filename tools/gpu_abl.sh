#!/bin/bash
# FSST decode ablation (temporary): for each VXG_FSST_ABL value, bench C4 (no verification: an
# ablated decode writes wrong bytes) and one SQ counter pass.
#   tools/gpu_abl.sh TAG 0 1 2 ...
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"; shift
for a in "$@"; do
  VXG_FSST_ABL=$a timeout -k 10 200 python -u bench.py --workloads c4 --no-cpu-baseline --no-verify > "$O/abl_${TAG}_$a.json" 2> "$O/abl_${TAG}_$a.err" || exit 4
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); v=d['encodings']['C4']; print('abl', sys.argv[2], 'C4 kernel_ms', v['kernel_ms_mean'])" "$O/abl_${TAG}_$a.json" $a
  (cd /tmp && VXG_FSST_ABL=$a TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$O/pmc_abl_${TAG}_$a" -o run -- python "$ROOTDIR/bench.py" --workloads c4 --steps 3 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_abl_${TAG}_$a.err") || exit 6
done
echo "abl done"

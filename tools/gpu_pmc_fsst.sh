#!/bin/bash
# PMC passes over the C4 (FSST) bench: instruction mix, wait/issue cycles, LDS, HBM bytes.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"
TAG="${1:-r02g}"
WL="${2:-c4}"
mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
B="$ROOTDIR/bench.py --workloads $WL --steps 3 --warmup 1 --no-cpu-baseline"
run() {  # name counters...
    local n=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$O/pmc_${TAG}_$n" -o run -- python3 $B > "$O/pmc_${TAG}_$n.log" 2>&1
    local rc=$?; echo "pass $n exit $rc"; return $rc
}
timeout -s KILL 60 rocprofv3 -L > "$O/pmc_list.txt" 2>&1; echo "list exit $?"
run a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE && \
run b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_ANY && \
run c FETCH_SIZE && run d WRITE_SIZE

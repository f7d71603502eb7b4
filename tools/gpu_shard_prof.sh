#!/bin/bash
# Kernel trace + SQ counters of one GPU's shard of the 8-GPU C5 scan (simulated in one process).
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"; B="$ROOTDIR/bench.py"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_shard_$TAG" -o run -- python "$B" --workloads c5 --simulate-world 8 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > "$O/prof_shard_$TAG.json" 2> "$O/prof_shard_$TAG.err" && \
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$O/pmc_shard_sq_$TAG" -o run -- python "$B" --workloads c5 --simulate-world 8 --steps 3 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_shard_sq_$TAG.err"
echo "shard prof exit $?"

#!/bin/bash
# Profiling session for the round's evidence: rocprofv3 kernel trace of the default bench, then
# separate PMC passes (FETCH_SIZE, WRITE_SIZE over C1-C5; two SQ passes over C4/C5) -- never
# combined with tracing.  Each GPU step has its own limit; steps are chained with &&.
#   tools/gpu_prof.sh TAG
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r03}"
B="$ROOTDIR/bench.py"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 60 rocprofv3 -L > "$O/counters_$TAG.txt" 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$B" --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_bench_$TAG.json" 2> "$O/prof_bench_$TAG.err" && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_$TAG" -o run -- python "$B" --steps 5 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_fetch_$TAG.err" && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_$TAG" -o run -- python "$B" --steps 5 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_write_$TAG.err" && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$O/pmc_sqa_$TAG" -o run -- python "$B" --workloads c1,c2,c4,c5 --steps 3 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_sqa_$TAG.err" && \
timeout -s KILL 200 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SMEM --output-format csv -d "$O/pmc_sqb_$TAG" -o run -- python "$B" --workloads c1,c2,c4,c5 --steps 3 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_sqb_$TAG.err"
echo "profiling exit $?"

#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel stats, then separate PMC passes for
# FETCH_SIZE and WRITE_SIZE (never combined with tracing).  Every GPU step has its own time
# limit and the steps are chained with && (a failure ends the call).
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r01}"
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 3
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.json 2> gpurun_out/bench.err && cat gpurun_out/bench.json && \
timeout -k 10 600 python bench.py --e2e --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_e2e.json 2> gpurun_out/bench_e2e.err && \
timeout -k 10 120 ./tools/ubench_k1 > gpurun_out/ubench_k1_$TAG.txt 2>&1 && \
timeout -k 10 120 ./tools/ubench_dict 16 > gpurun_out/ubench_dict_$TAG.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOTDIR/gpurun_out/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1,c2,c3,c4 --steps 10 --warmup 2 --no-cpu-baseline > "$ROOTDIR/gpurun_out/prof_bench_$TAG.json" 2> "$ROOTDIR/gpurun_out/prof_bench_$TAG.err" && \
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$ROOTDIR/gpurun_out/pmc_fetch_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1 --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> "$ROOTDIR/gpurun_out/pmc_fetch_$TAG.err" && \
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$ROOTDIR/gpurun_out/pmc_write_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1 --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> "$ROOTDIR/gpurun_out/pmc_write_$TAG.err" && \
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d "$ROOTDIR/gpurun_out/pmc_sq_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1,c4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$ROOTDIR/gpurun_out/pmc_sq_$TAG.err"
echo "profiling exit $?"

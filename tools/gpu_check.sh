#!/bin/bash
# One GPU session: parity tests, bench (+ host->host), microbenchmarks, rocprofv3 kernel stats,
# then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) -- never combined with tracing.  Every
# GPU step has its own time limit and the steps are chained with && (a failure ends the call).
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r01}"
O="$ROOTDIR/gpurun_out"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu_$TAG.log; tail -3 $O/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit 3
timeout -k 10 600 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err && cat $O/bench_$TAG.json && \
timeout -k 10 600 python bench.py --workloads c3,c5 --simulate-world 8 --no-cpu-baseline > $O/bench_sim8_$TAG.json 2> $O/bench_sim8_$TAG.err && \
timeout -k 10 600 python bench.py --e2e --steps 5 --warmup 2 --workloads c1,c2,c3,c4 --no-cpu-baseline > $O/bench_e2e_$TAG.json 2> $O/bench_e2e_$TAG.err && \
timeout -k 10 120 ./tools/ubench_k1 > $O/ubench_k1_$TAG.txt 2>&1 && \
timeout -k 10 120 ./tools/ubench_dict 16 > $O/ubench_dict_$TAG.txt 2>&1 && \
timeout -k 10 120 ./tools/ubench_lds > $O/ubench_lds_$TAG.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --steps 10 --warmup 2 --no-cpu-baseline > "$O/prof_bench_$TAG.json" 2> "$O/prof_bench_$TAG.err" && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1,c2,c3,c4 --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> "$O/pmc_fetch_$TAG.err" && \
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1,c2,c3,c4 --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> "$O/pmc_write_$TAG.err" && \
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$O/pmc_sq_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1,c4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$O/pmc_sq_$TAG.err"
echo "profiling exit $?"

#!/bin/bash
# One GPU session producing the round's committed evidence: the -m gpu suite, smoke(), the default
# bench line (driver-equivalent), the simulated 8-GPU C5/C3 shard, a rocprofv3 kernel trace of the
# default bench, then separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ) -- never combined with
# tracing.  Every GPU step has its own time limit; steps are chained with && (a failure ends it).
#   tools/gpu_round.sh TAG
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r02}"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 "$O/pytest_gpu_$TAG.log"
[ $rc -eq 0 ] || exit 3
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.log" 2>&1 && \
timeout -k 10 400 python -u bench.py > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" && cat "$O/bench_$TAG.json" && \
timeout -k 10 300 python -u bench.py --workloads c3,c5 --simulate-world 8 --no-cpu-baseline > "$O/bench_sim8_$TAG.json" 2> "$O/bench_sim8_$TAG.err" && \
timeout -k 10 200 python -u tools/plan_probe.py 1 > "$O/plan_probe_$TAG.txt" 2>&1 && \
timeout -k 10 200 python -u tools/plan_probe.py 8 >> "$O/plan_probe_$TAG.txt" 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_bench_$TAG.json" 2> "$O/prof_bench_$TAG.err" && \
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1,c2,c3,c4 --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> "$O/pmc_fetch_$TAG.err" && \
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1,c2,c3,c4 --steps 5 --warmup 1 --no-cpu-baseline > /dev/null 2> "$O/pmc_write_$TAG.err" && \
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d "$O/pmc_sq_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1,c4 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2> "$O/pmc_sq_$TAG.err"
echo "profiling exit $?"

#!/bin/bash
# One GPU session producing the round's committed evidence: the -m gpu suite, smoke(), the default
# bench line (driver-equivalent), the simulated 8/4/2-GPU shards (C3, C5), plan_probe, then
# tools/gpu_prof.sh (rocprofv3 kernel trace of the default bench and separate PMC passes --
# FETCH_SIZE, WRITE_SIZE, two SQ passes -- never combined with tracing).  Every GPU step has its
# own time limit; steps are chained with && (a failure ends it).
#   tools/gpu_round.sh TAG
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r03}"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_gpu_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 "$O/pytest_gpu_$TAG.log"
[ $rc -eq 0 ] || exit 3
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_$TAG.log" 2>&1 && \
timeout -k 10 400 python -u bench.py > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" && cat "$O/bench_$TAG.json" && \
timeout -k 10 300 python -u bench.py --workloads c3,c5 --simulate-world 8 --no-cpu-baseline > "$O/bench_sim8_$TAG.json" 2> "$O/bench_sim8_$TAG.err" && \
timeout -k 10 300 python -u bench.py --workloads c3,c5 --simulate-world 4 --no-cpu-baseline > "$O/bench_sim4_$TAG.json" 2> "$O/bench_sim4_$TAG.err" && \
timeout -k 10 300 python -u bench.py --workloads c3,c5 --simulate-world 2 --no-cpu-baseline > "$O/bench_sim2_$TAG.json" 2> "$O/bench_sim2_$TAG.err" && \
timeout -k 10 200 python -u tools/plan_probe.py 1 > "$O/plan_probe_$TAG.txt" 2>&1 && \
timeout -k 10 200 python -u tools/plan_probe.py 8 >> "$O/plan_probe_$TAG.txt" 2>&1 && \
bash tools/gpu_prof.sh "$TAG"
echo "round exit $?"

#!/bin/bash
# One rocprofv3 PMC pass over a short bench run: tools/pmc_pass.sh <tag> <workloads> <counters...>
# (counters of one pass must fit the hardware blocks: <= 8 SQ, <= 4 TCC, ...)
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
TAG="$1"; WL="$2"; shift 2
mkdir -p "$ROOTDIR/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$ROOTDIR/gpurun_out/pmc_$TAG" -o run -- \
    python "$ROOTDIR/bench.py" --workloads "$WL" --steps 3 --warmup 1 --no-cpu-baseline --no-verify \
    > "$ROOTDIR/gpurun_out/pmc_$TAG.out" 2> "$ROOTDIR/gpurun_out/pmc_$TAG.err"

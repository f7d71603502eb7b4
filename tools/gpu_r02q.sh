#!/bin/bash
# tests + bench (c1,c4,c5) + C5 columns, then a rocprofv3 kernel trace of the C1 bench for the
# two-event mean vs rocprof steady-average comparison.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r02q}"
bash "$ROOTDIR/tools/gpu_iter.sh" "$TAG" c1,c4,c5 || exit 1
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c1_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c1 --steps 20 --warmup 5 --no-cpu-baseline > "$O/prof_c1_$TAG.json" 2> "$O/prof_c1_$TAG.err" && \
cd "$ROOTDIR" && python tools/prof_summary.py --trace "$O/prof_c1_$TAG" --skip 5 | head -5 && \
python -c "
import json
d=json.loads(open('$O/prof_c1_$TAG.json').read().strip().splitlines()[-1])
print('bench C1 kernel_ms_mean', d['roofline']['kernel_ms_mean'], 'median', d['roofline']['kernel_ms_median'], 'frac', d['roofline']['frac'])"

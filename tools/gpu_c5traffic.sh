#!/bin/bash
# C5 evidence: per-column times (1 GPU and one 8-GPU shard), per-column and shard PMC traffic
# (separate FETCH_SIZE / WRITE_SIZE passes), simulated 2/4-GPU shards.
#   tools/gpu_c5traffic.sh TAG
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"
timeout -k 10 200 python -u tools/c5_columns.py --reps 10 > "$O/c5cols_w1_$TAG.jsonl" 2> "$O/c5cols_w1_$TAG.err" || exit 3
timeout -k 10 200 python -u tools/c5_columns.py --world 8 --reps 10 > "$O/c5cols_w8_$TAG.jsonl" 2> "$O/c5cols_w8_$TAG.err" || exit 3
for w in 2 4; do
  timeout -k 10 200 python -u bench.py --workloads c5 --no-cpu-baseline --simulate-world $w > "$O/bench_sim${w}_$TAG.json" 2> "$O/bench_sim${w}_$TAG.err" || exit 4
done
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_cols_${c}_$TAG" -o run -- python "$ROOTDIR/tools/c5_columns.py" --reps 3 --mark > "$O/pmc_cols_${c}_$TAG.jsonl" 2> "$O/pmc_cols_${c}_$TAG.err" || exit 5
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_shard_${c}_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c5 --simulate-world 8 --steps 3 --warmup 1 --no-cpu-baseline --no-verify > "$O/pmc_shard_${c}_$TAG.json" 2> "$O/pmc_shard_${c}_$TAG.err" || exit 6
done
echo "c5 traffic done"

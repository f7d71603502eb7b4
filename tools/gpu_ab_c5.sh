#!/bin/bash
# A/B of plan-recording options on C5 (N=1 and the simulated 8-GPU shard): the -m gpu suite,
# then bench c5 under each env setting given as arguments ("NAME:VAR=VAL,VAR=VAL" or "NAME:").
#   tools/gpu_ab_c5.sh TAG base: nobatch:VXG_PLAN_BATCH=0 ...
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"; shift
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -4 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
for spec in "$@"; do
  name="${spec%%:*}"; vars="${spec#*:}"
  envs=(); IFS=',' read -ra kv <<< "$vars"; for x in "${kv[@]}"; do [ -n "$x" ] && envs+=("$x"); done
  for sim in 1 8; do
    extra=""; [ $sim -gt 1 ] && extra="--simulate-world $sim"
    env "${envs[@]}" timeout -k 10 200 python -u bench.py --workloads c5 --no-cpu-baseline $extra > "$O/ab_${TAG}_${name}_w$sim.json" 2> "$O/ab_${TAG}_${name}_w$sim.err" || { echo "bench $name w$sim failed"; tail -3 "$O/ab_${TAG}_${name}_w$sim.err"; exit 4; }
    python - "$O/ab_${TAG}_${name}_w$sim.json" "$name" "$sim" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
v = d["encodings"]["C5"]
print(f"{sys.argv[2]:10s} world{sys.argv[3]} ms/step {v['ms_per_step']:.4f} kernel {v['kernel_ms_mean']:.4f} frac {v['hbm_frac_algorithmic']}")
PY
  done
done

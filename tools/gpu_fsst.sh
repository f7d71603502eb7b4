#!/bin/bash
# FSST iteration session: FSST parity tests, bench C4 (+ the given extra workloads) at N=1 and
# the simulated 8-GPU C5 shard, kernel stats and one SQ counter pass over C4.
#   tools/gpu_fsst.sh TAG [extra_workloads]
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="$1"; WL="c4${2:+,$2}"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "fsst or FSST or full_size_c4 or string" --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
timeout -k 10 300 python -u bench.py --workloads "$WL" --no-cpu-baseline > "$O/bench_$TAG.json" 2> "$O/bench_$TAG.err" || exit 4
timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --simulate-world 8 > "$O/bench_sim8_$TAG.json" 2> "$O/bench_sim8_$TAG.err" || exit 5
python - "$O/bench_$TAG.json" "$O/bench_sim8_$TAG.json" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    for k, v in d["encodings"].items():
        print(f"{f.split('/')[-1]:28s} {k} kernel_ms {v['kernel_ms_mean']:.4f} frac {v['hbm_frac_algorithmic']} verified {v.get('verified')}")
PY
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c4 --steps 20 --warmup 5 --no-cpu-baseline --no-verify > /dev/null 2> "$O/prof_$TAG.err" || exit 7
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$O/pmc_sq_$TAG" -o run -- python "$ROOTDIR/bench.py" --workloads c4 --steps 3 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> "$O/pmc_sq_$TAG.err" || exit 6
echo "fsst iter done"

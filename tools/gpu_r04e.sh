#!/bin/bash
# Round-4 session E: parity tests touched by this round's kernel changes (RunEnd K8r block-wise
# children, K1g string dictionaries in unbatched plans, KAT replays, Arrow validation), then
# A/B: K1w all-loads-first build (C1, C2; interleaved, two runs each) and VXG_PLAN_VB_K1G (C5),
# then e2e + C5 timeline + per-column (tools/gpu_c5e2e.sh).
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04e}"
timeout -k 10 900 python -u -m pytest tests/test_gpu_kats.py tests/test_gpu_arrow.py tests/test_gpu_parity.py tests/test_gpu_file.py -m gpu -x -q -k "kat or arrow or runend or RunEnd or plan or dict or string or chunked or file or lineitem or fused" --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/pytest_$TAG.log" 2>&1
rc=$?; echo "pytest exit $rc"; tail -5 "$O/pytest_$TAG.log"
[ $rc -eq 0 ] || exit 3
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --workloads c1,c2 --no-cpu-baseline --no-verify > "$O/ab_base_${TAG}_$i.json" 2> "$O/ab_base_${TAG}_$i.err" || exit 4
  VXG_GPU_LIB="$ROOTDIR/vortex_amd/libvortex_gpu_burst.so" timeout -k 10 300 python -u bench.py --workloads c1,c2 --no-cpu-baseline --no-verify > "$O/ab_burst_${TAG}_$i.json" 2> "$O/ab_burst_${TAG}_$i.err" || exit 5
done
timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline > "$O/c5_vb1_$TAG.json" 2> "$O/c5_vb1_$TAG.err" || exit 6
VXG_PLAN_VB_K1G=0 timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline > "$O/c5_vb0_$TAG.json" 2> "$O/c5_vb0_$TAG.err" || exit 7
timeout -k 10 300 python -u bench.py --workloads c5 --no-cpu-baseline --simulate-world 8 > "$O/c5_sim8_$TAG.json" 2> "$O/c5_sim8_$TAG.err" || exit 8
python - "$O" "$TAG" <<'PY'
import json, sys, glob
o, tag = sys.argv[1], sys.argv[2]
for f in sorted(glob.glob(f"{o}/ab_*_{tag}_*.json") + glob.glob(f"{o}/c5_*_{tag}.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], {k: (v['kernel_ms_mean'], v['hbm_frac_algorithmic']) for k, v in d['encodings'].items()})
PY
bash tools/gpu_c5e2e.sh "$TAG"

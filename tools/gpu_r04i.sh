#!/bin/bash
# Session I: tools/gpu_k1gbpw.sh (parity subset, C4, K1g bpw sweep), FSST ablation, C3 with K1w.
set -o pipefail
ROOTDIR="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$ROOTDIR"
O="$ROOTDIR/gpurun_out"; mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG="${1:-r04i}"
bash tools/gpu_k1gbpw.sh "$TAG" || exit $?
VXG_K1_WAVE=force timeout -k 10 300 python -u bench.py --workloads c3 --no-cpu-baseline > "$O/c3_k1w_$TAG.json" 2> "$O/c3_k1w_$TAG.err" || exit 10
timeout -k 10 300 python -u bench.py --workloads c3 --no-cpu-baseline > "$O/c3_base_$TAG.json" 2> "$O/c3_base_$TAG.err" || exit 11
python - "$O" "$TAG" <<'PY'
import json, sys
o, tag = sys.argv[1], sys.argv[2]
for n in ("c3_k1w", "c3_base"):
    d = json.loads(open(f"{o}/{n}_{tag}.json").read().strip().splitlines()[-1])
    e = d['encodings']['C3']
    print(n, e['kernel_ms_mean'], e['hbm_frac_algorithmic'], e['verified'])
PY
bash tools/gpu_fsst_abl.sh "$TAG"

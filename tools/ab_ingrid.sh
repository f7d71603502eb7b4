# A/B of the fused launch's in-grid FSST pre-pass against the separate pre-pass kernel at every
# C5 shard size (tools/gpu.sh-style; run on the GPU box).  Usage: bash tools/ab_ingrid.sh TAG [MAXTILES]
set -o pipefail
O=gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0; TAG=${1:-ab}; MT=${2:-100000}
summ() { python - $1 "$2" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k,v in d["encodings"].items(): print(sys.argv[2],k,v["kernel_ms_mean"],v["hbm_frac_algorithmic"],v.get("verified"),v.get("plan_mode",{}).get("batched"))
PY
}
for r in 1 2; do
  for w in 1 2 4 8; do
    for mt in $MT 0; do
      sim=""; [ $w -gt 1 ] && sim="--simulate-world $w"
      VXG_FUSED_PREPASS_MAX_TILES=$mt timeout -k 10 300 python -u bench.py --workloads c5 $sim --no-cpu-baseline > $O/${TAG}_${w}_$mt.json 2>$O/${TAG}_${w}_$mt.err || exit 4
      summ $O/${TAG}_${w}_$mt.json "w=$w maxtiles=$mt"
    done
  done
done

#!/bin/bash
# Resource usage of the fused FSST+K1g plan kernel only (fast: the standalone decode / pre-pass
# instantiations of fsst.hip are compiled out of a temporary copy).  tools/fsst_fused_kres.sh [-S]
set -eo pipefail
cd "$(dirname "$0")/../vortex_amd/csrc"
python3 - <<'PY'
import re
s = open("fsst.hip").read()
s = s.replace("hipLaunchKernelGGL((t.ext ? table_ext : table)[W]", "if (0) hipLaunchKernelGGL((t.ext ? table_ext : table)[W]")
s = re.sub(r"static constexpr Fn table\[\] = \{[^}]*\};", "static constexpr Fn table[] = {nullptr};", s)
s = re.sub(r"static constexpr Fn table_ext\[\] = \{[^}]*\};", "static constexpr Fn table_ext[] = {nullptr};", s)
s = s.replace("hipLaunchKernelGGL((fsst_tile_scan<", "if (0) hipLaunchKernelGGL((fsst_tile_scan<")
s = s.replace("hipLaunchKernelGGL((fsst_decode<", "if (0) hipLaunchKernelGGL((fsst_decode<")
open("/tmp/fsst_fused_only.hip", "w").write(s)
PY
cp /tmp/fsst_fused_only.hip ./.fsst_fused_only.hip
trap 'rm -f ./.fsst_fused_only.hip' EXIT
if [ "$1" = "-S" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off --cuda-device-only -S .fsst_fused_only.hip -o /tmp/fsst_fused.s
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off --cuda-device-only -c .fsst_fused_only.hip -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re,sys
cur=None; rows=[]
for l in sys.stdin:
    m=re.search(r"remark:\s+(Function Name|TotalSGPRs|VGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\S+)",l)
    if not m: continue
    k,v=m.groups()
    if k=="Function Name": cur={"name":v}; rows.append(cur)
    else: cur[k.split()[0]]=v
for r in rows:
    if "fsst_k1g" in r["name"]: print(r.get("VGPRs"), r.get("TotalSGPRs"), r.get("ScratchSize"), r.get("Occupancy"), r["name"][:110])
'

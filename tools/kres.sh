#!/bin/bash
# Per-kernel resource usage of one HIP source (VGPRs, SGPRs, scratch, occupancy): tools/kres.sh file.hip [filter]
f=$1; flt=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -ffp-contract=off --cuda-device-only -c "$f" -o /tmp/kres.o \
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
    if re.search(sys.argv[1], r["name"]): print(r.get("VGPRs"), r.get("TotalSGPRs"), r.get("ScratchSize"), r.get("Occupancy"), r["name"][:110])
' "$flt"

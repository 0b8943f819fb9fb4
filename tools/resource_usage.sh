#!/bin/bash
# resource_usage.sh FILE.hip -- per-kernel VGPR/AGPR/spill/LDS/occupancy summary
# (hipcc -Rpass-analysis=kernel-resource-usage), one line per kernel.
f=$1
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -c "$f" -o /tmp/ru.o \
    -Rpass-analysis=kernel-resource-usage 2>&1 |
python3 -c '
import sys,re
cur=None; rows=[]
for line in sys.stdin:
    m=re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|Occupancy \[waves/SIMD\]): (\S+)",line)
    if not m: continue
    k,v=m.groups()
    if k=="Function Name":
        cur={"name":v}; rows.append(cur)
    elif cur is not None: cur[k]=v
for r in rows:
    print(r["name"][:70].ljust(70), "V",r.get("VGPRs"),"A",r.get("AGPRs"),"vspill",r.get("VGPRs Spill"),"sspill",r.get("SGPRs Spill"),"LDS",r.get("LDS Size [bytes/block]"),"occ",r.get("Occupancy [waves/SIMD]"))
'

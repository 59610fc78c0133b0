#!/bin/bash
# usage: tools/kres.sh file.hip [extra hipcc flags] — per-kernel VGPR/AGPR/spill/occupancy
f=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I $(dirname $f) -I /root/repo/pipsort_amd/csrc "$@" -c $f -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import sys,re
cur=None
for l in sys.stdin:
    m=re.search(r"Function Name: (\S+)",l)
    if m: cur=m.group(1)[:60]; print(); print(cur,end=" ")
    for k in ("VGPRs","AGPRs","ScratchSize","Occupancy","VGPRs Spill","SGPRs Spill","LDS Size"):
        m=re.search(k+r"[^:]*: (\d+)",l)
        if m and cur and "remark:     "+k in l: print(f"{k}={m.group(1)}",end=" ")
print()'

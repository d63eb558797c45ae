#!/bin/sh
# kres.sh FILE.hip — per-kernel VGPR / occupancy / LDS summary (hipcc -Rpass-analysis)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -c "$1" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re,sys
cur=None
for line in sys.stdin:
    m=re.search(r"Function Name: (\S+)",line)
    if m: cur=m.group(1); out={}; continue
    for key in ("VGPRs","AGPRs","Occupancy \\[waves/SIMD\\]","LDS Size \\[bytes/block\\]","VGPRs Spill"):
        m=re.search(key+r": (\d+)",line)
        if m and cur: out[key.split()[0]]=m.group(1)
    if "LDS Size" in line and cur:
        print(cur[-70:], out); cur=None
'

# Per-kernel VGPR / SGPR / occupancy of a HIP source (compile-time resource report).
f=${1:?source}; shift
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -I "$(dirname "$0")/../include" "$@" -c "$f" -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 -c '
import re,sys
cur=None
for line in sys.stdin:
    m=re.search(r"Function Name: (\S+)",line)
    if m: cur=m.group(1); continue
    for key in ("VGPRs:","TotalSGPRs:","Occupancy \\[waves/SIMD\\]:","LDS Size \\[bytes/block\\]:","ScratchSize \\[bytes/lane\\]:"):
        m=re.search(key+r" (\d+)",line)
        if m and cur: print(f"{cur[:70]:70s} {key.split()[0]:12s} {m.group(1)}")
'

"""Total and per-launch kernel time by kernel from a rocprofv3 kernel-trace CSV (isolated durations)."""
import csv
import sys
from collections import defaultdict

tot, n = defaultdict(float), defaultdict(int)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
    tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    n[k] += 1
T = sum(tot.values())
for k in sorted(tot, key=lambda k: -tot[k]):
    print(f"{k[:45]:45s} {n[k]:5d} {tot[k]:9.2f} ms {tot[k] / n[k] * 1e3:9.1f} us/launch {tot[k] / T * 100:5.1f}%")
print(f"total {T:.1f} ms")

"""Median gap between consecutive kernels on one queue (rocprofv3 kernel traces): usage gaps.py DIR..."""
import csv
import glob
import statistics
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    by = defaultdict(list)
    for r in rows:
        by[r["Queue_Id"]].append(r)
    for q, rs in by.items():
        gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(rs, rs[1:])
                if "k_bounce" in a["Kernel_Name"] and "k_bounce<false" in b["Kernel_Name"].replace("(anonymous namespace)::", "")]
        if len(gaps) > 5:
            print(d.split("/")[-1], "queue", q, "bounce->bounce gaps:", len(gaps), "median us", round(statistics.median(gaps), 2),
                  "p10", round(sorted(gaps)[len(gaps) // 10], 2))

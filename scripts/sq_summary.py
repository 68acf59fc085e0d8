"""Per-kernel SQ counter means from a rocprofv3 --pmc csv directory (scripts/gpu_sq.sh)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
files = sorted(root.rglob("*counter_collection.csv"))
if not files:
    sys.exit(f"no counter_collection.csv under {root}")
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(set)
for f in files:
    for row in csv.DictReader(open(f)):
        k = row["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
        acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
        n[k].add(row.get("Dispatch_Id", row.get("Correlation_Id")))
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
    d = max(len(n[k]), 1)
    w = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k}  dispatches={d}")
    print("   per dispatch: " + "  ".join(f"{name}={v / d:.4g}" for name, v in sorted(c.items())))
    print(f"   fractions of WAVE_CYCLES: active={c.get('SQ_ACTIVE_INST_ANY', 0) / w:.3f} "
          f"wait_inst={c.get('SQ_WAIT_INST_ANY', 0) / w:.3f} wait_any={c.get('SQ_WAIT_ANY', 0) / w:.3f} "
          f"valu_active={c.get('SQ_ACTIVE_INST_VALU', 0) / w:.3f}; "
          f"VALU insts/wave={c.get('SQ_INSTS_VALU', 0) / max(c.get('SQ_WAVES', 1), 1):.0f}")

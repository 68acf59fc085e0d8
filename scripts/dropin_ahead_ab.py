"""Drop-in call sequence (bench.dropin_bench) with and without render-ahead (PT_AMD_AHEAD), alternating."""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

scene = str(ROOT / "tests" / "scenes" / "cornell.json")
for k in range(int(os.environ.get("RUNS", "3"))):
    for ahead in ("1", "0"):
        os.environ["PT_AMD_AHEAD"] = ahead
        r = bench.dropin_bench(scene, iters=int(os.environ.get("ITERS", "200")))
        print(json.dumps({"ahead": ahead, "value": round(r.get("value", 0), 1),
                          "ms_per_call": round(r.get("ms_per_call", 0), 4), "segments": r.get("segments"),
                          "error": r.get("error")}), flush=True)

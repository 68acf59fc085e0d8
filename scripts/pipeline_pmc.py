"""Per-kernel SQ counters of the fused pipelines (k_shift default vs k_bounce, PT_PIPELINE=fused) over
the same render-only workload: launches, isolated duration, VALU / SALU per launch, wave states,
instruction-fetch stalls.  usage: pipeline_pmc.py [spp] [passes]"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scripts"))
import pmc  # noqa: E402

pmc.GROUPS["ifetch"] = ["SQ_WAVE_CYCLES", "SQ_IFETCH", "SQ_IFETCH_LEVEL", "SQ_WAIT_INST_ANY", "SQ_INSTS_SMEM",
                        "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"]
spp = sys.argv[1] if len(sys.argv) > 1 else "128"
passes = sys.argv[2] if len(sys.argv) > 2 else "2"
out = {}
for v in ("shift", "fused"):
    if v == "fused":
        os.environ["PT_PIPELINE"] = "fused"
    else:
        os.environ.pop("PT_PIPELINE", None)
    res = pmc.collect([passes, f"spp={spp}"], ROOT / "gpurun_out" / "pipeline_pmc" / v, timeout=150,
                      groups=("sq", "ifetch"))
    out[v] = res
    print(v, "passes", res["_passes"], "segments", res.get("segments"))
    for k, m in sorted(res.get("kernels", {}).items()):
        if not k.startswith(("k_shift", "k_bounce", "k_finalize")):
            continue
        wc = max(m.get("SQ_WAVE_CYCLES", 1.0), 1.0)
        print(f"  {k:34s} n={m.get('launches')} dur={m.get('dur_ns_sq', 0) / 1e3:8.1f}us valu={m.get('SQ_INSTS_VALU', 0) / 1e6:8.2f}M "
              f"salu={m.get('SQ_INSTS_SALU', 0) / 1e6:7.2f}M waves={m.get('SQ_WAVES', 0):.0f} act={m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
              f"wi={m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} wa={m.get('SQ_WAIT_ANY', 0) / wc:.2f} ifetch={m.get('SQ_IFETCH', 0) / 1e6:.2f}M "
              f"ifl={m.get('SQ_IFETCH_LEVEL', 0) / wc:.2f} lds={m.get('SQ_INSTS_LDS', 0) / 1e6:.2f}M smem={m.get('SQ_INSTS_SMEM', 0) / 1e6:.2f}M "
              f"clk={m.get('GRBM_GUI_ACTIVE', 0) / 8 / max(m.get('dur_ns_sq', 1), 1):.2f}")
(ROOT / "gpurun_out" / "pipeline_pmc" / "summary.json").write_text(json.dumps(out, indent=1))

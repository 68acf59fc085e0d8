"""Stall breakdown of the bounce kernels (rocprofv3 PMC): issue-blocked cycles by unit, instruction
fetch, and average in-flight latency of vector-memory, LDS and scalar-memory instructions
(SQ_INST_LEVEL_x / SQ_INSTS_x, in cycles).  Workload: the bench's Cornell passes.  Usage:
python scripts/stall_pmc.py OUT_DIR [scene=PATH]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scripts"))
import pmc  # noqa: E402

out = Path(sys.argv[1]).resolve()
extra = [a for a in sys.argv[2:] if a.startswith("scene=")]
res = pmc.collect(["4", "spp=32"] + extra, out / "pmc", timeout=150, groups=("stall1", "stall2", "sq", "vmem"))
summ = {"passes": res["_passes"]}
for name in ("k_bounce<false, false, 0>", "k_bounce<true, false, 0>"):
    m = pmc.pick(res, name) or {}
    wc = max(m.get("SQ_WAVE_CYCLES", 0.0), 1.0)
    r = {k: m.get(k) for k in sorted(m)}
    r["frac_of_wave_cycles"] = {k: m.get(k, 0.0) / wc for k in ("SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                                                                 "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_ANY",
                                                                 "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU")}
    for lvl, cnt in (("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM"), ("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS"),
                     ("SQ_INST_LEVEL_SMEM", "SQ_INSTS_SMEM"), ("SQ_IFETCH_LEVEL", "SQ_IFETCH")):
        if m.get(cnt):
            r["avg_latency_" + cnt] = m.get(lvl, 0.0) / m[cnt]
    summ[name] = r
(out / "stall_pmc.json").write_text(json.dumps(summ, indent=1))
for name in ("k_bounce<false, false, 0>", "k_bounce<true, false, 0>"):
    r = summ[name]
    print(name, json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r["frac_of_wave_cycles"].items()}))
    print("   latencies", {k: round(v, 1) for k, v in r.items() if k.startswith("avg_latency")})

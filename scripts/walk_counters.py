"""Counters of the BVH walk (k_traverse4 / k_traverse) on config 5's scene: one rocprofv3 --pmc
pass per group over a render-only workload (scripts/prof_render.py), then per-launch means of the
later-bounce walk: VALU/SALU/VMEM/LDS instructions per ray, wave states, vector-L1 traffic and the
average L1->L2 request latency, L2 hit rate, TA busy.  Run on the GPU box:
python scripts/walk_counters.py OUT_DIR [spp] [groups...]"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))
import pmc  # noqa: E402
from cuda_pathtracer_amd import scenes  # noqa: E402

out = Path(sys.argv[1]).resolve()   # (rocprofv3 runs from /tmp)
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 16
groups = tuple(sys.argv[3:]) or ("sq", "stall1", "stall2", "tcp", "ta", "l2", "vmem")
scene = scenes.random_triangles(out / "scene", n=100_000)
res = pmc.collect(["1", f"spp={spp}", f"scene={scene}"], out / "pmc", timeout=240, groups=groups)
summ = {"passes": res["_passes"], "segments": res.get("segments"), "spp": spp}
for name in ("k_traverse4<false,", "k_traverse<false>", "k_traverse4<true,", "k_traverse<true>"):   # (k_traverse4<FIRST, K>)
    m = pmc.pick(res, name)
    if not m:
        continue
    wc = max(m.get("SQ_WAVE_CYCLES", 0.0), 1.0)
    d = {"launches": m.get("launches"), "dur_ms": (m.get("dur_ns_sq") or 0) / 1e6}
    for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_WAVES"):
        if c in m:
            d[c] = m[c]
    if "SQ_ACTIVE_INST_ANY" in m:
        d["issuing"] = m["SQ_ACTIVE_INST_ANY"] / wc
        d["waiting_on_issue"] = m.get("SQ_WAIT_INST_ANY", 0) / wc
        d["waiting_any"] = m.get("SQ_WAIT_ANY", 0) / wc
    if "SQ_INST_LEVEL_VMEM" in m and m.get("SQ_INSTS_VMEM"):
        d["vmem_latency_cycles"] = m["SQ_INST_LEVEL_VMEM"] / m["SQ_INSTS_VMEM"] * 4   # quad-cycles (pmc.py)
    if "SQ_INST_LEVEL_LDS" in m and m.get("SQ_INSTS_LDS"):
        d["lds_latency_cycles"] = m["SQ_INST_LEVEL_LDS"] / m["SQ_INSTS_LDS"] * 4
    if "TCP_TOTAL_ACCESSES_sum" in m:
        d["tcp_accesses"] = m["TCP_TOTAL_ACCESSES_sum"]
        d["tcp_to_l2_reqs"] = m["TCP_TCC_READ_REQ_sum"]
        d["l1_miss_ratio"] = m["TCP_TCC_READ_REQ_sum"] / max(m["TCP_TOTAL_ACCESSES_sum"], 1)
        d["l2_req_latency_cycles"] = m["TCP_TCC_READ_REQ_LATENCY_sum"] / max(m["TCP_TCC_READ_REQ_sum"], 1)
        d["tcp_latency_per_access"] = m["TCP_TCP_LATENCY_sum"] / max(m["TCP_TOTAL_ACCESSES_sum"], 1)
    if "TA_TA_BUSY_sum" in m and d["dur_ms"]:
        d["ta_busy_frac"] = m["TA_TA_BUSY_sum"] / 256 / (d["dur_ms"] * 1e-3 * 2.4e9)
        d["ta_addr_stalled_by_tc_frac"] = m["TA_ADDR_STALLED_BY_TC_CYCLES_sum"] / max(m["TA_TA_BUSY_sum"], 1)
    if "TCC_HIT_sum" in m:
        d["l2_hit"] = m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m["TCC_MISS_sum"], 1)
    summ[name] = d
(out / "walk_counters.json").write_text(json.dumps(summ, indent=1))
print(json.dumps(summ, indent=1))

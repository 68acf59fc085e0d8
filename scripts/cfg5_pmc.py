"""Counters of config 5's BVH walk (k_traverse): L2 hit rate, fabric bytes, VALU and memory
instructions per launch, and the gathered-bytes rate against the L2 bandwidth.  Workload: one pass of
`spp` iterations of the 100k-triangle scene at 4K (scripts/prof_render.py).  Run on the GPU box:
python scripts/cfg5_pmc.py OUT_DIR [spp]."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "scripts"))
import pmc  # noqa: E402
from cuda_pathtracer_amd import scenes  # noqa: E402

out = Path(sys.argv[1]).resolve()   # (rocprofv3 runs from /tmp)
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 2
scene = scenes.random_triangles(out / "scene", n=100_000)
res = pmc.collect(["1", f"spp={spp}", f"scene={scene}"], out / "pmc", timeout=240, groups=("fetch", "l2", "sq", "vmem"))
k = pmc.pick(res, "k_traverse<false>") or {}
k0 = pmc.pick(res, "k_traverse<true>") or {}
summ = {"passes": res["_passes"], "segments": res.get("segments"), "k_traverse_later": k, "k_traverse_first": k0}
for name, m in (("later", k), ("first", k0)):
    if m.get("TCC_HIT_sum") is not None:
        h, mi = m["TCC_HIT_sum"], m["TCC_MISS_sum"]
        summ[f"l2_hit_rate_{name}"] = h / max(h + mi, 1.0)
(out / "cfg5_pmc.json").write_text(json.dumps(summ, indent=1))
print(json.dumps({k: v for k, v in summ.items() if not isinstance(v, dict)}, indent=1))
for name, m in (("later", k), ("first", k0)):
    print(name, {c: m.get(c) for c in ("launches", "dur_ns_fetch", "FETCH_SIZE", "SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD",
                                        "SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY")})

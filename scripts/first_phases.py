"""Per-kernel VALU of the fused pipeline's kernels for phase-duplication builds (PT_DUP=6 raygen,
7 camera-ray closest hit, 2 shade of later bounces): rocprofv3 --pmc SQ counters over one pass of 128
iterations per variant.  usage: first_phases.py variant..."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "scripts"))
import pmc  # noqa: E402

for v in ["new"] + sys.argv[1:]:
    if v == "new":
        os.environ.pop("PT_AMD_LIB", None)
    else:
        os.environ["PT_AMD_LIB"] = str(ROOT / "cuda_pathtracer_amd" / "build" / f"libpt_amd_{v}.so")
    res = pmc.collect(["1", "spp=128"], ROOT / "gpurun_out" / "first_phases" / v, timeout=150, groups=("sq",))
    live = res.get("bounce_live") or [1]
    for k, m in sorted(res.get("kernels", {}).items()):
        if k.startswith("k_bounce"):
            n = m.get("launches", 1)
            print(f"{v:6s} {k:28s} n={n} VALU/launch={m.get('SQ_INSTS_VALU', 0) / 1e6:8.2f}M "
                  f"per camera path={m.get('SQ_INSTS_VALU', 0) * n / live[0] if 'true' in k else 0:.3f}")

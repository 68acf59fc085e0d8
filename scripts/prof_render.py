"""Render-only workload for rocprofv3 (no torch kernels, no scan): N passes of cornell 800x800,
`spp=K` iterations per pass (default 32, like bench.py)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import os
os.environ.setdefault("PT_AMD_NO_TORCH", "1")
import cuda_pathtracer_amd as P

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sort = "sort" in sys.argv[2:]
spp = next((int(a[4:]) for a in sys.argv[2:] if a.startswith("spp=")), 32)   # bench.py's default batch
s = P.Scene(str(ROOT / "tests" / "scenes" / "cornell.json"))
g = P.GuiDataContainer()
g.sortbyMaterial = sort
pt = P.PathTracer(s, g, spp=spp)
for k in range(passes):
    pt.render_pass(1 + k * spp)
st = pt.stats()
print(st["segments"], st["bounce_live"])
pt.free()

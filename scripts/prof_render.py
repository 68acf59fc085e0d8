"""Render-only workload for rocprofv3 (no torch kernels, no scan): N passes of cornell 800x800."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
import os
os.environ.setdefault("PT_AMD_NO_TORCH", "1")
import cuda_pathtracer_amd as P

passes = int(sys.argv[1]) if len(sys.argv) > 1 else 20
sort = len(sys.argv) > 2 and sys.argv[2] == "sort"
s = P.Scene(str(ROOT / "tests" / "scenes" / "cornell.json"))
g = P.GuiDataContainer()
g.sortbyMaterial = sort
pt = P.PathTracer(s, g)
for it in range(1, passes + 1):
    pt.render_pass(it)
st = pt.stats()
print(st["segments"], st["bounce_live"])
pt.free()

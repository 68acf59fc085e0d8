"""Phase attribution of the non-first bounce kernel from the -DPT_STAMPS diagnostic library."""
import ctypes as C
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("PT_AMD_LIB", str(ROOT / "cuda_pathtracer_amd" / "build" / "libpt_amd_stamps.so"))
os.environ.setdefault("PT_AMD_NO_TORCH", "1")
sys.path.insert(0, str(ROOT))
import cuda_pathtracer_amd as P  # noqa: E402
from cuda_pathtracer_amd._native import lib  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "tests" / "scenes" / "cornell.json")
pt = P.PathTracer(P.Scene(scene), P.GuiDataContainer(), spp=4)
buf = (C.c_ulonglong * 16)()
for k in range(3):
    pt.render_pass(1 + 4 * k)
lib().pt_debug_stamps(buf, 1)
for k in range(20):
    pt.render_pass(100 + 4 * k)
lib().pt_debug_stamps(buf, 0)
names = ["load", "intersect", "shade+retire", "ballot+barrier", "store+walk"]
tot = sum(buf[q] for q in range(5))
print(f"wave-tiles={buf[5]}  cycles/wave-tile={tot / max(buf[5], 1):.0f}")
for q, n in enumerate(names):
    print(f"  {n:16s} {buf[q] / max(buf[5], 1):8.0f} cycles  {100.0 * buf[q] / max(tot, 1):5.1f}%")
w = max(buf[8], 1)
print(f"closest-hit calls (wave-level) {buf[8]}: lanes with a hit candidate {buf[14] / w:.1f}/64")
print(f"  second candidate: {buf[9] / w:.2f} lanes/wave, {100.0 * buf[10] / w:.1f}% of waves")
print(f"  >=3 candidates:   {buf[11] / w:.3f} lanes/wave, {100.0 * buf[12] / w:.1f}% of waves")
print(f"  waves mixing cube+sphere first candidates: {100.0 * buf[13] / w:.1f}%")
pt.free()

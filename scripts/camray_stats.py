"""Camera rays' closest-hit work per wave (the -DPT_STAMPS diagnostic library, counters of
intersect_bounded): traced at DEPTH 1 so only the first bounce runs.  Per scene: waves, lanes with a
candidate, bounded geoms per wave (the camera mask's popcount), second / third exact tests."""
import ctypes as C
import os
import sys
import tempfile
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
os.environ.setdefault("PT_AMD_LIB", str(ROOT / "cuda_pathtracer_amd" / "build" / "libpt_amd_stamps.so"))
sys.path.insert(0, str(ROOT))
import cuda_pathtracer_amd as P  # noqa: E402
from cuda_pathtracer_amd import scenes  # noqa: E402
from cuda_pathtracer_amd._native import lib  # noqa: E402

tmp = tempfile.mkdtemp()
cases = [("cornell 800x800", str(ROOT / "tests" / "scenes" / "cornell.json")),
         ("cornell_hd 1920x1080", scenes.cornell_hd(tmp))]
buf = (C.c_ulonglong * 16)()
for name, path in cases:
    s = P.Scene(path)
    st = s.state()
    s.set_render(st.iterations, 1, st.imageName)
    s.finalize()
    pt = P.PathTracer(s, P.GuiDataContainer(), spp=8)
    pt.render_pass(1)
    lib().pt_debug_stamps(buf, 1)
    for k in range(4):
        pt.render_pass(9 + 8 * k)
    lib().pt_debug_stamps(buf, 0)
    w = max(buf[8], 1)
    print(f"{name}: closest-hit wave calls {buf[8]}")
    print(f"  lanes with a candidate {buf[14] / w:.1f}/64; bounded geoms per wave {buf[15] / w:.2f} (of {s.counts()[0]})")
    print(f"  second exact test: {buf[9] / w:.2f} lanes/wave, {100.0 * buf[10] / w:.1f}% of waves")
    print(f"  third+:            {buf[11] / w:.3f} lanes/wave, {100.0 * buf[12] / w:.1f}% of waves")
    print(f"  waves mixing cube+sphere first candidates {100.0 * buf[13] / w:.1f}%", flush=True)
    pt.free()

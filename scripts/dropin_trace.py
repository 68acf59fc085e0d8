"""Kernel trace helper for the drop-in sequence: 30 one-iteration pathtrace() calls (render pass on
the context's stream + synchronous image copy), run under rocprofv3 --kernel-trace."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from cuda_pathtracer_amd import GuiDataContainer, PathTracer, Scene  # noqa: E402
from cuda_pathtracer_amd._native import check_pt, lib  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
pt = PathTracer(Scene(str(ROOT / "tests" / "scenes" / "cornell.json")), GuiDataContainer())
st = C.c_void_p()
check_pt(lib().pt_stream_create(C.byref(st)))
img = np.empty((800, 800, 3), np.float32)
check_pt(lib().pt_host_register(img.ctypes.data, img.nbytes))
for it in range(1, 31):
    check_pt(lib().pt_render_pass(pt._h, it, st))
    check_pt(lib().pt_get_image(pt._h, img.ctypes.data))
check_pt(lib().pt_host_unregister(img.ctypes.data))
pt.free()
print("ok")

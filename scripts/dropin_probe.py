"""Where the drop-in pathtrace() call's time goes: one-iteration pass alone, the image copy into
pageable / registered / torch-pinned host memory, and the full call sequence."""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from cuda_pathtracer_amd import GuiDataContainer, PathTracer, Scene  # noqa: E402
from cuda_pathtracer_amd._native import check_pt, lib  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
scene = Scene(str(ROOT / "tests" / "scenes" / "cornell.json"))
pt = PathTracer(scene, GuiDataContainer())
st = C.c_void_p()
check_pt(lib().pt_stream_create(C.byref(st)))
N = 50
it = 1


def timed(fn, n=N):
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e3


def render():
    global it
    check_pt(lib().pt_render_pass(pt._h, it, st))
    it += 1


for _ in range(5):
    render()
pt.stats()
page = np.empty((800, 800, 3), np.float32)
reg = np.empty((800, 800, 3), np.float32)
check_pt(lib().pt_host_register(reg.ctypes.data, reg.nbytes))
pin = torch.empty((800, 800, 3), dtype=torch.float32, pin_memory=True)
res = {}
res["render+stats_ms"] = timed(lambda: (render(), pt.stats()))
res["copy_pageable_ms"] = timed(lambda: check_pt(lib().pt_get_image(pt._h, page.ctypes.data)))
res["copy_registered_ms"] = timed(lambda: check_pt(lib().pt_get_image(pt._h, reg.ctypes.data)))
res["copy_torch_pinned_ms"] = timed(lambda: check_pt(lib().pt_get_image(pt._h, pin.data_ptr())))
res["render_only_enqueue_ms"] = timed(render)
check_pt(lib().pt_get_image(pt._h, reg.ctypes.data))
res["render+copy_registered_ms"] = timed(lambda: (render(), check_pt(lib().pt_get_image(pt._h, reg.ctypes.data))))
res["render+copy_pageable_ms"] = timed(lambda: (render(), check_pt(lib().pt_get_image(pt._h, page.ctypes.data))))
d = torch.empty((800, 800, 3), dtype=torch.float32, device="cuda")
t0 = time.perf_counter()
for _ in range(N):
    d.copy_(pin.view_as(d), non_blocking=False)
torch.cuda.synchronize()
res["torch_h2d_pinned_ms"] = (time.perf_counter() - t0) / N * 1e3
t0 = time.perf_counter()
for _ in range(N):
    pin.copy_(d.view_as(pin))
torch.cuda.synchronize()
res["torch_d2h_pinned_ms"] = (time.perf_counter() - t0) / N * 1e3
print({k: round(v, 4) for k, v in res.items()})
check_pt(lib().pt_host_unregister(reg.ctypes.data))
pt.free()

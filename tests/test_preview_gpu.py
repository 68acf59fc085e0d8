"""Interactive preview on the GPU (cuda_pathtracer_amd/preview.py): the session's frames are the
HIP render's PBO (pt_preview_rgba) and its accumulator equals the oracle's for the loaded camera;
after an orbit the session restarts and renders what a fresh context of the moved camera renders;
the HTTP window serves the frames while its render thread runs the loop.

Reference: main.cpp:114-168 (runCuda), :228-271 (mouse), pathtrace.cu:64-86 (sendImageToPBO),
preview.cpp:289-322 (mainLoop).
"""
import io
import json
import time
import urllib.request

import numpy as np
import pytest

from oracle import binding as O

pytestmark = pytest.mark.gpu


def _scene(cornell_path, iterations=64, res=(64, 48)):
    from cuda_pathtracer_amd import Scene
    s = Scene(cornell_path)
    s.set_camera(res, 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    st = s.state()
    s.set_render(iterations, st.traceDepth, st.imageName)
    s.finalize()
    return s


def _direct(scene, iters):
    import torch
    from cuda_pathtracer_amd import PathTracer
    pt = PathTracer(scene)
    for it in range(1, iters + 1):
        pt.render_pass(it)
    cam = scene.camera()
    buf = torch.empty((cam.res[1], cam.res[0], 4), dtype=torch.uint8, device="cuda")
    pt.preview_rgba(iters, buf.data_ptr())
    out = buf.cpu().numpy(), pt.image()
    pt.free()
    return out


def test_session_frames_are_the_hip_render(cornell_path, tmp_path):
    from cuda_pathtracer_amd import preview as V
    s = _scene(cornell_path)
    ses = V.PreviewSession(s, out_dir=str(tmp_path))
    for _ in range(3):
        ses.run_cuda()
    assert ses.iteration == 3
    rgba, img = _direct(_scene(cornell_path), 3)
    assert np.array_equal(ses.rgba, rgba)
    assert np.array_equal(ses.ctx.image(), img)
    o = O.OracleScene.from_json(cornell_path)
    o.set_camera((64, 48), 45.0, (0, 5, 10.5), (0, 5, 0), (0, 1, 0))
    ref = None
    for it in range(1, 4):
        ref, _ = O.render_pass(o, O.flags(), it, image=ref)
    assert np.array_equal(img, ref)
    # orbit (left drag): the session restarts on the moved camera
    ses.mouse_move(10, 10)
    ses.mouse_button(V.MOUSE_LEFT, V.PRESS)
    ses.mouse_move(22, 16)
    ses.run_cuda()
    ses.run_cuda()
    assert ses.iteration == 2
    rgba2, img2 = _direct(s, 2)   # a fresh context of the same (moved) scene camera
    assert np.array_equal(ses.rgba, rgba2) and np.array_equal(ses.ctx.image(), img2)
    assert not np.array_equal(rgba2, _direct(_scene(cornell_path), 2)[0])
    ses.key("S")
    assert len(ses.saved) == 1 and ses.saved[0].endswith(".2samp.png")
    ses.close()


def test_http_window_with_render_thread(cornell_path, tmp_path):
    from PIL import Image
    from cuda_pathtracer_amd import preview as V
    ses = V.PreviewSession(_scene(cornell_path, iterations=12), out_dir=str(tmp_path))
    srv = V.PreviewServer(ses).start(render=True)
    try:
        deadline = time.time() + 60
        while not ses.done and time.time() < deadline:
            time.sleep(0.02)
        assert ses.done and ses.iteration == 12 and len(ses.saved) == 1
        with urllib.request.urlopen(srv.url + "state", timeout=10) as r:
            st = json.loads(r.read())
        assert st["iteration"] == 12 and st["done"] and st["fps"] > 0
        with urllib.request.urlopen(srv.url + "frame.png", timeout=10) as r:
            png = np.asarray(Image.open(io.BytesIO(r.read())))
        rgba, _ = _direct(_scene(cornell_path), 12)
        assert np.array_equal(png, rgba[:, ::-1, :3])
    finally:
        srv.stop()

"""Interactive preview (the reference's window, cuda_pathtracer_amd/preview.py) on the CPU: the
orbit camera recompute of the C ABI, main.cpp's mouse / key callbacks and runCuda's restart logic
driven with a stand-in render context, the PNG encoder, and the HTTP front end.

Reference: main.cpp:59-73 (orbit of the loaded camera), :114-168 (runCuda), :189-271 (callbacks),
preview.cpp:43-68 (display orientation), :212-282 (panel), :289-322 (mainLoop).
"""
from __future__ import annotations

import ctypes as C
import io
import json
import urllib.error
import urllib.request
from pathlib import Path

import numpy as np
import pytest

import cuda_pathtracer_amd as P
from cuda_pathtracer_amd import preview as V

ROOT = Path(__file__).resolve().parent.parent
SCENES = ROOT / "tests" / "scenes"
F = np.float32
_libm = C.CDLL("libm.so.6")
for _fn in ("sinf", "cosf"):
    getattr(_libm, _fn).restype = C.c_float
    getattr(_libm, _fn).argtypes = [C.c_float]


def _cam(scene):
    c = scene.camera()
    return {k: np.array(getattr(c, k)[:3], F) for k in ("position", "look_at", "view", "up", "right")}


def _orbit_restated(phi, theta, zoom, la):
    """main.cpp:117-136 in float32 (glm: normalize = v * (1 / sqrt(dot)), dot = (xx + yy) + zz)."""
    sp, st = F(_libm.sinf(phi)), F(_libm.sinf(theta))
    cp_, ct = F(_libm.cosf(phi)), F(_libm.cosf(theta))
    z = F(zoom)
    cp = np.array([(z * sp) * st, z * ct, (z * cp_) * st], F)
    d = (cp[0] * cp[0] + cp[1] * cp[1]) + cp[2] * cp[2]
    s = F(1.0) / np.sqrt(F(d))
    v = -(cp * s)
    u0 = np.array([0, 1, 0], F)

    def cross(a, b):
        return np.array([a[1] * b[2] - b[1] * a[2], a[2] * b[0] - b[2] * a[0], a[0] * b[1] - b[0] * a[1]], F)

    r = cross(v, u0)
    u = cross(r, v)
    return {"position": cp + np.asarray(la, F), "view": v, "right": r, "up": u, "look_at": np.asarray(la, F)}


@pytest.mark.parametrize("name", ["cornell.json", "sphere.json"])
def test_orbit_round_trip_reproduces_the_loaded_camera(name):
    path = SCENES / name
    if not path.exists():
        pytest.skip(f"{name} not bundled")
    s = P.Scene(str(path))
    before = _cam(s)
    s.set_orbit(*s.orbit(), before["look_at"])
    after = _cam(s)
    for k in before:
        assert before[k].tobytes() == after[k].tobytes(), k


@pytest.mark.parametrize("phi,theta,zoom,la", [(0.3, 1.2, 9.0, (0, 5, 0)), (-2.0, 0.001, 0.1, (1.5, -2, 3)),
                                               (3.0, 3.1415927, 25.0, (0, 0, 0))])
def test_set_orbit_is_runcudas_recompute(phi, theta, zoom, la):
    s = P.Scene(str(SCENES / "cornell.json"))
    s.set_orbit(phi, theta, zoom, la)
    got, want = _cam(s), _orbit_restated(F(phi), F(theta), F(zoom), la)
    for k in want:
        assert got[k].tobytes() == want[k].tobytes(), (k, got[k], want[k])
    assert got["right"][1] == 0.0   # view x (0,1,0) has no y component


def test_orbit_needs_a_finalized_scene():
    s = P.Scene()
    with pytest.raises(RuntimeError):
        s.orbit()
    with pytest.raises(RuntimeError):
        s.set_orbit(0.0, 1.0, 2.0, (0, 0, 0))


class FakeCtx:
    def __init__(self, h, w, log):
        self.h, self.w, self.log = h, w, log
        self.freed = False

    def set_flags(self, gui):
        self.log.append(("flags", gui.SSAA, gui.DoF, gui.aperture, gui.sortbyMaterial))

    def render_pass(self, it):
        self.log.append(("pass", it))

    def image(self):
        return np.full((self.h, self.w, 3), 0.5, np.float32)

    def free(self):
        self.freed = True


def _session(tmp_path, iterations=None):
    s = P.Scene(str(SCENES / "cornell.json"))
    if iterations is not None:
        st = s.state()
        s.set_render(iterations, st.traceDepth, st.imageName)
        s.finalize()
    log, made = [], []

    def factory(scene, gui):
        c = FakeCtx(scene.camera().res[1], scene.camera().res[0], log)
        made.append(c)
        return c

    def read(ctx, it):
        a = np.zeros((ctx.h, ctx.w, 4), np.uint8)
        a[..., 0] = it
        a[:, 0, 1] = 200   # column x = 0: shown at the window's right edge
        return a

    return V.PreviewSession(s, out_dir=str(tmp_path), tracer_factory=factory, read_preview=read), log, made


def test_runcuda_iterations_and_restart_on_camera_change(tmp_path):
    ses, log, made = _session(tmp_path)
    ses.run_cuda()
    ses.run_cuda()
    assert ses.iteration == 2 and len(made) == 1 and ("pass", 2) in log
    assert ses.title() == "Path Tracer | 2 Iterations"
    pos0 = _cam(ses.scene)["position"]
    # left drag: phi -= dx / width, theta -= dy / height (main.cpp:240-246)
    ses.mouse_move(100, 100)            # (both coordinates new: recorded, no button)
    ses.mouse_button(V.MOUSE_LEFT, V.PRESS)
    phi0, th0 = ses.phi, ses.theta
    ses.mouse_move(140, 120)
    assert ses.phi == F(float(phi0) - 40 / ses.width)
    assert ses.theta == F(float(th0) - 20 / ses.height)
    assert ses.camchanged
    ses.run_cuda()
    assert ses.iteration == 1 and len(made) == 2 and made[0].freed
    pos1 = _cam(ses.scene)["position"]
    assert not np.array_equal(pos0, pos1)
    want = _orbit_restated(ses.phi, ses.theta, ses.zoom, ses.look_at)["position"]
    assert pos1.tobytes() == want.tobytes()


def test_mouse_quirks_and_clamps(tmp_path):
    ses, _, _ = _session(tmp_path)
    ses.mouse_button(V.MOUSE_LEFT, V.PRESS)
    ses.mouse_move(10, 10)
    ses.camchanged = False
    ses.mouse_move(10, 50)              # x unchanged: dropped (main.cpp:230)
    assert not ses.camchanged and (ses.last_x, ses.last_y) == (10, 10)
    ses.mouse_move(11, 100000)          # far up: theta clamped at 0.001 (fmax(0.001f, ...))
    assert ses.theta == F(0.001)
    ses.mouse_move(12, -100000)
    assert ses.theta == V.PI
    ses.mouse_button(V.MOUSE_RIGHT, V.PRESS)   # a press of one button releases the others
    assert ses.right and not ses.left
    ses.mouse_move(13, -200000)
    assert ses.zoom == F(0.1)
    ses.mouse_button(V.MOUSE_RIGHT, V.RELEASE)
    assert not (ses.left or ses.right or ses.middle)


def test_middle_drag_pans_and_space_recentres(tmp_path):
    ses, _, _ = _session(tmp_path)
    ses.run_cuda()
    la0 = ses.look_at.copy()
    ses.mouse_move(50, 50)
    ses.mouse_button(V.MOUSE_MIDDLE, V.PRESS)
    ses.mouse_move(60, 45)
    cam = _cam(ses.scene)
    fwd = cam["view"].copy()
    fwd[1] = 0
    fwd = fwd * (F(1) / np.sqrt(F(np.dot(fwd, fwd))))
    rgt = cam["right"].copy()
    rgt[1] = 0
    rgt = rgt * (F(1) / np.sqrt(F(np.dot(rgt, rgt))))
    want = (la0 - (F(10) * rgt) * F(0.01)) + (F(-5) * fwd) * F(0.01)
    assert np.array_equal(ses.look_at, want)
    ses.run_cuda()
    assert np.array_equal(_cam(ses.scene)["look_at"], want)
    ses.key("SPACE")
    assert ses.camchanged and np.array_equal(ses.look_at, la0)
    ses.run_cuda()
    assert ses.iteration == 1 and np.array_equal(_cam(ses.scene)["look_at"], la0)


def test_panel_settings(tmp_path):
    ses, log, made = _session(tmp_path)
    ses.run_cuda()
    ses.set_setting("sortbyMaterial", True)   # general: applies to the next iteration, no restart
    ses.run_cuda()
    assert ses.iteration == 2 and len(made) == 1 and log[-2][4] is True
    ses.set_setting("aperture", 7.0)          # visual: clamped to the slider, restarts
    assert ses.gui.aperture == 1.0 and ses.visual_changed
    ses.run_cuda()
    assert ses.iteration == 1 and len(made) == 2
    ses.set_setting("SSAA", False)
    ses.run_cuda()
    assert ses.iteration == 1 and log[-2][1] is False
    with pytest.raises(ValueError):
        ses.set_setting("nope", 1)


def test_last_iteration_saves_and_escape_closes(tmp_path):
    ses, _, made = _session(tmp_path, iterations=3)
    for _ in range(3):
        ses.run_cuda()
    assert ses.iteration == 3 and not ses.done
    ses.run_cuda()                       # iteration == iterations: saveImage, pathtraceFree
    assert ses.done and made[0].freed and len(ses.saved) == 1
    assert ses.saved[0].endswith(".3samp.png") and Path(ses.saved[0]).exists()
    ses2, _, _ = _session(tmp_path, iterations=10)
    ses2.run_cuda()
    ses2.key("S")
    ses2.key("ESCAPE")
    assert ses2.should_close and len(ses2.saved) == 2


def test_display_orientation(tmp_path):
    ses, _, _ = _session(tmp_path)
    ses.run_cuda()
    rgb = ses.display_rgb()
    assert rgb.shape == (ses.height, ses.width, 3)
    assert (rgb[:, -1, 1] == 200).all() and (rgb[:, 0, 1] == 0).all()   # x mirrored (preview.cpp:52-57)


def test_png_bytes_decode():
    from PIL import Image
    a = np.random.default_rng(3).integers(0, 256, (37, 53, 3), dtype=np.uint8)
    im = Image.open(io.BytesIO(V.png_bytes(a)))
    assert im.mode == "RGB" and np.array_equal(np.asarray(im), a)


def _get(url):
    with urllib.request.urlopen(url, timeout=10) as r:
        return r.status, r.headers.get("Content-Type"), r.read()


def _post(url, obj):
    req = urllib.request.Request(url, data=json.dumps(obj).encode(), method="POST")
    with urllib.request.urlopen(req, timeout=10) as r:
        return r.status


def test_http_front_end(tmp_path):
    from PIL import Image
    ses, _, _ = _session(tmp_path)
    srv = V.PreviewServer(ses).start(render=False)
    try:
        ses.run_cuda()
        code, ctype, body = _get(srv.url)
        assert code == 200 and "text/html" in ctype and b"Path Tracer Analytics" in body
        st = json.loads(_get(srv.url + "state")[2])
        assert st["iteration"] == 1 and st["title"] == "Path Tracer | 1 Iterations"
        assert st["traced_depth"] == ses.traced_depth and st["settings"]["SSAA"] is True
        png = _get(srv.url + "frame.png?it=1")[2]
        assert np.array_equal(np.asarray(Image.open(io.BytesIO(png))), ses.display_rgb())
        assert _post(srv.url + "event", [{"kind": "move", "x": 5, "y": 5},
                                         {"kind": "button", "button": 1, "action": 1},
                                         {"kind": "move", "x": 6, "y": 30}]) == 200
        assert ses.camchanged and ses.zoom > F(10.5)
        assert _post(srv.url + "event", {"kind": "setting", "name": "DoF", "value": False}) == 200
        assert ses.gui.DoF is False
        ses.run_cuda()
        st = json.loads(_get(srv.url + "state")[2])
        assert st["iteration"] == 1 and st["settings"]["DoF"] is False
        with pytest.raises(urllib.error.HTTPError) as e:
            _post(srv.url + "event", {"kind": "bogus"})
        assert e.value.code == 400
        with pytest.raises(urllib.error.HTTPError) as e:
            _get(srv.url + "nothing")
        assert e.value.code == 404
    finally:
        srv.stop()


def test_render_loop_thread_runs_and_stops(tmp_path):
    ses, log, _ = _session(tmp_path, iterations=4)
    srv = V.PreviewServer(ses).start(render=True)
    try:
        for _ in range(200):
            if ses.done:
                break
            import time
            time.sleep(0.01)
        assert ses.done and ses.iteration == 4 and len(ses.saved) == 1
        assert [e for e in log if e[0] == "pass"] == [("pass", k) for k in range(1, 5)]
    finally:
        srv.stop()

"""Interactive preview: the reference's window (path_tracer/src/preview.cpp, main.cpp) without GL.

The reference shows the running render in a GLFW window (a PBO written by sendImageToPBO,
pathtrace.cu:64-86, blitted as a texture, preview.cpp:289-322), orbits the camera with the mouse
(main.cpp:228-271), takes ESC / S / SPACE (main.cpp:189-213) and draws an ImGui panel of toggles
(preview.cpp:212-282).  A GPU host has no display, so here the window is a web page served from the
render process:

  PreviewSession   main.cpp's state (zoom, theta, phi, look-at, mouse buttons, iteration) and its
                   callbacks, runCuda (main.cpp:114-168) and the panel's settings; the camera
                   recompute is pt_scene_set_orbit, the PBO write is pt_preview_rgba.
  PreviewServer    the window: GET / (page: the image, mouse and keys, the panel), GET /frame.png
                   (the PBO as the window shows it), GET /state (title, panel text, settings),
                   POST /event (GLFW-shaped input events and panel edits).

    python -m cuda_pathtracer_amd.preview SCENE.json [--port 8080]   (then open the printed URL)

Rendering stays on the HIP path (pt_render_pass + pt_preview_rgba on the device); the server only
encodes the latest frame.  Iterations restart at 1 whenever the camera or a visual setting changes,
as in the reference (runCuda: iteration = 0, pathtraceFree + pathtraceInit).
"""
from __future__ import annotations

import argparse
import json
import struct
import threading
import time
import zlib
from collections import deque
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path

import numpy as np

from .pathtrace import GuiDataContainer, PathTracer, Scene, save_image

F32 = np.float32
PI = F32(3.1415926535897932384626422832795028841971)   # utilities.h PI (a float)

# GLFW's codes (glfw3.h): mouse buttons and the key actions main.cpp tests
MOUSE_LEFT, MOUSE_RIGHT, MOUSE_MIDDLE = 0, 1, 2
RELEASE, PRESS = 0, 1
# panel settings that restart the accumulation (preview.cpp:258-271: visual_settings_changed)
VISUAL_SETTINGS = ("SSAA", "DoF", "aperture", "focal_len")
GENERAL_SETTINGS = ("russianRoulette", "sortbyMaterial", "useThrustPartition")
SLIDERS = {"aperture": (0.1, 1.0), "focal_len": (10.0, 80.0)}   # ImGui::SliderFloat ranges


def _normalize(v: np.ndarray) -> np.ndarray:   # glm::normalize: v * inversesqrt(dot(v, v))
    v = v.astype(F32)
    return v * (F32(1.0) / np.sqrt(F32(np.dot(v, v))))


class PreviewSession:
    """main.cpp's interactive state and callbacks for one scene (display-free).

    tracer_factory(scene, gui) -> a PathTracer-like context (pathtraceInit); read_preview(ctx, it)
    -> the (H, W, 4) uint8 PBO contents for `it` accumulated iterations.  The defaults render on the
    current HIP device; tests substitute both to drive the state machine on the CPU."""

    def __init__(self, scene: Scene, gui: GuiDataContainer | None = None, out_dir: str | None = None,
                 tracer_factory=None, read_preview=None):
        self.scene = scene
        cam = scene.camera()
        self.width, self.height = int(cam.res[0]), int(cam.res[1])
        # main.cpp:59-73: the orbit of the loaded camera
        phi, theta, zoom = scene.orbit()
        self.phi, self.theta, self.zoom = F32(phi), F32(theta), F32(zoom)
        self.og_look_at = np.array(cam.look_at[:3], dtype=F32)
        self.look_at = self.og_look_at.copy()
        st = scene.state()
        self.iterations, self.traced_depth, self.image_name = st.iterations, st.traceDepth, st.imageName
        self.gui = gui or GuiDataContainer()
        self.gui.TracedDepth = self.traced_depth   # pathtraceInit's guiData->TracedDepth
        self.out_dir = out_dir
        self.start_time = time.strftime("%Y-%m-%d_%H-%M-%Sz", time.gmtime())   # currentTimeString
        self.camchanged = True
        self.visual_changed = False
        self.left = self.right = self.middle = False
        self.last_x = self.last_y = 0.0
        self.iteration = 0
        self.ctx = None
        self.rgba = np.zeros((self.height, self.width, 4), np.uint8)   # the PBO
        self.done = False            # iterations reached: image saved, context freed (runCuda's exit)
        self.should_close = False    # ESC (glfwSetWindowShouldClose)
        self.saved: list[str] = []
        self._frame_times: deque[float] = deque(maxlen=120)   # ImGui's io.Framerate window
        self._last_frame = None
        self._factory = tracer_factory or (lambda sc, g: PathTracer(sc, g))
        self._read = read_preview or self._device_preview
        self._dbuf = None
        self.lock = threading.RLock()

    # ---- callbacks (main.cpp:189-271) --------------------------------------------------------
    def key(self, key: str) -> None:
        """keyCallback on GLFW_PRESS: ESCAPE saves and closes, S saves, SPACE re-centres the look-at."""
        with self.lock:
            k = key.upper()
            if k in ("ESCAPE", "ESC"):
                self.save_image()
                self.should_close = True
            elif k == "S":
                self.save_image()
            elif k in ("SPACE", " "):
                self.camchanged = True
                self.look_at = self.og_look_at.copy()

    def mouse_button(self, button: int, action: int) -> None:
        """mouseButtonCallback: each event sets all three button states (a press of one releases
        the others, any release clears them)."""
        with self.lock:
            self.left = button == MOUSE_LEFT and action == PRESS
            self.right = button == MOUSE_RIGHT and action == PRESS
            self.middle = button == MOUSE_MIDDLE and action == PRESS

    def mouse_move(self, x: float, y: float) -> None:
        """mousePositionCallback: orbit (left), zoom (right), pan the look-at (middle)."""
        with self.lock:
            x, y = float(x), float(y)
            if x == self.last_x or y == self.last_y:
                return   # main.cpp:230 (either coordinate unchanged: the event is dropped)
            if self.left:
                self.phi = F32(float(self.phi) - (x - self.last_x) / self.width)
                self.theta = F32(float(self.theta) - (y - self.last_y) / self.height)
                self.theta = max(F32(0.001), min(self.theta, PI))
                self.camchanged = True
            elif self.right:
                self.zoom = F32(float(self.zoom) + (y - self.last_y) / self.height)
                self.zoom = max(F32(0.1), self.zoom)
                self.camchanged = True
            elif self.middle:
                cam = self.scene.camera()
                fwd = np.array(cam.view[:3], dtype=F32)
                fwd[1] = 0
                fwd = _normalize(fwd)
                rgt = np.array(cam.right[:3], dtype=F32)
                rgt[1] = 0
                rgt = _normalize(rgt)
                self.look_at = self.look_at - (F32(x - self.last_x) * rgt) * F32(0.01)
                self.look_at = self.look_at + (F32(y - self.last_y) * fwd) * F32(0.01)
                self.camchanged = True
            self.last_x, self.last_y = x, y

    def set_setting(self, name: str, value) -> None:
        """An edit in the panel (preview.cpp:243-271).  The general settings apply to the next
        iteration; the visual ones restart the accumulation (visual_settings_changed)."""
        with self.lock:
            if name in GENERAL_SETTINGS or name in ("SSAA", "DoF"):
                setattr(self.gui, name, bool(value))
            elif name in SLIDERS:
                lo, hi = SLIDERS[name]
                setattr(self.gui, name, float(min(max(float(value), lo), hi)))
            else:
                raise ValueError(f"unknown setting {name!r}")
            if name in VISUAL_SETTINGS:
                self.visual_changed = True

    # ---- runCuda (main.cpp:114-168) -----------------------------------------------------------
    def run_cuda(self) -> None:
        with self.lock:
            if self.done:
                return
            t0 = time.perf_counter()
            if self.camchanged or self.visual_changed:
                self.iteration = 0
                self.scene.set_orbit(float(self.phi), float(self.theta), float(self.zoom), self.look_at)
                self.camchanged = False
                self.visual_changed = False
            if self.iteration == 0:   # pathtraceFree + pathtraceInit
                self._free()
                self.ctx = self._factory(self.scene, self.gui)
            if self.iteration < self.iterations:
                self.iteration += 1
                # pathtrace(pbo, frame, iteration): InitDataContainer's flags, one iteration, the PBO
                self.ctx.set_flags(self.gui)
                self.ctx.render_pass(self.iteration)
                self.rgba = self._read(self.ctx, self.iteration)
            else:
                self.save_image()
                self._free()
                self.done = True
            now = time.perf_counter()
            self._frame_times.append(now - (self._last_frame if self._last_frame is not None else t0))
            self._last_frame = now

    def _device_preview(self, ctx, it: int) -> np.ndarray:
        import torch
        if self._dbuf is None:
            self._dbuf = torch.empty((self.height, self.width, 4), dtype=torch.uint8, device="cuda")
        ctx.preview_rgba(it, self._dbuf.data_ptr())   # (the render's stream: NULL)
        return self._dbuf.cpu().numpy()

    def _free(self) -> None:
        if self.ctx is not None:
            if hasattr(self.ctx, "free"):
                self.ctx.free()
            self.ctx = None

    def save_image(self) -> str | None:
        """saveImage (main.cpp:88-112): the accumulator / iterations as imageName.<start>.<N>samp.png."""
        with self.lock:
            if self.ctx is None or self.iteration == 0 or self.out_dir is None:
                return None
            name = f"{self.image_name}.{self.start_time}.{self.iteration}samp.png"
            path = save_image(str(Path(self.out_dir) / name), self.ctx.image(), float(self.iteration))
            self.saved.append(path)
            return path

    def close(self) -> None:
        with self.lock:
            self._free()
            self._dbuf = None

    # ---- what the window shows ----------------------------------------------------------------
    def title(self) -> str:   # preview.cpp:297
        return f"Path Tracer | {self.iteration} Iterations"

    def display_rgb(self) -> np.ndarray:
        """The window's pixels: the PBO through the quad's texture coordinates (preview.cpp:43-68:
        u = 1 at the left edge, v = 0 at the top), i.e. x mirrored, rows top-down."""
        with self.lock:
            return np.ascontiguousarray(self.rgba[:, ::-1, :3])

    def state(self) -> dict:
        with self.lock:
            ft = sum(self._frame_times) / len(self._frame_times) if self._frame_times else 0.0
            cam = self.scene.camera()
            return {
                "title": self.title(), "iteration": self.iteration, "iterations": self.iterations,
                "done": self.done, "closed": self.should_close,
                "traced_depth": self.traced_depth,   # "Traced Depth %d"
                "ms_per_frame": ft * 1e3, "fps": (1.0 / ft) if ft > 0 else 0.0,
                "settings": {k: getattr(self.gui, k) for k in GENERAL_SETTINGS + VISUAL_SETTINGS},
                "camera": {"phi": float(self.phi), "theta": float(self.theta), "zoom": float(self.zoom),
                           "look_at": [float(v) for v in self.look_at],
                           "position": [float(v) for v in cam.position[:3]]},
                "size": [self.width, self.height], "saved": list(self.saved),
            }

    def handle_event(self, ev: dict) -> None:
        kind = ev.get("kind")
        if kind == "button":
            self.mouse_button(int(ev["button"]), int(ev["action"]))
        elif kind == "move":
            self.mouse_move(float(ev["x"]), float(ev["y"]))
        elif kind == "key":
            self.key(str(ev["key"]))
        elif kind == "setting":
            self.set_setting(str(ev["name"]), ev["value"])
        else:
            raise ValueError(f"unknown event kind {kind!r}")


def png_bytes(rgb: np.ndarray) -> bytes:
    """8-bit RGB PNG of an (H, W, 3) uint8 array (filter 0 rows, zlib level 1)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w = rgb.shape[:2]
    raw = np.concatenate([np.zeros((h, 1), np.uint8), rgb.reshape(h, w * 3)], axis=1).tobytes()

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
            + chunk(b"IDAT", zlib.compress(raw, 1)) + chunk(b"IEND", b""))


_PAGE = """<!doctype html><html><head><meta charset="utf-8"><title>Path Tracer</title>
<style>body{font:13px sans-serif;background:#222;color:#ddd;display:flex;gap:16px;margin:12px}
#img{image-rendering:pixelated;cursor:crosshair;user-select:none}
fieldset{border:1px solid #555;margin:0 0 8px 0} input[type=range]{width:160px}</style></head><body>
<img id="img" src="/frame.png" draggable="false" tabindex="0">
<div><div id="title"></div><fieldset><legend>Path Tracer Analytics</legend>
<div id="depth"></div><div id="rate"></div></fieldset>
<fieldset><legend>General settings</legend>
<label><input type="checkbox" id="russianRoulette"> Russian roulette</label><br>
<label><input type="checkbox" id="sortbyMaterial"> Sort by material (can harm performance)</label><br>
<label><input type="checkbox" id="useThrustPartition"> Use thrust library for path termination</label></fieldset>
<fieldset><legend>Visual settings</legend>
<label><input type="checkbox" id="SSAA"> Enable stochastic sampled antialiasing</label><br>
<label><input type="checkbox" id="DoF"> Enable DoF effects</label><br>
<label>Aperture radius <input type="range" id="aperture" min="0.1" max="1" step="0.01"></label><br>
<label>Focal distance <input type="range" id="focal_len" min="10" max="80" step="0.1"></label></fieldset>
<div>Left drag: orbit; right drag: zoom; middle drag: pan; S: save; Space: re-centre; Esc: save and quit</div>
</div><script>
const img=document.getElementById('img');let shown=-1;
function post(ev){fetch('/event',{method:'POST',body:JSON.stringify(ev)});}
function pos(e){const r=img.getBoundingClientRect();return{x:(e.clientX-r.left)*img.naturalWidth/r.width,
 y:(e.clientY-r.top)*img.naturalHeight/r.height};}
const btn={0:0,1:2,2:1};  // DOM -> GLFW (left, right, middle)
img.addEventListener('mousedown',e=>{e.preventDefault();img.focus();post({kind:'button',button:btn[e.button],action:1});});
window.addEventListener('mouseup',e=>post({kind:'button',button:btn[e.button],action:0}));
img.addEventListener('mousemove',e=>{const p=pos(e);post({kind:'move',x:p.x,y:p.y});});
img.addEventListener('contextmenu',e=>e.preventDefault());
window.addEventListener('keydown',e=>{const k=e.key==='Escape'?'ESCAPE':e.key===' '?'SPACE':e.key.toUpperCase();
 if(['ESCAPE','SPACE','S'].includes(k)){e.preventDefault();post({kind:'key',key:k});}});
for(const id of ['russianRoulette','sortbyMaterial','useThrustPartition','SSAA','DoF'])
 document.getElementById(id).addEventListener('change',e=>post({kind:'setting',name:id,value:e.target.checked}));
for(const id of ['aperture','focal_len'])
 document.getElementById(id).addEventListener('input',e=>post({kind:'setting',name:id,value:parseFloat(e.target.value)}));
async function poll(){try{const s=await (await fetch('/state')).json();
 document.getElementById('title').textContent=s.title;document.title=s.title;
 document.getElementById('depth').textContent='Traced Depth '+s.traced_depth;
 document.getElementById('rate').textContent='Application average '+s.ms_per_frame.toFixed(3)+' ms/frame ('+s.fps.toFixed(1)+' FPS)';
 for(const [k,v] of Object.entries(s.settings)){const el=document.getElementById(k);if(!el||el===document.activeElement)continue;
  if(el.type==='checkbox')el.checked=v;else el.value=v;}
 for(const id of ['aperture','focal_len'])document.getElementById(id).disabled=!s.settings.DoF;
 if(s.iteration!==shown){shown=s.iteration;img.src='/frame.png?it='+s.iteration+'&t='+Date.now();}
 if(s.closed){document.getElementById('title').textContent+=' (closed)';return;}}catch(e){}
 setTimeout(poll,100);}
poll();</script></body></html>"""


class PreviewServer:
    """The window: a render loop thread (preview.cpp:289-322's mainLoop) and an HTTP server."""

    def __init__(self, session: PreviewSession, host: str = "127.0.0.1", port: int = 0):
        self.session = session
        self._stop = threading.Event()
        self._png = (-1, b"")   # (iteration, bytes) of the last encoded frame
        srv = self

        class Handler(BaseHTTPRequestHandler):
            def log_message(self, *a):   # quiet
                pass

            def _send(self, code: int, body: bytes, ctype: str) -> None:
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(body)))
                self.send_header("Cache-Control", "no-store")
                self.end_headers()
                self.wfile.write(body)

            def do_GET(self):  # noqa: N802
                path = self.path.split("?", 1)[0]
                if path == "/":
                    self._send(200, _PAGE.encode(), "text/html; charset=utf-8")
                elif path == "/frame.png":
                    self._send(200, srv.frame_png(), "image/png")
                elif path == "/state":
                    self._send(200, json.dumps(srv.session.state()).encode(), "application/json")
                else:
                    self._send(404, b"not found", "text/plain")

            def do_POST(self):  # noqa: N802
                if self.path.split("?", 1)[0] != "/event":
                    self._send(404, b"not found", "text/plain")
                    return
                n = int(self.headers.get("Content-Length") or 0)
                try:
                    evs = json.loads(self.rfile.read(n) or b"[]")
                    for ev in evs if isinstance(evs, list) else [evs]:
                        srv.session.handle_event(ev)
                except (ValueError, KeyError, TypeError) as e:
                    self._send(400, str(e).encode(), "text/plain")
                    return
                self._send(200, b"{}", "application/json")

        self.httpd = ThreadingHTTPServer((host, port), Handler)
        self.httpd.daemon_threads = True
        self.url = f"http://{host}:{self.httpd.server_address[1]}/"
        self._threads: list[threading.Thread] = []
        self.error: BaseException | None = None

    def frame_png(self) -> bytes:
        s = self.session
        with s.lock:
            it = s.iteration
            if self._png[0] != it:
                self._png = (it, png_bytes(s.display_rgb()))
            return self._png[1]

    def _loop(self) -> None:
        try:
            while not self._stop.is_set() and not self.session.should_close:
                if self.session.done:
                    time.sleep(0.05)
                    continue
                self.session.run_cuda()
        except BaseException as e:   # surfaced by stop() / the CLI
            self.error = e
        finally:
            self.session.close()

    def start(self, render: bool = True) -> "PreviewServer":
        t = threading.Thread(target=self.httpd.serve_forever, name="preview-http", daemon=True)
        t.start()
        self._threads.append(t)
        if render:
            r = threading.Thread(target=self._loop, name="preview-render", daemon=True)
            r.start()
            self._threads.append(r)
        return self

    def stop(self) -> None:
        self._stop.set()
        self.httpd.shutdown()
        self.httpd.server_close()
        for t in self._threads:
            t.join(timeout=30)
        if self.error is not None:
            raise self.error

    def wait(self) -> None:
        """Block until ESC (should_close) or KeyboardInterrupt."""
        try:
            while not self.session.should_close and self.error is None:
                time.sleep(0.1)
        except KeyboardInterrupt:
            pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Interactive preview of a scene (the reference's window, served as a web page)")
    ap.add_argument("scene")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--out-dir", default=".", help="where S / ESC / the last iteration save the PNG")
    a = ap.parse_args(argv)
    scene = Scene(a.scene)
    print(f"Reading scene from {a.scene} ...", flush=True)
    srv = PreviewServer(PreviewSession(scene, out_dir=a.out_dir), a.host, a.port).start()
    print(f"preview at {srv.url}  (Esc in the page saves and quits)", flush=True)
    srv.wait()
    srv.stop()
    for p in srv.session.saved:
        print(f"Saved {p}.")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

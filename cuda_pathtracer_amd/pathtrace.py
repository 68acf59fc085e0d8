"""Python mirror of the reference's render boundary, backed by libpt_amd.so.

Reference interfaces (path_tracer/src):
  Scene::Scene(filename) / loadFromJSON           scene.h:17-35, scene.cpp:16-219   -> Scene(path)
  GuiDataContainer (runtime flags)                utilities.h:17-34                 -> GuiDataContainer
  InitDataContainer / pathtraceInit / pathtraceFree / pathtrace   pathtrace.h:6-9   -> same names
  runCuda's iteration loop + saveImage            main.cpp:88-168                   -> render(), save_image()
The reference keeps one implicit global render (file-static device buffers); the module-level
functions below reproduce that, while PathTracer objects allow any number of independent
contexts (one per GPU / pixel tile).
"""
from __future__ import annotations

import ctypes as C
import os
import time
from dataclasses import dataclass
from pathlib import Path

import numpy as np

from . import _native as N
from ._native import check_pt, lib

SPHERE, CUBE, MESH = 0, 1, 2


class GuiDataContainer:
    """Runtime flags with the reference defaults (utilities.h:17-34)."""

    def __init__(self):
        self.TracedDepth = 0
        self.russianRoulette = True
        self.useBVHtree = True
        self.useBBox = True
        self.sortbyMaterial = False
        self.useThrustPartition = False
        self.SSAA = True
        self.DoF = True
        self.aperture = 0.1
        self.focal_len = 10.0
        # extension, off = the reference: albedo applied once instead of twice (include/pt_amd.h)
        self.singleAlbedo = False
        # extension, off = the reference: cull BVH nodes beyond the closest hit so far
        self.bvhCull = False
        # tile schedule of the look-back kernels: False = static grid (fastest), True = claimed
        # tiles (other kernels / processes share the GPU); default from PT_AMD_SCHEDULE=claim
        self.sharedGPU = os.environ.get("PT_AMD_SCHEDULE", "") == "claim"
        # extension, off = the reference: shading RNG keyed by the global pixel, so the image does
        # not depend on the shard layout or the material sort (bitwise equal across GPU counts)
        self.rngKeyPixel = False

    def to_c(self) -> N.Flags:
        f = N.Flags()
        f.russian_roulette = int(bool(self.russianRoulette))
        f.use_bvh = int(bool(self.useBVHtree))
        f.use_bbox = int(bool(self.useBBox))
        f.sort_by_material = int(bool(self.sortbyMaterial))
        f.use_thrust_partition = int(bool(self.useThrustPartition))
        f.ssaa = int(bool(self.SSAA))
        f.dof = int(bool(self.DoF))
        f.aperture = float(self.aperture)
        f.focal_dist = float(self.focal_len)
        f.single_albedo = int(bool(self.singleAlbedo))
        f.bvh_cull = int(bool(self.bvhCull))
        f.shared_gpu = int(bool(self.sharedGPU))
        f.rng_key_pixel = int(bool(self.rngKeyPixel))
        return f


@dataclass
class RenderState:
    iterations: int
    traceDepth: int
    imageName: str


def decode_jpeg(data: bytes) -> np.ndarray:
    """Texture::load's stbi_load(file, &w, &h, &comp, 0) (sceneStructs.h:171-175) for JPEG bytes,
    by the native decoder (pt_decode_jpeg): an (h, w, components) uint8 array."""
    L = lib()
    w, h, c = C.c_int32(), C.c_int32(), C.c_int32()
    check_pt(L.pt_decode_jpeg(data, len(data), C.byref(w), C.byref(h), C.byref(c), None, 0))
    out = np.empty((h.value, w.value, c.value), np.uint8)
    check_pt(L.pt_decode_jpeg(data, len(data), C.byref(w), C.byref(h), C.byref(c),
                              out.ctypes.data_as(C.c_void_p), out.size))
    return out


class Scene:
    """Scene description; `Scene(path)` loads a reference JSON scene file (textures decoded
    natively, pt_decode_jpeg).  refraction=True reads the REFRACTIVE / IOR material keys the
    reference loader ignores (PT_LOAD_REFRACTION; a file may also opt in with
    "Extensions": {"REFRACTION": true}); by default they are ignored, like scene.cpp:46-56."""

    def __init__(self, filename: str | os.PathLike | None = None, refraction: bool = False,
                 device_bvh: bool = False):
        """device_bvh=True builds the BVH on the current HIP device (pt_scene_set_bvh_builder: the
        same tree as the host build, byte for byte)."""
        self._h = C.c_void_p()
        L = lib()
        if filename is None:
            check_pt(L.pt_scene_create(C.byref(self._h)))
            if device_bvh:
                check_pt(L.pt_scene_set_bvh_builder(self._h, 1))
            return
        opts = (1 if refraction else 0) | (2 if device_bvh else 0)
        check_pt(L.pt_scene_load_json_ex(str(filename).encode(), opts, C.byref(self._h)))
        self._fill_non_jpeg_textures()

    def set_bvh_builder(self, device: bool) -> None:
        check_pt(lib().pt_scene_set_bvh_builder(self._h, 1 if device else 0))

    def bvh_build_info(self) -> tuple[bool, float]:
        """(the last BVH build ran on the device, its wall time in ms)."""
        d, ms = C.c_int32(), C.c_double()
        check_pt(lib().pt_scene_bvh_build_info(self._h, C.byref(d), C.byref(ms)))
        return bool(d.value), float(ms.value)

    def texture_path(self, tid: int) -> str:
        buf = C.create_string_buffer(4096)
        check_pt(lib().pt_scene_texture_path(self._h, int(tid), buf, 4096))
        return buf.value.decode()

    def _fill_non_jpeg_textures(self) -> None:
        """Texture files that are not JPEG (PNG, BMP, TGA: stbi_load reads them too) are left
        undecoded by the native loader (include/pt_amd.h); decode them here.  These formats are
        lossless, so a decoder yields stbi_load(path, &w, &h, &comp, 0)'s texels once the modes are
        mapped as stb maps them: palette images expand to RGB, or RGBA with a tRNS chunk; a tRNS chunk
        adds an alpha channel to grey and RGB images too; 16-bit samples keep their high byte; 1-bit
        grey expands to 0/255.  A mode stb would not produce raises instead of converting silently
        (non-JPEG texels are parity-unpinned: no reference fixture covers them)."""
        ntex = self.counts()[4]
        for tid in range(ntex):
            path = self.texture_path(tid)
            with open(path, "rb") as f:
                head = f.read(2)
            if head == b"\xff\xd8":
                continue
            from PIL import Image   # (host-side file IO only; not on the render path)
            with Image.open(path) as im:
                px = _stb_texels(im, path)
            h, w = px.shape[:2]
            comps = 1 if px.ndim == 2 else px.shape[2]
            check_pt(lib().pt_scene_set_texture_pixels(self._h, tid, w, h, comps, px.ctypes.data_as(C.c_void_p)))

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().pt_scene_free(h)
            except Exception:
                pass
            self._h = None

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    # -- programmatic construction --
    def add_material(self, rgb=(0, 0, 0), specrgb=None, specex=1.0, reflective=0.0, refractive=0.0, ior=0.0,
                     emittance=0.0, texture_id=-1) -> int:
        m = N.Material()
        m.color[:] = [float(v) for v in rgb]
        m.spec_color[:] = [float(v) for v in (specrgb if specrgb is not None else rgb)]
        m.spec_exponent = specex
        m.has_reflective = reflective
        m.has_refractive = refractive
        m.ior = ior
        m.emittance = emittance
        m.texture_id = texture_id
        out = C.c_int32()
        check_pt(lib().pt_scene_add_material(self._h, C.byref(m), C.byref(out)))
        return out.value

    def add_geom(self, type_: int, material: int, trans, rotat, scale) -> int:
        out = C.c_int32()
        check_pt(lib().pt_scene_add_geom(self._h, type_, material, N.f3(trans), N.f3(rotat), N.f3(scale),
                                         C.byref(out)))
        return out.value

    def set_camera(self, res, fovy, eye, lookat, up=(0, 1, 0)) -> None:
        check_pt(lib().pt_scene_set_camera(self._h, int(res[0]), int(res[1]), float(fovy), N.f3(eye), N.f3(lookat),
                                           N.f3(up)))

    def set_render(self, iterations: int, depth: int, file: str = "render") -> None:
        check_pt(lib().pt_scene_set_render(self._h, iterations, depth, file.encode()))

    def finalize(self) -> None:
        check_pt(lib().pt_scene_finalize(self._h))

    # -- inspection --
    def counts(self):
        v = [C.c_int32() for _ in range(5)]
        check_pt(lib().pt_scene_counts(self._h, *[C.byref(x) for x in v]))
        return tuple(x.value for x in v)

    def camera(self) -> N.Camera:
        cam = N.Camera()
        check_pt(lib().pt_scene_get_camera(self._h, C.byref(cam)))
        return cam

    def orbit(self) -> tuple[float, float, float]:
        """(phi, theta, zoom) of the loaded camera, as main.cpp:59-73 derives them."""
        p, t, z = C.c_float(), C.c_float(), C.c_float()
        check_pt(lib().pt_scene_get_orbit(self._h, C.byref(p), C.byref(t), C.byref(z)))
        return p.value, t.value, z.value

    def set_orbit(self, phi: float, theta: float, zoom: float, look_at) -> None:
        """runCuda's camera recompute (main.cpp:117-136) for an orbit about look_at; contexts created
        afterwards render it."""
        check_pt(lib().pt_scene_set_orbit(self._h, float(phi), float(theta), float(zoom), N.f3(look_at)))

    def state(self) -> RenderState:
        it, d = C.c_int32(), C.c_int32()
        buf = C.create_string_buffer(1024)
        check_pt(lib().pt_scene_get_render(self._h, C.byref(it), C.byref(d), buf, 1024))
        return RenderState(it.value, d.value, buf.value.decode())

    def geoms(self):
        ng = self.counts()[0]
        arr = (N.Geom * max(ng, 1))()
        lib().pt_scene_get_geoms(self._h, arr, ng)
        return list(arr)[:ng]

    def materials(self):
        nm = self.counts()[1]
        arr = (N.Material * max(nm, 1))()
        lib().pt_scene_get_materials(self._h, arr, nm)
        return list(arr)[:nm]


def _stream_ptr(stream):
    if stream is None:
        return None
    return int(getattr(stream, "cuda_stream", stream))


def _stb_texels(im, path) -> np.ndarray:
    """PIL image -> the (h, w[, c]) uint8 texels stbi_load(..., 0) returns for the same file."""
    trans = "transparency" in im.info
    mode = im.mode
    if mode == "P":
        return np.ascontiguousarray(np.asarray(im.convert("RGBA" if trans else "RGB"), dtype=np.uint8))
    if mode == "1":
        im, mode = im.convert("L"), "L"
    if mode in ("I;16", "I;16B", "I;16L", "I"):   # 16-bit grey: stb keeps the high byte
        g = (np.asarray(im).astype(np.uint32) >> 8).astype(np.uint8)
        if trans:   # tRNS on grey: stb adds an alpha channel (opaque except the keyed value)
            key = int(im.info["transparency"])
            a = np.where(np.asarray(im).astype(np.uint32) == key, 0, 255).astype(np.uint8)
            return np.ascontiguousarray(np.stack([g, a], axis=-1))
        return np.ascontiguousarray(g)
    if mode == "L" and trans:
        return np.ascontiguousarray(np.asarray(im.convert("LA"), dtype=np.uint8))
    if mode == "RGB" and trans:
        return np.ascontiguousarray(np.asarray(im.convert("RGBA"), dtype=np.uint8))
    if mode in ("L", "LA", "RGB", "RGBA"):
        return np.ascontiguousarray(np.asarray(im, dtype=np.uint8))
    raise ValueError(f"texture {path}: image mode {mode!r} has no stbi_load equivalent here")


class PathTracer:
    """One render context (pathtraceInit ... pathtraceFree) for a pixel tile of the image.

    rank/world select the rows y % world == rank; spp iterations are traced per pass.
    """

    def __init__(self, scene: Scene, gui: GuiDataContainer | None = None, rank: int = 0, world: int = 1,
                 spp: int = 1):
        self.scene = scene
        self.gui = gui or GuiDataContainer()
        self._h = C.c_void_p()
        flags = self.gui.to_c()
        shard = N.Shard(rank, world, spp, 0)
        check_pt(lib().pt_create(scene.handle, C.byref(flags), C.byref(shard), C.byref(self._h)))
        w, rows, npix, npaths = (C.c_int32() for _ in range(4))
        check_pt(lib().pt_tile_info(self._h, C.byref(w), C.byref(rows), C.byref(npix), C.byref(npaths)))
        self.width, self.rows, self.npix, self.npaths = w.value, rows.value, npix.value, npaths.value
        self.rank, self.world, self.spp = rank, world, spp

    def free(self) -> None:
        if self._h is not None and self._h.value:
            check_pt(lib().pt_destroy(self._h))
        self._h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass

    def set_flags(self, gui: GuiDataContainer) -> None:
        self.gui = gui
        check_pt(lib().pt_set_flags(self._h, C.byref(gui.to_c())))

    def counters(self) -> dict:
        """Host-side counters (pt_ctx_counters): camera-mask builds and device-synchronising
        pt_set_flags calls."""
        b, y = C.c_uint64(), C.c_uint64()
        check_pt(lib().pt_ctx_counters(self._h, C.byref(b), C.byref(y)))
        return {"mask_builds": int(b.value), "flag_syncs": int(y.value)}

    def stream_info(self) -> dict:
        """Stream budget (pt_ctx_stream_info): the context's lanes and busy streams, the busy streams
        of every live context of the process, the hardware queues per priority, and whether pt_create
        capped the lanes to stay within them."""
        v = [C.c_int32() for _ in range(5)]
        check_pt(lib().pt_ctx_stream_info(self._h, *[C.byref(x) for x in v]))
        k = ("lanes", "busy_streams", "process_busy", "hw_queues", "lanes_capped")
        return {a: int(x.value) for a, x in zip(k, v)}

    def cmask_info(self) -> dict:
        """First-bounce camera masks (pt_ctx_cmask_info): built, share of empty 64-pixel blocks, and
        whether the fused first bounce skips those waves in its own instantiation."""
        on, sk, fr = C.c_int32(), C.c_int32(), C.c_double()
        check_pt(lib().pt_ctx_cmask_info(self._h, C.byref(on), C.byref(fr), C.byref(sk)))
        return {"on": bool(on.value), "empty_frac": float(fr.value), "skip_fused": bool(sk.value)}

    def walk_info(self) -> dict:
        """Mesh scenes: 4-wide walk on/off, its exact t-cull on/off and the share of slots whose
        cull margin can pay (pt_ctx_walk_info)."""
        qw, on, fr = C.c_int32(), C.c_int32(), C.c_double()
        check_pt(lib().pt_ctx_walk_info(self._h, C.byref(qw), C.byref(on), C.byref(fr)))
        return {"quad_walk": bool(qw.value), "tcull": bool(on.value), "tcull_frac": float(fr.value)}

    def render_pass(self, iter_first: int, stream=None) -> None:
        """pathtrace(): iterations [iter_first, iter_first + spp) for this tile, asynchronous."""
        check_pt(lib().pt_render_pass(self._h, int(iter_first), _stream_ptr(stream)))

    def render_ahead(self, iteration: int, stream=None) -> None:
        """One-iteration contexts: queue iteration `iteration`'s bounces now (pt_render_ahead); the
        render_pass(iteration) that follows with the same flags only adds their colours."""
        check_pt(lib().pt_render_ahead(self._h, int(iteration), _stream_ptr(stream)))

    def image(self) -> np.ndarray:
        """Tile accumulator (sum of radiance over iterations), shape (rows, width, 3) float32."""
        out = np.empty((self.rows, self.width, 3), dtype=np.float32)
        check_pt(lib().pt_get_image(self._h, out.ctypes.data))
        return out

    def set_image(self, image: np.ndarray) -> None:
        """Resume: load a tile accumulator saved from image() (pt_set_accum)."""
        img = np.ascontiguousarray(image, dtype=np.float32)
        if img.shape != (self.rows, self.width, 3):
            raise ValueError(f"accumulator shape {img.shape} != {(self.rows, self.width, 3)}")
        check_pt(lib().pt_set_accum(self._h, img.ctypes.data))

    def save_state(self, path: str, iterations_done: int) -> str:
        """Checkpoint the accumulator and the next iteration index (extension: resume a render)."""
        np.savez(path, image=self.image(), iterations_done=np.int64(iterations_done),
                 rank=np.int32(self.rank), world=np.int32(self.world))
        return str(path)

    def load_state(self, path: str) -> int:
        """Load a checkpoint written by save_state for the same tile; returns iterations_done."""
        with np.load(path, allow_pickle=False) as z:
            if int(z["rank"]) != self.rank or int(z["world"]) != self.world:
                raise ValueError("checkpoint is for another tile")
            self.set_image(z["image"])
            return int(z["iterations_done"])

    def copy_image_to(self, dst_ptr: int, stream=None) -> None:
        check_pt(lib().pt_copy_image(self._h, C.c_void_p(dst_ptr), _stream_ptr(stream)))

    def reset_image(self, stream=None) -> None:
        check_pt(lib().pt_reset_image(self._h, _stream_ptr(stream)))

    def preview_rgba(self, iteration: int, dst_ptr: int, stream=None) -> None:
        check_pt(lib().pt_preview_rgba(self._h, int(iteration), C.c_void_p(dst_ptr), _stream_ptr(stream)))

    def stats(self) -> dict:
        s = N.Stats()
        check_pt(lib().pt_stats(self._h, C.byref(s)))
        depth = self.scene.state().traceDepth
        return {"segments": int(s.segments), "passes": int(s.passes),
                "bounce_live": [int(s.bounce_live[k]) for k in range(depth)],
                "bounce_emit": [int(s.bounce_emit[k]) for k in range(depth)],
                "emissive_hits": int(s.emissive_hits), "bound_mismatch": int(s.bound_mismatch),
                "device_error": int(s.device_error)}

    def profile(self, on: bool = True) -> None:
        check_pt(lib().pt_profile_enable(self._h, int(on)))

    # PT_KIND_* of include/pt_amd.h, in order
    KINDS = ("first_bounce", "bounce", "compact", "sort", "traverse", "first_traverse")

    def profile_read(self) -> dict:
        """{kind: (summed ms, launches, busy ms)} since the previous read (HIP events on the launch
        streams); busy ms = the union of the kind's launch intervals (lanes overlap launches)."""
        k = len(self.KINDS)
        ms = (C.c_double * k)()
        busy = (C.c_double * k)()
        n = (C.c_uint64 * k)()
        check_pt(lib().pt_profile_read_kinds(self._h, k, ms, busy, n))
        return {name: (float(ms[i]), int(n[i]), float(busy[i])) for i, name in enumerate(self.KINDS)}


def tonemap(image: np.ndarray, samples: float) -> np.ndarray:
    """saveImage + Image::savePNG pixel math (x-mirrored, clamp, x255, truncation) -> (H, W, 3) uint8."""
    img = np.ascontiguousarray(image, dtype=np.float32)
    H, W = img.shape[0], img.shape[1]
    out = np.empty((H, W, 3), dtype=np.uint8)
    check_pt(lib().pt_tonemap(img.ctypes.data, W, H, float(samples), out.ctypes.data))
    return out


def save_image(path: str, image: np.ndarray, samples: float) -> str:
    img = np.ascontiguousarray(image, dtype=np.float32)
    check_pt(lib().pt_save_png(str(path).encode(), img.ctypes.data, img.shape[1], img.shape[0], float(samples)))
    return str(path)


def encode_hdr(image: np.ndarray, samples: float) -> bytes:
    """Image::saveHDR file bytes (Radiance RGBE, stb_image_write's run-length coding)."""
    img = np.ascontiguousarray(image, dtype=np.float32)
    n = C.c_int64(0)
    check_pt(lib().pt_encode_hdr(img.ctypes.data, img.shape[1], img.shape[0], float(samples), None, 0, C.byref(n)))
    buf = (C.c_uint8 * n.value)()
    check_pt(lib().pt_encode_hdr(img.ctypes.data, img.shape[1], img.shape[0], float(samples), buf, n.value,
                                 C.byref(n)))
    return bytes(buf)


def save_image_hdr(path: str, image: np.ndarray, samples: float) -> str:
    img = np.ascontiguousarray(image, dtype=np.float32)
    check_pt(lib().pt_save_hdr(str(path).encode(), img.ctypes.data, img.shape[1], img.shape[0], float(samples)))
    return str(path)


def render(scene_path: str, iterations: int | None = None, out_dir: str | None = None,
           gui: GuiDataContainer | None = None) -> tuple[np.ndarray, str | None]:
    """Headless runCuda loop (main.cpp:114-168): ITERATIONS passes, then saveImage."""
    scene = Scene(scene_path)
    st = scene.state()
    iters = iterations if iterations is not None else st.iterations
    pt = PathTracer(scene, gui)
    for it in range(1, iters + 1):
        pt.render_pass(it)
    img = pt.image()
    path = None
    if out_dir is not None:
        stamp = time.strftime("%Y-%m-%d_%H-%M-%Sz", time.gmtime())
        path = str(Path(out_dir) / f"{st.imageName}.{stamp}.{iters}samp.png")
        save_image(path, img, iters)
    pt.free()
    return img, path


# ---- the reference's global-state API (pathtrace.h:6-9) ------------------------------------
_GLOBAL: dict = {"gui": None, "ctx": None}


def InitDataContainer(gui: GuiDataContainer) -> None:  # noqa: N802
    _GLOBAL["gui"] = gui
    if _GLOBAL["ctx"] is not None:
        _GLOBAL["ctx"].set_flags(gui)


def pathtraceInit(scene: Scene) -> None:  # noqa: N802
    pathtraceFree()
    _GLOBAL["ctx"] = PathTracer(scene, _GLOBAL["gui"])


def pathtraceFree() -> None:  # noqa: N802
    if _GLOBAL["ctx"] is not None:
        _GLOBAL["ctx"].free()
    _GLOBAL["ctx"] = None


def pathtrace(pbo_ptr: int | None, frame: int, iteration: int) -> None:
    """One iteration; writes the RGBA preview into pbo_ptr (device) when given."""
    ctx = _GLOBAL["ctx"]
    if ctx is None:
        raise RuntimeError("pathtraceInit() was not called")
    if _GLOBAL["gui"] is not None:
        ctx.set_flags(_GLOBAL["gui"])
    ctx.render_pass(iteration)
    if pbo_ptr:
        ctx.preview_rgba(iteration, pbo_ptr)

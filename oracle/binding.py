"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/build/liboracle.so (the serial CPU restatement of the reference in
oracle/sc_oracle.cpp and oracle/pt_oracle.cpp).  Only tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py may import this module, and only as the checker; the product
package (cuda_pathtracer_amd) never imports, loads or calls it.

Also restates scene.cpp:33-219's JSON handling in Python (key defaults, alphabetical material
ids, object order) so scene parity is checked against an independent parse.
"""
from __future__ import annotations

import ctypes as C
import json
import subprocess
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
LIB = ORACLE_DIR / "build" / "liboracle.so"


class OGeom(C.Structure):
    _fields_ = [("type", C.c_int32), ("materialid", C.c_int32), ("translation", C.c_float * 3),
                ("rotation", C.c_float * 3), ("scale", C.c_float * 3), ("transform", C.c_float * 16),
                ("inverse_transform", C.c_float * 16), ("inv_transpose", C.c_float * 16),
                ("tri_start", C.c_int32), ("tri_end", C.c_int32), ("bbox_idx", C.c_int32),
                ("min_bound", C.c_float * 3), ("max_bound", C.c_float * 3)]


class OMaterial(C.Structure):
    _fields_ = [("color", C.c_float * 3), ("spec_exponent", C.c_float), ("spec_color", C.c_float * 3),
                ("has_reflective", C.c_float), ("has_refractive", C.c_float), ("ior", C.c_float),
                ("emittance", C.c_float), ("texture_id", C.c_int32)]


class OCamera(C.Structure):
    _fields_ = [("res", C.c_int32 * 2), ("position", C.c_float * 3), ("look_at", C.c_float * 3),
                ("view", C.c_float * 3), ("up", C.c_float * 3), ("right", C.c_float * 3),
                ("fov", C.c_float * 2), ("pixel_length", C.c_float * 2)]


class OTexture(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("components", C.c_int32), ("pad", C.c_int32),
                ("data", C.c_void_p)]


TRI_DTYPE = np.dtype([("id", "<i4"), ("v", "<f4", (3, 3)), ("uv", "<f4", (3, 2)), ("n", "<f4", (3, 3)),
                      ("bmin", "<f4", (3,)), ("bmax", "<f4", (3,))])
NODE_DTYPE = np.dtype([("bmin", "<f4", (3,)), ("bmax", "<f4", (3,)), ("sub_areas", "<i4"), ("axis", "<i4"),
                       ("first_area_idx", "<i4"), ("rchild_idx", "<i4")])
assert TRI_DTYPE.itemsize == 124 and NODE_DTYPE.itemsize == 40


class OFlags(C.Structure):
    _fields_ = [("russian_roulette", C.c_int32), ("use_bvh", C.c_int32), ("use_bbox", C.c_int32),
                ("sort_by_material", C.c_int32), ("use_thrust_partition", C.c_int32), ("ssaa", C.c_int32),
                ("dof", C.c_int32), ("aperture", C.c_float), ("focal_dist", C.c_float),
                ("single_albedo", C.c_int32), ("rng_key_pixel", C.c_int32)]


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not LIB.exists():
            subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)
        L = C.CDLL(str(LIB))
        P, I64 = C.c_void_p, C.c_int64
        L.oracle_scan.argtypes = [I64, P, P]
        L.oracle_compact_without_scan.argtypes = [I64, P, P]
        L.oracle_compact_without_scan.restype = I64
        L.oracle_compact_with_scan.argtypes = [I64, P, P]
        L.oracle_compact_with_scan.restype = I64
        L.oracle_partition_indices.argtypes = [I64, P, P]
        L.oracle_partition_indices.restype = I64
        L.oracle_time_scan_ms.argtypes = [I64, P, P, C.c_int]
        L.oracle_time_scan_ms.restype = C.c_double
        L.oracle_time_compact_ms.argtypes = [I64, P, P, C.c_int, C.POINTER(I64)]
        L.oracle_time_compact_ms.restype = C.c_double
        L.oracle_time_compact_without_scan_ms.argtypes = [I64, P, P, C.c_int, C.POINTER(I64)]
        L.oracle_time_compact_without_scan_ms.restype = C.c_double
        L.oracle_sincos.argtypes = [C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]
        L.oracle_u01_sequence.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float)]
        L.oracle_u01_sequence.restype = C.c_float
        L.oracle_build_transform.argtypes = [P, P, P, P, P, P]
        L.oracle_camera.argtypes = [C.c_int, C.c_int, C.c_float, P, P, P, C.POINTER(OCamera)]
        L.oracle_render_pass.argtypes = [C.POINTER(OGeom), C.c_int, C.POINTER(OMaterial), C.c_int,
                                         P, C.c_int, P, C.c_int, P, C.c_int,
                                         C.POINTER(OCamera), C.c_int, C.POINTER(OFlags),
                                         C.c_int, C.c_int, C.c_int, C.c_int, P, P]
        L.oracle_render_pass.restype = C.c_int
        L.oracle_render.argtypes = [C.POINTER(OGeom), C.c_int, C.POINTER(OMaterial), C.c_int,
                                    P, C.c_int, P, C.c_int, P, C.c_int,
                                    C.POINTER(OCamera), C.c_int, C.POINTER(OFlags), C.c_int, C.c_int, P, P]
        L.oracle_render.restype = C.c_double
        L.oracle_set_tap.argtypes = [C.c_int, P, P, C.c_int]
        L.oracle_set_threads.argtypes = [C.c_int]
        L.oracle_tap_count.restype = C.c_int
        L.oracle_tonemap.argtypes = [P, C.c_int, C.c_int, C.c_float, P]
        L.oracle_preview.argtypes = [P, C.c_int, C.c_int, C.c_int, P]
        L.oracle_load_obj.argtypes = [C.c_char_p, P, P, C.c_int, P, C.c_int, P, P]
        L.oracle_load_obj.restype = C.c_int
        L.oracle_build_bvh.argtypes = [P, C.c_int, P, C.c_int]
        L.oracle_build_bvh.restype = C.c_int
        _lib = L
    return _lib


# ---- stream compaction ---------------------------------------------------------------------
def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.int32)


def scan(a) -> np.ndarray:
    a = _i32(a)
    out = np.zeros_like(a)
    lib().oracle_scan(len(a), out.ctypes.data, a.ctypes.data)
    return out


def compact_without_scan(a) -> np.ndarray:
    a = _i32(a)
    out = np.zeros_like(a)
    n = lib().oracle_compact_without_scan(len(a), out.ctypes.data, a.ctypes.data)
    return out[:n]


def compact_with_scan(a) -> np.ndarray:
    a = _i32(a)
    out = np.zeros_like(a)
    n = lib().oracle_compact_with_scan(len(a), out.ctypes.data, a.ctypes.data)
    return out[:n]


def partition_indices(flags):
    f = _i32(flags)
    out = np.zeros_like(f)
    live = lib().oracle_partition_indices(len(f), f.ctypes.data, out.ctypes.data)
    return out, int(live)


# ---- scene (scene.cpp:33-219 restated) -----------------------------------------------------
def build_transform(t, r, s):
    T = np.zeros(16, np.float32); Inv = np.zeros(16, np.float32); InvT = np.zeros(16, np.float32)
    f = [np.asarray(x, np.float32) for x in (t, r, s)]
    lib().oracle_build_transform(f[0].ctypes.data, f[1].ctypes.data, f[2].ctypes.data,
                                 T.ctypes.data, Inv.ctypes.data, InvT.ctypes.data)
    return T, Inv, InvT


def camera(res, fovy, eye, lookat, up) -> OCamera:
    cam = OCamera()
    e, l, u = (np.asarray(x, np.float32) for x in (eye, lookat, up))
    lib().oracle_camera(int(res[0]), int(res[1]), float(np.float32(fovy)), e.ctypes.data, l.ctypes.data,
                        u.ctypes.data, C.byref(cam))
    return cam


_TEXTURES: dict = {}


def load_texture(path):
    """Decoded texels by the oracle's own restatement of stb_image 2.06's JPEG decoder
    (oracle/jpeg_oracle.py; the reference's Texture::load, sceneStructs.h:171-175).  Cached per path."""
    from oracle import jpeg_oracle
    key = str(path)
    if key not in _TEXTURES:
        px = jpeg_oracle.load(key)
        _TEXTURES[key] = (px.shape[1], px.shape[0], px.shape[2], np.ascontiguousarray(px).reshape(-1))
    return _TEXTURES[key]


class OracleScene:
    def __init__(self):
        self.geoms: list[OGeom] = []
        self.materials: list[OMaterial] = []
        self.cam: OCamera | None = None
        self.depth = 8
        self.iterations = 1
        self.file = "render"
        self.tris_load = np.zeros(0, TRI_DTYPE)     # mesh triangles, load order
        self.tris = np.zeros(0, TRI_DTYPE)          # BVH leaf order (after build_bvh)
        self.nodes = np.zeros(0, NODE_DTYPE)
        self.textures: list[tuple] = []             # (w, h, comps, uint8 array)

    def add_mesh_obj(self, obj_path, material, t, r, s) -> int:
        """scene.cpp:94-173: one mesh geom from an OBJ file (oracle/mesh_oracle.cpp)."""
        gid = self.add_geom(2, material, t, r, s)
        g = self.geoms[gid]
        T = np.array(g.transform[:], np.float32)
        IT = np.array(g.inv_transpose[:], np.float32)
        bmin, bmax = np.zeros(3, np.float32), np.zeros(3, np.float32)
        base = len(self.tris_load)
        n = lib().oracle_load_obj(str(obj_path).encode(), T.ctypes.data, IT.ctypes.data, base, None, 0,
                                  bmin.ctypes.data, bmax.ctypes.data)
        if n < 0:
            raise FileNotFoundError(obj_path)
        tr = np.zeros(n, TRI_DTYPE)
        lib().oracle_load_obj(str(obj_path).encode(), T.ctypes.data, IT.ctypes.data, base, tr.ctypes.data, n,
                              bmin.ctypes.data, bmax.ctypes.data)
        self.tris_load = np.concatenate([self.tris_load, tr])
        g.tri_start, g.tri_end, g.bbox_idx = base, base + n, 0
        g.min_bound[:] = bmin.tolist()
        g.max_bound[:] = bmax.tolist()
        return gid

    def build_bvh(self):
        """build_bvh_tree (BVH_tree.cpp:149-181) over every mesh triangle, load order in."""
        self.tris = self.tris_load.copy()
        n = len(self.tris)
        nodes = np.zeros(max(2 * n, 1), NODE_DTYPE)
        k = lib().oracle_build_bvh(self.tris.ctypes.data, n, nodes.ctypes.data, len(nodes)) if n else 0
        self.nodes = nodes[:k].copy()

    def add_texture(self, path) -> int:
        self.textures.append(load_texture(path))
        return len(self.textures) - 1

    def _tables(self):
        texs = (OTexture * max(len(self.textures), 1))()
        for i, (w, h, c, data) in enumerate(self.textures):
            texs[i] = OTexture(w, h, c, 0, data.ctypes.data)
        tris = self.tris if len(self.tris) else None
        nodes = self.nodes if len(self.nodes) else None
        return (tris.ctypes.data if tris is not None else None, len(self.tris),
                nodes.ctypes.data if nodes is not None else None, len(self.nodes),
                texs if self.textures else None, len(self.textures))

    def add_material(self, rgb=(0, 0, 0), specrgb=None, specex=1.0, reflective=0.0, refractive=0.0, ior=0.0,
                     emittance=0.0, texture_id=-1) -> int:
        m = OMaterial()
        m.color[:] = [float(np.float32(v)) for v in rgb]
        m.spec_color[:] = [float(np.float32(v)) for v in (specrgb if specrgb is not None else rgb)]
        m.spec_exponent, m.has_reflective, m.has_refractive = specex, reflective, refractive
        m.ior, m.emittance, m.texture_id = ior, emittance, texture_id
        self.materials.append(m)
        return len(self.materials) - 1

    def add_geom(self, type_, material, t, r, s) -> int:
        g = OGeom()
        g.type, g.materialid = type_, material
        g.translation[:], g.rotation[:], g.scale[:] = list(t), list(r), list(s)
        T, Inv, InvT = build_transform(t, r, s)
        g.transform[:], g.inverse_transform[:], g.inv_transpose[:] = T.tolist(), Inv.tolist(), InvT.tolist()
        g.bbox_idx = -1
        self.geoms.append(g)
        return len(self.geoms) - 1

    def set_camera(self, res, fovy, eye, lookat, up=(0, 1, 0)):
        self.cam = camera(res, fovy, eye, lookat, up)

    @classmethod
    def from_json(cls, path, refraction: bool = False) -> "OracleScene":
        """Scene::loadFromJSON (scene.cpp:33-219).  REFRACTIVE / IOR are read only with
        refraction=True or a top-level "Extensions": {"REFRACTION": true} (the build's loader
        extension; the reference reads neither key, scene.cpp:46-56)."""
        data = json.loads(Path(path).read_text())
        ext = data.get("Extensions", {})
        # as the native loader (pt_scene.cpp file_wants_refraction): an object's boolean
        # "REFRACTION": true, or the string "REFRACTION" inside an array; anything else is off
        if isinstance(ext, dict):
            wants = ext.get("REFRACTION") is True
        elif isinstance(ext, list):
            wants = any(isinstance(x, str) and x == "REFRACTION" for x in ext)
        else:
            wants = False
        refraction = refraction or wants
        sc = cls()
        ids = {}
        base = Path(path).resolve().parent
        for name in sorted(data["Materials"]):           # nlohmann::json objects are std::map
            p = data["Materials"][name]
            rgb = p.get("RGB", [0.0, 0.0, 0.0])
            tex = -1
            if p.get("TEXTURE_FILE"):
                tex = sc.add_texture(base / "Textures" / p["TEXTURE_FILE"])
            ids[name] = sc.add_material(rgb=rgb, specrgb=p.get("SPECRGB", rgb), specex=p.get("SPECEX", 1.0),
                                        reflective=p.get("REFLECTIVE", 0.0), emittance=p.get("EMITTANCE", 0.0),
                                        refractive=p.get("REFRACTIVE", 0.0) if refraction else 0.0,
                                        ior=p.get("IOR", 0.0) if refraction else 0.0, texture_id=tex)
        for o in data["Objects"]:
            typ = {"sphere": 0, "cube": 1, "mesh": 2}[o["TYPE"]]
            mat = ids.get(o["MATERIAL"], 0)
            if typ == 2:
                sc.add_mesh_obj(base / "Models" / o["OBJ_FILE"], mat, o["TRANS"], o["ROTAT"], o["SCALE"])
            else:
                sc.add_geom(typ, mat, o["TRANS"], o["ROTAT"], o["SCALE"])
        sc.build_bvh()
        c = data["Camera"]
        sc.set_camera(c["RES"], c["FOVY"], c["EYE"], c["LOOKAT"], c["UP"])
        sc.depth, sc.iterations, sc.file = int(c["DEPTH"]), int(c["ITERATIONS"]), c["FILE"]
        return sc


def flags(russian_roulette=True, use_bvh=True, use_bbox=True, sort_by_material=False, use_thrust_partition=False,
          ssaa=True, dof=True, aperture=0.1, focal_dist=10.0, single_albedo=False,
          rng_key_pixel=False) -> OFlags:
    return OFlags(int(russian_roulette), int(use_bvh), int(use_bbox), int(sort_by_material),
                  int(use_thrust_partition), int(ssaa), int(dof), float(aperture), float(focal_dist),
                  int(single_albedo), int(rng_key_pixel))


def render_pass(sc: OracleScene, fl: OFlags, iter_first: int, spp: int = 1, rank: int = 0, world: int = 1,
                image: np.ndarray | None = None, depth: int | None = None):
    """One pass on the tile; returns (image (rows, W, 3) float32, bounce_live list)."""
    W, H = sc.cam.res[0], sc.cam.res[1]
    rows = (H - rank + world - 1) // world
    if image is None:
        image = np.zeros((rows, W, 3), np.float32)
    d = depth if depth is not None else sc.depth
    live = np.zeros(64, np.uint64)
    G = (OGeom * len(sc.geoms))(*sc.geoms)
    M = (OMaterial * len(sc.materials))(*sc.materials)
    lib().oracle_render_pass(G, len(sc.geoms), M, len(sc.materials), *sc._tables(),
                             C.byref(sc.cam), d, C.byref(fl), iter_first, spp, rank, world,
                             image.ctypes.data, live.ctypes.data)
    return image, [int(x) for x in live[:d]]


def set_threads(n: int) -> None:
    """Worker threads of render_pass's per-path loops (the result does not depend on it)."""
    lib().oracle_set_threads(int(n))


def bounce_records(sc: OracleScene, fl: OFlags, iteration: int, bounce: int):
    """Real per-bounce records of a one-iteration render: the material key of every live path as
    computeIntersections leaves it (before the material sort) and its remainingBounces after
    shading (before the compaction).  Test input for pinning sort/partition against rocThrust."""
    cap = sc.cam.res[0] * sc.cam.res[1]
    keys = np.zeros(cap, np.int32)
    rem = np.zeros(cap, np.int32)
    lib().oracle_set_tap(bounce, keys.ctypes.data, rem.ctypes.data, cap)
    try:
        render_pass(sc, fl, iteration)
        n = lib().oracle_tap_count()
    finally:
        lib().oracle_set_tap(-1, None, None, 0)
    return keys[:n].copy(), rem[:n].copy()


def render(sc: OracleScene, fl: OFlags, iters: int, iter_first: int = 1):
    W, H = sc.cam.res[0], sc.cam.res[1]
    image = np.zeros((H, W, 3), np.float32)
    live = np.zeros(64, np.uint64)
    G = (OGeom * len(sc.geoms))(*sc.geoms)
    M = (OMaterial * len(sc.materials))(*sc.materials)
    secs = lib().oracle_render(G, len(sc.geoms), M, len(sc.materials), *sc._tables(),
                               C.byref(sc.cam), sc.depth, C.byref(fl), iter_first, iters, image.ctypes.data,
                               live.ctypes.data)
    return image, [int(x) for x in live[:sc.depth]], secs


def tonemap(image: np.ndarray, samples: float) -> np.ndarray:
    img = np.ascontiguousarray(image, np.float32)
    H, W = img.shape[:2]
    out = np.zeros((H, W, 3), np.uint8)
    lib().oracle_tonemap(img.ctypes.data, W, H, float(samples), out.ctypes.data)
    return out


def u01_sequence(it, index, depth, count) -> np.ndarray:
    out = (C.c_float * count)()
    lib().oracle_u01_sequence(it, index, depth, count, out)
    return np.frombuffer(out, dtype=np.float32).copy()


def sincos(x: float):
    s, c = C.c_float(), C.c_float()
    lib().oracle_sincos(float(x), C.byref(s), C.byref(c))
    return s.value, c.value

"""ctypes binding of libpt_amd.so (the C ABI declared in include/pt_amd.h and include/sc_amd.h).

The library is REQUIRED: there is no CPU fallback anywhere in this package.  If the shared object
is missing or fails to load, every entry point raises NativeLibraryError.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
from pathlib import Path

_PKG = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ["PT_AMD_LIB"]) if os.environ.get("PT_AMD_LIB") else _PKG / "libpt_amd.so"


class NativeLibraryError(RuntimeError):
    pass


class PtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[pt error {code}] {msg}")
        self.code = code


# ---- C structs (same layout as include/pt_amd.h) -------------------------------------------
class Flags(C.Structure):
    _fields_ = [("russian_roulette", C.c_int32), ("use_bvh", C.c_int32), ("use_bbox", C.c_int32),
                ("sort_by_material", C.c_int32), ("use_thrust_partition", C.c_int32), ("ssaa", C.c_int32),
                ("dof", C.c_int32), ("aperture", C.c_float), ("focal_dist", C.c_float),
                ("single_albedo", C.c_int32), ("bvh_cull", C.c_int32), ("shared_gpu", C.c_int32),
                ("rng_key_pixel", C.c_int32)]


class Material(C.Structure):
    _fields_ = [("color", C.c_float * 3), ("spec_exponent", C.c_float), ("spec_color", C.c_float * 3),
                ("has_reflective", C.c_float), ("has_refractive", C.c_float), ("ior", C.c_float),
                ("emittance", C.c_float), ("texture_id", C.c_int32)]


class Geom(C.Structure):
    _fields_ = [("type", C.c_int32), ("material_id", C.c_int32), ("translation", C.c_float * 3),
                ("rotation", C.c_float * 3), ("scale", C.c_float * 3), ("transform", C.c_float * 16),
                ("inverse_transform", C.c_float * 16), ("inv_transpose", C.c_float * 16),
                ("tri_start", C.c_int32), ("tri_end", C.c_int32), ("bbox_idx", C.c_int32),
                ("min_bound", C.c_float * 3), ("max_bound", C.c_float * 3)]


class Camera(C.Structure):
    _fields_ = [("res", C.c_int32 * 2), ("position", C.c_float * 3), ("look_at", C.c_float * 3),
                ("view", C.c_float * 3), ("up", C.c_float * 3), ("right", C.c_float * 3),
                ("fov", C.c_float * 2), ("pixel_length", C.c_float * 2)]


class Triangle(C.Structure):
    _fields_ = [("id", C.c_int32), ("v", (C.c_float * 3) * 3), ("uv", (C.c_float * 2) * 3),
                ("n", (C.c_float * 3) * 3), ("bmin", C.c_float * 3), ("bmax", C.c_float * 3)]


class BvhNode(C.Structure):
    _fields_ = [("bmin", C.c_float * 3), ("bmax", C.c_float * 3), ("sub_areas", C.c_int32),
                ("axis", C.c_int32), ("first_area_idx", C.c_int32), ("rchild_idx", C.c_int32)]


class Shard(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("spp", C.c_int32), ("reserved", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("passes", C.c_uint64), ("bounce_live", C.c_uint64 * 64),
                ("emissive_hits", C.c_uint64), ("bounce_emit", C.c_uint64 * 64), ("device_error", C.c_uint32),
                ("bound_mismatch", C.c_uint32)]


assert C.sizeof(Geom) == 272 and C.sizeof(Material) == 48 and C.sizeof(Triangle) == 124
assert C.sizeof(BvhNode) == 40

_P = C.c_void_p
_I = C.c_int32
_F = C.c_float
_FP = C.POINTER(C.c_float)
_IP = C.POINTER(C.c_int32)

# name -> (restype, argtypes).  Every function declared in include/*.h appears here.
SIGNATURES = {
    # sc_amd.h
    "sc_last_error": (C.c_char_p, []),
    "sc_workspace_bytes": (C.c_size_t, [C.c_int64]),
    "sc_scan_exclusive_i32": (_I, [_P, _P, C.c_int64, _P, _P]),
    "sc_compact_i32": (_I, [_P, _P, C.c_int64, _P, _P, _P]),
    "sc_partition_i32": (_I, [_P, _P, C.c_int64, _P, _P, _P]),
    "sc_partition_indices": (_I, [_P, _P, C.c_int64, _P, _P, _P]),
    "sc_efficient_scan": (_I, [C.c_int, _P, _P]),
    "sc_efficient_compact": (_I, [C.c_int, _P, _P, _IP]),
    "sc_timer_gpu_ms": (C.c_float, []),
    "sc_cpu_scan": (_I, [C.c_int, _P, _P]),
    "sc_cpu_compact_without_scan": (_I, [C.c_int, _P, _P, _IP]),
    "sc_cpu_compact_with_scan": (_I, [C.c_int, _P, _P, _IP]),
    "sc_naive_scan_i32": (_I, [_P, _P, C.c_int64, _P, _P]),
    "sc_thrust_scan_i32": (_I, [_P, _P, C.c_int64, _P]),
    "sc_naive_scan": (_I, [C.c_int, _P, _P]),
    "sc_thrust_scan": (_I, [C.c_int, _P, _P]),
    "sc_set_tile_schedule": (_I, [_I]),
    "sc_workspace_check": (_I, [_P]),
    "sc_workspace_error_word": (_P, [_P]),
    # pt_amd.h
    "pt_last_error": (C.c_char_p, []),
    "pt_flags_default": (None, [C.POINTER(Flags)]),
    "pt_scene_load_json": (_I, [C.c_char_p, C.POINTER(_P)]),
    "pt_scene_load_json_ex": (_I, [C.c_char_p, C.c_uint32, C.POINTER(_P)]),
    "pt_scene_create": (_I, [C.POINTER(_P)]),
    "pt_scene_free": (None, [_P]),
    "pt_scene_add_material": (_I, [_P, C.POINTER(Material), _IP]),
    "pt_scene_add_texture": (_I, [_P, _I, _I, _I, _P, _IP]),
    "pt_scene_texture_path": (_I, [_P, _I, C.c_char_p, _I]),
    "pt_scene_set_texture_pixels": (_I, [_P, _I, _I, _I, _I, _P]),
    "pt_scene_add_geom": (_I, [_P, _I, _I, _FP, _FP, _FP, _IP]),
    "pt_scene_add_mesh": (_I, [_P, _I, _FP, _FP, _FP, _FP, _I, _FP, _I, _FP, _I, _IP, _I, _IP, _IP, _IP, _IP]),
    "pt_scene_set_camera": (_I, [_P, _I, _I, _F, _FP, _FP, _FP]),
    "pt_scene_set_render": (_I, [_P, _I, _I, C.c_char_p]),
    "pt_scene_finalize": (_I, [_P]),
    "pt_scene_set_bvh_builder": (_I, [_P, _I]),
    "pt_scene_bvh_build_info": (_I, [_P, _IP, C.POINTER(C.c_double)]),
    "pt_scene_counts": (_I, [_P, _IP, _IP, _IP, _IP, _IP]),
    "pt_scene_get_camera": (_I, [_P, C.POINTER(Camera)]),
    "pt_scene_get_render": (_I, [_P, _IP, _IP, C.c_char_p, _I]),
    "pt_scene_get_orbit": (_I, [_P, _FP, _FP, _FP]),
    "pt_scene_set_orbit": (_I, [_P, _F, _F, _F, _FP]),
    "pt_scene_get_geoms": (_I, [_P, C.POINTER(Geom), _I]),
    "pt_scene_get_materials": (_I, [_P, C.POINTER(Material), _I]),
    "pt_scene_get_triangles": (_I, [_P, C.POINTER(Triangle), _I]),
    "pt_scene_get_bvh": (_I, [_P, C.POINTER(BvhNode), _I]),
    "pt_scene_bvh_quads": (_I, [_P, _P, _I, _IP, _IP]),
    "pt_scene_bvh_tcull": (_I, [_P, C.POINTER(C.c_uint32), _I, C.POINTER(C.c_double)]),
    "pt_create": (_I, [_P, C.POINTER(Flags), C.POINTER(Shard), C.POINTER(_P)]),
    "pt_destroy": (_I, [_P]),
    "pt_set_flags": (_I, [_P, C.POINTER(Flags)]),
    "pt_ctx_cmask_info": (_I, [_P, _IP, C.POINTER(C.c_double), _IP]),
    "pt_ctx_counters": (_I, [_P, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "pt_ctx_stream_info": (_I, [_P] + [C.POINTER(C.c_int32)] * 5),
    "pt_ctx_walk_info": (_I, [_P, C.POINTER(_I), C.POINTER(_I), C.POINTER(C.c_double)]),
    "pt_render_pass": (_I, [_P, _I, _P]),
    "pt_render_ahead": (_I, [_P, _I, _P]),
    "pt_host_register": (_I, [_P, C.c_uint64]),
    "pt_host_unregister": (_I, [_P]),
    "pt_stream_create": (_I, [C.POINTER(_P)]),
    "pt_stream_destroy": (_I, [_P]),
    "pt_preview_rgba": (_I, [_P, _I, _P, _P]),
    "pt_tile_info": (_I, [_P, _IP, _IP, _IP, _IP]),
    "pt_get_image": (_I, [_P, _P]),
    "pt_get_accum": (_I, [_P, _P]),
    "pt_render_iteration": (_I, [_P, _I, _P, _P]),
    "pt_copy_image": (_I, [_P, _P, _P]),
    "pt_reset_image": (_I, [_P, _P]),
    "pt_stats": (_I, [_P, C.POINTER(Stats)]),
    "pt_profile_enable": (_I, [_P, _I]),
    "pt_selftest_math": (_I, [C.c_uint64, C.c_uint32, C.POINTER(C.c_uint64)]),
    "pt_profile_read": (_I, [_P, C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "pt_profile_read_busy": (_I, [_P, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "pt_profile_read_kinds": (_I, [_P, _I, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint64)]),
    "pt_tonemap": (_I, [_P, _I, _I, _F, _P]),
    "pt_save_png": (_I, [C.c_char_p, _P, _I, _I, _F]),
    "pt_save_hdr": (_I, [C.c_char_p, _P, _I, _I, _F]),
    "pt_encode_hdr": (_I, [_P, _I, _I, _F, _P, C.c_int64, _P]),
    "pt_set_accum": (_I, [_P, _P]),
    "pt_decode_jpeg": (_I, [C.c_char_p, C.c_int64, _IP, _IP, _IP, _P, C.c_int64]),
}

_lib = None


def _preload_torch() -> None:
    # torch ships its own libamdhip64.so.7; importing torch first makes this library bind to the
    # same HIP runtime instance (same SONAME), so device pointers and streams are shared.
    if "torch" not in sys.modules:
        try:
            import torch  # noqa: F401
        except Exception:
            pass


_OPTIONAL = {"pt_selftest_math", "pt_profile_read_kinds"}


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise NativeLibraryError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(there is no CPU fallback)")
    if os.environ.get("PT_AMD_NO_TORCH", "0") != "1":
        _preload_torch()
    try:
        L = C.CDLL(str(LIB_PATH), mode=C.RTLD_GLOBAL)
    except OSError as e:
        raise NativeLibraryError(f"failed to load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        if name in _OPTIONAL and not hasattr(L, name):   # (an older build timed beside this one)
            continue
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check_pt(rc: int) -> None:
    if rc != 0:
        raise PtError(rc, lib().pt_last_error().decode())


def check_sc(rc: int) -> None:
    if rc != 0:
        raise PtError(rc, lib().sc_last_error().decode())


def f3(x) -> C.Array:
    return (C.c_float * 3)(*[float(v) for v in x])

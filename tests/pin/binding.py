"""ctypes binding of tests/pin/build/libthrust_pin.so (test infrastructure only): rocThrust's
default_random_engine + uniform_real_distribution, sort_by_key and stable_partition as the
reference calls them (pathtrace.cu:57-62, 479-503), on the host (thrust::host) and the device."""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

_LIB = Path(__file__).resolve().parent / "build" / "libthrust_pin.so"
_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not _LIB.exists():
            from cuda_pathtracer_amd import build as B
            B.build_pin()
        L = C.CDLL(str(_LIB))
        P = C.c_void_p
        for side in ("host", "device"):
            getattr(L, f"pin_rng_{side}").argtypes = [C.c_int, P, P, P, C.c_int, P]
            getattr(L, f"pin_sort_by_key_{side}").argtypes = [C.c_int, P, P]
            getattr(L, f"pin_stable_partition_{side}").argtypes = [C.c_int, P, P, P]
        _lib = L
    return _lib


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def rng(iters, indices, depths, draws: int, device: bool = False) -> np.ndarray:
    it, ix, dp = _i32(iters), _i32(indices), _i32(depths)
    out = np.zeros((len(it), draws), np.float32)
    f = lib().pin_rng_device if device else lib().pin_rng_host
    assert f(len(it), it.ctypes.data, ix.ctypes.data, dp.ctypes.data, draws, out.ctypes.data) == 0
    return out


def sort_by_key_order(mat, device: bool = False) -> np.ndarray:
    m = _i32(mat)
    out = np.zeros(len(m), np.int32)
    f = lib().pin_sort_by_key_device if device else lib().pin_sort_by_key_host
    assert f(len(m), m.ctypes.data, out.ctypes.data) == 0
    return out


def stable_partition_order(remaining, device: bool = False):
    r = _i32(remaining)
    out = np.zeros(len(r), np.int32)
    live = C.c_int(0)
    f = lib().pin_stable_partition_device if device else lib().pin_stable_partition_host
    assert f(len(r), r.ctypes.data, out.ctypes.data, C.byref(live)) == 0
    return out, live.value

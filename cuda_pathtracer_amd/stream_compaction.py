"""Python mirror of the reference's StreamCompaction API, backed by the HIP kernels.

Reference: path_tracer/stream_compaction/{efficient,cpu,naive,thrust,common}.{h,cu}.
  StreamCompaction::Efficient::scan(n, odata, idata)     -> Efficient.scan
  StreamCompaction::Efficient::compact(n, odata, idata)  -> Efficient.compact
  StreamCompaction::Efficient::timer()                   -> Efficient.timer()
  StreamCompaction::CPU::{scan, compactWithoutScan, compactWithScan}, CPU::timer()  -> CPU
  StreamCompaction::Naive::scan, Naive::timer()          -> Naive
  StreamCompaction::Thrust::scan, Thrust::timer()        -> Thrust
The host-array calls keep the reference semantics (host arrays in, host arrays out, GPU time of
the device work only).  The device-tensor functions (scan_device, compact_device,
partition_device, naive_scan_device) take torch tensors already resident on the GPU and never
synchronise; thrust_scan_device synchronises the device (rocThrust allocates and frees its
temporary storage on every call).  CPU's functions are the library's own host loops (sc_cpu_*), the
reference's CPU namespace; they are not a fallback of any device path and not the test oracle
(oracle/ checks them).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._native import check_sc, lib


class _Timer:
    """PerformanceTimer (common.h:46-130), GPU side only."""

    def getGpuElapsedTimeForPreviousOperation(self) -> float:  # noqa: N802 (reference name)
        return float(lib().sc_timer_gpu_ms())


_TIMER = _Timer()


class _CpuTimer:
    """PerformanceTimer's CPU side (common.h:63-80): wall time of the previous CPU:: call."""

    def __init__(self):
        self._ms = 0.0

    def getCpuElapsedTimeForPreviousOperation(self) -> float:  # noqa: N802 (reference name)
        return self._ms


_CPU_TIMER = _CpuTimer()


def _i32(a: np.ndarray, name: str) -> np.ndarray:
    if not isinstance(a, np.ndarray) or a.dtype != np.int32 or not a.flags.c_contiguous:
        raise TypeError(f"{name} must be a C-contiguous numpy int32 array")
    return a


class Efficient:
    @staticmethod
    def timer() -> _Timer:
        return _TIMER

    @staticmethod
    def scan(n: int, odata: np.ndarray, idata: np.ndarray) -> None:
        """Exclusive prefix sum of idata[:n] into odata[:n] (int32, wrapping)."""
        _i32(odata, "odata"); _i32(idata, "idata")
        if n < 0 or n > len(idata) or n > len(odata):
            raise ValueError("n out of range")
        check_sc(lib().sc_efficient_scan(n, odata.ctypes.data, idata.ctypes.data))

    @staticmethod
    def compact(n: int, odata: np.ndarray, idata: np.ndarray) -> int:
        """Keep the non-zero elements of idata[:n] in order; returns how many were kept."""
        _i32(odata, "odata"); _i32(idata, "idata")
        if n < 0 or n > len(idata) or n > len(odata):
            raise ValueError("n out of range")
        cnt = C.c_int32(0)
        check_sc(lib().sc_efficient_compact(n, odata.ctypes.data, idata.ctypes.data, C.byref(cnt)))
        return int(cnt.value)


def _host_args(n, odata, idata):
    _i32(odata, "odata"); _i32(idata, "idata")
    if n < 0 or n > len(idata) or n > len(odata):
        raise ValueError("n out of range")


class CPU:
    """StreamCompaction::CPU (cpu.h:9-13): sequential host loops in libpt_amd.so (sc_cpu_*)."""

    @staticmethod
    def timer() -> _CpuTimer:
        return _CPU_TIMER

    @staticmethod
    def _timed(fn, *args):
        import time
        t0 = time.perf_counter()
        rc = fn(*args)
        _CPU_TIMER._ms = (time.perf_counter() - t0) * 1e3
        check_sc(rc)

    @staticmethod
    def scan(n: int, odata: np.ndarray, idata: np.ndarray) -> None:
        _host_args(n, odata, idata)
        CPU._timed(lib().sc_cpu_scan, n, odata.ctypes.data, idata.ctypes.data)

    @staticmethod
    def compactWithoutScan(n: int, odata: np.ndarray, idata: np.ndarray) -> int:  # noqa: N802
        _host_args(n, odata, idata)
        cnt = C.c_int32(0)
        CPU._timed(lib().sc_cpu_compact_without_scan, n, odata.ctypes.data, idata.ctypes.data, C.byref(cnt))
        return int(cnt.value)

    @staticmethod
    def compactWithScan(n: int, odata: np.ndarray, idata: np.ndarray) -> int:  # noqa: N802
        _host_args(n, odata, idata)
        cnt = C.c_int32(0)
        CPU._timed(lib().sc_cpu_compact_with_scan, n, odata.ctypes.data, idata.ctypes.data, C.byref(cnt))
        return int(cnt.value)


class Naive:
    """StreamCompaction::Naive (naive.h:9): Hillis & Steele on the device (sc_naive_scan)."""

    @staticmethod
    def timer() -> _Timer:
        return _TIMER

    @staticmethod
    def scan(n: int, odata: np.ndarray, idata: np.ndarray) -> None:
        _host_args(n, odata, idata)
        check_sc(lib().sc_naive_scan(n, odata.ctypes.data, idata.ctypes.data))


class Thrust:
    """StreamCompaction::Thrust (thrust.h:9): rocThrust's exclusive_scan (sc_thrust_scan)."""

    @staticmethod
    def timer() -> _Timer:
        return _TIMER

    @staticmethod
    def scan(n: int, odata: np.ndarray, idata: np.ndarray) -> None:
        _host_args(n, odata, idata)
        check_sc(lib().sc_thrust_scan(n, odata.ctypes.data, idata.ctypes.data))


def _stream_ptr(stream) -> int:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return int(getattr(stream, "cuda_stream", stream))


def _check_dev_i32(t, name: str):
    import torch
    if not (isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.int32 and t.is_contiguous()):
        raise TypeError(f"{name} must be a contiguous int32 CUDA tensor")


def _checked(stream, check: bool) -> None:
    """check=True: wait for the call and read the workspace's device error word (sc_workspace_check).
    The device-pointer entry points are asynchronous; a static-schedule look-back that could not get
    the whole GPU (another process or stream holding part of it) drains with wrong results and sets
    that word instead of failing the call — check=True (or sc_set_tile_schedule(1) for shared GPUs)
    turns it into an exception."""
    if check:
        import torch
        torch.cuda.synchronize()
        check_sc(lib().sc_workspace_check(None))


def scan_device(d_in, d_out=None, stream=None, check: bool = False):
    """Exclusive scan of a device int32 tensor (single-pass decoupled look-back).  check: see _checked."""
    import torch
    _check_dev_i32(d_in, "d_in")
    if d_out is None:
        d_out = torch.empty_like(d_in)
    _check_dev_i32(d_out, "d_out")
    check_sc(lib().sc_scan_exclusive_i32(d_in.data_ptr(), d_out.data_ptr(), d_in.numel(), None, _stream_ptr(stream)))
    _checked(stream, check)
    return d_out


def compact_device(d_in, d_out=None, stream=None, check: bool = False):
    """Returns (d_out, d_count): non-zero elements first (in order), count as a 1-element int64 tensor.
    check: see _checked."""
    import torch
    _check_dev_i32(d_in, "d_in")
    if d_out is None:
        d_out = torch.empty_like(d_in)
    _check_dev_i32(d_out, "d_out")
    cnt = torch.zeros(1, dtype=torch.int64, device=d_in.device)
    check_sc(lib().sc_compact_i32(d_in.data_ptr(), d_out.data_ptr(), d_in.numel(), cnt.data_ptr(), None,
                                  _stream_ptr(stream)))
    _checked(stream, check)
    return d_out, cnt


def partition_device(d_flags, d_perm=None, stream=None, check: bool = False):
    """Stable partition of indices (live first, then dead), like pathtrace.cu:366-376 `keep`.
    check: see _checked."""
    import torch
    _check_dev_i32(d_flags, "d_flags")
    if d_perm is None:
        d_perm = torch.empty_like(d_flags)
    live = torch.zeros(1, dtype=torch.int64, device=d_flags.device)
    check_sc(lib().sc_partition_i32(d_flags.data_ptr(), d_perm.data_ptr(), d_flags.numel(), live.data_ptr(), None,
                                    _stream_ptr(stream)))
    _checked(stream, check)
    return d_perm, live


def live_indices_device(d_flags, d_idx=None, stream=None, check: bool = False):
    """Index list of the non-zero flags, in order (sc_partition_indices): returns (d_idx, count)
    with the count as a 1-element int32 tensor; d_idx beyond the count is untouched.  check: see _checked."""
    import torch
    _check_dev_i32(d_flags, "d_flags")
    if d_idx is None:
        d_idx = torch.empty_like(d_flags)
    _check_dev_i32(d_idx, "d_idx")
    cnt = torch.zeros(1, dtype=torch.int32, device=d_flags.device)
    check_sc(lib().sc_partition_indices(d_flags.data_ptr(), d_idx.data_ptr(), d_flags.numel(), cnt.data_ptr(), None,
                                        _stream_ptr(stream)))
    _checked(stream, check)
    return d_idx, cnt


def _check_len(d_in, **bufs) -> None:
    """Output and scratch tensors must hold at least d_in.numel() elements (the kernels write n)."""
    for name, t in bufs.items():
        if t.numel() < d_in.numel():
            raise ValueError(f"{name} holds {t.numel()} elements < n = {d_in.numel()}")


def naive_scan_device(d_in, d_out=None, d_tmp=None, stream=None):
    """Naive::scan on device tensors (sc_naive_scan_i32): d_in unchanged, d_tmp = n int32 of scratch."""
    import torch
    _check_dev_i32(d_in, "d_in")
    d_out = torch.empty_like(d_in) if d_out is None else d_out
    d_tmp = torch.empty_like(d_in) if d_tmp is None else d_tmp
    _check_dev_i32(d_out, "d_out"); _check_dev_i32(d_tmp, "d_tmp")
    _check_len(d_in, d_out=d_out, d_tmp=d_tmp)
    check_sc(lib().sc_naive_scan_i32(d_in.data_ptr(), d_out.data_ptr(), d_in.numel(), d_tmp.data_ptr(),
                                     _stream_ptr(stream)))
    return d_out


def thrust_scan_device(d_in, d_out=None, stream=None):
    """Thrust::scan on device tensors (sc_thrust_scan_i32: rocThrust exclusive_scan).  Synchronises
    the device (rocThrust's per-call temporary storage)."""
    import torch
    _check_dev_i32(d_in, "d_in")
    d_out = torch.empty_like(d_in) if d_out is None else d_out
    _check_dev_i32(d_out, "d_out")
    _check_len(d_in, d_out=d_out)
    check_sc(lib().sc_thrust_scan_i32(d_in.data_ptr(), d_out.data_ptr(), d_in.numel(), _stream_ptr(stream)))
    return d_out

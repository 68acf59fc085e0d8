"""MI355X-native Monte-Carlo path tracer (drop-in for the render loop of sgong-0224/CUDA_Pathtracer).

The hot path (ray generation, intersection, shading, stream compaction) is hand-written HIP for
gfx950 in csrc/, exported through the C ABI in include/pt_amd.h and include/sc_amd.h and bound
here with ctypes.  There is no CPU fallback: importing works without the shared object, but every
entry point raises NativeLibraryError if libpt_amd.so is missing.
"""
from ._native import LIB_PATH, NativeLibraryError, PtError, lib  # noqa: F401
from .pathtrace import (  # noqa: F401
    CUBE, MESH, SPHERE, GuiDataContainer, InitDataContainer, PathTracer, Scene, pathtrace, pathtraceFree,
    pathtraceInit, render, save_image, save_image_hdr, encode_hdr, tonemap)
from . import distributed  # noqa: F401
from .stream_compaction import (CPU, Efficient, Naive, Thrust, compact_device, live_indices_device,  # noqa: F401
                                naive_scan_device, partition_device, scan_device, thrust_scan_device)

__all__ = ["Scene", "PathTracer", "GuiDataContainer", "Efficient", "CPU", "Naive", "Thrust", "scan_device",
           "compact_device", "naive_scan_device", "thrust_scan_device",
           "partition_device", "live_indices_device", "render", "save_image", "save_image_hdr", "encode_hdr", "tonemap", "pathtraceInit",
           "pathtraceFree", "pathtrace",
           "InitDataContainer", "lib", "LIB_PATH", "NativeLibraryError", "PtError"]

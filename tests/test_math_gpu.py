"""The range-gated correctly rounded sqrt / division cores of the device code (pt_device.h
sqrt_cr, div_cr, div2_cr, normalize, length) return the same bits as hipcc's library sqrtf and
'/' — the evaluation contract's premise that keeps GPU == oracle bit for bit."""
import ctypes as C

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", [1, 0xC0FFEE])
def test_fast_sqrt_div_cores_equal_library(gpu_device, seed):
    from cuda_pathtracer_amd._native import check_pt, lib
    bad = C.c_uint64(0)
    check_pt(lib().pt_selftest_math(1 << 26, seed, C.byref(bad)))
    assert bad.value == 0, f"{bad.value} mismatching operations"

"""The reference's other StreamCompaction namespaces: CPU (cpu.h:9-13, cpu.cu:16-79), Naive
(naive.h:9, naive.cu:14-66) and Thrust (thrust.h:9, thrust.cu:14-28), through the C ABI
(sc_cpu_*, sc_naive_scan*, sc_thrust_scan*) and the Python mirror (CPU, Naive, Thrust).

CPU::* are host loops of the product library, so they are checked here without a GPU: against
the reference's known answers (INSTRUCTION.md:262-302), the committed golden vectors and the
oracle.  Naive and Thrust run on the device (-m gpu): bit-exact against the oracle at the shapes
main.cpp uses (POT / NPOT, last element 0, values < 50) plus odd/even pass counts, wrap-around and
the argument checks.
"""
import ctypes as C
from pathlib import Path

import numpy as np
import pytest

import cuda_pathtracer_amd as P
from cuda_pathtracer_amd._native import PtError, lib
from oracle import binding as O

GOLDEN = Path(__file__).resolve().parent / "golden"


def _gen(n, maxval, seed):
    a = np.random.default_rng(seed).integers(0, maxval, size=n, dtype=np.int32)
    if n:
        a[-1] = 0          # main.cpp:23,98 "leave a 0 at the end"
    return a


# ---- CPU (no GPU needed) --------------------------------------------------------------------
def test_cpu_known_answers():
    a = np.array([1, 5, 0, 1, 2, 0, 3], np.int32)
    o = np.zeros_like(a)
    P.CPU.scan(7, o, a)
    assert o.tolist() == [0, 1, 6, 6, 7, 9, 9]
    o[:] = 0
    assert P.CPU.compactWithoutScan(7, o, a) == 5 and o[:5].tolist() == [1, 5, 1, 2, 3]
    o[:] = 0
    assert P.CPU.compactWithScan(7, o, a) == 5 and o[:5].tolist() == [1, 5, 1, 2, 3]
    assert P.CPU.timer().getCpuElapsedTimeForPreviousOperation() >= 0.0


def test_cpu_golden_vectors():
    g = np.load(GOLDEN / "scan_compact.npz")
    for tag in ("pot", "npot", "small"):
        a = g[f"{tag}_scan_in"]
        o = np.zeros_like(a)
        P.CPU.scan(len(a), o, a)
        np.testing.assert_array_equal(o, g[f"{tag}_scan_out"])
        c = g[f"{tag}_compact_in"]
        exp = g[f"{tag}_compact_out"]
        for fn in (P.CPU.compactWithoutScan, P.CPU.compactWithScan):
            o = np.zeros_like(c)
            k = fn(len(c), o, c)
            assert k == len(exp)
            np.testing.assert_array_equal(o[:k], exp)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 255, 256, 257, (1 << 16) - 3, 1 << 16, (1 << 20) + 7])
def test_cpu_matches_oracle(n):
    rng = np.random.default_rng(n)
    a = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)   # wrap-around
    o = np.full(max(n, 1), 7, np.int32)
    P.CPU.scan(n, o, a)
    np.testing.assert_array_equal(o[:n], O.scan(a))
    b = (a & 3).astype(np.int32)
    for fn, ofn in ((P.CPU.compactWithoutScan, O.compact_without_scan), (P.CPU.compactWithScan, O.compact_with_scan)):
        o = np.zeros(max(n, 1), np.int32)
        k = fn(n, o, b)
        exp = ofn(b)
        assert k == len(exp)
        np.testing.assert_array_equal(o[:k], exp)


def test_cpu_scan_in_place_and_errors():
    a = _gen(1001, 50, 4)
    exp = O.scan(a)
    b = a.copy()
    assert lib().sc_cpu_scan(len(b), b.ctypes.data, b.ctypes.data) == 0
    np.testing.assert_array_equal(b, exp)
    cnt = C.c_int32(0)
    assert lib().sc_cpu_scan(-1, b.ctypes.data, a.ctypes.data) != 0
    assert lib().sc_cpu_compact_with_scan(5, None, a.ctypes.data, C.byref(cnt)) != 0
    assert b"null" in lib().sc_last_error()
    assert lib().sc_cpu_compact_without_scan(0, None, None, C.byref(cnt)) == 0 and cnt.value == 0


# ---- Naive and Thrust (device) --------------------------------------------------------------
SIZES = [1, 2, 3, 4, 5, 63, 64, 65, 1000, 4095, 4096, 4097, 65536 + 17, (1 << 20) - 3, 1 << 20]


@pytest.mark.gpu
@pytest.mark.parametrize("n", SIZES)
def test_naive_and_thrust_host_api(gpu_device, n):
    a = _gen(n, 50, n)
    exp = O.scan(a)
    for ns in (P.Naive, P.Thrust):
        o = np.full(n, -1, np.int32)
        ns.scan(n, o, a)
        np.testing.assert_array_equal(o, exp, err_msg=ns.__name__)
        assert ns.timer().getGpuElapsedTimeForPreviousOperation() >= 0.0


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 3, 129, 4097, 100003, (1 << 22) + 5])
def test_naive_and_thrust_device_wrap(gpu_device, n):
    import torch
    rng = np.random.default_rng(11)
    a = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
    d = torch.from_numpy(a).to(gpu_device)
    keep = d.clone()
    out_n = P.naive_scan_device(d)
    out_t = P.thrust_scan_device(d)
    torch.cuda.synchronize()
    exp = O.scan(a)
    np.testing.assert_array_equal(out_n.cpu().numpy(), exp)
    np.testing.assert_array_equal(out_t.cpu().numpy(), exp)
    assert torch.equal(d, keep), "the input is left unchanged"
    P.thrust_scan_device(d, d)    # in place
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy(), exp)


@pytest.mark.gpu
def test_naive_argument_checks(gpu_device):
    import torch
    d = torch.zeros(100, dtype=torch.int32, device=gpu_device)
    t = torch.empty_like(d)
    with pytest.raises(PtError):
        P.naive_scan_device(d, d, t)          # out aliases in
    with pytest.raises(PtError):
        P.naive_scan_device(d, t, t)          # tmp aliases out
    assert lib().sc_naive_scan_i32(None, None, 0, None, None) == 0
    assert lib().sc_thrust_scan_i32(None, None, 0, None) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("off_in,off_out,off_tmp", [(1, 0, 0), (0, 3, 0), (0, 0, 2), (1, 1, 1)])
def test_naive_unaligned_views(gpu_device, off_in, off_out, off_tmp):
    """sc_naive_scan_i32 on torch views with a storage offset (4-byte aligned only): the 16-byte
    vector path is taken only when every base is 16-byte aligned, the scalar path otherwise (ADVICE
    r03); results equal the oracle.  Too-short output or scratch tensors are refused."""
    import torch
    n = 4099
    rng = np.random.default_rng(off_in * 7 + off_out * 3 + off_tmp)
    a = rng.integers(-1000, 1000, size=n, dtype=np.int64).astype(np.int32)
    big_in = torch.zeros(n + 8, dtype=torch.int32, device=gpu_device)
    big_in[off_in:off_in + n] = torch.from_numpy(a).to(gpu_device)
    d_in = big_in[off_in:off_in + n]
    d_out = torch.zeros(n + 8, dtype=torch.int32, device=gpu_device)[off_out:off_out + n]
    d_tmp = torch.zeros(n + 8, dtype=torch.int32, device=gpu_device)[off_tmp:off_tmp + n]
    P.naive_scan_device(d_in, d_out, d_tmp)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_out.cpu().numpy(), O.scan(a))
    with pytest.raises(ValueError):
        P.naive_scan_device(d_in, d_out[:-1], d_tmp)
    with pytest.raises(ValueError):
        P.naive_scan_device(d_in, d_out, d_tmp[:-1])
    with pytest.raises(ValueError):
        P.thrust_scan_device(d_in, d_out[:-1])

"""GPU parity of the stream-compaction kernels against the serial CPU oracle (bit-exact).

Reference behaviour: path_tracer/stream_compaction/cpu.cu:16-79 (oracle), efficient.cu:150-219
(product API), stream_compaction/src/main.cpp:14-146 (test shape: POT and NPOT sizes, last element
forced to 0, values rand()%50 for scan and rand()%4 for compaction).
"""
import numpy as np
import pytest

from oracle import binding as O

pytestmark = pytest.mark.gpu

SIZES = [1, 2, 3, 5, 63, 64, 65, 127, 128, 129, 255, 256, 257, 1000, 4095, 4096, 4097, 8191, 65536 + 17,
         (1 << 20) - 3, 1 << 20]


def _gen(n, maxval, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, maxval, size=n, dtype=np.int32)
    if n:
        a[-1] = 0          # main.cpp:23,98 "leave a 0 at the end"
    return a


@pytest.mark.parametrize("n", SIZES)
def test_scan_matches_oracle(gpu_device, n):
    import torch
    from cuda_pathtracer_amd import scan_device
    a = _gen(n, 50, n)
    d = torch.from_numpy(a).to(gpu_device)
    out = scan_device(d)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), O.scan(a))


@pytest.mark.parametrize("n", [1, 3, 129, 4097, 100003])
def test_scan_wraps_and_negatives(gpu_device, n):
    import torch
    from cuda_pathtracer_amd import scan_device
    rng = np.random.default_rng(7)
    a = rng.integers(-2**31, 2**31 - 1, size=n, dtype=np.int64).astype(np.int32)
    out = scan_device(torch.from_numpy(a).to(gpu_device)).cpu().numpy()
    np.testing.assert_array_equal(out, O.scan(a))


def test_scan_inplace_and_unaligned(gpu_device):
    import torch
    from cuda_pathtracer_amd import scan_device
    a = _gen(10000 + 3, 50, 3)
    d = torch.from_numpy(a).to(gpu_device)
    scan_device(d, d)                                    # in place
    np.testing.assert_array_equal(d.cpu().numpy(), O.scan(a))
    big = torch.from_numpy(np.concatenate([np.array([9], np.int32), a])).to(gpu_device)
    sub = big[1:]                                        # 4-byte aligned, not 16
    out = torch.empty_like(sub)
    scan_device(sub, out)
    np.testing.assert_array_equal(out.cpu().numpy(), O.scan(a))


@pytest.mark.parametrize("n", SIZES)
def test_compact_matches_oracle(gpu_device, n):
    import torch
    from cuda_pathtracer_amd import compact_device
    a = _gen(n, 4, n + 1)
    out, cnt = compact_device(torch.from_numpy(a).to(gpu_device))
    c = int(cnt.item())
    ref = O.compact_without_scan(a)
    assert c == len(ref)
    np.testing.assert_array_equal(out[:c].cpu().numpy(), ref)
    np.testing.assert_array_equal(ref, O.compact_with_scan(a))


@pytest.mark.parametrize("n", [1, 2, 65, 4097, 100000])
def test_partition_matches_keep(gpu_device, n):
    import torch
    from cuda_pathtracer_amd import partition_device
    f = _gen(n, 2, n + 5)
    perm, live = partition_device(torch.from_numpy(f).to(gpu_device))
    ref, ref_live = O.partition_indices(f)
    assert int(live.item()) == ref_live
    np.testing.assert_array_equal(perm.cpu().numpy(), ref)


@pytest.mark.parametrize("n", [1, 2, 65, 8192, 8193, 100000, 1 << 20])
def test_live_indices_match_keep(gpu_device, n):
    """sc_partition_indices: the live prefix of the stable partition, int32 count."""
    import torch
    from cuda_pathtracer_amd import live_indices_device
    f = _gen(n, 3, n + 7) * (np.arange(n) % 5 != 0)
    sentinel = torch.full((n,), -7, dtype=torch.int32, device=gpu_device)
    idx, cnt = live_indices_device(torch.from_numpy(f.astype(np.int32)).to(gpu_device), sentinel)
    ref, ref_live = O.partition_indices(f.astype(np.int32))
    assert cnt.dtype == torch.int32 and int(cnt.item()) == ref_live
    got = idx.cpu().numpy()
    np.testing.assert_array_equal(got[:ref_live], ref[:ref_live])
    assert (got[ref_live:] == -7).all()


def test_device_wrappers_check_option(gpu_device):
    """the asynchronous device entry points report a look-back stall only through the
    workspace's error word; check=True synchronises and reads it (sc_workspace_check).  On a GPU this
    process has to itself every call succeeds, and the results are the oracle's."""
    import torch
    from cuda_pathtracer_amd import compact_device, live_indices_device, partition_device, scan_device
    a = _gen(300_001, 50, 3)
    d = torch.from_numpy(a).to(gpu_device)
    np.testing.assert_array_equal(scan_device(d, check=True).cpu().numpy(), O.scan(a))
    out, cnt = compact_device(torch.from_numpy(_gen(300_001, 4, 4)).to(gpu_device), check=True)
    assert int(cnt.item()) == len(O.compact_without_scan(_gen(300_001, 4, 4)))
    f = _gen(100_000, 2, 5)
    perm, live = partition_device(torch.from_numpy(f).to(gpu_device), check=True)
    assert int(live.item()) == O.partition_indices(f)[1]
    idx, c2 = live_indices_device(torch.from_numpy(f).to(gpu_device), check=True)
    assert int(c2.item()) == O.partition_indices(f)[1]


def test_edge_cases(gpu_device):
    import torch
    from cuda_pathtracer_amd import compact_device, scan_device
    empty = torch.zeros(0, dtype=torch.int32, device=gpu_device)
    assert scan_device(empty).numel() == 0
    _, cnt = compact_device(empty)
    assert int(cnt.item()) == 0
    zeros = torch.zeros(5000, dtype=torch.int32, device=gpu_device)
    _, cnt = compact_device(zeros)
    assert int(cnt.item()) == 0
    ones = torch.ones(5000, dtype=torch.int32, device=gpu_device)
    np.testing.assert_array_equal(scan_device(ones).cpu().numpy(), np.arange(5000, dtype=np.int32))
    out, cnt = compact_device(ones)
    assert int(cnt.item()) == 5000


def test_host_api_reference_semantics(gpu_device):
    """Efficient::scan / compact with host arrays (efficient.cu:150-219), incl. n == 1."""
    from cuda_pathtracer_amd import Efficient
    for n in (1, 2, 7, 1 << 16, (1 << 16) - 3):
        a = _gen(n, 50, n)
        o = np.zeros(n, np.int32)
        Efficient.scan(n, o, a)
        np.testing.assert_array_equal(o, O.scan(a))
        assert Efficient.timer().getGpuElapsedTimeForPreviousOperation() >= 0.0
        b = _gen(n, 4, n + 9)
        o2 = np.zeros(n, np.int32)
        cnt = Efficient.compact(n, o2, b)
        ref = O.compact_without_scan(b)
        assert cnt == len(ref)
        np.testing.assert_array_equal(o2[:cnt], ref)
    # the reference's known-answer vectors (stream_compaction/INSTRUCTION.md:262-302)
    a = np.array([1, 5, 0, 1, 2, 0, 3], np.int32)
    o = np.zeros(7, np.int32)
    Efficient.scan(7, o, a)
    assert o.tolist() == [0, 1, 6, 6, 7, 9, 9]
    assert Efficient.compact(7, o, a) == 5 and o[:5].tolist() == [1, 5, 1, 2, 3]


@pytest.mark.parametrize("n", [1 << 26, (1 << 26) + 12345, (1 << 27) + 5])
def test_large_inputs_match_oracle(gpu_device, n):
    """Inputs past the 256 MiB Infinity Cache take the two-pass super-round kernel
    (sc_kernels.hip k_scan_mall): full-array parity for scan, compaction and partition."""
    import torch
    from cuda_pathtracer_amd import compact_device, partition_device, scan_device
    a = _gen(n, 50, n)
    d = torch.from_numpy(a).to(gpu_device)
    np.testing.assert_array_equal(scan_device(d).cpu().numpy(), O.scan(a))
    f = (a % 4).astype(np.int32)
    df = torch.from_numpy(f).to(gpu_device)
    out, cnt = compact_device(df)
    ref = O.compact_without_scan(f)
    assert int(cnt.item()) == len(ref)
    np.testing.assert_array_equal(out[:len(ref)].cpu().numpy(), ref)
    del out
    perm, live = partition_device(df)
    ref_perm, ref_live = O.partition_indices(f)
    assert int(live.item()) == ref_live
    np.testing.assert_array_equal(perm.cpu().numpy(), ref_perm)
    del d, df, perm
    torch.cuda.empty_cache()


@pytest.mark.slow
def test_reference_size_2e28_properties(gpu_device):
    """SIZE = 1<<28 and NPOT = SIZE-3 (main.cpp:8-9): the whole scan against the oracle, plus the
    size-independent checks on the device (difference identity, compaction count and order)."""
    import torch
    from cuda_pathtracer_amd import compact_device, scan_device
    for n in ((1 << 28), (1 << 28) - 3):
        g = torch.Generator(device=gpu_device).manual_seed(1234)
        a = torch.randint(0, 50, (n,), dtype=torch.int32, device=gpu_device, generator=g)
        a[-1] = 0
        s = scan_device(a)
        # exclusive scan: s[i+1] - s[i] == a[i] (int32 wrap), s[0] == 0
        assert int(s[0].item()) == 0
        diff = (s[1:] - s[:-1])
        assert bool(torch.equal(diff, a[:-1]))
        # the whole array against the oracle (O.scan: ~0.1 s on the host at 2^28)
        ah = a.cpu().numpy()
        np.testing.assert_array_equal(s.cpu().numpy(), O.scan(ah))
        del s, diff, ah
        f = (a % 4).to(torch.int32)
        out, cnt = compact_device(f)
        nz = int((f != 0).sum().item())
        assert int(cnt.item()) == nz
        assert bool(torch.equal(out[:nz], f[f != 0]))
        del a, f, out
        torch.cuda.empty_cache()


def test_concurrent_streams_make_progress(gpu_device):
    """Two large scans and two compactions in flight at once on separate streams: each kernel is
    sized to fill the GPU, so neither can have its whole grid resident.  In the claimed tile
    schedule (lookback.h TileSeq) tiles are claimed in order from a ticket, so the look-back still
    completes (the static schedule assumes a fully resident grid)."""
    import torch
    from cuda_pathtracer_amd._native import check_sc, lib
    n = (1 << 24) + 777
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    a = torch.randint(0, 50, (n,), dtype=torch.int32, device=gpu_device)
    b = torch.randint(0, 4, (n,), dtype=torch.int32, device=gpu_device)
    oa, ob = torch.empty_like(a), torch.empty_like(b)
    cnt = torch.zeros(1, dtype=torch.int64, device=gpu_device)
    wa = torch.empty(int(lib().sc_workspace_bytes(n)), dtype=torch.uint8, device=gpu_device)
    wb = torch.empty_like(wa)
    torch.cuda.synchronize()
    check_sc(lib().sc_set_tile_schedule(1))      # claimed tiles: safe when kernels share the GPU
    try:
        for _ in range(4):
            check_sc(lib().sc_scan_exclusive_i32(a.data_ptr(), oa.data_ptr(), n, wa.data_ptr(), s1.cuda_stream))
            check_sc(lib().sc_compact_i32(b.data_ptr(), ob.data_ptr(), n, cnt.data_ptr(), wb.data_ptr(),
                                          s2.cuda_stream))
        torch.cuda.synchronize()
    finally:
        check_sc(lib().sc_set_tile_schedule(0))
    ha, hb = a.cpu().numpy(), b.cpu().numpy()
    np.testing.assert_array_equal(oa.cpu().numpy(), O.scan(ha))
    ref = O.compact_without_scan(hb)
    assert int(cnt.item()) == len(ref)
    np.testing.assert_array_equal(ob[:len(ref)].cpu().numpy(), ref)


@pytest.mark.parametrize("n", [1, 8191, 8193, 100003, (1 << 20) + 5, (1 << 24) + 3])
def test_claimed_schedule_matches_oracle(gpu_device, n):
    """The claimed tile schedule gives the same bits as the static one (scan, compact, partition)."""
    import torch
    from cuda_pathtracer_amd import compact_device, partition_device, scan_device
    from cuda_pathtracer_amd._native import check_sc, lib
    a = _gen(n, 50, n + 11)
    f = (a % 4).astype(np.int32)
    check_sc(lib().sc_set_tile_schedule(1))
    try:
        s = scan_device(torch.from_numpy(a).to(gpu_device)).cpu().numpy()
        out, cnt = compact_device(torch.from_numpy(f).to(gpu_device))
        perm, live = partition_device(torch.from_numpy(f).to(gpu_device))
        torch.cuda.synchronize()
    finally:
        check_sc(lib().sc_set_tile_schedule(0))
    np.testing.assert_array_equal(s, O.scan(a))
    ref = O.compact_without_scan(f)
    assert int(cnt.item()) == len(ref)
    np.testing.assert_array_equal(out[:len(ref)].cpu().numpy(), ref)
    ref_perm, ref_live = O.partition_indices(f)
    assert int(live.item()) == ref_live
    np.testing.assert_array_equal(perm.cpu().numpy(), ref_perm)


_STALL_SCRIPT = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
from cuda_pathtracer_amd._native import lib
L = lib()
torch.cuda.set_device(0)
n = 1 << 25
a = torch.randint(0, 50, (n,), dtype=torch.int32, device="cuda")
out = torch.empty_like(a)
ws = torch.empty(int(L.sc_workspace_bytes(n)), dtype=torch.uint8, device="cuda")
assert L.sc_scan_exclusive_i32(a.data_ptr(), out.data_ptr(), n, ws.data_ptr(), None) == 0   # async: no error yet
rc = L.sc_workspace_check(ws.data_ptr())
msg = L.sc_last_error().decode()
h = np.random.default_rng(0).integers(0, 50, n, dtype=np.int32)
ho = np.zeros_like(h)
rc2 = L.sc_efficient_scan(n, ho.ctypes.data, h.ctypes.data)
L.sc_set_tile_schedule(1)                                   # claimed tiles: no co-residency needed
rc3 = L.sc_efficient_scan(n, ho.ctypes.data, h.ctypes.data)
ok3 = bool((ho[1:] - ho[:-1] == h[:-1]).all()) and ho[0] == 0
print("RESULT", rc, rc2, rc3, ok3, "|", msg)
"""


def test_static_schedule_stall_is_reported(gpu_device, tmp_path):
    """a static-schedule scan whose grid is not co-resident (forced here with the
    PT_AMD_TEST_SCAN_OVERSUB=4 hook of the test-hook build: 4x the resident grid) hits its bounded spin; the device
    error word is read back — sc_workspace_check and the host-pointer helper return SC_ERR_HIP
    instead of SC_OK with wrong prefixes — and the claimed schedule still completes correctly."""
    import os
    import subprocess
    import sys
    from pathlib import Path
    root = str(Path(__file__).resolve().parent.parent)
    hooks = Path(root) / "cuda_pathtracer_amd" / "build" / "libpt_amd_testhooks.so"   # build.build_test_hooks
    assert hooks.exists(), "test-hook library missing (build() builds it)"
    env = dict(os.environ, PT_AMD_TEST_SCAN_OVERSUB="4", PT_AMD_LIB=str(hooks))
    res = subprocess.run([sys.executable, "-c", _STALL_SCRIPT, root], env=env, capture_output=True, text=True,
                         timeout=120)
    line = [x for x in res.stdout.splitlines() if x.startswith("RESULT")]
    assert res.returncode == 0 and line, res.stdout + res.stderr
    rc, rc2, rc3, ok3 = line[0].split("|")[0].split()[1:5]
    assert int(rc) == 2 and int(rc2) == 2, line[0]          # SC_ERR_HIP: spin bound reported
    assert "spin bound" in line[0]
    assert int(rc3) == 0 and ok3 == "True", line[0]

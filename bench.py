"""Benchmark: Mray/s (paths x bounces / s) on the bundled Cornell scene + scan GB/s vs HBM peak.

Workload (BASELINE.json configs[1]): path_tracer/scenes/cornell.json as-is — 800x800, DEPTH 8,
default flags.  A step renders a FIXED 256 samples per pixel of the whole image (strong scaling,
the default): on N GPUs (one process per GPU, torchrun) rank r owns the image rows y % N == r and
traces its rows' 256 iterations as passes of `--spp` iterations (default: one pass of 256 at every
N; 2 x 128 at N = 1 measured 0.5% slower), so the work per step is the same at every N and the driver's 1/2/4/8
values measure speed-up.  Batching iterations into one pass is bit-identical to tracing them one
pass at a time (tests/test_render_gpu.py::test_batched_pass_equals_sequential_passes); --spp 1
--samples 1 is exactly the reference's pathtrace() per step.  --scaling weak: a step is one pass of
spp x N iterations of the rank's rows per GPU.  After the timed passes the float tiles are gathered
to rank 0 with one RCCL gather (inside the timed region, timed separately as gather_ms; one
untimed gather of the same shape before the timed region sets up RCCL's connections).
value = all ranks' traced segments / max-over-ranks wall time / 1e6.

Roofline: the dominant kernel of analytic scenes is the fused bounce kernel k_bounce<false,...>
(bounces >= 1); of mesh scenes (config 5) the BVH walk k_traverse4<false> (bounces >= 1), with the
bounce kernel that follows it reported beside it (roofline.bounce_kernel).  Launch times come from HIP
events recorded on the launch stream, per kernel kind, over a profiled segment of the same workload;
the kernel's time per launch is the union of its launch intervals / launches (effective_launch_ms:
the two lanes' launches overlap, and launches x it fits the step; rocprofv3 --kernel-trace of the same
command agrees: profiles/r0*_union_check.txt).  The roofline names the BINDING resource
(_finalize_roofline): the in-run rocprofv3 --pmc passes (scripts/pmc.py) give the kernel's fabric
traffic (FETCH_SIZE x 2 + WRITE_SIZE) and its VALU wave-instructions per launch; when the traffic is
below half the HBM peak the bound is "issue" and achieved / peak / frac are the VALU issue rate's
(256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction, MI355X_MICROARCH.md).  The byte
figures stay beside it under roofline.hbm: SURVEY.md §8d's 184 B per traced segment (a MODEL — ray 24
+ hit write 28 + hit read 28 + path read 48 + write 48 + compaction 8; the fused kernel keeps the hit
in registers), the kernel's own minimum bytes (40 B in + 40 B per survivor + 24 B per emissive hit;
path planes of 16 + 16 + 8 B) and the counters' traffic, each over effective_launch_ms.
roofline.step_model_ratio = the §8d bytes of every bounce of a step / ms_per_step / 8 TB/s (a model
ratio: above 1 it is flagged in model_ratios_above_1).  For the BVH walk also its memory
instructions, L2 hit rate and, with the diagnostic counter build (build.py build_trav_stats), the
walk's lane counters (scripts/trav_stats.py).
The scan kernel is measured separately at n = 2^28 (8 B/element, 2 GiB, beyond the 256 MiB MALL).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "Mray/s (paths×bounces/s) on Cornell scene + scan GB/s vs HBM peak, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
HBM_COPY_GBS = 6290.0          # same guide: measured float4 copy, the achievable streaming rate (79%)
VALU_PEAK = 256 * 4 * 2.4e9 / 2   # wave64 VALU instructions/s: 4 SIMD-32 per CU, 2 cycles each (same guide)
SEGMENT_BYTES = 184            # SURVEY.md §8d algorithmic bytes per traced segment
PATH_BYTES = 40                # fused kernel's path state: planes (o, d.x) 16 + (d.yz, c.rg) 16 + (c.b, slot) 8
FB_RMW_BYTES = 24              # float3 read + write


def _log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def _host_cpu() -> str:
    """lscpu-style model name and logical CPU count of this host (SURVEY.md §8d asks for both)."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return f"{model}; nproc={os.cpu_count()}"


def cpu_baseline_render(seconds_target: float) -> dict:
    """The oracle (serial C++ restatement of the reference renderer) on this host, 1 thread."""
    from oracle import binding as O
    sc = O.OracleScene.from_json(ROOT / "tests" / "scenes" / "cornell.json")
    fl = O.flags()
    total_seg, total_t, iters = 0, 0.0, 0
    while total_t < seconds_target and iters < 64:
        _, live, secs = O.render(sc, fl, 1, iter_first=iters + 1)
        total_seg += sum(live)
        total_t += secs
        iters += 1
    return {"value": total_seg / total_t / 1e6, "unit": "Mray/s", "cores": 1, "kind": "port", "host": _host_cpu(),
            "sample": f"{iters} iteration(s) of cornell.json 800x800 DEPTH 8 default flags, "
                      f"{total_seg} segments in {total_t:.2f} s (oracle/pt_oracle.cpp, g++ -O2, 1 thread)"}


def cpu_baseline_render_mt(seconds_target: float, threads: int) -> dict:
    """The same oracle on `threads` host cores: each thread renders the rows y % threads == t of
    every iteration (independent pixel shards, as the GPUs of bench.py do; ctypes releases the
    GIL during the C call).  A labelled multithreaded variant of the reference's serial CPU path."""
    import threading
    from oracle import binding as O
    sc = O.OracleScene.from_json(ROOT / "tests" / "scenes" / "cornell.json")
    fl = O.flags()
    total_seg, iters = 0, 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds_target and iters < 256:
        lives = [None] * threads

        def work(r, it=iters + 1):
            lives[r] = O.render_pass(sc, fl, it, rank=r, world=threads)[1]
        ts = [threading.Thread(target=work, args=(r,)) for r in range(threads)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        total_seg += sum(sum(lv) for lv in lives)
        iters += 1
    secs = time.perf_counter() - t0
    return {"value": total_seg / secs / 1e6, "unit": "Mray/s", "cores": threads, "kind": "port", "host": _host_cpu(),
            "sample": f"{iters} iteration(s) of cornell.json 800x800 DEPTH 8 default flags on {threads} threads "
                      f"(row shards), {total_seg} segments in {secs:.2f} s (oracle/pt_oracle.cpp, g++ -O2)"}


def cpu_baseline_scan(n: int = 1 << 20, reps: int = 50) -> dict:
    """CPU::scan (cpu.cu:16-33) restated, 1 thread, timed like PerformanceTimer (common.h:61-80)."""
    from oracle import binding as O
    a = np.random.default_rng(1234).integers(0, 50, n, dtype=np.int32)
    a[-1] = 0
    out = np.zeros_like(a)
    O.lib().oracle_scan(n, out.ctypes.data, a.ctypes.data)  # warm
    ms = O.lib().oracle_time_scan_ms(n, a.ctypes.data, out.ctypes.data, reps) / reps
    return {"n": n, "ms": ms, "GB/s": 8.0 * n / (ms * 1e-3) / 1e9, "cores": 1, "kind": "port", "host": _host_cpu(),
            "sample": f"CPU::scan restated (oracle/sc_oracle.cpp), {reps} reps, U[0,50) seed 1234"}


def cpu_baseline_compact(n: int = 1 << 20, reps: int = 20) -> dict:
    """CPU::compactWithScan and CPU::compactWithoutScan (cpu.cu:40-79) restated, 1 thread, on
    SC/src/main.cpp's compaction input shape (U[0,4), last element 0; ~75% kept).  GB/s at the
    algorithmic 4 B read per element + 4 B written per kept element."""
    import ctypes as C
    from oracle import binding as O
    a = np.random.default_rng(4321).integers(0, 4, n, dtype=np.int32)
    a[-1] = 0
    out = np.zeros_like(a)
    res = {"n": n, "cores": 1, "kind": "port", "host": _host_cpu(),
           "sample": f"oracle/sc_oracle.cpp, {reps} reps, U[0,4) seed 4321"}
    for name, fn in (("with_scan", O.lib().oracle_time_compact_ms),
                     ("without_scan", O.lib().oracle_time_compact_without_scan_ms)):
        cnt = C.c_int64(0)
        fn(n, a.ctypes.data, out.ctypes.data, 1, C.byref(cnt))  # warm
        ms = fn(n, a.ctypes.data, out.ctypes.data, reps, C.byref(cnt)) / reps
        res[name] = {"ms": ms, "kept": cnt.value, "GB/s": (4.0 * n + 4.0 * cnt.value) / (ms * 1e-3) / 1e9}
    return res


def scan_bench(torch, dev, n: int, reps: int) -> dict:
    import cuda_pathtracer_amd as P
    from cuda_pathtracer_amd._native import check_sc, lib
    g = torch.Generator(device=dev).manual_seed(1234)
    a = torch.randint(0, 50, (n,), dtype=torch.int32, device=dev, generator=g)
    out = torch.empty_like(a)
    ws = torch.empty(int(lib().sc_workspace_bytes(n)), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    for _ in range(3):
        check_sc(lib().sc_scan_exclusive_i32(a.data_ptr(), out.data_ptr(), n, ws.data_ptr(), st.cuda_stream))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st)
        check_sc(lib().sc_scan_exclusive_i32(a.data_ptr(), out.data_ptr(), n, ws.data_ptr(), st.cuda_stream))
        e1.record(st)
    torch.cuda.synchronize()
    times = sorted(e0.elapsed_time(e1) for e0, e1 in ev)
    ms = float(np.mean(times))
    # correctness of the timed output: exclusive-scan identity on the device
    ok = bool(torch.equal(out[1:] - out[:-1], a[:-1])) and int(out[0].item()) == 0
    del P
    gbs = 8.0 * n / (ms * 1e-3) / 1e9
    return {"n": n, "ms": ms, "ms_min": times[0], "GB/s": gbs, "verified": ok,
            "roofline": {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": gbs / HBM_PEAK_GBS, "copy_ceiling": HBM_COPY_GBS,
                         "frac_of_copy_ceiling": gbs / HBM_COPY_GBS,
                         "copy_ceiling_source": "MI355X_MICROARCH.md: float4 copy measured at 6.29 TB/s"}}


def compact_bench(torch, dev, n: int, reps: int) -> dict:
    """sc_compact_i32 (Efficient::compact, efficient.cu:185-219) on n ints U[0,4) (SC/src/main.cpp's
    compaction input shape, ~75% kept): algorithmic bytes = 4 B read per element + 4 B per kept."""
    from cuda_pathtracer_amd._native import check_sc, lib
    g = torch.Generator(device=dev).manual_seed(4321)
    a = torch.randint(0, 4, (n,), dtype=torch.int32, device=dev, generator=g)
    out = torch.empty_like(a)
    cnt = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = torch.empty(int(lib().sc_workspace_bytes(n)), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    for _ in range(3):
        check_sc(lib().sc_compact_i32(a.data_ptr(), out.data_ptr(), n, cnt.data_ptr(), ws.data_ptr(), st.cuda_stream))
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for e0, e1 in ev:
        e0.record(st)
        check_sc(lib().sc_compact_i32(a.data_ptr(), out.data_ptr(), n, cnt.data_ptr(), ws.data_ptr(), st.cuda_stream))
        e1.record(st)
    torch.cuda.synchronize()
    ms = float(np.mean([e0.elapsed_time(e1) for e0, e1 in ev]))
    kept = int(cnt.item())
    ok = kept == int((a != 0).sum().item()) and bool(torch.equal(out[:kept], a[a != 0]))
    gbs = (4.0 * n + 4.0 * kept) / (ms * 1e-3) / 1e9
    return {"n": n, "kept": kept, "ms": ms, "GB/s": gbs, "frac": gbs / HBM_PEAK_GBS, "verified": ok}


def dropin_bench(scene_path: str, iters: int = 50, warmup: int = 3) -> dict:
    """The drop-in call sequence a reference caller gets: `iters` calls of the C++ mirror's
    pathtrace(nullptr, 0, it) (host/pathtrace.cpp: the per-call pt_set_flags of pathtrace.cu:438-463,
    one iteration, and the synchronous image copy of pathtrace.cu:524), as main.cpp:114-168's loop
    issues them (host/dropin_bench.cpp through libpt_dropin.so)."""
    import ctypes as C
    lib = C.CDLL(str(ROOT / "cuda_pathtracer_amd" / "libpt_dropin.so"))
    fn = lib.pt_dropin_bench
    fn.restype = C.c_int
    fn.argtypes = [C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
    ms, seg, syncs = C.c_double(), C.c_uint64(), C.c_uint64()
    rc = fn(str(scene_path).encode(), warmup, iters, C.byref(ms), C.byref(seg), C.byref(syncs))
    if rc != 0:
        return {"error": f"pt_dropin_bench rc={rc}"}
    return {"value": seg.value / (ms.value * 1e-3) / 1e6, "unit": "Mray/s", "calls": iters,
            "ms_per_call": ms.value / iters, "segments": seg.value, "flag_syncs": syncs.value,
            "render_ahead": os.environ.get("PT_AMD_AHEAD", "1") != "0",
            "definition": f"{iters} calls of the C++ mirror's pathtrace(nullptr, 0, it) on the same scene (one "
                          "iteration each: per-call pt_set_flags, pt_render_pass, synchronous 7.7 MB image copy "
                          f"to the host, as pathtrace.cu:438-524), after {warmup} warm-up calls; segments / wall time. "
                          "Each call queues the next iteration's bounces before its copy (pt_render_ahead), and "
                          "the next call claims them; segments count claimed iterations only"}


def _pmc_leg(args, scene_path, spp_pass, sorted_, avg_ms, kernel_prefix, seg_per_launch, busy_ms, launches,
             walk=False):
    """rocprofv3 --pmc passes over the same workload (scripts/pmc.py): fabric traffic and VALU
    wave-instructions per launch of the dominant kernel, and its wave-state split; for the BVH walk
    (walk=True) also its memory instructions and L2 hit rate."""
    sys.path.insert(0, str(ROOT / "scripts"))
    import pmc
    wl = [str(args.pmc_passes), f"spp={spp_pass}", f"scene={scene_path}"] + (["sort"] if sorted_ else []) + \
         (["bvhcull"] if args.bvh_cull else [])
    out_dir = ROOT / "gpurun_out" / "bench_pmc"
    groups = ("fetch", "write", "sq") + (("l2", "vmem") if walk else ())
    res = pmc.collect(wl, out_dir, timeout=args.pmc_timeout, groups=groups)
    (out_dir / "summary.json").write_text(json.dumps(res, indent=1))
    if sorted_:   # the sorted pipeline: every kernel of a bounce, per traced segment
        # bounces >= 1 only, like the numerator: the first producer (camera rays, k_sort_produce<true>)
        # is left out of the bytes, and bounce 0's paths out of the segments
        ks = {k: m for k, m in res.get("kernels", {}).items()
              if k.startswith(("k_sort_", "k_hist_", "k_scan_lag", "k_scan_tiles"))
              and not k.startswith("k_sort_produce<true")}
        if not ks or not all("bytes_per_launch" in m for m in ks.values()):
            return {"pmc": res["_passes"]}
        total = sum(m["bytes_per_launch"] * m["launches"] for m in ks.values())
        live = res.get("bounce_live")
        segs = sum(live[1:]) if live else 0
        first = next((m for k, m in res.get("kernels", {}).items() if k.startswith("k_sort_produce<true")), None)
        out = {"pmc": res["_passes"], "traffic_per_segment": total / segs if segs else None,
               "traffic_definition": "FETCH_SIZE x 2 + WRITE_SIZE of the sorted-pipeline kernels of bounces >= 1 "
                                     "(every k_sort_produce<false> + the histogram scans) over the profiled passes "
                                     "/ their traced segments of bounces >= 1; traffic = that x segments per "
                                     "pipeline bounce, like algorithmic_bytes_per_launch",
               "first_producer_bytes_per_path": (first["bytes_per_launch"] * first["launches"] / live[0])
               if first and "bytes_per_launch" in first and live and live[0] else None,
               "traffic_kernels": sorted(ks)}
        if segs:
            out["traffic"] = total / segs * seg_per_launch
            out["traffic_frac"] = out["traffic"] / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS
            if out["traffic_frac"] < 0.5:   # measured traffic far below the HBM peak (as for k_bounce)
                out["bound"] = "issue"
            if all("SQ_INSTS_VALU" in m for m in ks.values()):
                valu = sum(m["SQ_INSTS_VALU"] * m["launches"] for m in ks.values()) / segs * seg_per_launch
                out["valu_issue"] = {
                    "unit": "wave64 VALU instr/s", "peak": VALU_PEAK, "instructions_per_launch": valu,
                    "instructions_per_segment": valu / max(seg_per_launch, 1.0),
                    "achieved": valu / (avg_ms * 1e-3), "frac": valu / (avg_ms * 1e-3) / VALU_PEAK,
                    "definition": "SQ_INSTS_VALU of the sorted-pipeline kernels of bounces >= 1 (as traffic_kernels) "
                                  "per traced segment x segments per pipeline bounce / the pipeline bounce's time "
                                  "(roofline.effective_launch_ms) / (256 CUs x 4 SIMDs x 2.4 GHz / 2)"}
        return out
    m = pmc.pick(res, kernel_prefix)
    if m is None or "bytes_per_launch" not in m:
        return {"pmc": res["_passes"]}
    out = {"pmc": res["_passes"], "traffic": m["bytes_per_launch"],
           "traffic_per_segment": m["bytes_per_launch"] / max(seg_per_launch, 1.0),
           "traffic_frac": m["bytes_per_launch"] / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    iso_ns = m.get("dur_ns_sq") or m.get("dur_ns_fetch")
    if iso_ns:   # rocprofv3 --pmc serialises the dispatches: each launch alone on the GPU
        iso_ms = iso_ns * 1e-6
        out["isolated"] = {
            "avg_launch_ms": iso_ms,
            "achieved": SEGMENT_BYTES * seg_per_launch / (iso_ms * 1e-3) / 1e9,
            "frac": SEGMENT_BYTES * seg_per_launch / (iso_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "definition": "the same 184 B x segments per launch over the launch's duration in the rocprofv3 --pmc "
                          "passes, where dispatches run one at a time (the line's avg_launch_ms shares the GPU "
                          "with the other lane's launches)"}
    if "SQ_INSTS_VALU" in m:
        valu = m["SQ_INSTS_VALU"]
        wc = max(m.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        act, wi, wa = (m.get("SQ_ACTIVE_INST_ANY", 0.0) / wc, m.get("SQ_WAIT_INST_ANY", 0.0) / wc,
                       m.get("SQ_WAIT_ANY", 0.0) / wc)
        dur = m.get("dur_ns_sq", 0.0)
        out["valu_issue"] = {
            "unit": "wave64 VALU instr/s", "peak": VALU_PEAK,
            "instructions_per_launch": valu, "instructions_per_segment": valu / max(seg_per_launch, 1.0),
            "achieved": valu / (avg_ms * 1e-3), "frac": valu / (avg_ms * 1e-3) / VALU_PEAK,
            "aggregate_frac": valu * launches / (busy_ms * 1e-3) / VALU_PEAK if busy_ms > 0 else None,
            "salu_per_launch": m.get("SQ_INSTS_SALU"),
            "effective_clock_ghz": m["GRBM_GUI_ACTIVE"] / 8.0 / dur if dur > 0 and "GRBM_GUI_ACTIVE" in m else None,
            "definition": "SQ_INSTS_VALU per launch / the kernel's time per launch (roofline.effective_launch_ms) "
                          "/ (256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction)"}
        out["wave_states"] = {"issuing": act, "waiting_on_issue": wi, "waiting_on_memory_or_barrier": wa,
                              "waves_per_launch": m.get("SQ_WAVES")}
        out["limiter"] = (f"VALU issue + latency, not bandwidth: waves issue {act:.0%} of their cycles, wait on "
                          f"dependencies/arbitration {wi:.0%}, on memory/LDS/barriers {wa:.0%}; fabric traffic "
                          f"{out['traffic_frac']:.0%} of the HBM peak")
        # the bound, from the counters: the measured fabric traffic is far below the HBM peak while
        # the waves spend their cycles issuing or waiting to issue -> issue/latency-bound (`frac`
        # stays the prescribed 184 B / launch time / HBM peak)
        if out["traffic_frac"] < 0.5:
            out["bound"] = "issue"
    if walk:
        if "TCC_HIT_sum" in m:
            out["l2_hit_rate"] = m["TCC_HIT_sum"] / max(m["TCC_HIT_sum"] + m.get("TCC_MISS_sum", 0.0), 1.0)
        if "SQ_INSTS_VMEM_RD" in m:
            out["vmem_rd_per_launch"] = m["SQ_INSTS_VMEM_RD"]
            out["vmem_rd_per_segment"] = m["SQ_INSTS_VMEM_RD"] / max(seg_per_launch, 1.0)
        out["salu_per_segment"] = (m.get("SQ_INSTS_SALU") or 0.0) / max(seg_per_launch, 1.0)
    return out


def _finalize_roofline(r: dict) -> None:
    """The line's roofline names the kernel's BINDING resource.

    Byte figures, each over the kernel's time per launch (effective_launch_ms, the union of its launch
    intervals / launches: launches x it fits the step):
      hbm.model_184B     — SURVEY.md §8d's 184 B per traced segment (ray 24 + hit 28 + 28 + path 48 + 48 +
                           compaction 8).  A MODEL: the fused kernel keeps the hit record in registers and
                           never moves most of these bytes;
      hbm.kernel_min     — the fused kernel's own minimum bytes (path planes in, survivors out, emissive
                           colour read-modify-write: kernel_min_bytes_per_launch);
      hbm.counter_traffic— measured fabric traffic (rocprofv3 --pmc FETCH_SIZE x 2 + WRITE_SIZE, in-run).
    VALU issue (when the --pmc passes ran): SQ_INSTS_VALU per launch / effective_launch_ms / VALU_PEAK.
    bound = "hbm" when the measured traffic reaches half the HBM peak, else "issue" — then the top-level
    achieved / peak / unit / frac are the VALU issue rate's, and the byte figures stay under "hbm".
    Without --pmc: the §8d model's fraction, labelled as such.  Every reported fraction is <= 1 unless
    listed in fractions_above_1 (with the reason)."""
    eff = r.get("effective_launch_ms") or r.get("avg_launch_ms") or 0.0
    secs = eff * 1e-3
    hbm = {"peak": HBM_PEAK_GBS, "unit": "GB/s"}
    model = r.get("algorithmic_bytes_per_launch")
    if model is not None and secs > 0:
        hbm["model_184B"] = {"bytes_per_launch": model, "achieved": model / secs / 1e9,
                             "frac": model / secs / 1e9 / HBM_PEAK_GBS,
                             "definition": "SURVEY.md §8d model: 184 B x segments per launch / effective_launch_ms"}
    kmin = r.get("kernel_min_bytes_per_launch")
    if kmin is not None and secs > 0:
        hbm["kernel_min"] = {"bytes_per_launch": kmin, "achieved": kmin / secs / 1e9,
                             "frac": kmin / secs / 1e9 / HBM_PEAK_GBS,
                             "per_segment": kmin / max(r.get("segments_per_launch") or 1.0, 1.0),
                             "definition": "the fused kernel's own minimum bytes (40 B path in, 40 B per survivor "
                                           "out, 24 B per emissive hit) / effective_launch_ms"}
    if r.get("traffic") is not None and secs > 0:
        hbm["counter_traffic"] = {"bytes_per_launch": r["traffic"], "achieved": r["traffic"] / secs / 1e9,
                                  "frac": r["traffic"] / secs / 1e9 / HBM_PEAK_GBS,
                                  "per_segment": r.get("traffic_per_segment"),
                                  "definition": "rocprofv3 --pmc FETCH_SIZE x 2 + WRITE_SIZE per launch (in-run "
                                                "passes of the same workload) / effective_launch_ms"}
    r["hbm"] = hbm
    v = r.get("valu_issue")
    counters = hbm.get("counter_traffic")
    if v and v.get("instructions_per_launch") and secs > 0:
        v["frac"] = v["instructions_per_launch"] / secs / VALU_PEAK
        v["achieved"] = v["instructions_per_launch"] / secs
    if v and counters and counters["frac"] < 0.5:
        r["bound"] = "issue"
        r["achieved"], r["peak"], r["unit"], r["frac"] = v["achieved"], VALU_PEAK, "wave64 VALU instr/s", v["frac"]
        r["definition"] = ("binding resource: VALU issue — SQ_INSTS_VALU per launch (rocprofv3 --pmc, in-run) / "
                           "effective_launch_ms (union of the kernel's launch intervals / launches) / "
                           "(256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction); measured fabric "
                           f"traffic is {counters['frac']:.2f} of the HBM peak (hbm.counter_traffic)")
    elif counters and counters["frac"] >= 0.5:
        r["bound"] = "hbm"
        r["achieved"], r["peak"], r["unit"], r["frac"] = counters["achieved"], HBM_PEAK_GBS, "GB/s", counters["frac"]
        r["definition"] = "binding resource: HBM — measured fabric traffic per launch / effective_launch_ms / 8 TB/s"
    elif "model_184B" in hbm:
        r["bound"] = "hbm"
        r["achieved"], r["peak"], r["unit"], r["frac"] = (hbm["model_184B"]["achieved"], HBM_PEAK_GBS, "GB/s",
                                                          hbm["model_184B"]["frac"])
        r["definition"] = ("no counters in this run (--no-pmc): SURVEY.md §8d MODEL bytes (184 B per segment) / "
                           "effective_launch_ms / 8 TB/s — a model, not measured traffic")
    above = []
    def walk(d, path):
        for k, x in d.items():
            if isinstance(x, dict):
                walk(x, path + [k])
            elif k in ("frac", "aggregate_frac") and isinstance(x, (int, float)) and x > 1.0:
                above.append(".".join(path + [k]))
    walk(r, [])
    notes = {}
    if (r.get("step_model_ratio") or 0) > 1.0:
        notes["step_model_ratio"] = ("> 1: the §8d model counts bytes the fused kernel never moves (hit records "
                                     "stay in registers), so the model saturates; it is not an HBM fraction")
    r["fractions_above_1"] = above
    r["model_ratios_above_1"] = notes


def _walk_counters(scene_path, spp_pass, timeout=300) -> dict | None:
    """The BVH walk's lane counters from the diagnostic build (cuda_pathtracer_amd/build.py build_trav_stats ->
    cuda_pathtracer_amd/build/libpt_amd_trav.so; scripts/trav_stats.py), one pass of the same
    scene in a subprocess, or None when the diagnostic library is absent."""
    import subprocess
    if not (ROOT / "cuda_pathtracer_amd" / "build" / "libpt_amd_trav.so").exists():
        return None
    try:
        r = subprocess.run([sys.executable, str(ROOT / "scripts" / "trav_stats.py"), str(scene_path), str(spp_pass)],
                           capture_output=True, text=True, timeout=timeout, cwd=str(ROOT))
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    line = (r.stdout.strip().splitlines() or [""])[-1]
    out: dict = {"rc": r.returncode}
    for kv in line.split():
        if "=" in kv:
            k, v = kv.split("=", 1)
            try:
                out[k] = float(v) if "." in v else int(v)
            except ValueError:
                out[k] = v
    out["definition"] = "scripts/trav_stats.py (diagnostic -DPT_TRAV_STATS build, one pass of the same scene)"
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--scan-n", type=int, default=1 << 28)
    ap.add_argument("--scan-reps", type=int, default=20)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-scan", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 --pmc passes (traffic, VALU issue)")
    ap.add_argument("--pmc-passes", type=int, default=6)
    ap.add_argument("--no-walk-counters", action="store_true",
                    help="mesh scenes: skip the BVH walk's lane counters (diagnostic build, scripts/trav_stats.py)")
    ap.add_argument("--pmc-timeout", type=int, default=150)
    ap.add_argument("--scene", default=str(ROOT / "tests" / "scenes" / "cornell.json"))
    ap.add_argument("--config", default="cornell", choices=["cornell", "cornell_hd_sorted", "multi_object_4k",
                                                           "random_triangles_100k", "tessellated_meshes_100k"],
                    help="BASELINE.json workload: cornell (configs[1], the default line) or configs 3-5 "
                         "generated by cuda_pathtracer_amd.scenes")
    ap.add_argument("--bvh-cull", action="store_true", help="pt_flags.bvh_cull extension (mesh scenes)")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the drop-in leg (50 per-iteration pathtrace() calls of the C++ mirror, N = 1)")
    ap.add_argument("--spp", type=int, default=None,
                    help="iterations per pass and GPU-share: a pass traces spp x N iterations of the rank's rows "
                         "(so every GPU's pass has the 1-GPU pass's size); results are bit-identical to one "
                         "iteration per pass (default: 256 for cornell and config 3, 128 for configs 4 and 5)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong (default): a step renders a FIXED batch of --samples samples per pixel of the "
                         "whole image, split over the N GPUs by rows (cornell: one pass of 256 iterations of the "
                         "rank's rows at every N); "
                         "weak: a step is one pass of spp x N iterations of the rank's rows")
    ap.add_argument("--samples", type=int, default=256, help="strong scaling: samples per pixel per step")
    args = ap.parse_args()
    if args.spp is None:   # iterations per pass, measured per workload
        args.spp = {"cornell": 256, "cornell_hd_sorted": 256, "multi_object_4k": 128, "random_triangles_100k": 128,
                    "tessellated_meshes_100k": 128}[args.config]

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    # One process per GPU.  PT_BENCH_REHEARSAL=1 lets several ranks share the visible GPUs
    # (device = local_rank % count) and uses gloo for the collectives: a functional rehearsal of
    # the N > 1 path on a 1-GPU box, never a measurement.
    rehearsal = os.environ.get("PT_BENCH_REHEARSAL", "0") == "1"
    ndev = torch.cuda.device_count()
    dev_index = local_rank % ndev if rehearsal else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rehearsal:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    import cuda_pathtracer_amd as P
    from cuda_pathtracer_amd import distributed as D
    from cuda_pathtracer_amd._native import lib as _native_lib
    P.lib()

    from cuda_pathtracer_amd import scenes as SG
    gui = P.GuiDataContainer()
    scene_path, workload = args.scene, None
    if args.config != "cornell":
        gen_dir = ROOT / "gpurun_out" / "bench_scenes"
        if rank == 0:
            scene_path = SG.CONFIGS[args.config](gen_dir)
        if dist is not None:
            box = [scene_path]
            dist.broadcast_object_list(box, src=0)
            scene_path = box[0]
        gui.sortbyMaterial = args.config == "cornell_hd_sorted"
        workload = {"cornell_hd_sorted": "config 3: cornell geometry 1920x1080 DEPTH 16, material-sorted shading",
                    "multi_object_4k": "config 4: 4K multi-object (spheres+boxes; diffuse, mirror, glass) DEPTH 8",
                    "random_triangles_100k": "config 5: 100k random triangles via OBJ+BVH, 4K, DEPTH 32",
                    "tessellated_meshes_100k": "not a BASELINE config: 100k small triangles (tessellated sphere "
                                               "+ torus) via OBJ+BVH, 1920x1080, DEPTH 16 (the exact t-cull's case)",
                    }[args.config]
    gui.bvhCull = bool(args.bvh_cull)
    scene = P.Scene(scene_path)
    st_r = scene.state()
    # PT_BENCH_SHARD_OF=N (1 process only): trace exactly rank 0's share of an N-GPU strong-scaling
    # step alone on one GPU, no gather — a rehearsal of the per-rank time at N GPUs (value = rank 0's
    # segments / time, not a whole-job number), never the bench line of an N-GPU run
    shard_of = int(os.environ.get("PT_BENCH_SHARD_OF", "0") or 0)
    if shard_of and world != 1:
        raise SystemExit("PT_BENCH_SHARD_OF is a single-process rehearsal")
    sw = shard_of or world                  # the shard layout: rows y % sw == rank
    spp = sw * max(1, args.spp)             # iterations per pass of this rank's rows
    passes_per_step = 1
    if args.scaling == "strong":
        passes_per_step = max(1, args.samples // spp)
        if args.samples % passes_per_step:
            raise SystemExit(f"--samples {args.samples} does not split into {passes_per_step} equal passes")
        spp = args.samples // passes_per_step
    if spp > 256:   # pt_shard.spp limit (one thread of the bounce kernel's workgroup per iteration)
        raise SystemExit(f"{spp} iterations per pass > 256 (pt_shard.spp limit)")
    pt = P.PathTracer(scene, gui, rank=rank, world=sw, spp=spp)
    walk_info = pt.walk_info() if scene.counts()[2] > 0 else None
    stream = torch.cuda.current_stream()
    _log(rank, f"[bench] {args.scaling} scaling: tile rows={pt.rows} npix={pt.npix} paths/pass={pt.npaths} "
               f"passes/step={passes_per_step} depth={st_r.traceDepth}")

    it = 1
    for _ in range(args.warmup * passes_per_step):
        pt.render_pass(it, stream)
        it += spp
    torch.cuda.synchronize()
    s0 = pt.stats()

    rows_all = None
    tile = torch.empty((pt.rows, pt.width, 3), dtype=torch.float32, device=dev)
    H = scene.camera().res[1]
    if dist is not None:   # untimed gather of the real tile shape: RCCL connects its peers on first use
        pt.copy_image_to(tile.data_ptr(), stream)
        D.gather_tiles(torch, dist, tile, H)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps * passes_per_step):
        pt.render_pass(it, stream)
        it += spp
    # single RCCL gather of the framebuffer tiles to rank 0
    pt.copy_image_to(tile.data_ptr(), stream)
    gather_ms = None
    if dist is not None:
        torch.cuda.synchronize()   # (the render had to finish before the gather anyway)
        tg = time.perf_counter()
        rows_all = D.gather_tiles(torch, dist, tile, H)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3
    barrier()
    elapsed = time.perf_counter() - t0
    s1 = pt.stats()
    gather_ms_min = None
    if dist is not None:   # the last rank to arrive waits least: its gather time is the collective's own
        gather_ms_min = -D.max_over_ranks(torch, dist, -gather_ms, dev)

    # Kernel-level timing for the roofline: a profiled segment of the same workload right after
    # the timed region (HIP events bracket every launch on its stream; events inside the timed
    # region would add inter-kernel gaps to `value`).
    prof_passes = min(args.steps * passes_per_step, 50)
    pt.profile(True)
    pt.profile_read()
    sp0 = pt.stats()
    for _ in range(prof_passes):
        pt.render_pass(it, stream)
        it += spp
    prof = pt.profile_read()
    pt.profile(False)
    sp1 = pt.stats()

    seg = s1["segments"] - s0["segments"]
    live = [b - a for a, b in zip(s0["bounce_live"], s1["bounce_live"])]
    t_max = elapsed
    seg_all = seg
    ranks = None
    if dist is not None:
        t_max = D.max_over_ranks(torch, dist, elapsed, dev)
        seg_all = D.sum_over_ranks(torch, dist, seg, dev)
        # per-rank elapsed time and segments (min, max, spread): an imbalanced N-GPU line is
        # diagnosable from the line itself
        ranks = D.rank_spread(D.per_rank(torch, dist, (elapsed, seg), dev))
        ranks["gather_ms_per_rank"] = [r[0] for r in D.per_rank(torch, dist, (gather_ms,), dev)]

    # roofline of the dominant kernel (bounces >= 1), over the profiled segment
    depth = st_r.traceDepth
    plive = [b - a for a, b in zip(sp0["bounce_live"], sp1["bounce_live"])]
    pemit = [b - a for a, b in zip(sp0["bounce_emit"], sp1["bounce_emit"])]
    seg_bounce = sum(plive[1:depth])
    sorted_ = bool(gui.sortbyMaterial)
    b_ms, b_n, b_busy = prof["bounce"]
    if sorted_:   # material-sorted pipeline: every producer after the first + its histogram scans
        b_ms, b_n, b_busy = prof["sort"]
    t_ms, t_n, t_busy = prof["traverse"]
    walk = t_n > 0   # mesh scene with the BVH walk in its own kernel (k_traverse / k_traverse4)
    f_ms, f_n, _ = prof["first_bounce"]
    mesh = scene.counts()[2] > 0
    quads = walk and not args.bvh_cull and os.environ.get("PT_AMD_TRAV") != "pairs" and \
        _native_lib().pt_scene_bvh_quads(scene.handle, None, 0, None, None) > 0
    # k_bounce<FIRST, SPP1, MESH mode>: mesh scenes run mode 2 (closest mesh hit from k_traverse)
    bprefix = f"k_bounce<false, {'true' if spp == 1 else 'false'}, {2 if mesh else 0}>"
    # (k_traverse4<FIRST, K>: K triangle tasks per lane, 2, or 1 where the exact t-cull is on)
    wprefix = "k_traverse4<false," if quads else "k_traverse<false>"
    kprefix = wprefix if walk else bprefix
    kernel_name = ("material-sorted pipeline (k_sort_produce: shade + compact + intersect / histogram scan + permutation)"
                   if sorted_ else ("k_traverse4<false, K>" if kprefix == "k_traverse4<false," else kprefix))
    kernel_min = 0
    for b in range(1, depth):
        n_out = plive[b + 1] if b + 1 < depth else 0
        kernel_min += PATH_BYTES * plive[b] + PATH_BYTES * n_out + FB_RMW_BYTES * pemit[b]
    k_ms, k_n, k_busy = (t_ms, t_n, t_busy) if walk else (b_ms, b_n, b_busy)
    per_launch_bytes = SEGMENT_BYTES * seg_bounce / max(k_n, 1)
    avg_ms = k_ms / max(k_n, 1)
    # The lanes' launches overlap (two streams), so a launch's own duration is shared with the other
    # lane's work: launches x avg_ms exceeds the step.  The kernel's time per launch that fits the
    # step is the union of its launch intervals / launches (launches x eff_ms = union <= the step):
    # that is the roofline's duration; the HIP-event average (= rocprofv3's) is reported beside it.
    eff_ms = k_busy / max(k_n, 1) if k_busy > 0 else avg_ms
    achieved = per_launch_bytes / (eff_ms * 1e-3) / 1e9 if eff_ms > 0 else 0.0
    achieved_overlapped = per_launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    # pt_kernels.hip pt_create: 3 lanes for large sorted passes (kThreeLanePaths), 1 with the BVH walk
    default_lanes = 3 if sorted_ and pt.npaths >= (48 << 20) else (1 if quads else 2)
    lanes = min(int(os.environ.get("PT_AMD_LANES", str(default_lanes))), spp, 4) \
        if (spp > 1 and (sorted_ or os.environ.get("PT_PIPELINE") != "split")) else 1
    # every bounce's algorithmic bytes (184 B per segment) of one step over the step time: the
    # byte metric at step level (near 1.0 it is saturated and stops being evidence; VALU issue is
    # the limiter then, roofline.valu_issue)
    step_seg = seg / max(args.steps, 1)
    prof_steps = prof_passes / max(passes_per_step, 1)
    roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                "definition": "184 B (SURVEY.md §8d) x segments per launch / the kernel's time per launch "
                              "(union of its launch intervals over the profiled passes / launches, HIP events "
                              "on the launch streams: launches x that time fits the step)",
                "kernel": kernel_name, "effective_launch_ms": eff_ms, "avg_launch_ms": avg_ms, "launches": k_n,
                "lanes": lanes,
                "launches_per_step": k_n / max(prof_steps, 1e-9),
                "kernel_ms_per_step": k_busy / max(prof_steps, 1e-9),
                "overlapped": {"avg_launch_ms": avg_ms, "achieved": achieved_overlapped,
                               "frac": achieved_overlapped / HBM_PEAK_GBS,
                               "definition": "the same bytes / the HIP-event average launch duration (= rocprofv3 "
                                             "--kernel-trace --stats' average; each launch shares the GPU with the "
                                             "other lane's, so launches x this exceeds the step)"},
                "segments_per_launch": seg_bounce / max(k_n, 1),
                "algorithmic_bytes_per_launch": per_launch_bytes,
                "step_model_ratio": SEGMENT_BYTES * step_seg / (elapsed / max(args.steps, 1)) / 1e9 / HBM_PEAK_GBS
                if world == 1 else None,
                "step_model_ratio_definition": "§8d model bytes (184 B x traced segments of one step, all bounces) / "
                                               "ms_per_step / 8 TB/s — a model ratio, not a measured HBM fraction",
                # two lanes' launches overlap: the same bytes over the union of the launch intervals
                "aggregate": {"busy_ms": k_busy,
                              "achieved": SEGMENT_BYTES * seg_bounce / (k_busy * 1e-3) / 1e9 if k_busy > 0 else 0.0,
                              "frac": SEGMENT_BYTES * seg_bounce / (k_busy * 1e-3) / 1e9 / HBM_PEAK_GBS
                              if k_busy > 0 else 0.0,
                              "definition": "184 B x segments of bounces >= 1 / union of their launch intervals"}}
    if not walk:
        roofline["kernel_min_bytes_per_launch"] = kernel_min / max(b_n, 1)
    else:   # the bounce kernel after the walk (bounded closest hit with the mesh hit + shade + compact)
        bb = SEGMENT_BYTES * seg_bounce / max(b_n, 1)
        b_avg = b_ms / max(b_n, 1)
        roofline["bounce_kernel"] = {
            "kernel": bprefix, "avg_launch_ms": b_avg, "launches": b_n,
            "achieved": bb / (b_avg * 1e-3) / 1e9 if b_avg > 0 else 0.0,
            "frac": bb / (b_avg * 1e-3) / 1e9 / HBM_PEAK_GBS if b_avg > 0 else 0.0,
            "kernel_min_bytes_per_launch": kernel_min / max(b_n, 1)}
        roofline["walk_share_of_gpu_time"] = t_ms / max(t_ms + b_ms + f_ms + prof["first_traverse"][0], 1e-9)
        roofline["walk_info"] = walk_info   # 4-wide walk, its exact t-cull on/off, share of slots it can cull
        roofline["first_traverse_avg_ms"] = prof["first_traverse"][0] / max(prof["first_traverse"][1], 1)

    result = None
    if rank == 0:
        if rows_all is not None:
            full = D.assemble([t.cpu().numpy() for t in rows_all], scene.camera().res[1], world)
            assert np.isfinite(full).all()
        if world > 1:   # the N-GPU line's parts (the driver's scaling run): every rank's segments, the gather
            assert gather_ms is not None and gather_ms_min is not None, "N > 1: the tile gather was not timed"
            assert seg_all >= seg > 0 and rows_all is not None and len(rows_all) == world, \
                "N > 1: per-rank segment sums or gathered tiles missing"
            assert ranks is not None and len(ranks["segments"]) == world and sum(ranks["segments"]) == seg_all \
                and abs(ranks["elapsed_max_s"] - t_max) < 1e-9, "N > 1: per-rank diagnostics inconsistent"
        value = seg_all / t_max / 1e6
        strong = args.scaling == "strong"
        desc = (f"cornell.json 800x800 DEPTH 8 default flags; a step = {args.samples} samples per pixel of the whole "
                f"image, split over the GPUs by rows (each rank: {passes_per_step} pass(es) of {spp} iterations of "
                f"its rows y%N==rank; bit-identical to one iteration per pass); fused bounce kernel" if strong else
                f"cornell.json 800x800 DEPTH 8 default flags; a step = one pass of {spp} iteration(s) of the rank's "
                f"rows y%N==rank per GPU (bit-identical to one iteration per pass); fused bounce kernel")
        result = {
            "metric": METRIC,
            "value": value,
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (bundled cornell.json scene; camera rays generated on device)" if workload is None
                    else "synthetic (generated scene, cuda_pathtracer_amd/scenes.py; camera rays generated on device)",
            "config": {"workload": workload or desc,
                       "scene": Path(scene_path).name, "resolution": list(scene.camera().res), "depth": depth,
                       "samples_per_step": (args.samples if strong else spp * world),
                       "iterations_per_pass": spp, "passes_per_step": passes_per_step,
                       "paths_per_gpu_per_pass": pt.npaths,
                       "parallelism": (f"pixel rows x{world} (world_size {world}, backend "
                                       f"{dist.get_backend() if dist is not None else 'none'}) + one gather")
                                      if not shard_of else
                                      f"REHEARSAL: rank 0's rows of a x{shard_of} shard, alone on one GPU"},
            "roofline": roofline,
            "segments": seg_all,
            "bounce_live_per_step": [x / args.steps for x in live],
            # SURVEY.md §8d's nominal rate: every path of every sample traced to full depth
            "nominal_mrays": scene.camera().res[0] * scene.camera().res[1] * (args.samples if strong else spp * world)
            * depth / (t_max / args.steps) / 1e6,
            "nominal_definition": "W x H x samples per step x DEPTH / ms_per_step (no early termination counted)",
            "first_bounce_avg_ms": f_ms / max(f_n, 1),
            "gather_ms": gather_ms,
            "gather_ms_last_rank": gather_ms_min,
            "ranks": ranks,
        }
        if not args.no_scan:
            result["scan"] = scan_bench(torch, dev, args.scan_n, args.scan_reps)
            result["compact"] = compact_bench(torch, dev, args.scan_n, max(3, args.scan_reps // 2))
        if world == 1 and not args.no_cpu_baseline:
            result["cpu_baseline"] = cpu_baseline_render(args.cpu_seconds)
            # labelled multithreaded variant: 16 host threads (the box's CPU share per GPU)
            result["cpu_baseline_mt"] = cpu_baseline_render_mt(args.cpu_seconds / 2, min(16, os.cpu_count() or 1))
            result["cpu_baseline_scan"] = cpu_baseline_scan()
            result["cpu_baseline_scan_2e28"] = cpu_baseline_scan(1 << 28, 3)
            result["cpu_baseline_compact"] = cpu_baseline_compact()
        else:
            result["cpu_baseline"] = None
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    pt.free()
    if rank == 0 and world == 1 and not args.no_dropin and not shard_of and args.config == "cornell":
        try:
            result["dropin"] = dropin_bench(scene_path)
            result["dropin"]["vs_batched"] = result["dropin"]["value"] / result["value"]
        except Exception as e:   # a reported side leg: never fail the bench line
            result["dropin"] = {"error": repr(e)}
    if rank == 0 and world == 1 and not args.no_pmc:
        try:
            extra = _pmc_leg(args, scene_path, spp, sorted_, eff_ms, kprefix, seg_bounce / max(k_n, 1), k_busy, k_n,
                             walk=walk)
        except Exception as e:   # profiling is evidence, not the measurement: never fail the bench line
            extra = {"pmc_error": repr(e)}
        roofline.update(extra)
        if "isolated" in roofline and roofline.get("launches"):
            lps = roofline["launches"] / max(prof_passes, 1) * passes_per_step   # launches per step
            roofline["isolated"]["launches_per_step"] = lps
            roofline["isolated"]["ms_per_step_if_serial"] = lps * roofline["isolated"]["avg_launch_ms"]
    if rank == 0 and world == 1 and walk and not args.no_walk_counters:
        roofline["walk_counters"] = _walk_counters(scene_path, spp)
    if rank == 0:
        _finalize_roofline(roofline)
    if rank == 0:
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()

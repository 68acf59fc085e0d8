// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called from the
// product library (cuda_pathtracer_amd).  Only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py may load liboracle.so, and only as the checker.
//
// Serial CPU restatement of the reference's stream-compaction CPU path:
//   path_tracer/stream_compaction/cpu.cu:16-22   calc_prefix_sum  (exclusive scan)
//   path_tracer/stream_compaction/cpu.cu:28-33   CPU::scan
//   path_tracer/stream_compaction/cpu.cu:40-51   CPU::compactWithoutScan
//   path_tracer/stream_compaction/cpu.cu:58-79   CPU::compactWithScan
//   path_tracer/stream_compaction/common.cu:25-46 kernMapToBoolean / kernScatter (map + scatter)
//   path_tracer/src/pathtrace.cu:359-407          mark_valid / keep (stable partition of paths)
//
// Semantics pinned here:
//   * The reference's `#pragma omp` lines are inert (no -fopenmp anywhere), so the oracle is
//     the SERIAL loop.  Sums wrap in int32: we add in uint32 to make the wrap defined.
//   * n <= 0 writes nothing (the reference writes odata[0] for n == 0: out of contract).
//
// Pinned against the reference's own known-answer vectors (stream_compaction/INSTRUCTION.md
// :262-302) in tests/test_oracle.py.
#include <cstdint>
#include <cstring>
#include <chrono>
#include <vector>

extern "C" {

// CPU::scan -> calc_prefix_sum (cpu.cu:16-22): out[0] = 0, out[i] = out[i-1] + in[i-1].
void oracle_scan(int64_t n, int32_t* out, const int32_t* in) {
    if (n <= 0) return;
    uint32_t acc = 0;
    for (int64_t i = 0; i < n; ++i) {
        uint32_t v = (uint32_t)in[i];
        out[i] = (int32_t)acc;
        acc += v;
    }
}

// CPU::compactWithoutScan (cpu.cu:40-51): keep non-zero values in order, return count.
int64_t oracle_compact_without_scan(int64_t n, int32_t* out, const int32_t* in) {
    int64_t cnt = 0;
    for (int64_t i = 0; i < n; ++i)
        if (in[i] != 0) out[cnt++] = in[i];
    return cnt;
}

// CPU::compactWithScan (cpu.cu:58-79): map -> exclusive scan -> scatter, count = scan[n-1]+keep[n-1].
int64_t oracle_compact_with_scan(int64_t n, int32_t* out, const int32_t* in) {
    if (n <= 0) return 0;
    std::vector<int32_t> keep((size_t)n), pos((size_t)n);
    for (int64_t i = 0; i < n; ++i) keep[i] = in[i] != 0 ? 1 : 0;
    oracle_scan(n, pos.data(), keep.data());
    for (int64_t i = 0; i < n; ++i)
        if (keep[i]) out[pos[i]] = in[i];
    return (int64_t)pos[n - 1] + keep[n - 1];
}

// Stable partition used by relocate_terminated_paths (pathtrace.cu:359-407): element i with
// flag != 0 goes to scan[i]; element with flag == 0 goes to live + i - scan[i].
// Writes the source index of every destination slot into perm_out (size n); returns #live.
int64_t oracle_partition_indices(int64_t n, const int32_t* flags, int32_t* perm_out) {
    if (n <= 0) return 0;
    std::vector<int32_t> keep((size_t)n), pos((size_t)n);
    for (int64_t i = 0; i < n; ++i) keep[i] = flags[i] != 0 ? 1 : 0;
    oracle_scan(n, pos.data(), keep.data());
    int64_t live = (int64_t)pos[n - 1] + keep[n - 1];
    for (int64_t i = 0; i < n; ++i) {
        int64_t dst = keep[i] ? pos[i] : live + i - pos[i];
        perm_out[dst] = (int32_t)i;
    }
    return live;
}

// CPU baseline timing: median-free helper, returns the wall time of `reps`
// back-to-back scans in milliseconds, measured like PerformanceTimer (common.h:61-80).
double oracle_time_scan_ms(int64_t n, const int32_t* in, int32_t* out, int reps) {
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int r = 0; r < reps; ++r) oracle_scan(n, out, in);
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

// CPU::compactWithScan (with_scan != 0) or CPU::compactWithoutScan, timed the same way.
double oracle_time_compact_ms(int64_t n, const int32_t* in, int32_t* out, int reps, int64_t* count) {
    auto t0 = std::chrono::high_resolution_clock::now();
    int64_t c = 0;
    for (int r = 0; r < reps; ++r) c = oracle_compact_with_scan(n, out, in);
    auto t1 = std::chrono::high_resolution_clock::now();
    if (count) *count = c;
    return std::chrono::duration<double, std::milli>(t1 - t0).count();
}
double oracle_time_compact_without_scan_ms(int64_t n, const int32_t* in, int32_t* out, int reps, int64_t* count) {
    auto t0 = std::chrono::high_resolution_clock::now();
    int64_t c = 0;
    for (int r = 0; r < reps; ++r) c = oracle_compact_without_scan(n, out, in);
    auto t1 = std::chrono::high_resolution_clock::now();
    if (count) *count = c;
    return std::chrono::duration<double, std::milli>(t1 - t0).count();
}

}  // extern "C"

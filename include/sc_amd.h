/* sc_amd.h — C ABI of the MI355X stream-compaction library (libpt_amd.so).
 *
 * Replaces the reference's StreamCompaction namespace (path_tracer/stream_compaction/ and the
 * standalone stream_compaction/stream_compaction/ copy):
 *   Efficient::scan      efficient.h:9   / efficient.cu:150-174   -> sc_efficient_scan, sc_scan_exclusive_i32
 *   Efficient::compact   efficient.h:11  / efficient.cu:185-219   -> sc_efficient_compact, sc_compact_i32
 *   Efficient::timer()   efficient.h:7   / common.h:46-130        -> sc_timer_gpu_ms
 *   Common::kernMapToBoolean / kernScatter  common.cu:25-46       -> fused into sc_compact_i32
 *   mark_valid + scan + keep  path_tracer/src/pathtrace.cu:359-407 -> sc_partition_i32 (stable partition)
 *                                                                    and sc_partition_indices (live index list)
 * The reference's other three namespaces (sc_variants.hip; not on the path tracer's hot path, which
 * calls Efficient only — they let the reference's self-test, stream_compaction/src/main.cpp:31-85,
 * compare the four implementations against the C++ mirror):
 *   CPU::scan / compactWithoutScan / compactWithScan  cpu.h:9-13 / cpu.cu:16-79 -> sc_cpu_*
 *   Naive::scan                                       naive.h:9 / naive.cu:14-66 -> sc_naive_scan(_i32)
 *   Thrust::scan                                      thrust.h:9 / thrust.cu:14-28 -> sc_thrust_scan(_i32)
 * sc_cpu_* are host loops of their own, not the test oracle (oracle/sc_oracle.cpp checks them) and
 * not a fallback of the device entry points: nothing here falls back to the CPU.
 *
 * Differences from the reference, by design:
 *   - every entry point returns a status code (SC_OK / SC_ERR_*) instead of exit()ing
 *     (common.cu:3-15); sc_last_error() gives the message;
 *   - device-pointer entry points take an explicit hipStream_t (passed as void*) and never
 *     allocate or synchronise (graph-capturable when given a workspace);
 *   - no power-of-two padding: n is any value in [0, 2^31 - 1]; the reference's n == 1 failure
 *      does not exist here;
 *   - sums wrap in int32 exactly like the reference (two's complement).
 * All functions are thread-compatible (no hidden globals besides a per-device workspace cache
 * used only by the *_auto / host-pointer helpers, guarded by a mutex).
 */
#ifndef SC_AMD_H
#define SC_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SC_OK 0
#define SC_ERR_ARG 1
#define SC_ERR_HIP 2
#define SC_ERR_NOMEM 3

/* Last error message of the calling thread ("" if none). */
const char* sc_last_error(void);

/* Bytes of device workspace the device-pointer entry points need for n elements
 * (decoupled look-back tile status words + control words). */
size_t sc_workspace_bytes(int64_t n);

/* Exclusive prefix sum of int32 (wrapping), device pointers, single pass (decoupled look-back).
 * d_out may alias d_in.  workspace: >= sc_workspace_bytes(n) bytes of device memory, or NULL
 * to use the library's cached per-device workspace.  Replaces Efficient::scan. */
int sc_scan_exclusive_i32(const int32_t* d_in, int32_t* d_out, int64_t n,
                          void* workspace, void* stream);

/* Stream compaction of int32: keeps the non-zero elements in order.  Writes the kept count to
 * *d_count (device int64).  Replaces Efficient::compact (map + scan + scatter fused). */
int sc_compact_i32(const int32_t* d_in, int32_t* d_out, int64_t n, int64_t* d_count,
                   void* workspace, void* stream);

/* Stable partition of indices by flags: d_perm[j] = source index of output slot j, live
 * (flag != 0) elements first in original order, then dead ones in original order — exactly the
 * `keep` placement of pathtrace.cu:366-376.  *d_live (device int64) = number of live elements. */
int sc_partition_i32(const int32_t* d_flags, int32_t* d_perm, int64_t n, int64_t* d_live,
                     void* workspace, void* stream);

/* Index list of the live elements: d_idx[j] = index of the j-th non-zero flag, in order;
 * *d_count (device int32) = their number.  The 8 B/path path-compaction primitive of SURVEY.md
 * §8b (flag read + index write); d_idx beyond the count is left untouched. */
int sc_partition_indices(const int32_t* d_flags, int32_t* d_idx, int64_t n, int32_t* d_count,
                         void* workspace, void* stream);

/* Host-pointer helpers with the reference's exact call semantics (Efficient::scan / compact take
 * host arrays and return after the result is on the host).  They allocate device buffers from a
 * per-device cache and time the device work with hipEvents like PerformanceTimer::startGpuTimer. */
int sc_efficient_scan(int n, int* odata, const int* idata);
int sc_efficient_compact(int n, int* odata, const int* idata, int* count_out);

/* The device-pointer entry points are asynchronous, so a look-back stall (static schedule on a
 * GPU shared with other work: the grid is not co-resident, a wait hits its spin bound and the
 * grid drains with invalid results) is reported here: synchronises the device and returns
 * SC_ERR_HIP if the most recent call that used `workspace` (NULL: the cached per-device one) hit
 * the bound, SC_OK otherwise.  The host-pointer helpers check this themselves. */
int sc_workspace_check(const void* workspace);

/* Device address of `workspace`'s error word (uint32, non-zero after a stall), for callers that
 * fold it into their own device-side status without a host round trip (the renderer does). */
const uint32_t* sc_workspace_error_word(const void* workspace);

/* Tile schedule of the look-back kernels (process-wide).  0 (default, fastest): a static
 * assignment over a grid that must be fully resident — if another kernel or process holds part of
 * the GPU the call stalls until a bounded spin gives up (~0.25 s) and sc_workspace_check reports
 * SC_ERR_HIP ("look-back spin bound") instead of hanging.
 * 1: tiles claimed in order from a ticket — correct whatever else runs on the GPU, ~15% slower.
 * The environment variable PT_AMD_SCHEDULE=claim selects 1 at load time. */
int sc_set_tile_schedule(int32_t claimed);

/* ---- the reference's CPU / Naive / Thrust namespaces (sc_variants.hip) ----------------------- */

/* CPU::scan (cpu.cu:16-33): exclusive prefix sum on the host, wrapping; odata may equal idata. */
int sc_cpu_scan(int n, int* odata, const int* idata);
/* CPU::compactWithoutScan (cpu.cu:40-52): the non-zero elements in order; *count_out = how many. */
int sc_cpu_compact_without_scan(int n, int* odata, const int* idata, int* count_out);
/* CPU::compactWithScan (cpu.cu:59-79): map to 0/1, exclusive scan, scatter; *count_out = kept. */
int sc_cpu_compact_with_scan(int n, int* odata, const int* idata, int* count_out);

/* Naive::scan (naive.cu:14-66): Hillis & Steele, ceil(log2 n) launches ping-ponging between d_out
 * and d_tmp (n int32 of device scratch), then the inclusive -> exclusive shift.  d_in is left
 * unchanged; d_in, d_out and d_tmp must not alias (SC_ERR_ARG).  Asynchronous on `stream`. */
int sc_naive_scan_i32(const int32_t* d_in, int32_t* d_out, int64_t n, int32_t* d_tmp, void* stream);
/* Thrust::scan (thrust.cu:14-28): rocThrust's exclusive_scan on `stream` (d_out may equal d_in). */
int sc_thrust_scan_i32(const int32_t* d_in, int32_t* d_out, int64_t n, void* stream);
/* Host-array forms with the reference's signatures (upload, device work timed by sc_timer_gpu_ms,
 * download), like sc_efficient_scan. */
int sc_naive_scan(int n, int* odata, const int* idata);
int sc_thrust_scan(int n, int* odata, const int* idata);

/* Elapsed device time (ms) of the previous host-pointer operation
 * (PerformanceTimer::getGpuElapsedTimeForPreviousOperation, common.h:98-101). */
float sc_timer_gpu_ms(void);

#ifdef __cplusplus
}
#endif
#endif /* SC_AMD_H */

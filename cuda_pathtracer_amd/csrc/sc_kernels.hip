// MI355X stream compaction: single-pass exclusive scan / compaction / stable partition of int32.
//
// Replaces StreamCompaction::Efficient (path_tracer/stream_compaction/efficient.cu:46-219) and
// Common::kernMapToBoolean / kernScatter (common.cu:25-46).  The reference runs a recursive
// Blelloch scan with 64 elements per block (blockDim = warpSize = 32), pads n to a power of two
// and allocates/frees device memory on every call.  Here one launch streams each element once:
//   tile = 256 threads x 8 x int4 = 8192 elements, loaded as wave-contiguous 16-byte vectors
//   (chunk k of a tile is 1 KiB per wave-instruction), per-thread 4-element scan, wave64 DPP scan
//   of the per-thread sums, 16 wave totals through LDS, then the tile's prefix from the
//   aggregates of the tiles before it (lookback.h: a window sum under the static schedule, a
//   decoupled look-back when tiles are claimed).  Algorithmic traffic: 8 B/element for scan
//   (4 read + 4 write), 4 B/element + 4 B/kept for compaction.
//
// Kernels: k_scan_lag (16-byte aligned pointers; the prefix of each tile is resolved one
// iteration late, see below) and k_scan_tiles (unaligned pointers and the partial tail tile;
// look-back resolved immediately).  Design history with measurements: DESIGN.md §4,
// profiles/r01_scan_ab.txt.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "lookback.h"
#include "../../include/sc_amd.h"

namespace {

constexpr int kThreads = 256;
constexpr int kChunks = 8;                       // int4 chunks per thread
constexpr int kTile = kThreads * kChunks * 4;    // 8192 elements (32 KiB)
constexpr size_t kCtlBytes = 256;                // [1] device error word, [2] tile ticket (padded)
constexpr int kLagWindows = 4;                   // look-back predecessors per round trip: 4 x 64
constexpr int kTicket = 2;                       // ctl word of the tile ticket

thread_local std::string g_err;
thread_local float g_timer_ms = 0.f;
// Tile schedule (lookback.h TileSeq): static co-resident grid, or claimed tiles for shared GPUs.
// Default from PT_AMD_SCHEDULE=claim|static; sc_set_tile_schedule() overrides.
std::atomic<bool> g_schedule_claimed{[] {
    const char* v = std::getenv("PT_AMD_SCHEDULE");
    return v && std::strcmp(v, "claim") == 0;
}()};

#ifdef PT_SC_TEST_HOOKS
// Test build only (build/libpt_amd_testhooks.so, tests/test_scan_gpu.py): PT_AMD_TEST_SCAN_OVERSUB=k
// launches the look-back kernels on k x the co-resident grid, so the static schedule stalls and must
// report its spin bound.  The shipping library has no such hook.
const int g_test_oversub = [] {
    const char* v = std::getenv("PT_AMD_TEST_SCAN_OVERSUB");
    const int k = v ? std::atoi(v) : 1;
    return k >= 1 && k <= 16 ? k : 1;
}();
#else
constexpr int g_test_oversub = 1;
#endif

int fail(int code, const std::string& msg) { g_err = msg; return code; }
int hip_fail(hipError_t e, const char* where) {
    return fail(SC_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

enum Mode { kScan = 0, kCompact = 1, kPartition = 2, kIndices = 3 };
typedef int v4i __attribute__((ext_vector_type(4)));

// LDS-only workgroup barrier: waits for this wave's LDS traffic, not for its outstanding global
// loads, so a prefetched tile stays in flight across it (cdna_hip_programming.md §5 "Pipelining
// across barriers").
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void load_full(const int32_t* __restrict__ in, int64_t base, int tid, v4i (&v)[kChunks]) {
#pragma unroll
    for (int k = 0; k < kChunks; ++k)
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(in + base + (int64_t)k * (kThreads * 4) + 4 * tid));
}
__device__ __forceinline__ void load_guarded(const int32_t* __restrict__ in, int64_t n, int64_t base, int tid,
                                             v4i (&v)[kChunks]) {
#pragma unroll
    for (int k = 0; k < kChunks; ++k) {
        const int64_t e0 = base + (int64_t)k * (kThreads * 4) + 4 * tid;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t j = e0 + e < n ? e0 + e : n - 1;   // branch-free: clamp, then mask
            const int32_t x = in[j];
            v[k][e] = e0 + e < n ? x : 0;
        }
    }
}

template <int MODE>
__device__ __forceinline__ uint32_t chunk_count(const v4i& v) {
    if (MODE == kScan) return ((uint32_t)v[0] + (uint32_t)v[1]) + ((uint32_t)v[2] + (uint32_t)v[3]);
    return (uint32_t)(v[0] != 0) + (uint32_t)(v[1] != 0) + (uint32_t)(v[2] != 0) + (uint32_t)(v[3] != 0);
}

// Block-local part shared by both kernels: per-chunk sums, wave scans, the 4 wave totals of every
// chunk through LDS.  On return pre[k] = this thread's exclusive local offset for chunk k and the
// tile aggregate is returned.  Starts with a barrier (the previous readers of s_wsum are done).
template <int MODE>
__device__ __forceinline__ uint32_t tile_offsets(const v4i (&cur)[kChunks], uint32_t (&s_wsum)[kChunks][4],
                                                 uint32_t (&pre)[kChunks]) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t sv[kChunks], incl[kChunks];
#pragma unroll
    for (int k = 0; k < kChunks; ++k) {
        sv[k] = chunk_count<MODE>(cur[k]);
        incl[k] = lb::wave_inclusive_scan(sv[k]);
    }
    lds_barrier();
    if (lane == 63) {
#pragma unroll
        for (int k = 0; k < kChunks; ++k) s_wsum[k][wave] = incl[k];
    }
    lds_barrier();
    uint32_t run = 0;
#pragma unroll
    for (int k = 0; k < kChunks; ++k) {
        uint32_t before = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t x = s_wsum[k][w];
            before += (w < wave) ? x : 0u;
        }
        pre[k] = run + before + (incl[k] - sv[k]);
#pragma unroll
        for (int w = 0; w < 4; ++w) run += s_wsum[k][w];
    }
    return run;
}

// Outputs of chunk k of a tile whose prefix is known: scan values, kept values, live indices, or
// partition indices (live in order; dead ones to `dead` in order, appended by k_append_dead).
// Padding lanes of a partial tile load as 0, so they are never counted or kept.
template <int MODE, bool FULL>
__device__ __forceinline__ void write_chunk(const v4i& v, int64_t e0, uint32_t run, int64_t n,
                                            int32_t* __restrict__ out, int32_t* __restrict__ dead) {
    if (MODE == kScan) {
        v4i o;
#pragma unroll
        for (int e = 0; e < 4; ++e) { o[e] = (int32_t)run; run += (uint32_t)v[e]; }
        if (FULL) {
            __builtin_nontemporal_store(o, reinterpret_cast<v4i*>(out + e0));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
                if (e0 + e < n) out[e0 + e] = o[e];
        }
    } else if (MODE == kCompact) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (v[e] != 0) out[run++] = v[e];
    } else if (MODE == kIndices) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (v[e] != 0) out[run++] = (int32_t)(e0 + e);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int64_t idx = e0 + e;
            if (FULL || idx < n) {
                if (v[e] != 0) out[run++] = (int32_t)idx;
                else dead[idx - (int64_t)run] = (int32_t)idx;
            }
        }
    }
}

// The kept count, written once by the last tile: int64 for compact / partition, int32 for the
// index list (sc_partition_indices' contract).
template <int MODE>
__device__ __forceinline__ void store_count(int64_t* __restrict__ d_count, uint32_t v) {
    if (MODE == kIndices) *reinterpret_cast<int32_t*>(d_count) = (int32_t)v;
    else *d_count = (int64_t)v;
}

// One tile with the look-back resolved immediately (unaligned inputs, the partial tail tile).
template <int MODE>
__device__ __forceinline__ void process_tile(const v4i (&cur)[kChunks], int tile, int num_tiles, int64_t n,
                                             int32_t* __restrict__ out, uint64_t* __restrict__ status,
                                             uint32_t* __restrict__ ctl, int64_t* __restrict__ d_count,
                                             int32_t* __restrict__ dead, uint32_t (&s_wsum)[kChunks][4],
                                             uint32_t* s_excl) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t pre[kChunks];
    const uint32_t total = tile_offsets<MODE>(cur, s_wsum, pre);
    if (wave == 0) {
        uint32_t excl = 0;
        if (tile == 0) {
            if (lane == 0) lb::publish(status, 0, lb::kFlagPre, total);
        } else {
            if (lane == 0) lb::publish(status, tile, lb::kFlagAgg, total);
            excl = lb::lookback(status, tile, lane, &ctl[1]);
            if (lane == 0) lb::publish(status, tile, lb::kFlagPre, excl + total);
        }
        if (lane == 0) *s_excl = excl;
    }
    lds_barrier();
    const uint32_t excl = *s_excl;
    const int64_t base = (int64_t)tile * kTile;
#pragma unroll
    for (int k = 0; k < kChunks; ++k)
        write_chunk<MODE, false>(cur[k], base + (int64_t)k * (kThreads * 4) + 4 * tid, excl + pre[k], n, out, dead);
    if (MODE != kScan && tid == 0 && tile == num_tiles - 1) store_count<MODE>(d_count, excl + total);
}

// ---- lagged look-back -----------------------------------------------------------------------
// Measured on MI355X (profiles/r01_scan_ab.txt): resolving each tile's prefix right after
// reducing it put the look-back round trip on every iteration's critical path (0.69 ms for 2^28
// ints, 0.39 ms with the look-back removed).  Here a workgroup publishes tile t's aggregate as
// soon as t is reduced, and resolves t's prefix in the NEXT iteration, after issuing the loads
// of t+2G and reducing t+G: by then every predecessor's aggregate is out, so the look-back
// rarely spins, and its round trip overlaps the loads in flight.  The deferred tile's raw values
// wait in LDS (2 x 32 KiB ping-pong); each thread keeps only its 8 per-chunk local offsets.
// Under the static schedule the look-back itself is replaced by a window sum (lag_resolve):
// 0.50 -> 0.39 ms for 2^28 ints, 4.2 -> 5.5 TB/s.
struct LagTile {
    uint32_t pre[kChunks];   // this thread's exclusive local offset of each of its chunks
    uint32_t total;          // tile aggregate
    int tile;
};

// Reduce tile `cur` into LDS parity `par` and publish its aggregate.
template <int MODE, bool WINDOW>
__device__ __forceinline__ void lag_reduce(const v4i (&cur)[kChunks], int tile, int par, int32_t (*s_data)[kTile],
                                           uint32_t (*s_wsum)[kChunks][4], uint64_t* __restrict__ status,
                                           LagTile& L) {
    const int tid = threadIdx.x;
    // tile_offsets' leading barrier also orders these writes after the previous readers of
    // s_data[par] (the store phase of the step before last)
    L.total = tile_offsets<MODE>(cur, s_wsum[par], L.pre);
    if (MODE != kScan) {
        // The kept elements' tile-local positions are known now: compact into LDS here, so the
        // deferred store is a plain copy once the tile's prefix is resolved.  Partition: the
        // dropped indices follow the kept ones, in order (local position li - kept before li).
        const int64_t base = (int64_t)tile * kTile;
#pragma unroll
        for (int k = 0; k < kChunks; ++k) {
            uint32_t run = L.pre[k];
            const int li0 = k * (kThreads * 4) + 4 * tid;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int32_t idx = (int32_t)(base + li0 + e);
                if (cur[k][e] != 0) s_data[par][run++] = MODE == kCompact ? cur[k][e] : idx;
                else if (MODE == kPartition) s_data[par][L.total + (uint32_t)(li0 + e) - run] = idx;
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < kChunks; ++k)
            *reinterpret_cast<v4i*>(&s_data[par][k * (kThreads * 4) + 4 * tid]) = cur[k];
    }
    L.tile = tile;
    if (tid == 0) lb::publish(status, tile, tile == 0 && !WINDOW ? lb::kFlagPre : lb::kFlagAgg, L.total);
}

// Wave 0: resolve the deferred tile's prefix, publish it, share it through LDS.
// WINDOW (static schedule): workgroup b owns tiles b, b+G, ..., so
//   excl(t) = excl(t-G) + agg(t-G) + sum of agg(t') for t-G < t' < t,
// where the first two terms are this workgroup's own `carry`.  Only aggregates are ever
// published and a tile waits for the G-1 aggregates before it, not for a chain of inclusive
// prefixes hopping from workgroup to workgroup (lb::window_sum).  Otherwise (claimed tiles):
// decoupled look-back.
template <bool WINDOW>
__device__ __forceinline__ void lag_resolve(const LagTile& L, uint32_t* s_excl, uint64_t* __restrict__ status,
                                            uint32_t* __restrict__ ctl, uint32_t& carry) {
    const int lane = threadIdx.x & 63;
    uint32_t excl = 0;
    if (WINDOW) {
        excl = carry + lb::window_sum(status, L.tile, (int)gridDim.x, lane, &ctl[1]);
        carry = excl + L.total;
    } else if (L.tile != 0) {
        excl = lb::lookback<kLagWindows>(status, L.tile, lane, &ctl[1]);
        if (lane == 0) lb::publish(status, L.tile, lb::kFlagPre, excl + L.total);
    }
    if (lane == 0) *s_excl = excl;
}

// count consecutive ints from LDS to global memory with wave-contiguous 16-byte stores (a
// per-lane `out[run++]` store scatters 4-byte writes across the wave's 64 runs); up to 3 head
// elements bring dst to a 16-byte boundary.
__device__ __forceinline__ void copy_out(const int32_t* src, int32_t* __restrict__ dst, uint32_t count) {
    const uint32_t tid = threadIdx.x;
    const uint32_t head = min((4u - (uint32_t)((reinterpret_cast<uintptr_t>(dst) >> 2) & 3u)) & 3u, count);
    const uint32_t quads = (count - head) >> 2;
    if (tid < head) dst[tid] = src[tid];
    for (uint32_t q = tid; q < quads; q += kThreads) {
        const uint32_t j = head + 4 * q;
        const v4i v = {src[j], src[j + 1], src[j + 2], src[j + 3]};
        __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(dst + j));
    }
    const uint32_t rest = head + 4 * quads;
    if (tid < count - rest) dst[rest + tid] = src[rest + tid];
}

// Outputs of a resolved tile, values from LDS parity `par`.
template <int MODE>
__device__ __forceinline__ void lag_store(const LagTile& L, int par, int32_t (*s_data)[kTile],
                                          const uint32_t* s_excl, int num_tiles, int32_t* __restrict__ out,
                                          int64_t* __restrict__ d_count, int32_t* __restrict__ dead) {
    const int tid = threadIdx.x;
    const uint32_t excl = *s_excl;
    const int64_t base = (int64_t)L.tile * kTile;
    if (MODE != kScan) {
        // The tile was compacted in LDS by lag_reduce: kept values / indices, then (partition)
        // the dropped indices.
        copy_out(s_data[par], out + excl, L.total);
        if (MODE == kPartition) copy_out(s_data[par] + L.total, dead + (base - excl), kTile - L.total);
        if (tid == 0 && L.tile == num_tiles - 1) store_count<MODE>(d_count, excl + L.total);
        return;
    }
#pragma unroll
    for (int k = 0; k < kChunks; ++k) {
        const v4i v = *reinterpret_cast<const v4i*>(&s_data[par][k * (kThreads * 4) + 4 * tid]);
        write_chunk<MODE, true>(v, base + (int64_t)k * (kThreads * 4) + 4 * tid, excl + L.pre[k], 0, out, dead);
    }
}

// One step: prefetch `next` into `pf`, reduce `cur` (= tile), resolve + write the deferred tile.
template <int MODE, bool WINDOW>
__device__ __forceinline__ void lag_step(const int32_t* __restrict__ in, const v4i (&cur)[kChunks],
                                         v4i (&pf)[kChunks], int tile, int next, int num_full, int num_tiles,
                                         int par, LagTile& prev, bool& have_prev, int32_t (*s_data)[kTile],
                                         uint32_t (*s_wsum)[kChunks][4], uint32_t* s_excl,
                                         int32_t* __restrict__ out, uint64_t* __restrict__ status,
                                         uint32_t* __restrict__ ctl, int64_t* __restrict__ d_count,
                                         int32_t* __restrict__ dead, uint32_t& carry) {
    // unconditional (clamped) prefetch: a branch here would make the wait-count pass merge
    // "issued"/"skipped" states and drain the prefetch at the first use of the other buffer
    load_full(in, (int64_t)(next < num_full ? next : tile) * kTile, (int)threadIdx.x, pf);
    LagTile L;
    lag_reduce<MODE, WINDOW>(cur, tile, par, s_data, s_wsum, status, L);
    if (have_prev) {
        if ((threadIdx.x >> 6) == 0) lag_resolve<WINDOW>(prev, s_excl, status, ctl, carry);
        lds_barrier();
        lag_store<MODE>(prev, par ^ 1, s_data, s_excl, num_tiles, out, d_count, dead);
    }
    prev = L;
    have_prev = true;
}

// Unaligned pointers: claimed tiles (above) with guarded scalar loads, prefix resolved at once.
template <int MODE>
__global__ __launch_bounds__(kThreads) void k_scan_tiles(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                         int64_t n, uint64_t* __restrict__ status,
                                                         uint32_t* __restrict__ ctl, int64_t* __restrict__ d_count,
                                                         int32_t* __restrict__ dead, int claimed) {
    __shared__ uint32_t s_wsum[kChunks][4];
    __shared__ uint32_t s_excl;
    __shared__ int s_ring[lb::kRing];
    const int num_tiles = (int)((n + kTile - 1) / kTile);
    lb::TileSeq q = lb::seq_start(claimed != 0, &ctl[kTicket], s_ring, num_tiles);
    while (q.tile != INT_MAX) {
        lb::seq_step(q, &ctl[kTicket]);
        v4i cur[kChunks];
        load_guarded(in, n, (int64_t)q.tile * kTile, threadIdx.x, cur);
        process_tile<MODE>(cur, q.tile, num_tiles, n, out, status, ctl, d_count, dead, s_wsum, &s_excl);
        lb::seq_advance(q, s_ring);
    }
}

// The partial tail tile under the static schedule (window prefix, see lag_resolve).
template <int MODE>
__device__ __forceinline__ void window_tail(const v4i (&cur)[kChunks], int tile, int num_tiles, int64_t n,
                                            int32_t* __restrict__ out, uint64_t* __restrict__ status,
                                            uint32_t* __restrict__ ctl, int64_t* __restrict__ d_count,
                                            int32_t* __restrict__ dead, uint32_t (&s_wsum)[kChunks][4],
                                            uint32_t* s_excl, uint32_t carry) {
    const int tid = threadIdx.x, lane = tid & 63;
    uint32_t pre[kChunks];
    const uint32_t total = tile_offsets<MODE>(cur, s_wsum, pre);
    if ((tid >> 6) == 0) {
        const uint32_t excl = carry + lb::window_sum(status, tile, (int)gridDim.x, lane, &ctl[1]);
        if (lane == 0) *s_excl = excl;
    }
    lds_barrier();
    const uint32_t excl = *s_excl;
    const int64_t base = (int64_t)tile * kTile;
#pragma unroll
    for (int k = 0; k < kChunks; ++k)
        write_chunk<MODE, false>(cur[k], base + (int64_t)k * (kThreads * 4) + 4 * tid, excl + pre[k], n, out, dead);
    if (MODE != kScan && tid == 0 && tile == num_tiles - 1) store_count<MODE>(d_count, excl + total);
}

// 16-byte aligned pointers: each tile's prefix resolved one step late (above).
template <int MODE, bool WINDOW>
__device__ __forceinline__ void scan_lag_body(const int32_t* __restrict__ in, int32_t* __restrict__ out, int64_t n,
                                              uint64_t* __restrict__ status, uint32_t* __restrict__ ctl,
                                              int64_t* __restrict__ d_count, int32_t* __restrict__ dead,
                                              int32_t (*s_data)[kTile], uint32_t (*s_wsum)[kChunks][4],
                                              uint32_t* s_excl, int* s_ring, bool claimed) {
    const int tid = threadIdx.x;
    const int num_tiles = (int)((n + kTile - 1) / kTile);
    const int num_full = (int)(n / kTile);
    lb::TileSeq q = lb::seq_start(claimed, &ctl[kTicket], s_ring, num_tiles);
    uint32_t carry = 0;   // WINDOW: excl + aggregate of this workgroup's previous tile (wave 0)
    if (q.tile < num_full) {
        // two named register buffers, loop unrolled by two: no load destination is ever copied,
        // so the wait-count pass keeps each prefetch in flight across the other buffer's step
        v4i bA[kChunks], bB[kChunks];
        LagTile prev;
        bool have_prev = false;
        int par = 0;
        load_full(in, (int64_t)q.tile * kTile, tid, bA);
        for (;;) {
            lb::seq_step(q, &ctl[kTicket]);
            lag_step<MODE, WINDOW>(in, bA, bB, q.tile, q.next, num_full, num_tiles, par, prev, have_prev, s_data,
                                   s_wsum, s_excl, out, status, ctl, d_count, dead, carry);
            lb::seq_advance(q, s_ring);
            par ^= 1;
            if (q.tile >= num_full) break;
            lb::seq_step(q, &ctl[kTicket]);
            lag_step<MODE, WINDOW>(in, bB, bA, q.tile, q.next, num_full, num_tiles, par, prev, have_prev, s_data,
                                   s_wsum, s_excl, out, status, ctl, d_count, dead, carry);
            lb::seq_advance(q, s_ring);
            par ^= 1;
            if (q.tile >= num_full) break;
        }
        // drain: the last reduced tile
        if ((tid >> 6) == 0) lag_resolve<WINDOW>(prev, s_excl, status, ctl, carry);
        lds_barrier();
        lag_store<MODE>(prev, par ^ 1, s_data, s_excl, num_tiles, out, d_count, dead);
    }
    // the partial tail tile (the last tile, so nothing waits on this workgroup after it)
    if (q.tile == num_full && num_full < num_tiles) {
        v4i cur[kChunks];
        load_guarded(in, n, (int64_t)q.tile * kTile, tid, cur);
        if (WINDOW)
            window_tail<MODE>(cur, q.tile, num_tiles, n, out, status, ctl, d_count, dead, s_wsum[0], s_excl, carry);
        else
            process_tile<MODE>(cur, q.tile, num_tiles, n, out, status, ctl, d_count, dead, s_wsum[0], s_excl);
    }
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void k_scan_lag(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                       int64_t n, uint64_t* __restrict__ status,
                                                       uint32_t* __restrict__ ctl, int64_t* __restrict__ d_count,
                                                       int32_t* __restrict__ dead, int claimed) {
    __shared__ __attribute__((aligned(16))) int32_t s_data[2][kTile];
    __shared__ uint32_t s_wsum[2][kChunks][4];
    __shared__ uint32_t s_excl;
    __shared__ int s_ring[lb::kRing];
    if (claimed)
        scan_lag_body<MODE, false>(in, out, n, status, ctl, d_count, dead, s_data, s_wsum, &s_excl, s_ring, true);
    else
        scan_lag_body<MODE, true>(in, out, n, status, ctl, d_count, dead, s_data, s_wsum, &s_excl, s_ring, false);
}

__global__ void k_append_dead(const int32_t* __restrict__ dead, int32_t* __restrict__ perm,
                              int64_t n, const int64_t* __restrict__ d_live) {
    const int64_t live = *d_live;
    const int64_t ndead = n - live;
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < ndead;
         j += (int64_t)gridDim.x * blockDim.x)
        perm[live + j] = dead[j];
}

// ---- host ---------------------------------------------------------------------------------
int resident_grid(const void* kernel) {
    // Persistent look-back kernels need every workgroup co-resident.  The occupancy API can
    // over-report when a resource is filled (almost) exactly (see resident_per_cu in
    // pt_kernels.hip for the measurements), so a per-CU count is accepted only while LDS
    // (<= 152 of 160 KiB) and VGPRs (<= 448 of 512 per SIMD lane) keep headroom.
    static std::mutex mu;
    static std::vector<std::pair<const void*, int>> cache;
    std::lock_guard<std::mutex> lk(mu);
    for (auto& e : cache)
        if (e.first == kernel) return e.second;
    int dev = 0, cus = 256, per_cu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kThreads, 0) != hipSuccess || per_cu <= 0)
        per_cu = 2;
    per_cu = std::min(per_cu, 8);
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, kernel) == hipSuccess) {
        const int vgpr = ((fa.numRegs + 7) / 8) * 8;
        const size_t lds = fa.sharedSizeBytes;
        while (per_cu > 1 && ((size_t)per_cu * lds > (size_t)(152 * 1024) || per_cu * vgpr > 448)) --per_cu;
    } else {
        per_cu = std::max(1, per_cu - 1);
    }
    const int g = cus * per_cu;
    cache.push_back({kernel, g});
    return g;
}

size_t status_bytes(int64_t n) {
    const int64_t tiles = (n + kTile - 1) / kTile;
    return (size_t)(tiles > 0 ? tiles : 1) * sizeof(uint64_t);
}

struct Workspace {
    void* ptr = nullptr;
    size_t bytes = 0;
};
std::mutex g_ws_mu;
std::vector<Workspace> g_ws;   // per device

int get_cached_ws(size_t need, void** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    std::lock_guard<std::mutex> lk(g_ws_mu);
    if ((int)g_ws.size() <= dev) g_ws.resize(dev + 1);
    Workspace& w = g_ws[dev];
    if (w.bytes < need) {
        if (w.ptr) (void)hipFree(w.ptr);
        w.ptr = nullptr;
        w.bytes = 0;
        e = hipMalloc(&w.ptr, need);
        if (e != hipSuccess) return hip_fail(e, "hipMalloc(workspace)");
        w.bytes = need;
    }
    *out = w.ptr;
    return SC_OK;
}

template <int MODE>
int launch(const int32_t* d_in, int32_t* d_out, int64_t n, int64_t* d_count, void* workspace,
           hipStream_t stream) {
    if (n < 0 || n > 0x7fffffffLL) return fail(SC_ERR_ARG, "n out of range [0, 2^31-1]");
    if (n > 0 && (!d_in || !d_out)) return fail(SC_ERR_ARG, "null pointer");
    if (MODE != kScan && !d_count) return fail(SC_ERR_ARG, "null count pointer");
    const size_t need = sc_workspace_bytes(n);
    if (!workspace) {
        const int rc = get_cached_ws(need, &workspace);
        if (rc) return rc;
    }
    uint8_t* ws = static_cast<uint8_t*>(workspace);
    uint32_t* ctl = reinterpret_cast<uint32_t*>(ws);
    uint64_t* status = reinterpret_cast<uint64_t*>(ws + kCtlBytes);
    int32_t* dead = reinterpret_cast<int32_t*>(ws + kCtlBytes + status_bytes(n));
    if (n == 0) {
        if (MODE != kScan) {
            hipError_t e = hipMemsetAsync(d_count, 0, MODE == kIndices ? sizeof(int32_t) : sizeof(int64_t), stream);
            if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
        }
        return SC_OK;
    }
    hipError_t e = hipMemsetAsync(ws, 0, kCtlBytes + status_bytes(n), stream);
    if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync(workspace)");
    const int64_t tiles = (n + kTile - 1) / kTile;
    const bool aligned = ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out)) & 15) == 0;
    const bool claimed = g_schedule_claimed.load(std::memory_order_relaxed);
    if (aligned) {
        const int g = (int)std::min<int64_t>(tiles, resident_grid((const void*)k_scan_lag<MODE>) * g_test_oversub);
        hipLaunchKernelGGL((k_scan_lag<MODE>), dim3(g), dim3(kThreads), 0, stream, d_in, d_out, n, status, ctl,
                           d_count, dead, (int)claimed);
    } else {
        const int g = (int)std::min<int64_t>(tiles, resident_grid((const void*)k_scan_tiles<MODE>) * g_test_oversub);
        hipLaunchKernelGGL((k_scan_tiles<MODE>), dim3(g), dim3(kThreads), 0, stream, d_in, d_out, n, status, ctl,
                           d_count, dead, (int)claimed);
    }
    e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "scan kernel launch");
    if (MODE == kPartition) {
        const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4096);
        hipLaunchKernelGGL(k_append_dead, dim3((unsigned)blocks), dim3(256), 0, stream, dead, d_out, n,
                           (const int64_t*)d_count);
        e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(e, "k_append_dead launch");
    }
    return SC_OK;
}

// The device error word of a workspace (ctl[1]): set by a look-back / window-sum wait that hit its
// spin bound (lookback.h), i.e. the static schedule's grid was not co-resident.  Each launch
// re-zeroes it, so it reports the most recent call on that workspace.  Caller has synchronised.
int read_ws_error(const void* ws) {
    uint32_t err = 0;
    hipError_t e = hipMemcpy(&err, static_cast<const uint8_t*>(ws) + sizeof(uint32_t), sizeof err, hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "hipMemcpy(workspace error word)");
    if (err) return fail(SC_ERR_HIP, "look-back spin bound hit: the scan grid was not co-resident (GPU shared? use "
                                     "sc_set_tile_schedule(1)); results of that call are invalid");
    return SC_OK;
}

// Host-pointer helper buffers (per device).
struct HostBufs {
    int32_t* in = nullptr;
    int32_t* out = nullptr;
    int64_t* cnt = nullptr;
    int64_t cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};
std::mutex g_hb_mu;
std::vector<HostBufs> g_hb;

int get_host_bufs(int64_t n, HostBufs** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    if ((int)g_hb.size() <= dev) g_hb.resize(dev + 1);
    HostBufs& b = g_hb[dev];
    if (!b.ev0) {
        if ((e = hipEventCreate(&b.ev0)) != hipSuccess) return hip_fail(e, "hipEventCreate");
        if ((e = hipEventCreate(&b.ev1)) != hipSuccess) return hip_fail(e, "hipEventCreate");
        if ((e = hipMalloc(&b.cnt, sizeof(int64_t))) != hipSuccess) return hip_fail(e, "hipMalloc");
    }
    if (b.cap < n) {
        if (b.in) (void)hipFree(b.in);
        if (b.out) (void)hipFree(b.out);
        b.in = b.out = nullptr;
        b.cap = 0;
        const size_t bytes = (size_t)(n > 0 ? n : 1) * sizeof(int32_t);
        if ((e = hipMalloc(&b.in, bytes)) != hipSuccess) return hip_fail(e, "hipMalloc(in)");
        if ((e = hipMalloc(&b.out, bytes)) != hipSuccess) return hip_fail(e, "hipMalloc(out)");
        b.cap = n;
    }
    *out = &b;
    return SC_OK;
}

template <int MODE>
int host_op(int n, int* odata, const int* idata, int* count_out) {
    if (n < 0) return fail(SC_ERR_ARG, "n < 0");
    if (n > 0 && (!odata || !idata)) return fail(SC_ERR_ARG, "null pointer");
    std::lock_guard<std::mutex> lk(g_hb_mu);
    HostBufs* b = nullptr;
    int rc = get_host_bufs(n, &b);
    if (rc) return rc;
    hipError_t e;
    if (n > 0 && (e = hipMemcpy(b->in, idata, (size_t)n * 4, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy H2D");
    void* ws = nullptr;
    if ((rc = get_cached_ws(sc_workspace_bytes(n), &ws))) return rc;
    (void)hipEventRecord(b->ev0, nullptr);
    rc = launch<MODE>(b->in, b->out, n, b->cnt, ws, nullptr);
    if (rc) return rc;
    (void)hipEventRecord(b->ev1, nullptr);
    if ((e = hipEventSynchronize(b->ev1)) != hipSuccess) return hip_fail(e, "hipEventSynchronize");
    (void)hipEventElapsedTime(&g_timer_ms, b->ev0, b->ev1);
    if ((rc = read_ws_error(ws))) return rc;
    int64_t cnt = n;
    if (MODE != kScan) {
        if ((e = hipMemcpy(&cnt, b->cnt, sizeof cnt, hipMemcpyDeviceToHost)) != hipSuccess)
            return hip_fail(e, "hipMemcpy count");
        if (count_out) *count_out = (int)cnt;
    }
    if (cnt > 0 && (e = hipMemcpy(odata, b->out, (size_t)cnt * 4, hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "hipMemcpy D2H");
    return SC_OK;
}

}  // namespace

// Shared with sc_variants.hip (the CPU / Naive / Thrust entry points): one error message and one
// "previous operation" timer per thread for the whole sc_* ABI.
namespace sc_internal {
int fail(int code, const std::string& msg) { return ::fail(code, msg); }
void set_timer_ms(float ms) { g_timer_ms = ms; }
}  // namespace sc_internal

extern "C" {

const char* sc_last_error(void) { return g_err.c_str(); }

size_t sc_workspace_bytes(int64_t n) {
    return kCtlBytes + status_bytes(n) + (size_t)(n > 0 ? n : 0) * sizeof(int32_t);
}

int sc_scan_exclusive_i32(const int32_t* d_in, int32_t* d_out, int64_t n, void* workspace, void* stream) {
    return launch<kScan>(d_in, d_out, n, nullptr, workspace, (hipStream_t)stream);
}

int sc_compact_i32(const int32_t* d_in, int32_t* d_out, int64_t n, int64_t* d_count, void* workspace,
                   void* stream) {
    return launch<kCompact>(d_in, d_out, n, d_count, workspace, (hipStream_t)stream);
}

int sc_partition_i32(const int32_t* d_flags, int32_t* d_perm, int64_t n, int64_t* d_live, void* workspace,
                     void* stream) {
    return launch<kPartition>(d_flags, d_perm, n, d_live, workspace, (hipStream_t)stream);
}

int sc_partition_indices(const int32_t* d_flags, int32_t* d_idx, int64_t n, int32_t* d_count, void* workspace,
                         void* stream) {
    return launch<kIndices>(d_flags, d_idx, n, reinterpret_cast<int64_t*>(d_count), workspace, (hipStream_t)stream);
}

int sc_efficient_scan(int n, int* odata, const int* idata) { return host_op<kScan>(n, odata, idata, nullptr); }

int sc_efficient_compact(int n, int* odata, const int* idata, int* count_out) {
    return host_op<kCompact>(n, odata, idata, count_out);
}

float sc_timer_gpu_ms(void) { return g_timer_ms; }

int sc_workspace_check(const void* workspace) {
    void* ws = const_cast<void*>(workspace);
    if (!ws) {
        int dev = 0;
        hipError_t e = hipGetDevice(&dev);
        if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
        std::lock_guard<std::mutex> lk(g_ws_mu);
        if ((int)g_ws.size() <= dev || !g_ws[dev].ptr) return SC_OK;   // never used
        ws = g_ws[dev].ptr;
    }
    hipError_t e = hipDeviceSynchronize();
    if (e != hipSuccess) return hip_fail(e, "hipDeviceSynchronize");
    return read_ws_error(ws);
}

const uint32_t* sc_workspace_error_word(const void* workspace) {
    return reinterpret_cast<const uint32_t*>(static_cast<const uint8_t*>(workspace) + sizeof(uint32_t));
}

int sc_set_tile_schedule(int32_t claimed) {
    g_schedule_claimed.store(claimed != 0, std::memory_order_relaxed);
    return SC_OK;
}

}  // extern "C"

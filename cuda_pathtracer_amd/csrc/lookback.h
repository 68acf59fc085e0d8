// Single-pass decoupled look-back prefix machinery for 256-thread (4 x wave64) workgroups.
//
// Each tile publishes one 64-bit status word {flag:2 @ bit 62 | value:32 @ bit 0} with ONE
// relaxed agent-scope atomic store (the "granule" form: the value is its own flag, so no
// release/acquire fence is needed — cdna_hip_programming.md §6 Guideline 16, R2), first the
// tile AGGREGATE, later the INCLUSIVE prefix.  A successor's wave 0 reads 4 x 64 predecessors
// per round trip with relaxed agent-scope loads and stops at the nearest inclusive prefix.
//
// Tile assignment: TileSeq below (static co-resident grid, or tiles claimed from a ticket for
// shared GPUs).  Every spin is bounded; on timeout the tile proceeds and raises *err (results
// then wrong and reported, but the kernel always drains — a hung wave would take the GPU down).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>

namespace lb {

constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagPre = 2ull << 62;
constexpr uint32_t kSpinLimit = 1u << 18;   // ~0.25 s of polling; a live chain resolves in us
constexpr int kWindows = 4;

__device__ __forceinline__ void publish(uint64_t* st, int tile, uint64_t flag, uint32_t v) {
    __hip_atomic_store(st + tile, flag | (uint64_t)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
    return v;
}

// Inclusive scan across one wave64 using DPP row shifts + row broadcasts (GFX9 family).
__device__ __forceinline__ uint32_t wave_inclusive_scan(uint32_t v) {
    // row_shr:1,2,4,8 within 16-lane rows (bound_ctrl: lanes without a source read 0)
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
    // row_bcast:15 -> rows 1 and 3; row_bcast:31 -> rows 2 and 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
    return v;
}

__device__ __forceinline__ uint64_t poll(const uint64_t* st, int j) {
    return j >= 0 ? __hip_atomic_load(st + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagPre;
}

// First-round polls of a look-back, issued early so their latency overlaps other work.
template <int WINDOWS>
__device__ __forceinline__ void prepoll(const uint64_t* st, int tile, int lane, uint64_t (&w)[WINDOWS]) {
#pragma unroll
    for (int k = 0; k < WINDOWS; ++k) w[k] = poll(st, tile - 1 - 64 * k - lane);
}

// Called by one full wave (all 64 lanes).  Returns the exclusive prefix of `tile` (> 0).
// Window w of a round covers predecessors base - 64w - lane; windows are consumed in order.
// WINDOWS x 64 predecessors are polled per round trip; `w` holds the first round's polls
// (from prepoll, or issued here when PREPOLLED is false).
template <int WINDOWS, bool PREPOLLED>
__device__ __forceinline__ uint32_t lookback_impl(uint64_t* st, int tile, int lane, uint32_t* err,
                                                  uint64_t (&w)[WINDOWS]) {
    uint32_t excl = 0;
    int base = tile - 1;
    uint32_t spins = 0;
    bool polled = PREPOLLED;
    for (;;) {
        if (!polled) {
#pragma unroll
            for (int k = 0; k < WINDOWS; ++k) w[k] = poll(st, base - 64 * k - lane);
        }
        polled = false;
        int consumed = 0;   // windows fully summed this round
        bool stalled = false;
#pragma unroll
        for (int k = 0; k < WINDOWS; ++k) {
            if (stalled) break;
            const uint64_t nr = __ballot((w[k] >> 62) == 0);
            const uint64_t pre = __ballot((w[k] >> 62) == 2);
            const int first_pre = pre ? __builtin_ctzll(pre) : 64;
            const int first_nr = nr ? __builtin_ctzll(nr) : 64;
            if (first_pre < first_nr) {
                excl += wave_sum(lane <= first_pre ? (uint32_t)w[k] : 0u);
                return excl;
            }
            if (first_nr < 64) { stalled = true; break; }
            excl += wave_sum((uint32_t)w[k]);
            ++consumed;
        }
        base -= 64 * consumed;
        if (stalled) {
            // Give up when this wave has spun too long or any other wave already gave up (so one
            // stuck chain costs ~0.25 s, not one timeout per tile): results are then wrong and
            // flagged, but the grid always drains.
            if (++spins > kSpinLimit ||
                ((spins & 63) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
                if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                return excl;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
}

template <int WINDOWS = kWindows>
__device__ __forceinline__ uint32_t lookback(uint64_t* st, int tile, int lane, uint32_t* err) {
    uint64_t w[WINDOWS];
    return lookback_impl<WINDOWS, false>(st, tile, lane, err, w);
}

// Static-schedule alternative to the look-back (sc_kernels.hip lag_resolve): the sum of the
// aggregates of tiles max(0, tile-G+1) .. tile-1, read by one full wave, kWinPolls x 64 per
// round trip.  Nothing here waits on another tile's look-back, only on aggregates, which every
// workgroup publishes as soon as it has reduced a tile.
constexpr int kWinPolls = 8;

__device__ __forceinline__ uint32_t window_sum(const uint64_t* st, int tile, int G, int lane, uint32_t* err) {
    const int lo = tile - G + 1 > 0 ? tile - G + 1 : 0;
    uint32_t acc = 0;
    uint32_t spins = 0;
    for (int top = tile - 1; top >= lo; top -= 64 * kWinPolls) {
        uint64_t w[kWinPolls];
#pragma unroll
        for (int k = 0; k < kWinPolls; ++k) {
            const int j = top - 64 * k - lane;
            w[k] = j >= lo ? poll(st, j) : kFlagAgg;
        }
        for (;;) {
            bool nr = false;
#pragma unroll
            for (int k = 0; k < kWinPolls; ++k) nr |= (w[k] >> 62) == 0;
            if (__ballot(nr) == 0) break;
            if (++spins > kSpinLimit ||
                ((spins & 63) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
                if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;   // results wrong and reported; the grid still drains
            }
            __builtin_amdgcn_s_sleep(1);
#pragma unroll
            for (int k = 0; k < kWinPolls; ++k)
                if ((w[k] >> 62) == 0) w[k] = poll(st, top - 64 * k - lane);
        }
#pragma unroll
        for (int k = 0; k < kWinPolls; ++k) acc += (uint32_t)w[k];
    }
    return wave_sum(acc);
}

// ---- tile schedules ------------------------------------------------------------------------
// STATIC (default, fastest): a grid of G workgroups that must all be resident at once (sized by
// the host from the occupancy with headroom); workgroup b owns tiles b, b+G, b+2G, ...  No
// atomics.  If part of the grid cannot become resident — another kernel or process holding the
// GPU — the look-back stalls, hits its spin bound and the launch reports an error (it never
// hangs).
// CLAIMED (shared GPUs): each tile is claimed from a ticket on its own, so claim order == tile
// order: every predecessor of a claimed tile was claimed earlier by a running workgroup and the
// lowest unfinished tile always progresses, whatever else runs on the GPU.  A workgroup claims
// kAhead steps ahead, so the claim's round trip overlaps its current work and consecutive tiles
// go to different workgroups (contiguous multi-tile claims would chain each chunk's first
// look-back to the previous chunk's last tile — measured 100x slower).  The cost is one
// device-scope atomic per tile on one address, which saturates at ~88/us on MI355X: about 2x
// slower bounce kernels at 256-path tiles, ~15% slower scans.
//   Claimed mode plumbing: the claim returned at step k is written to the LDS ring at the END of
// step k (so the wave does not stall on the atomic) and read at the top of step k + 2, after step
// k + 1's barriers; the caller's per-step work must contain a workgroup barrier.
constexpr int kAhead = 3;   // claims in flight: next, next + 1, next + 2
constexpr int kRing = 4;

struct TileSeq {
    int tile;      // current tile (INT_MAX: done)
    int next;      // the tile after it (INT_MAX: none)
    int k;         // step index (ring position)
    int limit;
    bool claimed;
    uint32_t pending;   // thread 0: claim issued this step, stored at seq_advance
};

// Block-wide start (contains a barrier in claimed mode).
__device__ __forceinline__ TileSeq seq_start(bool claimed, uint32_t* ticket, int* s_ring, int limit) {
    TileSeq q;
    q.k = 0;
    q.limit = limit;
    q.claimed = claimed;
    q.pending = 0;
    if (!claimed) {
        q.tile = (int)blockIdx.x < limit ? (int)blockIdx.x : INT_MAX;
        const int n = (int)blockIdx.x + (int)gridDim.x;
        q.next = n < limit ? n : INT_MAX;
        return q;
    }
    if (threadIdx.x == 0)
        for (int i = 0; i < kAhead; ++i) s_ring[i] = (int)atomicAdd(ticket, 1u);
    __syncthreads();
    q.tile = s_ring[0] < limit ? s_ring[0] : INT_MAX;
    q.next = s_ring[1] < limit ? s_ring[1] : INT_MAX;
    return q;
}

// Top of a step: claimed mode, thread 0 claims the tile for step k + kAhead (kept in a register).
__device__ __forceinline__ void seq_step(TileSeq& q, uint32_t* ticket) {
    if (q.claimed && q.next != INT_MAX && threadIdx.x == 0) q.pending = atomicAdd(ticket, 1u);
}

// Bottom of a step: publish the claim, then move on.
__device__ __forceinline__ void seq_advance(TileSeq& q, int* s_ring) {
    if (q.tile == INT_MAX) return;
    if (!q.claimed) {
        q.tile = q.next;
        if (q.tile == INT_MAX) return;
        const int n = q.tile + (int)gridDim.x;
        q.next = n < q.limit ? n : INT_MAX;
        return;
    }
    if (threadIdx.x == 0) s_ring[(q.k + kAhead) % kRing] = q.next != INT_MAX ? (int)q.pending : INT_MAX;
    ++q.k;
    q.tile = q.next;
    if (q.tile == INT_MAX) return;
    const int c = s_ring[(q.k + 1) % kRing];   // claimed at step k - 1, published before its barriers
    q.next = c < q.limit ? c : INT_MAX;
}

}  // namespace lb

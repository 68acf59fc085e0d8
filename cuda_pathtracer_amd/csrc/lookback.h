// Single-pass decoupled look-back prefix machinery for 256-thread (4 x wave64) workgroups.
//
// Each tile publishes one 64-bit status word {flag:2 @ bit 62 | value:32 @ bit 0} with ONE
// relaxed agent-scope atomic store (the "granule" form: the value is its own flag, so no
// release/acquire fence is needed — cdna_hip_programming.md §6 Guideline 16, R2), first the
// tile AGGREGATE, later the INCLUSIVE prefix.  A successor's wave 0 reads 4 x 64 predecessors
// per round trip with relaxed agent-scope loads and stops at the nearest inclusive prefix.
//
// Tile assignment is STATIC and persistent: a grid of G co-resident workgroups, workgroup b
// owns tiles b, b+G, b+2G, ... and processes them in increasing order.  There is no ticket
// counter (a single returning atomic saturates at ~88 dequeues/us on MI355X, which made the
// ticket the bottleneck).  Forward progress: the lowest unpublished tile's predecessors are all
// published and its workgroup is resident (G <= resident capacity, see grid_for()), so it
// completes.  Every spin is still bounded; on timeout the tile proceeds and raises *err
// (results then wrong, but the kernel always drains — a hung wave would take the GPU down).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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

}  // namespace lb

// Single-pass decoupled look-back prefix machinery for 256-thread (4 x wave64) workgroups.
//
// Each tile publishes one 64-bit status word {flag:2 @ bit 62 | value:32 @ bit 0} with ONE
// relaxed agent-scope atomic store (the "granule" form: the value is its own flag, so no
// release/acquire fence is needed — cdna_hip_programming.md §6 Guideline 16, R2), first the
// tile AGGREGATE, later the INCLUSIVE prefix.  A successor's wave 0 reads 64 predecessors per
// step with relaxed agent-scope loads (sc1: bypass the stale per-CU L1) and stops at the
// nearest inclusive prefix.  Tile ids come from an atomic ticket so every predecessor of a
// running tile is already resident (forward progress without co-residency assumptions).
// Every spin is bounded; on timeout the tile proceeds and raises *err (results then wrong,
// but the kernel always drains — a hung wave would take the GPU down).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lb {

constexpr uint64_t kFlagAgg = 1ull << 62;
constexpr uint64_t kFlagPre = 2ull << 62;
constexpr uint32_t kSpinLimit = 1u << 22;

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

// Called by one full wave (all 64 lanes).  Returns the exclusive prefix of `tile` (> 0).
__device__ __forceinline__ uint32_t lookback(uint64_t* st, int tile, int lane, uint32_t* err) {
    uint32_t excl = 0;
    int base = tile - 1;
    for (;;) {
        const int j = base - lane;
        uint64_t w;
        uint32_t spins = 0;
        int first_pre;
        for (;;) {
            w = j >= 0 ? __hip_atomic_load(st + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagPre;
            const uint64_t not_ready = __ballot((w >> 62) == 0);
            const uint64_t pre = __ballot((w >> 62) == 2);
            first_pre = pre ? __builtin_ctzll(pre) : 64;
            const int first_nr = not_ready ? __builtin_ctzll(not_ready) : 64;
            if (first_nr > first_pre || first_nr == 64) break;
            if (++spins > kSpinLimit) {
                if (lane == 0) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                first_pre = first_nr;   // give up: treat the unready word as a zero prefix
                w = (lane == first_nr) ? kFlagPre : w;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t v = (lane <= first_pre) ? (uint32_t)w : 0u;
        excl += wave_sum(v);
        if (first_pre < 64) return excl;
        base -= 64;
    }
}

}  // namespace lb

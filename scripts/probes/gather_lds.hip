// Probe (round 4): a divergent gather of 128-byte rows (k_traverse4's quads: 112 B used), per wave
// of 64 rows, five ways.  Prints ps per row for tables of 20k rows (2.5 MB, config 5's quad table),
// 200k and 2M rows.
//   A : each lane loads its own row, 7 dwordx4 (the shipped walk).
//   B : 8 lanes per row per instruction (8 instructions), pieces stay in the loading lanes.
//   C : as B, pieces through LDS rows of 128 B (ds_write_b128; 8-way read conflicts) to the owner.
//   S : as C with the 16-byte columns of row s rotated by s >> 1: conflict-free ds_read_b128.
//   G : as S, but the pieces go global -> LDS directly (global_load_lds_dwordx4): the lane computes
//       which chunk lands in its fixed LDS slot (base + 16 lane).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned hsh(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void kA(const v4f* __restrict__ rows, unsigned R, int iters, float* out) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        const unsigned r = hsh(t * 977u + it) % R;
        const v4f* p = rows + (size_t)r * 8;
        v4f v[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < 7; ++k) acc += v[k][0] + v[k][1] + v[k][2] + v[k][3];
    }
    out[t] = acc;
}

__global__ __launch_bounds__(256) void kB(const v4f* __restrict__ rows, unsigned R, int iters, float* out) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        const unsigned r = hsh(t * 977u + it) % R;
        v4f v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned rr = __shfl(r, j * 8 + (lane >> 3), 64);
            v[j] = rows[(size_t)rr * 8 + (lane & 7)];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += v[j][0] + v[j][1] + v[j][2] + v[j][3];
    }
    out[t] = acc;
}

template <bool SWZ>
__global__ __launch_bounds__(256) void kCS(const v4f* __restrict__ rows, unsigned R, int iters, float* out) {
    __shared__ v4f lds[4][64 * 8];
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        const unsigned r = hsh(t * 977u + it) % R;
        v4f v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned rr = __shfl(r, j * 8 + (lane >> 3), 64);
            v[j] = rows[(size_t)rr * 8 + (lane & 7)];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int s = j * 8 + (lane >> 3), c = lane & 7;
            lds[w][s * 8 + (SWZ ? ((c + (s >> 1)) & 7) : c)] = v[j];
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0)
        __builtin_amdgcn_wave_barrier();
        v4f u[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) u[k] = lds[w][lane * 8 + (SWZ ? ((k + (lane >> 1)) & 7) : k)];
#pragma unroll
        for (int k = 0; k < 7; ++k) acc += u[k][0] + u[k][1] + u[k][2] + u[k][3];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
    out[t] = acc;
}

__global__ __launch_bounds__(256) void kG(const v4f* __restrict__ rows, unsigned R, int iters, float* out) {
    __shared__ v4f lds[4][64 * 8];
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        const unsigned r = hsh(t * 977u + it) % R;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int s = j * 8 + (lane >> 3);
            const unsigned rr = __shfl(r, s, 64);
            const int c = ((lane & 7) - (s >> 1)) & 7;   // the chunk whose rotated column is lane & 7
            __builtin_amdgcn_global_load_lds(
                reinterpret_cast<const void*>(rows + (size_t)rr * 8 + c),
                reinterpret_cast<__attribute__((address_space(3))) void*>(
                    reinterpret_cast<uintptr_t>(&lds[w][j * 64])), 16, 0, 0);
        }
        __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): the DMA landed
        __builtin_amdgcn_wave_barrier();
        v4f u[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) u[k] = lds[w][lane * 8 + ((k + (lane >> 1)) & 7)];
#pragma unroll
        for (int k = 0; k < 7; ++k) acc += u[k][0] + u[k][1] + u[k][2] + u[k][3];
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
    }
    out[t] = acc;
}

int main() {
    const int iters = 64, blocks = 4096;
    v4f* rows; float* out;
    const unsigned Rs[3] = {20000u, 200000u, 2000000u};
    hipMalloc(&rows, (size_t)2000000 * 128);
    // row r, chunk k = (r, k, r + k, 1): the sums differ between variants only by summation order
    v4f* h = (v4f*)malloc((size_t)2000000 * 128);
    for (size_t i = 0; i < (size_t)2000000 * 8; ++i) h[i] = v4f{(float)(i >> 3), (float)(i & 7), 1.f, 0.f};
    hipMemcpy(rows, h, (size_t)2000000 * 128, hipMemcpyHostToDevice);
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    float* ho = (float*)malloc((size_t)blocks * 256 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (unsigned R : Rs) {
        double ref = 0;
        for (int k = 0; k < 5; ++k) {
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                hipEventRecord(a);
                if (k == 0) kA<<<blocks, 256>>>(rows, R, iters, out);
                if (k == 1) kB<<<blocks, 256>>>(rows, R, iters, out);
                if (k == 2) kCS<false><<<blocks, 256>>>(rows, R, iters, out);
                if (k == 3) kCS<true><<<blocks, 256>>>(rows, R, iters, out);
                if (k == 4) kG<<<blocks, 256>>>(rows, R, iters, out);
                hipEventRecord(b); hipEventSynchronize(b);
                float ms; hipEventElapsedTime(&ms, a, b);
                if (rep) best = ms < best ? ms : best;
            }
            hipMemcpy(ho, out, (size_t)blocks * 256 * 4, hipMemcpyDeviceToHost);
            double sum = 0;   // checksum of the 7 used chunks (B sums all 8: reported, not compared)
            for (int i = 0; i < blocks * 256; ++i) sum += ho[i];
            if (k == 0) ref = sum;
            const double nrows = (double)blocks * 256 * iters;
            printf("R=%u kernel %c: %.3f ms, %.3f ps per row, %.2f Grows/s, checksum %s\n", R, "ABCSG"[k], best,
                   best * 1e9 / nrows, nrows / best / 1e6, k == 1 ? "(8 chunks)" : (sum == ref ? "ok" : "DIFF"));
        }
    }
    return 0;
}

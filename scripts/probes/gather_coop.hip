// Probe: does a divergent 128-byte-row gather cost per lane-line or per instruction?
//   A  : each lane loads its own row with 7 dwordx4 loads (k_traverse4's quad fetch).
//   B  : the wave loads the same 64 rows cooperatively, 8 lanes per row per instruction (8 loads),
//        pieces stay in the loading lanes (load cost only).
//   C  : as B, then the pieces go through LDS to the owning lane (7 ds_read_b128 each).
// Rows are random in a table of R rows (2.5 MB ~ config 5's quads, or larger).  Prints ns per row.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ unsigned hsh(unsigned x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ __launch_bounds__(256) void kA(const float4* __restrict__ rows, unsigned R, int iters, float* out) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        const unsigned r = hsh(t * 977u + it) % R;
        const float4* p = rows + (size_t)r * 8;
        float4 v[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < 7; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
    }
    out[t] = acc;
}

__global__ __launch_bounds__(256) void kB(const float4* __restrict__ rows, unsigned R, int iters, float* out) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        const unsigned r = hsh(t * 977u + it) % R;
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned rr = __shfl(r, j * 8 + (lane >> 3), 64);
            v[j] = (lane & 7) < 7 ? rows[(size_t)rr * 8 + (lane & 7)] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += v[j].x + v[j].y + v[j].z + v[j].w;
    }
    out[t] = acc;
}

__global__ __launch_bounds__(256) void kC(const float4* __restrict__ rows, unsigned R, int iters, float* out) {
    __shared__ float4 lds[4][64 * 8];
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    float acc = 0.f;
    for (int it = 0; it < iters; ++it) {
        const unsigned r = hsh(t * 977u + it) % R;
        float4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const unsigned rr = __shfl(r, j * 8 + (lane >> 3), 64);
            v[j] = (lane & 7) < 7 ? rows[(size_t)rr * 8 + (lane & 7)] : make_float4(0, 0, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) lds[w][(j * 8 + (lane >> 3)) * 8 + (lane & 7)] = v[j];
        __builtin_amdgcn_s_waitcnt(0xc07f);   // lgkmcnt(0): the wave's own LDS writes
        __builtin_amdgcn_wave_barrier();
        float4 u[7];
#pragma unroll
        for (int k = 0; k < 7; ++k) u[k] = lds[w][lane * 8 + k];
#pragma unroll
        for (int k = 0; k < 7; ++k) acc += u[k].x + u[k].y + u[k].z + u[k].w;
        __builtin_amdgcn_wave_barrier();
    }
    out[t] = acc;
}


// D: two lanes per row (lanes 2i, 2i+1 load the row's halves: 4 dwordx4 each); 32 rows per wave-iteration
// E: four lanes per row (2 dwordx4 each); 16 rows per wave-iteration.  Same rows per thread-iteration as A/2, A/4.
template <int L>
__global__ __launch_bounds__(256) void kDE(const float4* __restrict__ rows, unsigned R, int iters, float* out) {
    const unsigned t = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    float acc = 0.f;
    for (int it = 0; it < iters * L; ++it) {
        const unsigned r = hsh((t / L) * 977u + it) % R;
        const float4* p = rows + (size_t)r * 8 + (lane % L) * (8 / L);
        float4 v[8 / L];
#pragma unroll
        for (int k = 0; k < 8 / L; ++k) v[k] = p[k];
#pragma unroll
        for (int k = 0; k < 8 / L; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
    }
    out[t] = acc;
}

int main(int argc, char** argv) {
    const int iters = 64, blocks = 4096;
    float4* rows; float* out;
    const unsigned Rs[3] = {20000u, 200000u, 2000000u};
    hipMalloc(&rows, (size_t)2000000 * 128);
    hipMemset(rows, 0, (size_t)2000000 * 128);
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (unsigned R : Rs) {
        for (int k = 0; k < 5; ++k) {
            float best = 1e30f;
            for (int rep = 0; rep < 5; ++rep) {
                hipEventRecord(a);
                if (k == 0) kA<<<blocks, 256>>>(rows, R, iters, out);
                if (k == 1) kB<<<blocks, 256>>>(rows, R, iters, out);
                if (k == 2) kC<<<blocks, 256>>>(rows, R, iters, out);
                if (k == 3) kDE<2><<<blocks, 256>>>(rows, R, iters, out);
                if (k == 4) kDE<4><<<blocks, 256>>>(rows, R, iters, out);
                hipEventRecord(b); hipEventSynchronize(b);
                float ms; hipEventElapsedTime(&ms, a, b);
                if (rep) best = ms < best ? ms : best;
            }
            const double nrows = (double)blocks * 256 * iters;
            printf("R=%u kernel %c: %.3f ms, %.3f ps per row, %.2f Grows/s\n", R, "ABCDE"[k], best,
                   best * 1e9 / nrows, nrows / best / 1e6);
        }
    }
    return 0;
}

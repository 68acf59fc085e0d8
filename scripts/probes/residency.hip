// Co-residency probe: can cus * k workgroups of 256 threads with L bytes of LDS all be resident
// at once?  Each workgroup bumps a counter and spins (bounded) until every workgroup arrived.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void probe(unsigned* counter, unsigned total, unsigned* ok, unsigned long long limit) {
    extern __shared__ int lds[];
    if (threadIdx.x == 0) {
        lds[0] = 1;
        __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned long long spins = 0;
        while (__hip_atomic_load(counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < total && ++spins < limit)
            __builtin_amdgcn_s_sleep(2);
        if (spins < limit) __hip_atomic_fetch_add(ok, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (lds[0] != 1) ok[1] = 1;
}

int main() {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    unsigned *counter, *ok;
    hipMalloc(&counter, 4);
    hipMalloc(&ok, 8);
    const int lds_kb[] = {64, 48, 40, 32, 24, 16};
    for (int kb : lds_kb) {
        int occ = 0;
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, probe, 256, kb * 1024);
        for (int per = occ - 1; per <= occ; ++per) {
            if (per < 1) continue;
            const unsigned total = (unsigned)(cus * per);
            hipMemset(counter, 0, 4);
            hipMemset(ok, 0, 8);
            hipLaunchKernelGGL(probe, dim3(total), dim3(256), kb * 1024, 0, counter, total, ok, 200000ull);
            hipDeviceSynchronize();
            unsigned h[2];
            hipMemcpy(h, ok, 8, hipMemcpyDeviceToHost);
            printf("LDS %2d KiB: occupancy %d, %d/CU x %d CUs = %u workgroups: %u co-resident%s\n", kb, occ, per, cus,
                   total, h[0], h[0] == total ? " (all)" : "  <-- NOT all");
        }
    }
    return 0;
}

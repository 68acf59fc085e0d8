// StreamCompaction::{Efficient, CPU, Naive, Thrust} over the C ABI (see stream_compaction.h).
#include "stream_compaction.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "sc_amd.h"

namespace {

// checkCUDAError (common.cu:3-15): print the message and exit.
void check(int rc, const char* what) {
    if (rc == SC_OK) return;
    std::fprintf(stderr, "StreamCompaction error: %s: %s\n", what, sc_last_error());
    std::exit(EXIT_FAILURE);
}

bool on_device(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

struct DeviceCount {   // one int64 on the device for the kept count
    int64_t* p = nullptr;
    ~DeviceCount() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

namespace StreamCompaction {
namespace Efficient {

Common::PerformanceTimer& timer() {
    static Common::PerformanceTimer t;
    return t;
}

void scan(int n, int* odata, const int* idata) {
    if (on_device(odata) && on_device(idata)) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        (void)hipEventRecord(a, nullptr);
        check(sc_scan_exclusive_i32(idata, odata, n, nullptr, nullptr), "scan");
        (void)hipEventRecord(b, nullptr);
        (void)hipEventSynchronize(b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        timer().setGpuElapsed(ms);
        return;
    }
    check(sc_efficient_scan(n, odata, idata), "scan");
    timer().setGpuElapsed(sc_timer_gpu_ms());
}

int compact(int n, int* odata, const int* idata) {
    if (on_device(odata) && on_device(idata)) {
        static DeviceCount cnt;
        if (!cnt.p && hipMalloc(&cnt.p, sizeof(int64_t)) != hipSuccess) check(SC_ERR_NOMEM, "hipMalloc");
        check(sc_compact_i32(idata, odata, n, cnt.p, nullptr, nullptr), "compact");
        int64_t h = 0;
        if (hipMemcpy(&h, cnt.p, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) check(SC_ERR_HIP, "hipMemcpy");
        return (int)h;
    }
    int count = 0;
    check(sc_efficient_compact(n, odata, idata, &count), "compact");
    timer().setGpuElapsed(sc_timer_gpu_ms());
    return count;
}

}  // namespace Efficient

namespace CPU {

Common::PerformanceTimer& timer() {
    static Common::PerformanceTimer t;
    return t;
}

void scan(int n, int* odata, const int* idata) {
    timer().startCpuTimer();
    const int rc = sc_cpu_scan(n, odata, idata);
    timer().endCpuTimer();
    check(rc, "CPU::scan");
}

int compactWithoutScan(int n, int* odata, const int* idata) {
    int count = 0;
    timer().startCpuTimer();
    const int rc = sc_cpu_compact_without_scan(n, odata, idata, &count);
    timer().endCpuTimer();
    check(rc, "CPU::compactWithoutScan");
    return count;
}

int compactWithScan(int n, int* odata, const int* idata) {
    int count = 0;
    timer().startCpuTimer();
    const int rc = sc_cpu_compact_with_scan(n, odata, idata, &count);
    timer().endCpuTimer();
    check(rc, "CPU::compactWithScan");
    return count;
}

}  // namespace CPU

namespace Naive {

Common::PerformanceTimer& timer() {
    static Common::PerformanceTimer t;
    return t;
}

void scan(int n, int* odata, const int* idata) {
    check(sc_naive_scan(n, odata, idata), "Naive::scan");
    timer().setGpuElapsed(sc_timer_gpu_ms());
}

}  // namespace Naive

namespace Thrust {

Common::PerformanceTimer& timer() {
    static Common::PerformanceTimer t;
    return t;
}

void scan(int n, int* odata, const int* idata) {
    check(sc_thrust_scan(n, odata, idata), "Thrust::scan");
    timer().setGpuElapsed(sc_timer_gpu_ms());
}

}  // namespace Thrust
}  // namespace StreamCompaction

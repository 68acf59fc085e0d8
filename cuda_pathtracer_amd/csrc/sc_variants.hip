// StreamCompaction's other three namespaces, behind the same C ABI as Efficient (include/sc_amd.h):
//   CPU::scan / compactWithoutScan / compactWithScan   cpu.h:9-13,  cpu.cu:16-79
//   Naive::scan                                        naive.h:9,   naive.cu:14-66
//   Thrust::scan                                       thrust.h:9,  thrust.cu:14-28
// These are not on the path tracer's hot path (pathtrace.cu calls Efficient only); they exist so
// that the reference's stream_compaction self-test (stream_compaction/src/main.cpp:31-85) builds
// against the C++ mirror unchanged and compares the four implementations, as it does there.
//
// CPU: sequential host loops (the reference's loops carry `#pragma omp parallel for` over a
// loop-carried sum and a shared counter; what its tests check is the sequential result, which is
// what these compute).  The scan may run in place (odata == idata).
// Naive: Hillis & Steele on the device, one launch per distance 1, 2, 4, ... < n, ping-ponging
// between two buffers, then a shift to the exclusive result — the reference's algorithm.  Each
// thread handles 4 consecutive elements: 16-byte loads of its own four and, when the distance is
// a multiple of 4, of the four `distance` before them.
// Thrust: rocThrust's exclusive_scan (the reference calls thrust::exclusive_scan).  rocThrust
// allocates and frees its temporary storage on every call, which synchronises the device: unlike
// the Efficient and Naive entry points, the Thrust one is not asynchronous on its stream.
// Sums wrap in int32 like the reference's (two's complement; computed in uint32 here, so the
// wrap is defined behaviour).
#include <hip/hip_runtime.h>
#include <thrust/execution_policy.h>
#include <thrust/scan.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sc_amd.h"

namespace sc_internal {
int fail(int code, const std::string& msg);   // sc_kernels.hip: sets sc_last_error()
void set_timer_ms(float ms);                  // sc_kernels.hip: sc_timer_gpu_ms()
}  // namespace sc_internal

namespace {

using sc_internal::fail;

int hip_fail(hipError_t e, const char* where) {
    return fail(SC_ERR_HIP, std::string(where) + ": " + hipGetErrorString(e));
}

int host_args(int n, const void* odata, const void* idata) {
    if (n < 0) return fail(SC_ERR_ARG, "n < 0");
    if (n > 0 && (!odata || !idata)) return fail(SC_ERR_ARG, "null pointer");
    return SC_OK;
}

// ---- Naive: Hillis & Steele ----------------------------------------------------------------------
constexpr int kNaiveThreads = 256;
typedef int v4i __attribute__((ext_vector_type(4)));

// out[i] = in[i] + in[i - dist] (i >= dist), in[i] otherwise, for i in [4t, 4t + 4) of thread t.
__global__ __launch_bounds__(kNaiveThreads) void k_naive_pass(const int32_t* __restrict__ in,
                                                            int32_t* __restrict__ out, int64_t n, int64_t dist,
                                                            bool vec) {
    const int64_t stride = (int64_t)gridDim.x * kNaiveThreads * 4;
    for (int64_t i = ((int64_t)blockIdx.x * kNaiveThreads + threadIdx.x) * 4; i < n; i += stride) {
        if (vec && i + 4 <= n && i >= dist && (dist & 3) == 0) {
            const v4i a = *reinterpret_cast<const v4i*>(in + i);
            const v4i b = *reinterpret_cast<const v4i*>(in + i - dist);
            v4i c;
            for (int k = 0; k < 4; ++k) c[k] = (int32_t)((uint32_t)a[k] + (uint32_t)b[k]);
            *reinterpret_cast<v4i*>(out + i) = c;
        } else {
            for (int64_t j = i; j < i + 4 && j < n; ++j)
                out[j] = j >= dist ? (int32_t)((uint32_t)in[j] + (uint32_t)in[j - dist]) : in[j];
        }
    }
}

// Inclusive -> exclusive (naive.cu gpu_incl2excl_pfxsum): out[i] = i == 0 ? 0 : in[i - 1].
__global__ __launch_bounds__(kNaiveThreads) void k_naive_shift(const int32_t* __restrict__ in,
                                                             int32_t* __restrict__ out, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * kNaiveThreads;
    for (int64_t i = (int64_t)blockIdx.x * kNaiveThreads + threadIdx.x; i < n; i += stride)
        out[i] = i == 0 ? 0 : in[i - 1];
}

int naive_grid(int64_t elems_per_thread, int64_t n) {
    const int64_t want = (n + kNaiveThreads * elems_per_thread - 1) / (kNaiveThreads * elems_per_thread);
    return (int)std::max<int64_t>(1, std::min<int64_t>(want, 256 * 16));   // grid-stride beyond 16 per CU
}

int naive_device(const int32_t* d_in, int32_t* d_out, int64_t n, int32_t* d_tmp, hipStream_t st) {
    if (n < 0 || n > 0x7fffffffLL) return fail(SC_ERR_ARG, "n out of range [0, 2^31-1]");
    if (n == 0) return SC_OK;
    if (!d_in || !d_out || (n > 1 && !d_tmp)) return fail(SC_ERR_ARG, "null pointer");
    if (d_out == d_in || d_tmp == d_in || d_tmp == d_out) return fail(SC_ERR_ARG, "buffers must not alias");
    // 16-byte vector loads and stores only when every base is 16-byte aligned (a torch view with a
    // storage offset is only 4-byte aligned); the scalar path otherwise
    const bool vec = ((reinterpret_cast<uintptr_t>(d_in) | reinterpret_cast<uintptr_t>(d_out) |
                       reinterpret_cast<uintptr_t>(d_tmp)) & 15) == 0;
    int passes = 0;
    while ((int64_t)1 << passes < n) ++passes;   // ilog2ceil(n) (common.h:24-26); 0 for n == 1
    // ping-pong so that the last pass writes d_tmp, from which the shift writes d_out
    const int32_t* src = d_in;
    for (int p = 0; p < passes; ++p) {
        int32_t* dst = ((passes - 1 - p) & 1) ? d_out : d_tmp;
        hipLaunchKernelGGL(k_naive_pass, dim3(naive_grid(4, n)), dim3(kNaiveThreads), 0, st, src, dst, n,
                           (int64_t)1 << p, vec);
        src = dst;
    }
    hipLaunchKernelGGL(k_naive_shift, dim3(naive_grid(1, n)), dim3(kNaiveThreads), 0, st, src, d_out, n);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SC_OK : hip_fail(e, "naive scan launch");
}

int thrust_device(const int32_t* d_in, int32_t* d_out, int64_t n, hipStream_t st) {
    if (n < 0 || n > 0x7fffffffLL) return fail(SC_ERR_ARG, "n out of range [0, 2^31-1]");
    if (n == 0) return SC_OK;
    if (!d_in || !d_out) return fail(SC_ERR_ARG, "null pointer");
    // uint32 arithmetic: the int32 wrap of the reference's sums, without signed overflow
    const uint32_t* in = reinterpret_cast<const uint32_t*>(d_in);
    uint32_t* out = reinterpret_cast<uint32_t*>(d_out);
    try {
        thrust::exclusive_scan(thrust::hip::par.on(st), in, in + n, out, 0u);
    } catch (const std::exception& ex) {
        return fail(SC_ERR_HIP, std::string("thrust::exclusive_scan: ") + ex.what());
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? SC_OK : hip_fail(e, "thrust::exclusive_scan");
}

// Host-array calls (the reference's signatures): device buffers cached per device, the device
// work timed with hipEvents after the upload (PerformanceTimer::startGpuTimer's placement).
struct Bufs {
    int32_t* a = nullptr;
    int32_t* b = nullptr;
    int32_t* c = nullptr;
    int64_t cap = 0;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
};
std::mutex g_mu;
std::vector<Bufs> g_bufs;

int get_bufs(int64_t n, Bufs** out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
    if ((int)g_bufs.size() <= dev) g_bufs.resize(dev + 1);
    Bufs& b = g_bufs[dev];
    if (!b.ev0) {
        if ((e = hipEventCreate(&b.ev0)) != hipSuccess) return hip_fail(e, "hipEventCreate");
        if ((e = hipEventCreate(&b.ev1)) != hipSuccess) return hip_fail(e, "hipEventCreate");
    }
    if (b.cap < n) {
        for (int32_t** p : {&b.a, &b.b, &b.c})
            if (*p) { (void)hipFree(*p); *p = nullptr; }
        b.cap = 0;
        const size_t bytes = (size_t)std::max<int64_t>(n, 1) * sizeof(int32_t);
        for (int32_t** p : {&b.a, &b.b, &b.c})
            if ((e = hipMalloc(p, bytes)) != hipSuccess) return hip_fail(e, "hipMalloc");
        b.cap = n;
    }
    *out = &b;
    return SC_OK;
}

template <class Op>
int host_scan(int n, int* odata, const int* idata, Op op) {
    int rc = host_args(n, odata, idata);
    if (rc) return rc;
    std::lock_guard<std::mutex> lk(g_mu);
    Bufs* b = nullptr;
    if ((rc = get_bufs(n, &b))) return rc;
    hipError_t e;
    if (n > 0 && (e = hipMemcpy(b->a, idata, (size_t)n * 4, hipMemcpyHostToDevice)) != hipSuccess)
        return hip_fail(e, "hipMemcpy H2D");
    (void)hipEventRecord(b->ev0, nullptr);
    if ((rc = op(b->a, b->b, (int64_t)n, b->c))) return rc;
    (void)hipEventRecord(b->ev1, nullptr);
    if ((e = hipEventSynchronize(b->ev1)) != hipSuccess) return hip_fail(e, "hipEventSynchronize");
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, b->ev0, b->ev1);
    sc_internal::set_timer_ms(ms);
    if (n > 0 && (e = hipMemcpy(odata, b->b, (size_t)n * 4, hipMemcpyDeviceToHost)) != hipSuccess)
        return hip_fail(e, "hipMemcpy D2H");
    return SC_OK;
}

}  // namespace

extern "C" {

int sc_cpu_scan(int n, int* odata, const int* idata) {
    const int rc = host_args(n, odata, idata);
    if (rc) return rc;
    uint32_t run = 0;
    for (int i = 0; i < n; ++i) {   // (idata[i] read before odata[i] is written: in place is fine)
        const uint32_t v = (uint32_t)idata[i];
        odata[i] = (int32_t)run;
        run += v;
    }
    return SC_OK;
}

int sc_cpu_compact_without_scan(int n, int* odata, const int* idata, int* count_out) {
    const int rc = host_args(n, odata, idata);
    if (rc) return rc;
    int cnt = 0;
    for (int i = 0; i < n; ++i)
        if (idata[i] != 0) odata[cnt++] = idata[i];
    if (count_out) *count_out = cnt;
    return SC_OK;
}

int sc_cpu_compact_with_scan(int n, int* odata, const int* idata, int* count_out) {
    const int rc = host_args(n, odata, idata);
    if (rc) return rc;
    // map to booleans, exclusive scan of the booleans, scatter (cpu.cu:59-79's three steps)
    std::vector<int32_t> keep((size_t)n), pos((size_t)n);
    for (int i = 0; i < n; ++i) keep[(size_t)i] = idata[i] != 0 ? 1 : 0;
    int32_t run = 0;
    for (int i = 0; i < n; ++i) { pos[(size_t)i] = run; run += keep[(size_t)i]; }
    for (int i = 0; i < n; ++i)
        if (keep[(size_t)i]) odata[pos[(size_t)i]] = idata[i];
    if (count_out) *count_out = run;
    return SC_OK;
}

int sc_naive_scan_i32(const int32_t* d_in, int32_t* d_out, int64_t n, int32_t* d_tmp, void* stream) {
    return naive_device(d_in, d_out, n, d_tmp, (hipStream_t)stream);
}

int sc_thrust_scan_i32(const int32_t* d_in, int32_t* d_out, int64_t n, void* stream) {
    return thrust_device(d_in, d_out, n, (hipStream_t)stream);
}

int sc_naive_scan(int n, int* odata, const int* idata) {
    return host_scan(n, odata, idata, [](int32_t* in, int32_t* out, int64_t m, int32_t* tmp) {
        return naive_device(in, out, m, tmp, nullptr);
    });
}

int sc_thrust_scan(int n, int* odata, const int* idata) {
    return host_scan(n, odata, idata, [](int32_t* in, int32_t* out, int64_t m, int32_t*) {
        return thrust_device(in, out, m, nullptr);
    });
}

}  // extern "C"

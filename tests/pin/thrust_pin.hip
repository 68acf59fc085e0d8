// TEST INFRASTRUCTURE ONLY — pins the oracle's restatement of the reference's third-party
// arithmetic against the real implementation of that library: rocThrust (system ROCm 7.2,
// /opt/rocm/include/thrust; the reference uses CUDA Thrust with the same API), not reference code.
// Built by cuda_pathtracer_amd/build.py (build_pin) into tests/pin/build/libthrust_pin.so and
// called only by tests/ (test_pin_cpu.py on the host, test_pin_gpu.py on the device).
//
// What the reference calls (path_tracer/src):
//   thrust::default_random_engine(h) seeded by makeSeededRandomEngine   pathtrace.cu:57-62
//   thrust::uniform_real_distribution<float> u01(0, 1)                  pathtrace.cu:197,314;
//                                                                       interactions.cu:7,58
//   thrust::sort_by_key(device, ShadeableIntersection*, ..., PathSegment*, material_compare)
//                                                                       pathtrace.cu:410-414,479-491
//   thrust::stable_partition(device, PathSegment*, ..., is_valid)       pathtrace.cu:416-420,498-503
// The element types below have the reference's layouts (sceneStructs.h:80-99): 28-byte keys and
// 48-byte values, so rocThrust takes the same (non-radix, comparator) dispatch path.
#include <hip/hip_runtime.h>
#include <thrust/device_ptr.h>
#include <thrust/execution_policy.h>
#include <thrust/partition.h>
#include <thrust/random.h>
#include <thrust/sort.h>

#include <cstdint>
#include <vector>

namespace {

struct V3 { float x, y, z; };
struct V2 { float x, y; };
struct Isect {          // ShadeableIntersection (sceneStructs.h:92-99), 28 bytes
    float t;
    V3 n;
    int materialId;
    V2 uv;
};
struct Path {           // PathSegment (sceneStructs.h:80-87), 48 bytes
    V3 o, d, color;
    int pixelIndex, remainingBounces, bounces;
};
static_assert(sizeof(Isect) == 28 && sizeof(Path) == 48, "reference layouts");

struct material_compare {   // pathtrace.cu:410-414
    __host__ __device__ bool operator()(const Isect& a, const Isect& b) const { return a.materialId < b.materialId; }
};
struct is_valid {           // pathtrace.cu:416-420
    __host__ __device__ bool operator()(const Path& p) const { return p.remainingBounces > 0; }
};

// utilhash (intersections.h:13-22) and makeSeededRandomEngine (pathtrace.cu:57-62): the seed
// arithmetic around the library engine, as the reference writes it (int h, then the engine's
// unsigned constructor).
__host__ __device__ unsigned int utilhash(unsigned int a) {
    a = (a + 0x7ed55d16) + (a << 12);
    a = (a ^ 0xc761c23c) ^ (a >> 19);
    a = (a + 0x165667b1) + (a << 5);
    a = (a + 0xd3a2646c) ^ (a << 9);
    a = (a + 0xfd7046c5) + (a << 3);
    a = (a ^ 0xb55a4f09) ^ (a >> 16);
    return a;
}
__host__ __device__ thrust::default_random_engine seeded(int iter, int index, int depth) {
    int h = (int)(utilhash((1u << 31) | ((unsigned)depth << 22) | (unsigned)iter) ^ utilhash((unsigned)index));
    return thrust::default_random_engine(h);
}
__host__ __device__ void draw(int iter, int index, int depth, int draws, float* out) {
    thrust::default_random_engine rng = seeded(iter, index, depth);
    thrust::uniform_real_distribution<float> u01(0, 1);
    for (int k = 0; k < draws; ++k) out[k] = u01(rng);
}

__global__ void k_draw(int n, const int* it, const int* ix, const int* dp, int draws, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) draw(it[i], ix[i], dp[i], draws, out + (size_t)i * draws);
}

template <class T>
T* dev_copy(const T* h, size_t n) {
    T* d = nullptr;
    if (hipMalloc(&d, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    if (n && hipMemcpy(d, h, n * sizeof(T), hipMemcpyHostToDevice) != hipSuccess) { (void)hipFree(d); return nullptr; }
    return d;
}

std::vector<Isect> make_keys(int n, const int* mat) {
    std::vector<Isect> k((size_t)n);
    for (int i = 0; i < n; ++i) k[i] = Isect{1.0f + i, {0.f, 1.f, 0.f}, mat[i], {0.f, 0.f}};
    return k;
}
std::vector<Path> make_paths(int n, const int* remaining) {
    std::vector<Path> p((size_t)n);
    for (int i = 0; i < n; ++i)
        p[i] = Path{{0.f, 0.f, 0.f}, {0.f, 0.f, 1.f}, {1.f, 1.f, 1.f}, i, remaining ? remaining[i] : 1, 0};
    return p;
}

}  // namespace

extern "C" {

// out[i * draws + k] = k-th u01 draw of the engine makeSeededRandomEngine(iter[i], index[i], depth[i]).
int pin_rng_host(int n, const int* iter, const int* index, const int* depth, int draws, float* out) {
    for (int i = 0; i < n; ++i) draw(iter[i], index[i], depth[i], draws, out + (size_t)i * draws);
    return 0;
}
int pin_rng_device(int n, const int* iter, const int* index, const int* depth, int draws, float* out) {
    int *a = dev_copy(iter, n), *b = dev_copy(index, n), *c = dev_copy(depth, n);
    float* o = nullptr;
    int rc = (a && b && c && hipMalloc(&o, std::max(1, n * draws) * sizeof(float)) == hipSuccess) ? 0 : 1;
    if (!rc && n > 0) {
        hipLaunchKernelGGL(k_draw, dim3((n + 255) / 256), dim3(256), 0, nullptr, n, a, b, c, draws, o);
        rc = hipGetLastError() != hipSuccess ||
             hipMemcpy(out, o, (size_t)n * draws * sizeof(float), hipMemcpyDeviceToHost) != hipSuccess;
    }
    (void)hipFree(a); (void)hipFree(b); (void)hipFree(c); (void)hipFree(o);
    return rc;
}

// thrust::sort_by_key(policy, keys = ShadeableIntersection[n] with materialId = mat[i],
// values = PathSegment[n] with pixelIndex = i, material_compare): order[j] = pixelIndex of value j.
int pin_sort_by_key_host(int n, const int* mat, int* order) {
    auto k = make_keys(n, mat);
    auto v = make_paths(n, nullptr);
    thrust::sort_by_key(thrust::host, k.data(), k.data() + n, v.data(), material_compare());
    for (int i = 0; i < n; ++i) order[i] = v[i].pixelIndex;
    return 0;
}
int pin_sort_by_key_device(int n, const int* mat, int* order) {
    auto k = make_keys(n, mat);
    auto v = make_paths(n, nullptr);
    Isect* dk = dev_copy(k.data(), k.size());
    Path* dv = dev_copy(v.data(), v.size());
    int rc = dk && dv ? 0 : 1;
    if (!rc) {
        thrust::sort_by_key(thrust::device, thrust::device_pointer_cast(dk), thrust::device_pointer_cast(dk + n),
                            thrust::device_pointer_cast(dv), material_compare());
        rc = hipMemcpy(v.data(), dv, v.size() * sizeof(Path), hipMemcpyDeviceToHost) != hipSuccess;
    }
    for (int i = 0; !rc && i < n; ++i) order[i] = v[i].pixelIndex;
    (void)hipFree(dk); (void)hipFree(dv);
    return rc;
}

// thrust::stable_partition(policy, PathSegment[n] with remainingBounces = remaining[i] and
// pixelIndex = i, is_valid): order[j] = pixelIndex at position j; *live = the partition point.
int pin_stable_partition_host(int n, const int* remaining, int* order, int* live) {
    auto v = make_paths(n, remaining);
    Path* mid = thrust::stable_partition(thrust::host, v.data(), v.data() + n, is_valid());
    *live = (int)(mid - v.data());
    for (int i = 0; i < n; ++i) order[i] = v[i].pixelIndex;
    return 0;
}
int pin_stable_partition_device(int n, const int* remaining, int* order, int* live) {
    auto v = make_paths(n, remaining);
    Path* dv = dev_copy(v.data(), v.size());
    int rc = dv ? 0 : 1;
    if (!rc) {
        auto mid = thrust::stable_partition(thrust::device, thrust::device_pointer_cast(dv),
                                            thrust::device_pointer_cast(dv + n), is_valid());
        *live = (int)(mid - thrust::device_pointer_cast(dv));
        rc = hipMemcpy(v.data(), dv, v.size() * sizeof(Path), hipMemcpyDeviceToHost) != hipSuccess;
    }
    for (int i = 0; !rc && i < n; ++i) order[i] = v[i].pixelIndex;
    (void)hipFree(dv);
    return rc;
}

}  // extern "C"

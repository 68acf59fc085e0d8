// Device-side math for the MI355X path tracer (gfx950, wave64).
//
// Evaluation contract: this file is compiled with -ffp-contract=off, so every
// a*b+c below is a separate correctly-rounded multiply and add unless fmaf() is written; the
// association follows glm 0.9.6.3 as used by the reference (dot = (xx'+yy')+zz',
// mat*vec = (m0 v0 + m1 v1) + (m2 v2 + m3 v3), normalize = v * (1/sqrt(dot))).  hipcc lowers
// sqrtf and '/' to correctly-rounded sequences on gfx950, so the kernels reproduce the CPU
// oracle bit for bit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ptd {

constexpr float kPI = 3.1415926535897932384626422832795028841971f;       // utilities.h:12
constexpr float kTWO_PI = 6.2831853071795864769252867665590057683943f;   // utilities.h:13
constexpr float kSQRT_1_3 = 0.5773502691896257645091487805019574556476f; // utilities.h:14
constexpr float kFLT_MAX = 3.402823466e+38f;
constexpr float kFLT_EPS = 1.192092896e-07f;

struct f3 { float x, y, z; };
__device__ __forceinline__ f3 F3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return F3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return F3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator-(f3 a) { return F3(-a.x, -a.y, -a.z); }
__device__ __forceinline__ f3 hadamard(f3 a, f3 b) { return F3(a.x * b.x, a.y * b.y, a.z * b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return F3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ f3 operator*(float s, f3 a) { return F3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ f3 operator/(f3 a, float s) { return F3(a.x / s, a.y / s, a.z / s); }
__device__ __forceinline__ float dot(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return F3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}

// ---- correctly rounded sqrt and division, range-gated --------------------------------------
// hipcc expands sqrtf into v_sqrt + two neighbour corrections, wrapped in a scaling step for tiny
// inputs and a zero/inf fix-up (16 instructions), and '/' into v_div_scale x2, v_rcp, a Newton
// step, two residual corrections (v_div_fmas) and v_div_fixup (11 instructions + hazard nops).
// For operands in a safe range the wrapping steps are identities, so the cores below — the same
// operations in the same order — return the same bits; outside it (or for 0, NaN, inf, denormal
// intermediates) the library form runs instead (a divergent branch, skipped when no lane needs it).
//   sqrt:  x in [2^-96, FLT_MAX]: no scaling, not zero/inf.
//   n / d: |n|, |d| in [2^-40, 2^40]: exponent gap < 96, no denormal 1/d or quotient, no tiny n,
//          no zero (a zero numerator's sign would not survive the residual steps).
// pt_selftest_math checks cores == library ops on the device over random and edge operands.
__device__ __forceinline__ float sqrt_core(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float r1 = fmaf(-sm, s, x);
    const float s1 = r1 <= 0.0f ? sm : s;
    const float r2 = fmaf(-sp, s, x);
    return r2 > 0.0f ? sp : s1;
}
__device__ __forceinline__ bool sqrt_ok(float x) { return x >= 0x1p-96f && x <= 3.402823466e+38f; }
__device__ __forceinline__ float recip_core(float d) {   // v_rcp + one Newton step (the divisor's part)
    const float r = __builtin_amdgcn_rcpf(d);
    return fmaf(fmaf(-d, r, 1.0f), r, r);
}
__device__ __forceinline__ float div_core(float n, float d, float r) {
    float q = n * r;
    float e = fmaf(-d, q, n);
    q = fmaf(e, r, q);
    e = fmaf(-d, q, n);
    return fmaf(e, r, q);
}
__device__ __forceinline__ bool div_ok(float v) {
    const float a = fabsf(v);
    return a >= 0x1p-40f && a <= 0x1p+40f;
}
__device__ __forceinline__ float sqrt_cr(float x) {
    float s = sqrt_core(x);
    if (__builtin_expect(!sqrt_ok(x), 0)) s = sqrtf(x);
    return s;
}
__device__ __forceinline__ float div_cr(float n, float d) {
    float q = div_core(n, d, recip_core(d));
    if (__builtin_expect(!(div_ok(n) && div_ok(d)), 0)) q = n / d;
    return q;
}
// n1 / d and n2 / d sharing the divisor's reciprocal step
__device__ __forceinline__ void div2_cr(float n1, float n2, float d, float& q1, float& q2) {
    const float r = recip_core(d);
    q1 = div_core(n1, d, r);
    q2 = div_core(n2, d, r);
    if (__builtin_expect(!(div_ok(n1) && div_ok(n2) && div_ok(d)), 0)) {
        q1 = n1 / d;
        q2 = n2 / d;
    }
}
// glm normalize: v * (1 / sqrt(dot(v, v))); dot in [2^-80, 2^80] keeps sqrt and 1/sqrt in range
__device__ __forceinline__ f3 normalize(f3 v) {
    const float x = dot(v, v);
    const float s = sqrt_core(x);
    float inv = div_core(1.0f, s, recip_core(s));
    if (__builtin_expect(!(x >= 0x1p-80f && x <= 0x1p+80f), 0)) inv = 1.0f / sqrtf(x);
    return v * inv;
}
__device__ __forceinline__ float length(f3 v) { return sqrt_cr(dot(v, v)); }
__device__ __forceinline__ float gmin(float a, float b) { return a < b ? a : b; }
__device__ __forceinline__ float gmax(float a, float b) { return a > b ? a : b; }
__device__ __forceinline__ float at(f3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

// Affine 3x4 in glm column order + the exact glm w-term constants.
//   point  (w=1): (c0 x + c1 y) + (c2 z + c3)
//   vector (w=0): (c0 x + c1 y) + (c2 z + z3),  z3 = c3 * 0.0f (a signed zero)
struct Affine {
    float c[4][3];
    float z3[3];
};
// Scene tables that every lane of a wave reads at the same address are accessed through the
// constant address space so hipcc emits scalar (s_load) reads into SGPRs instead of 64 copies.
#define PT_CONST_AS __attribute__((address_space(4)))
template <class T>
__device__ __forceinline__ const T PT_CONST_AS* as_const(const T* p) {
    return (const T PT_CONST_AS*)(p);
}
template <class M>
__device__ __forceinline__ f3 xform_point(const M& m, f3 v) {
    return F3((m.c[0][0] * v.x + m.c[1][0] * v.y) + (m.c[2][0] * v.z + m.c[3][0]),
              (m.c[0][1] * v.x + m.c[1][1] * v.y) + (m.c[2][1] * v.z + m.c[3][1]),
              (m.c[0][2] * v.x + m.c[1][2] * v.y) + (m.c[2][2] * v.z + m.c[3][2]));
}
template <class M>
__device__ __forceinline__ f3 xform_vector(const M& m, f3 v) {
    return F3((m.c[0][0] * v.x + m.c[1][0] * v.y) + (m.c[2][0] * v.z + m.z3[0]),
              (m.c[0][1] * v.x + m.c[1][1] * v.y) + (m.c[2][1] * v.z + m.z3[1]),
              (m.c[0][2] * v.x + m.c[1][2] * v.y) + (m.c[2][2] * v.z + m.z3[2]));
}

// Device copy of a Geom: what intersection needs, nothing else (176 bytes, scalar-loaded).
struct DGeom {
    int32_t type, material, tri_start, tri_end;
    Affine inv;      // inverseTransform
    Affine xf;       // transform
    Affine itr;      // invTranspose
    float bmin[3], bmax[3];
    // Conservative bounds test (pt_kernels.hip bound_geom), filled by pt_create: the unit cube's
    // slabs widened to [slo, shi] = [-0.5 - mu_a, 0.5 + mu_a], the sphere's radius^2 widened to
    // r2w = 0.25 + kappa (mu, kappa exceed the rounding of both the exact test and the bounds
    // test for every ray origin in the scene), and tslack < 1, the relative slack that turns a
    // lower bound on the hit parameter into one on the reference's world distance.
    //   A sphere ray whose origin is outside the exact sphere by more than
    // kappa_ray = (|qo|^2 + 1) (kcs |ro|_inf + kc3) and moves away from its centre surely misses
    // (the ray leaving the sphere it just hit; the widened radius alone cannot tell).
    //   Axis-aligned cubes (bkind 3: the Cornell walls, incl. 90-degree rotations) are bounded by
    // their widened WORLD box [wlo, whi] (of the exact inverse of `inv`): a 6-plane slab test on the
    // world ray, with `back` >= 1e-4 * (largest stretch of the transform) for pointOnRay's pull-back.
    float slo[3], shi[3];
    float r2w, tslack;
    float kcs, kc3;
    float wlo[3], whi[3], back;
    int32_t bkind;   // 0: never hit (mesh), 1: oriented cube, 2: sphere, 3: world-box cube,
                     // 4: uniformly scaled sphere (world-space dot products)
    int32_t orig;    // SceneDev::bgeoms rows: index of this geom in SceneDev::geoms
    // Cubes: the world normal of each slab code (axis * 2 + sign) — boxIntersectionTest's
    // normalize(multiplyMV(invTranspose, (n, 0))) of a unit axis vector depends on the geom and
    // the code only, so pt_create evaluates it once with the same float32 operations (glm's
    // association, correctly rounded sqrt and division: the same bits as the per-hit evaluation).
    float nrm[6][3];
    // Cubes: the tangent frame calculateRandomDirectionInHemisphere builds from each of those
    // normals (interactions.cu:23-33: p1 = normalize(cross(n, dnn)), p2 = normalize(cross(n, p1))),
    // also a function of (geom, code) only: frm[code] = (p1, p2), evaluated once by pt_create.
    float frm[6][6];
    // bkind 3: the widened world box with each axis's two planes side by side, (wlo[k], whi[k]) at
    // wbox[2k], so one packed f32 operation (v_pk_add_f32 / v_pk_mul_f32, IEEE per component) takes
    // both planes of an axis from one SGPR pair (pt_kernels.hip slab2)
    float wbox[6];
    float wback;   // bkind 3: back * SceneDev::wb_tslack rounded up (bound_wbox_tagged)
    float pad_;
};

struct DMaterial {   // == pt_material
    float color[3];
    float spec_exponent;
    float spec_color[3];
    float has_reflective, has_refractive, ior, emittance;
    int32_t texture_id;
};

struct DTexture {
    int32_t width, height, components, pad;
    const uint8_t* data;
};

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v2f __attribute__((ext_vector_type(2)));

// Triangle hot data, 48 bytes = three 16-byte loads: (v0, id bits), (e1, 0), (e2, 0).  The edges
// e1 = v1 - v0, e2 = v2 - v0 are computed on the host with the same single subtraction glm
// performs, so the per-test arithmetic is unchanged.
struct alignas(16) DTri {
    v4f a, b, c;
};
struct DTriAttr {    // read once for the closest hit
    float n[3][3];
    float uv[3][2];
};
// BVH node, 32 bytes = two 16-byte loads: lo = (bmin, meta), hi = (bmax, link)
//   leaf:     meta = sub_areas (> 0),  link = first triangle
//   interior: meta = -(axis + 1),      link = right child (the left child is this node + 1)
struct alignas(16) DNode {
    v4f lo, hi;
};

// ---- RNG: thrust::default_random_engine (minstd_rand) seeded like makeSeededRandomEngine ----
__device__ __forceinline__ uint32_t utilhash(uint32_t a) {   // intersections.h:13-22
    a = (a + 0x7ed55d16u) + (a << 12);
    a = (a ^ 0xc761c23cu) ^ (a >> 19);
    a = (a + 0x165667b1u) + (a << 5);
    a = (a + 0xd3a2646cu) ^ (a << 9);
    a = (a + 0xfd7046c5u) + (a << 3);
    a = (a ^ 0xb55a4f09u) ^ (a >> 16);
    return a;
}
struct Rng {
    uint32_t x;
    __device__ __forceinline__ Rng(int iter, int index, int depth) {
        const uint32_t key = 0x80000000u | ((uint32_t)depth << 22) | (uint32_t)iter;
        const uint32_t h = utilhash(key) ^ utilhash((uint32_t)index);
        const uint32_t s = h % 2147483647u;
        x = s == 0u ? 1u : s;
    }
    // x <- 48271 x mod (2^31 - 1) via the Mersenne fold (exact), u = float(x-1) / 2^31.
    __device__ __forceinline__ float u01() {
        const uint64_t p = (uint64_t)48271u * x;
        uint32_t r = (uint32_t)(p & 0x7fffffffu) + (uint32_t)(p >> 31);
        if (r >= 2147483647u) r -= 2147483647u;
        x = r;
        return (float)(x - 1u) * 4.656612873077392578125e-10f;   // / 2147483648.0f (exact)
    }
};

// ---- deterministic sin/cos (evaluation contract; mirrored by the oracle) --------------------
__device__ __forceinline__ void sincos_c(float x, float* s_out, float* c_out) {
    const float j = rintf(x * 0.636619772367581343f);
    float r = fmaf(-j, 1.5707962513e+00f, x);
    r = fmaf(-j, 7.5497894159e-08f, r);
    r = fmaf(-j, 5.3903029534e-15f, r);
    const float z = r * r;
    const float ps = fmaf(fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), z, -1.6666654611e-1f);
    const float s = fmaf(r * z, ps, r);
    const float pc = fmaf(fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    const float c = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
    const int q = ((int)j) & 3;
    const float sa = (q & 1) ? c : s;
    const float ca = (q & 1) ? s : c;
    *s_out = (q & 2) ? -sa : sa;
    *c_out = ((q + 1) & 2) ? -ca : ca;
}

// getPointOnRay (intersections.h:29-32)
__device__ __forceinline__ f3 point_on_ray(f3 o, f3 d, float t) { return o + (t - .0001f) * normalize(d); }

}  // namespace ptd

// ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by or called from the
// product library (cuda_pathtracer_amd).  Only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py may load liboracle.so, and only as the checker.
//
// Serial CPU restatement of the reference renderer's per-iteration hot path.  Every function
// cites the reference file:line it restates (paths relative to /root/reference/path_tracer).
//
// Evaluation contract (shared with the HIP kernels, written independently on each side):
//   * float32 everywhere, IEEE round-to-nearest, NO fused multiply-add except where this file
//     calls fmaf() explicitly (compile with -ffp-contract=off; x86-64 SSE arithmetic);
//   * operations in the order the reference source writes them, with glm 0.9.6.3's own
//     association (dot = (x*x' + y*y') + z*z'; mat*vec = (m0*v0 + m1*v1) + (m2*v2 + m3*v3);
//     normalize = v * (1/sqrt(dot(v,v))); glm::min/max are ternaries);
//   * sqrtf and '/' correctly rounded;
//   * sin/cos of the two sampling angles use one fixed, published algorithm (pt_sincos below:
//     Cody-Waite reduction by pi/2 + Cephes-style minimax polynomials, evaluated with fmaf)
//     because libm/ocml sinf differ in the last ulp.  Host-side set-up (camera, transforms)
//     uses libm (acosf, sinf, cosf, tanf, atanf) exactly like the reference host code.
// Under this contract the product's GPU output is bit-identical to this oracle
// (tests/test_render_gpu.py).
//
// Pinned pieces (tests/test_pin_thrust.py, against rocThrust 7.2 from the system ROCm headers —
// the third-party library the reference calls through the same Thrust API, not reference code —
// under thrust::host and thrust::device):
//   * oracle_u01_sequence (makeSeededRandomEngine + thrust::default_random_engine +
//     uniform_real_distribution<float>(0,1), pathtrace.cu:57-62,197,314; interactions.cu:7,58):
//     bit for bit over 3,900 (iteration, index, depth) keys x 8 draws;
//   * the material order of the sort (thrust::sort_by_key with material_compare,
//     pathtrace.cu:410-414,479-491): this file's std::stable_sort order on real per-bounce keys;
//   * relocate_terminated_paths (thrust::stable_partition, pathtrace.cu:416-420,498-503).
// Parity caveat ("parity unpinned" for radiance): the reference ships no renderer test or
// golden vector that can pin per-pixel radiance; its CUDA build cannot run
// here and compiling/running reference sources was denied.  The geometry,
// shading and accumulation arithmetic is pinned by reading the reference source, and the
// radiance statistically by the reference's course render.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

extern "C" {

// ---- data layouts (same field order as the reference structs; sceneStructs.h) ----------
struct OGeom {                 // sceneStructs.h:25-41 (272 bytes)
    int32_t type;              // 0 SPHERE, 1 CUBE, 2 MESH  (sceneStructs.h:12-17)
    int32_t materialid;
    float translation[3], rotation[3], scale[3];
    float transform[16];       // glm column-major: m[c][r] == a[4*c + r]
    float inverse_transform[16];
    float inv_transpose[16];
    int32_t tri_start, tri_end, bbox_idx;
    float min_bound[3], max_bound[3];
};
struct OMaterial {             // sceneStructs.h:43-57 (48 bytes)
    float color[3];
    float spec_exponent;
    float spec_color[3];
    float has_reflective, has_refractive, ior, emittance;
    int32_t texture_id;
};
struct OCamera {               // sceneStructs.h:59-69
    int32_t res[2];
    float position[3], look_at[3], view[3], up[3], right[3], fov[2], pixel_length[2];
};
struct OFlags {                // utilities.h:17-34 (GuiDataContainer) / pathtrace.cu:31-42 (Settings)
    int32_t russian_roulette, use_bvh, use_bbox, sort_by_material, use_thrust_partition, ssaa, dof;
    float aperture, focal_dist;
    int32_t single_albedo;     // extension (pt_amd.h); 0 = the reference
    int32_t rng_key_pixel;     // extension (pt_amd.h): shading RNG keyed by the global pixel
};
struct OTriangle {             // sceneStructs.h:103-161 (124 bytes)
    int32_t id;
    float v[3][3];
    float uv[3][2];
    float n[3][3];
    float bmin[3], bmax[3];
};
struct ONode {                 // BVH_tree.h:54-61 (40 bytes)
    float bmin[3], bmax[3];
    int32_t sub_areas, axis, first_area_idx, rchild_idx;
};
struct OTexture {              // sceneStructs.h:162-189
    int32_t width, height, components, pad;
    const uint8_t* data;
};

}  // extern "C"

namespace {

constexpr float kPI = 3.1415926535897932384626422832795028841971f;        // utilities.h:12
constexpr float kTWO_PI = 6.2831853071795864769252867665590057683943f;    // utilities.h:13
constexpr float kSQRT_ONE_THIRD = 0.5773502691896257645091487805019574556476f;  // utilities.h:14

// ---- small float3 helpers with glm 0.9.6.3 association ---------------------------------
struct V3 { float x, y, z; };
inline V3 mk(float x, float y, float z) { return V3{x, y, z}; }
inline V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
inline V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
inline V3 mulv(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 muls(V3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }   // vec * scalar
inline V3 smul(float s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }   // scalar * vec
inline V3 divs(V3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
inline V3 neg(V3 a) { return mk(-a.x, -a.y, -a.z); }
inline float dot3(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }   // func_geometric.inl compute_dot
inline V3 cross3(V3 a, V3 b) {                                                   // func_geometric.inl cross
    return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
inline V3 normalize3(V3 v) { return muls(v, 1.0f / sqrtf(dot3(v, v))); }       // x * inversesqrt(dot(x,x))
inline float length3(V3 v) { return sqrtf(dot3(v, v)); }
inline float gmin(float a, float b) { return a < b ? a : b; }                    // func_common.inl:409-414
inline float gmax(float a, float b) { return a > b ? a : b; }                    // func_common.inl:430-435
inline V3 ld3(const float* p) { return mk(p[0], p[1], p[2]); }
inline float comp(V3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
inline void setc(V3& v, int i, float f) { if (i == 0) v.x = f; else if (i == 1) v.y = f; else v.z = f; }

// glm mat4 * vec4 (type_mat4x4.inl:592-627): (m0*v0 + m1*v1) + (m2*v2 + m3*v3); xyz kept
// (intersections.h:37-40 multiplyMV).
inline V3 mul_mv(const float* m, V3 v, float w) {
    float r[3];
    for (int i = 0; i < 3; ++i) {
        float a0 = m[0 + i] * v.x, a1 = m[4 + i] * v.y, a2 = m[8 + i] * v.z, a3 = m[12 + i] * w;
        r[i] = (a0 + a1) + (a2 + a3);
    }
    return mk(r[0], r[1], r[2]);
}

// ---- 4x4 matrix helpers (host set-up; glm 0.9.6.3 association) ----------------------------
typedef float M4[16];
inline void m4_identity(float* m) { for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.0f : 0.0f; }
// glm operator*(mat4, mat4) (type_mat4x4.inl:686-705): Result[c] = ((A0*B[c][0] + A1*B[c][1]) + A2*B[c][2]) + A3*B[c][3]
void m4_mul(const float* a, const float* b, float* out) {
    float r[16];
    for (int c = 0; c < 4; ++c)
        for (int i = 0; i < 4; ++i)
            r[4 * c + i] = ((a[i] * b[4 * c + 0] + a[4 + i] * b[4 * c + 1]) + a[8 + i] * b[4 * c + 2]) + a[12 + i] * b[4 * c + 3];
    std::memcpy(out, r, sizeof r);
}
// glm::translate(mat4(), v) (gtc/matrix_transform.inl:40-49)
void m4_translate(const float* v, float* out) {
    float m[16]; m4_identity(m);
    std::memcpy(out, m, sizeof m);
    for (int i = 0; i < 4; ++i) out[12 + i] = ((m[i] * v[0] + m[4 + i] * v[1]) + m[8 + i] * v[2]) + m[12 + i];
}
// glm::rotate(mat4(), angle, axis) (gtc/matrix_transform.inl:52-85)
void m4_rotate(float angle, V3 axis_in, float* out) {
    const float c = cosf(angle), s = sinf(angle);
    V3 ax = normalize3(axis_in);
    V3 tp = smul(1.0f - c, ax);
    float R[3][3];
    R[0][0] = c + tp.x * ax.x;
    R[0][1] = (0.0f + tp.x * ax.y) + s * ax.z;
    R[0][2] = (0.0f + tp.x * ax.z) - s * ax.y;
    R[1][0] = (0.0f + tp.y * ax.x) - s * ax.z;
    R[1][1] = c + tp.y * ax.y;
    R[1][2] = (0.0f + tp.y * ax.z) + s * ax.x;
    R[2][0] = (0.0f + tp.z * ax.x) + s * ax.y;
    R[2][1] = (0.0f + tp.z * ax.y) - s * ax.x;
    R[2][2] = c + tp.z * ax.z;
    float m[16]; m4_identity(m);
    for (int col = 0; col < 3; ++col)
        for (int i = 0; i < 4; ++i)
            out[4 * col + i] = (m[i] * R[col][0] + m[4 + i] * R[col][1]) + m[8 + i] * R[col][2];
    for (int i = 0; i < 4; ++i) out[12 + i] = m[12 + i];
}
// glm::scale(mat4(), v) (gtc/matrix_transform.inl:122-134)
void m4_scale(const float* v, float* out) {
    float m[16]; m4_identity(m);
    for (int col = 0; col < 3; ++col)
        for (int i = 0; i < 4; ++i) out[4 * col + i] = m[4 * col + i] * v[col];
    for (int i = 0; i < 4; ++i) out[12 + i] = m[12 + i];
}
#define MM(c, r) m[4 * (c) + (r)]
// glm::inverse for mat4 (detail/type_mat4x4.inl:37-92)
void m4_inverse(const float* m, float* out) {
    const float c00 = MM(2,2) * MM(3,3) - MM(3,2) * MM(2,3), c02 = MM(1,2) * MM(3,3) - MM(3,2) * MM(1,3), c03 = MM(1,2) * MM(2,3) - MM(2,2) * MM(1,3);
    const float c04 = MM(2,1) * MM(3,3) - MM(3,1) * MM(2,3), c06 = MM(1,1) * MM(3,3) - MM(3,1) * MM(1,3), c07 = MM(1,1) * MM(2,3) - MM(2,1) * MM(1,3);
    const float c08 = MM(2,1) * MM(3,2) - MM(3,1) * MM(2,2), c10 = MM(1,1) * MM(3,2) - MM(3,1) * MM(1,2), c11 = MM(1,1) * MM(2,2) - MM(2,1) * MM(1,2);
    const float c12 = MM(2,0) * MM(3,3) - MM(3,0) * MM(2,3), c14 = MM(1,0) * MM(3,3) - MM(3,0) * MM(1,3), c15 = MM(1,0) * MM(2,3) - MM(2,0) * MM(1,3);
    const float c16 = MM(2,0) * MM(3,2) - MM(3,0) * MM(2,2), c18 = MM(1,0) * MM(3,2) - MM(3,0) * MM(1,2), c19 = MM(1,0) * MM(2,2) - MM(2,0) * MM(1,2);
    const float c20 = MM(2,0) * MM(3,1) - MM(3,0) * MM(2,1), c22 = MM(1,0) * MM(3,1) - MM(3,0) * MM(1,1), c23 = MM(1,0) * MM(2,1) - MM(2,0) * MM(1,1);
    const float F0[4] = {c00, c00, c02, c03}, F1[4] = {c04, c04, c06, c07}, F2[4] = {c08, c08, c10, c11};
    const float F3[4] = {c12, c12, c14, c15}, F4[4] = {c16, c16, c18, c19}, F5[4] = {c20, c20, c22, c23};
    const float V0[4] = {MM(1,0), MM(0,0), MM(0,0), MM(0,0)}, V1[4] = {MM(1,1), MM(0,1), MM(0,1), MM(0,1)};
    const float V2[4] = {MM(1,2), MM(0,2), MM(0,2), MM(0,2)}, V3_[4] = {MM(1,3), MM(0,3), MM(0,3), MM(0,3)};
    const float sA[4] = {1, -1, 1, -1}, sB[4] = {-1, 1, -1, 1};
    float inv[16];
    for (int k = 0; k < 4; ++k) {
        inv[0 + k] = ((V1[k] * F0[k] - V2[k] * F1[k]) + V3_[k] * F2[k]) * sA[k];
        inv[4 + k] = ((V0[k] * F0[k] - V2[k] * F3[k]) + V3_[k] * F4[k]) * sB[k];
        inv[8 + k] = ((V0[k] * F1[k] - V1[k] * F3[k]) + V3_[k] * F5[k]) * sA[k];
        inv[12 + k] = ((V0[k] * F2[k] - V1[k] * F4[k]) + V2[k] * F5[k]) * sB[k];
    }
    const float row0[4] = {inv[0], inv[4], inv[8], inv[12]};
    float d[4];
    for (int k = 0; k < 4; ++k) d[k] = m[k] * row0[k];
    const float det = (d[0] + d[1]) + (d[2] + d[3]);
    const float one_over = 1.0f / det;
    for (int i = 0; i < 16; ++i) out[i] = inv[i] * one_over;
}
// glm::inverseTranspose for mat4 (gtc/matrix_inverse.inl:95-147)
void m4_inverse_transpose(const float* m, float* out) {
    const float s00 = MM(2,2) * MM(3,3) - MM(3,2) * MM(2,3), s01 = MM(2,1) * MM(3,3) - MM(3,1) * MM(2,3);
    const float s02 = MM(2,1) * MM(3,2) - MM(3,1) * MM(2,2), s03 = MM(2,0) * MM(3,3) - MM(3,0) * MM(2,3);
    const float s04 = MM(2,0) * MM(3,2) - MM(3,0) * MM(2,2), s05 = MM(2,0) * MM(3,1) - MM(3,0) * MM(2,1);
    const float s06 = MM(1,2) * MM(3,3) - MM(3,2) * MM(1,3), s07 = MM(1,1) * MM(3,3) - MM(3,1) * MM(1,3);
    const float s08 = MM(1,1) * MM(3,2) - MM(3,1) * MM(1,2), s09 = MM(1,0) * MM(3,3) - MM(3,0) * MM(1,3);
    const float s10 = MM(1,0) * MM(3,2) - MM(3,0) * MM(1,2), s11 = MM(1,1) * MM(3,3) - MM(3,1) * MM(1,3);
    const float s12 = MM(1,0) * MM(3,1) - MM(3,0) * MM(1,1), s13 = MM(1,2) * MM(2,3) - MM(2,2) * MM(1,3);
    const float s14 = MM(1,1) * MM(2,3) - MM(2,1) * MM(1,3), s15 = MM(1,1) * MM(2,2) - MM(2,1) * MM(1,2);
    const float s16 = MM(1,0) * MM(2,3) - MM(2,0) * MM(1,3), s17 = MM(1,0) * MM(2,2) - MM(2,0) * MM(1,2);
    const float s18 = MM(1,0) * MM(2,1) - MM(2,0) * MM(1,1);
    float r[16];
    r[0]  = +((MM(1,1) * s00 - MM(1,2) * s01) + MM(1,3) * s02);
    r[1]  = -((MM(1,0) * s00 - MM(1,2) * s03) + MM(1,3) * s04);
    r[2]  = +((MM(1,0) * s01 - MM(1,1) * s03) + MM(1,3) * s05);
    r[3]  = -((MM(1,0) * s02 - MM(1,1) * s04) + MM(1,2) * s05);
    r[4]  = -((MM(0,1) * s00 - MM(0,2) * s01) + MM(0,3) * s02);
    r[5]  = +((MM(0,0) * s00 - MM(0,2) * s03) + MM(0,3) * s04);
    r[6]  = -((MM(0,0) * s01 - MM(0,1) * s03) + MM(0,3) * s05);
    r[7]  = +((MM(0,0) * s02 - MM(0,1) * s04) + MM(0,2) * s05);
    r[8]  = +((MM(0,1) * s06 - MM(0,2) * s07) + MM(0,3) * s08);
    r[9]  = -((MM(0,0) * s06 - MM(0,2) * s09) + MM(0,3) * s10);
    r[10] = +((MM(0,0) * s11 - MM(0,1) * s09) + MM(0,3) * s12);
    r[11] = -((MM(0,0) * s08 - MM(0,1) * s10) + MM(0,2) * s12);
    r[12] = -((MM(0,1) * s13 - MM(0,2) * s14) + MM(0,3) * s15);
    r[13] = +((MM(0,0) * s13 - MM(0,2) * s16) + MM(0,3) * s17);
    r[14] = -((MM(0,0) * s14 - MM(0,1) * s16) + MM(0,3) * s18);
    r[15] = +((MM(0,0) * s15 - MM(0,1) * s17) + MM(0,2) * s18);
    const float det = ((+MM(0,0) * r[0] + MM(0,1) * r[1]) + MM(0,2) * r[2]) + MM(0,3) * r[3];
    for (int i = 0; i < 16; ++i) out[i] = r[i] / det;
}
#undef MM

// ---- RNG: thrust::default_random_engine (minstd_rand) + uniform_real_distribution<float> ----
// intersections.h:13-22 utilhash; pathtrace.cu:57-62 makeSeededRandomEngine;
// rocThrust 7.2 linear_congruential_engine.inl:43-61 (seed, x==0 -> 1), random/detail/mod.h
// (Schrage: exact 48271*x mod (2^31-1)), uniform_real_distribution.inl:67-80.
inline uint32_t utilhash(uint32_t a) {
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
    Rng(int iter, int index, int depth) {
        uint32_t key = 0x80000000u | ((uint32_t)depth << 22) | (uint32_t)iter;
        uint32_t h = utilhash(key) ^ utilhash((uint32_t)index);
        uint32_t s = h % 2147483647u;
        x = s == 0 ? 1u : s;
    }
    float u01() {
        x = (uint32_t)(((uint64_t)48271u * x) % 2147483647ull);
        float r = (float)(x - 1u);
        r /= (1.0f + (float)(2147483646u - 1u));
        return r * (1.0f - 0.0f) + 0.0f;
    }
};

// ---- pt_sincos: the deterministic sin/cos of the evaluation contract ---------------------
// Cody-Waite reduction by pi/2 (three-part constant), Cephes single-precision polynomials on
// [-pi/4, pi/4], every step with an explicit fmaf or a plain correctly-rounded op.
void pt_sincos(float x, float* s_out, float* c_out) {
    const float two_over_pi = 0.636619772367581343f;
    const float p1 = 1.5707962513e+00f, p2 = 7.5497894159e-08f, p3 = 5.3903029534e-15f;
    float j = rintf(x * two_over_pi);
    float r = fmaf(-j, p1, x);
    r = fmaf(-j, p2, r);
    r = fmaf(-j, p3, r);
    float z = r * r;
    float ps = fmaf(fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), z, -1.6666654611e-1f);
    float s = fmaf(r * z, ps, r);
    float pc = fmaf(fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    float c = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
    int q = ((int)j) & 3;
    float so, co;
    if (q == 0) { so = s; co = c; }
    else if (q == 1) { so = c; co = -s; }
    else if (q == 2) { so = -s; co = -c; }
    else { so = -c; co = s; }
    *s_out = so; *c_out = co;
}

// ---- path + intersection records (sceneStructs.h:80-99) ----------------------------------
struct Path {
    V3 o, d, c;
    int pixel;       // global pixel index
    int slot;        // tile-local slot: sample * npix_tile + local pixel
    int iter;        // iteration index used for the RNG
    int remaining, bounces;
};
struct Isect {
    float t;
    V3 n;
    int mat;
    float uv[2];
};

struct Scene {
    const OGeom* geoms; int ngeoms;
    const OMaterial* mats; int nmats;
    const OTriangle* tris; int ntris;
    const ONode* nodes; int nnodes;
    const OTexture* texs; int ntexs;
};

// getPointOnRay (intersections.h:29-32)
inline V3 point_on_ray(V3 o, V3 d, float t) { return add(o, smul(t - .0001f, normalize3(d))); }

// boxIntersectionTest (intersections.cu:3-58)
float box_test(const OGeom& g, V3 ro, V3 rd, V3& ip, V3& nrm, bool& outside) {
    V3 qo = mul_mv(g.inverse_transform, ro, 1.0f);
    V3 qd = normalize3(mul_mv(g.inverse_transform, rd, 0.0f));
    float tmin = -1e38f, tmax = 1e38f;
    V3 tmin_n = mk(0, 0, 0), tmax_n = mk(0, 0, 0);
    for (int a = 0; a < 3; ++a) {
        float qda = comp(qd, a);
        float t1 = (-0.5f - comp(qo, a)) / qda;
        float t2 = (+0.5f - comp(qo, a)) / qda;
        float ta = gmin(t1, t2), tb = gmax(t1, t2);
        V3 n = mk(0, 0, 0);
        setc(n, a, t2 < t1 ? +1.0f : -1.0f);
        if (ta > 0 && ta > tmin) { tmin = ta; tmin_n = n; }
        if (tb < tmax) { tmax = tb; tmax_n = n; }
    }
    if (tmax >= tmin && tmax > 0) {
        outside = true;
        if (tmin <= 0) { tmin = tmax; tmin_n = tmax_n; outside = false; }
        ip = mul_mv(g.transform, point_on_ray(qo, qd, tmin), 1.0f);
        nrm = normalize3(mul_mv(g.inv_transpose, tmin_n, 0.0f));
        return length3(sub(ro, ip));
    }
    return -1;
}

// sphereIntersectionTest (intersections.cu:60-115)
float sphere_test(const OGeom& g, V3 r_o, V3 r_d, V3& ip, V3& nrm, bool& outside) {
    const float radius = .5f;
    V3 ro = mul_mv(g.inverse_transform, r_o, 1.0f);
    V3 rd = normalize3(mul_mv(g.inverse_transform, r_d, 0.0f));
    float vdd = dot3(ro, rd);
    float radicand = vdd * vdd - (dot3(ro, ro) - powf(radius, 2));
    if (radicand < 0) return -1;
    float sq = sqrtf(radicand);
    float first = -vdd;
    float t1 = first + sq, t2 = first - sq;
    float t = 0;
    if (t1 < 0 && t2 < 0) return -1;
    else if (t1 > 0 && t2 > 0) { t = gmin(t1, t2); outside = true; }
    else { t = gmax(t1, t2); outside = false; }
    V3 obj = point_on_ray(ro, rd, t);
    ip = mul_mv(g.transform, obj, 1.0f);
    nrm = normalize3(mul_mv(g.inv_transpose, obj, 0.0f));
    if (!outside) nrm = neg(nrm);
    return length3(sub(r_o, ip));
}

// glm::intersectRayTriangle (external/include/glm/gtx/intersect.inl:37-74): one-sided, eps=FLT_EPSILON
bool ray_tri(V3 orig, V3 dir, V3 v0, V3 v1, V3 v2, float bary[3]) {
    V3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    V3 p = cross3(dir, e2);
    float a = dot3(e1, p);
    if (a < FLT_EPSILON) return false;
    float f = 1.0f / a;
    V3 s = sub(orig, v0);
    bary[0] = f * dot3(s, p);
    if (bary[0] < 0.0f) return false;
    if (bary[0] > 1.0f) return false;
    V3 q = cross3(s, e1);
    bary[1] = f * dot3(dir, q);
    if (bary[1] < 0.0f) return false;
    if (bary[1] + bary[0] > 1.0f) return false;
    bary[2] = f * dot3(e2, q);
    return bary[2] >= 0.0f;
}

// Triangle::intersect (sceneStructs.h:145-160): uv with correct weights, normal with the
// mis-weighted barycentrics (quirk 10).
bool tri_intersect(const OTriangle& tr, V3 o, V3 d, Isect& out) {
    float b[3] = {0, 0, 0};
    if (ray_tri(o, d, ld3(tr.v[0]), ld3(tr.v[1]), ld3(tr.v[2]), b)) {
        out.t = b[2];
        float w = (1.0f - b[0]) - b[1];
        for (int k = 0; k < 2; ++k) out.uv[k] = (tr.uv[0][k] * w + tr.uv[1][k] * b[0]) + tr.uv[2][k] * b[1];
        V3 n = add(add(muls(ld3(tr.n[0]), b[0]), muls(ld3(tr.n[1]), b[1])), muls(ld3(tr.n[2]), (1.0f - b[0]) - b[1]));
        out.n = normalize3(n);
        return true;
    }
    out.t = -1.0f;
    return false;
}

// BoundingBox::intersect (boundingbox.h:73-92)
bool aabb_hit(const float* bmin, const float* bmax, V3 o, V3 inv) {
    float mx = (bmin[0] - o.x) * inv.x, Mx = (bmax[0] - o.x) * inv.x;
    float my = (bmin[1] - o.y) * inv.y, My = (bmax[1] - o.y) * inv.y;
    float mz = (bmin[2] - o.z) * inv.z, Mz = (bmax[2] - o.z) * inv.z;
    float lo = gmax(gmax(gmin(mx, Mx), gmin(my, My)), gmin(mz, Mz));
    float hi = gmin(gmin(gmax(mx, Mx), gmax(my, My)), gmax(mz, Mz));
    if (hi < 0) return false;
    if (lo > hi) return false;
    return true;
}

// BVHIntersectionTest (intersections.cu:169-224): stack 64, near-child-first by dir sign,
// silent pop on overflow, no t-culling.
bool bvh_test(const Scene& sc, V3 o, V3 d, int& hit_tri_id, Isect& isec) {
    if (!sc.nodes || sc.nnodes == 0) return false;
    bool hit = false;
    const int MAXD = 64;
    int top = 0, cur = 0;
    int stack[MAXD];
    bool neg[3] = {d.x < 0.0f, d.y < 0.0f, d.z < 0.0f};
    V3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    for (;;) {
        const ONode& nd = sc.nodes[cur];
        if (aabb_hit(nd.bmin, nd.bmax, o, inv)) {
            if (nd.sub_areas > 0) {
                for (int i = 0; i < nd.sub_areas; ++i) {
                    Isect tmp;
                    const OTriangle& tr = sc.tris[nd.first_area_idx + i];
                    if (tri_intersect(tr, o, d, tmp)) {
                        hit = true;
                        if ((isec.t == -1.0f) || (tmp.t < isec.t)) { isec = tmp; hit_tri_id = tr.id; }
                    }
                }
                if (top == 0) break;
                cur = stack[--top];
            } else {
                if (top == MAXD) { cur = stack[--top]; continue; }
                if (neg[nd.axis]) { stack[top++] = cur + 1; cur = nd.rchild_idx; }
                else { stack[top++] = nd.rchild_idx; cur = cur + 1; }
            }
        } else {
            if (top == 0) break;
            cur = stack[--top];
        }
    }
    return hit;
}

// meshIntersectionTest (intersections.cu:119-167): linear loop with optional world AABB cull.
float mesh_linear_test(const Scene& sc, const OGeom& g, V3 o, V3 d, float uv[2], V3& nrm, bool use_bbox) {
    if (use_bbox) {
        V3 inv = mk(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        float mx = (g.min_bound[0] - o.x) * inv.x, Mx = (g.max_bound[0] - o.x) * inv.x;
        float my = (g.min_bound[1] - o.y) * inv.y, My = (g.max_bound[1] - o.y) * inv.y;
        float mz = (g.min_bound[2] - o.z) * inv.z, Mz = (g.max_bound[2] - o.z) * inv.z;
        float lo = gmax(gmax(gmin(mx, Mx), gmin(my, My)), gmin(mz, Mz));
        float hi = gmin(gmin(gmax(mx, Mx), gmax(my, My)), gmax(mz, Mz));
        if (hi < 0 || lo > hi) return -1.0f;
    }
    int best = -1;
    float tmin = FLT_MAX;
    float bb[3] = {0, 0, 0}, mb[3] = {0, 0, 0};
    for (int i = g.tri_start; i < g.tri_end; ++i) {
        const OTriangle& tr = sc.tris[i];
        if (ray_tri(o, d, ld3(tr.v[0]), ld3(tr.v[1]), ld3(tr.v[2]), bb)) {
            if (bb[2] > 0.0f && bb[2] < tmin) { best = i; tmin = bb[2]; mb[0] = bb[0]; mb[1] = bb[1]; mb[2] = bb[2]; }
        }
    }
    if (best == -1) return -1.0f;
    float az = (1.0f - mb[0]) - mb[1];
    const OTriangle& tr = sc.tris[best];
    nrm = normalize3(add(add(smul(az, ld3(tr.n[0])), ld3(tr.n[1])), ld3(tr.n[2])));
    for (int k = 0; k < 2; ++k) uv[k] = (az * tr.uv[0][k] + tr.uv[1][k]) + tr.uv[2][k];
    return tmin;
}

// computeIntersections (pathtrace.cu:229-298) for one ray.  `rec` starts as the memset state
// (all zero); a miss only writes t = -1.
void compute_isect(const Scene& sc, const OFlags& fl, V3 o, V3 d, Isect& rec) {
    float t = 0, t_min = FLT_MAX;
    int hit_geom = -1, hit_tri = -1;
    bool outside = true;
    V3 tmp_ip = mk(0, 0, 0), tmp_n = mk(0, 0, 0), nrm = mk(0, 0, 0);
    float tmp_uv[2] = {0, 0}, uv[2] = {0, 0};
    for (int i = 0; i < sc.ngeoms; ++i) {
        const OGeom& g = sc.geoms[i];
        if (g.type == 1) t = box_test(g, o, d, tmp_ip, tmp_n, outside);
        else if (g.type == 0) t = sphere_test(g, o, d, tmp_ip, tmp_n, outside);
        else if (g.type == 2) {
            if (fl.use_bvh) {
                Isect is; is.t = FLT_MAX; is.n = mk(0, 0, 0); is.mat = 0; is.uv[0] = is.uv[1] = 0;
                t = -1.0f;
                if (bvh_test(sc, o, d, hit_tri, is)) {
                    if (hit_tri >= g.tri_start && hit_tri < g.tri_end) {
                        t = is.t; tmp_uv[0] = is.uv[0]; tmp_uv[1] = is.uv[1]; tmp_n = is.n;
                    }
                }
            } else {
                t = mesh_linear_test(sc, g, o, d, tmp_uv, tmp_n, fl.use_bbox != 0);
            }
        }
        if (t > 0.0f && t_min > t) {
            t_min = t; hit_geom = i; uv[0] = tmp_uv[0]; uv[1] = tmp_uv[1]; nrm = tmp_n;
        }
    }
    if (hit_geom == -1) {
        rec.t = -1.0f;
    } else {
        rec.t = t_min;
        rec.mat = sc.geoms[hit_geom].materialid;
        rec.uv[0] = uv[0]; rec.uv[1] = uv[1];
        rec.n = nrm;
    }
}

// Texture::get_color (sceneStructs.h:176-189); negative texel indices are clamped to 0
// (the reference reads out of bounds there).
V3 tex_color(const OTexture& tx, const float uv[2]) {
    int X = (int)gmin(1.f * tx.width * uv[0], 1.f * tx.width - 1.0f);
    int Y = (int)gmin(1.f * tx.height * (1.0f - uv[1]), 1.f * tx.height - 1.0f);
    if (X < 0) X = 0;
    if (Y < 0) Y = 0;
    int id = Y * tx.width + X;
    if (tx.components == 3) {
        V3 c = mk((float)tx.data[id * 3], (float)tx.data[id * 3 + 1], (float)tx.data[id * 3 + 2]);
        return smul(0.003921568627f, c);
    }
    return mk(0, 0, 0);
}

// calculateRandomDirectionInHemisphere (interactions.cu:3-41)
V3 hemisphere(V3 n, Rng& rng) {
    float up = sqrtf(rng.u01());
    float over = sqrtf(1 - up * up);
    float around = rng.u01() * kTWO_PI;
    V3 dnn;
    if (fabsf(n.x) < kSQRT_ONE_THIRD) dnn = mk(1, 0, 0);
    else if (fabsf(n.y) < kSQRT_ONE_THIRD) dnn = mk(0, 1, 0);
    else dnn = mk(0, 0, 1);
    V3 p1 = normalize3(cross3(n, dnn));
    V3 p2 = normalize3(cross3(n, p1));
    float sa, ca;
    pt_sincos(around, &sa, &ca);
    return add(add(smul(up, n), smul(ca * over, p1)), smul(sa * over, p2));
}

// glm::reflect (detail/func_geometric.inl:176-181): I - N * dot(N, I) * 2
inline V3 reflect3(V3 I, V3 N) { return sub(I, mulv(muls(N, dot3(N, I)), mk(2, 2, 2))); }
// glm::refract(vec, vec, T) (detail/func_geometric.inl:193-199); NaN when k < 0 as in glm.
inline V3 refract3(V3 I, V3 N, float eta) {
    float dv = dot3(N, I);
    float k = 1.0f - eta * eta * (1.0f - dv * dv);
    return muls(sub(smul(eta, I), smul(eta * dv + sqrtf(k), N)), (float)(k >= 0.0f));
}

// scatterRay (interactions.cu:43-85)
void scatter(const Scene& sc, Path& p, V3 hit_point, Isect& is, const OMaterial& m, Rng& rng, bool fl_single_albedo) {
    V3 nrm = is.n;
    p.o = add(hit_point, smul(0.0001f, nrm));
    V3 alb = m.texture_id != -1 ? tex_color(sc.texs[m.texture_id], is.uv) : ld3(m.color);
    p.c = mulv(p.c, alb);
    if (m.has_refractive != 0.0f) {
        float n = m.ior;
        float R0 = ((n - 1) * (n - 1)) / ((n + 1) * (n + 1));
        float X = 1 - fabsf(dot3(p.d, nrm));
        float X2 = X * X;
        float R = R0 + (1 - R0) * ((X * X2) * X2);
        if (R < rng.u01()) {
            p.d = refract3(p.d, nrm, n);
            is.n = neg(nrm);
            p.c = mulv(p.c, ld3(m.color));
        } else {
            p.d = reflect3(p.d, nrm);
            p.c = mulv(p.c, ld3(m.spec_color));
        }
    } else if (rng.u01() < m.has_reflective) {
        p.d = reflect3(p.d, nrm);
        p.c = mulv(p.c, ld3(m.spec_color));
    } else {
        p.d = hemisphere(nrm, rng);
    }
    if (!fl_single_albedo) p.c = mulv(p.c, ld3(m.color));   // interactions.cu:83
}

// shadeMaterials (pathtrace.cu:300-344) for the path at array position idx.
void shade(const Scene& sc, const OFlags& fl, Path& p, Isect& is, int idx) {
    if (is.t <= 0.0f) { p.c = mk(0, 0, 0); p.remaining = 0; return; }
    Rng rng(p.iter, idx, p.remaining);
    const OMaterial& m = sc.mats[is.mat];
    if (m.emittance > 0.0f) {
        p.c = mulv(p.c, muls(ld3(m.color), m.emittance));
        p.remaining = 0;
        return;
    }
    scatter(sc, p, point_on_ray(p.o, p.d, is.t), is, m, rng, fl.single_albedo != 0);
    p.bounces += 1;
    if (--p.remaining == 0) { p.c = mk(0, 0, 0); return; }
    if (fl.russian_roulette && p.bounces > 3) {
        const V3 luma = mk((float)0.2126, (float)0.7152, (float)0.0722);
        float l = dot3(p.c, luma);
        float q = gmax(0.05f, 1 - l);
        if (rng.u01() < q) { p.c = mk(0, 0, 0); p.remaining = 0; return; }
        p.c = divs(p.c, 1.0f - q);
    }
}

// generateRayFromCamera (pathtrace.cu:183-227) for global pixel (x, y).
void raygen(const OCamera& cam, const OFlags& fl, int iter, int depth, int x, int y, Path& p) {
    int index = x + y * cam.res[0];
    p.o = ld3(cam.position);
    p.c = mk(1.0f, 1.0f, 1.0f);
    Rng rng(iter, index, depth);
    V3 view = ld3(cam.view), right = ld3(cam.right), up = ld3(cam.up);
    float jx = 0.0f, jy = 0.0f;
    float ax, ay;
    if (fl.ssaa) {
        jx = rng.u01();
        ax = ((float)x - (float)cam.res[0] * 0.5f) + jx;
        jy = rng.u01();
        ay = ((float)y - (float)cam.res[1] * 0.5f) + jy;
    } else {
        ax = (float)x - (float)cam.res[0] * 0.5f;
        ay = (float)y - (float)cam.res[1] * 0.5f;
    }
    V3 dir = sub(sub(view, muls(muls(right, cam.pixel_length[0]), ax)), muls(muls(up, cam.pixel_length[1]), ay));
    p.d = normalize3(dir);
    if (fl.dof) {
        float r = rng.u01() * fl.aperture;
        float th = (rng.u01() * 2) * kPI;
        float sth, cth;
        pt_sincos(th, &sth, &cth);
        V3 lens = mk(r * cth, r * sth, 0.0f);
        float ft = fl.focal_dist / fabsf(p.d.z);
        V3 focus = add(p.o, smul(ft, p.d));
        p.o = add(p.o, lens);
        p.d = normalize3(sub(focus, p.o));
    }
    p.pixel = index;
    p.remaining = depth;
    p.bounces = 0;
}

}  // namespace

extern "C" {

void oracle_sincos(float x, float* s, float* c) { pt_sincos(x, s, c); }

float oracle_u01_sequence(int iter, int index, int depth, int count, float* out) {
    Rng r(iter, index, depth);
    for (int i = 0; i < count; ++i) out[i] = r.u01();
    return count > 0 ? out[0] : 0.0f;
}

// utilityCore::buildTransformationMatrix (utilities.cpp:84-92) + scene.cpp:89-91.
void oracle_build_transform(const float* t, const float* r, const float* s, float* T, float* Inv, float* InvT) {
    float mt[16], rx[16], ry[16], rz[16], rot[16], ms[16], tr[16];
    m4_translate(t, mt);
    m4_rotate(r[0] * (float)kPI / 180, mk(1, 0, 0), rx);
    m4_rotate(r[1] * (float)kPI / 180, mk(0, 1, 0), ry);
    m4_rotate(r[2] * (float)kPI / 180, mk(0, 0, 1), rz);
    m4_mul(rx, ry, rot);
    m4_mul(rot, rz, rot);
    m4_scale(s, ms);
    m4_mul(mt, rot, tr);
    m4_mul(tr, ms, T);
    m4_inverse(T, Inv);
    m4_inverse_transpose(T, InvT);
}

// Camera as the reference ends up using it on frame 1: scene.cpp:185-211 (load) +
// main.cpp:59-73 (phi/theta/zoom) + main.cpp:117-136 (runCuda first-frame recompute).
void oracle_camera(int resx, int resy, float fovy, const float* eye, const float* lookat, const float* upv, OCamera* cam) {
    std::memset(cam, 0, sizeof *cam);
    cam->res[0] = resx; cam->res[1] = resy;
    V3 pos = ld3(eye), la = ld3(lookat), up = ld3(upv);
    float yscaled = tanf(fovy * (kPI / 180));
    float xscaled = (yscaled * resx) / resy;
    float fovx = (atanf(xscaled) * 180) / kPI;
    cam->fov[0] = fovx; cam->fov[1] = fovy;
    cam->pixel_length[0] = 2 * xscaled / (float)resx;
    cam->pixel_length[1] = 2 * yscaled / (float)resy;
    V3 view = normalize3(sub(la, pos));
    // main.cpp:65-73
    V3 vxz = mk(view.x, 0.0f, view.z), vzy = mk(0.0f, view.y, view.z);
    float phi = acosf(dot3(normalize3(vxz), mk(0, 0, -1)));
    float theta = acosf(dot3(normalize3(vzy), mk(0, 1, 0)));
    float zoom = length3(sub(pos, la));
    // main.cpp:121-134
    V3 cp = mk((zoom * sinf(phi)) * sinf(theta), zoom * cosf(theta), (zoom * cosf(phi)) * sinf(theta));
    V3 v = neg(normalize3(cp));
    V3 rr = cross3(v, mk(0, 1, 0));
    V3 uu = cross3(rr, v);
    V3 p = add(cp, la);
    const V3 out[5] = {p, la, v, uu, rr};
    float* dst[5] = {cam->position, cam->look_at, cam->view, cam->up, cam->right};
    for (int k = 0; k < 5; ++k) { dst[k][0] = out[k].x; dst[k][1] = out[k].y; dst[k][2] = out[k].z; }
    (void)up;
}

// One render pass = `spp` consecutive iterations [iter_first, iter_first+spp) traced together
// for the pixel tile {rows y : y % world == rank} (world == 1: the whole image; spp == 1:
// exactly the reference's pathtrace(), pathtrace.cu:423-528).  `image` is the tile
// accumulator (npix_tile x float3, tile-local row-major), updated in place.  `bounce_live`
// (optional, depth entries) accumulates the live-path count entering each bounce.
// Per pixel, contributions are added in sample order (as `spp` sequential iterations would).
// Test tap (tests/test_pin_*.py): the material keys of bounce `bounce` as computeIntersections
// leaves them (before the sort, pathtrace.cu:470-491) and the survivor flags as shadeMaterials
// leaves them (remainingBounces > 0, before the compaction, pathtrace.cu:495-505) — real inputs
// for pinning the sort and partition semantics against rocThrust.
struct Tap {
    int bounce = -1, cap = 0, n = 0;
    int32_t *keys = nullptr, *flags = nullptr;
};
static Tap g_tap;
void oracle_set_tap(int bounce, int32_t* keys, int32_t* flags, int cap) {
    g_tap = Tap{};
    g_tap.bounce = bounce;
    g_tap.keys = keys;
    g_tap.flags = flags;
    g_tap.cap = cap;
}
int oracle_tap_count() { return g_tap.n; }

// Worker threads of oracle_render_pass's per-path loops (raygen, intersection, shading): each
// path's work is independent given its index, and the sort and the compaction stay sequential, so
// the result is the same for every thread count (default 1).  Lets a test check a 4K frame
// (BASELINE.json configs 4 and 5 at their benched size) in seconds on the host's cores.
static int g_threads = 1;
void oracle_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
}  // extern "C"

template <class F>
static void par_for(int n, F f) {
    const int T = std::min(g_threads, std::max(1, n / 256));
    if (T <= 1) {
        for (int i = 0; i < n; ++i) f(i);
        return;
    }
    std::vector<std::thread> ts;
    ts.reserve((size_t)T);
    for (int t = 0; t < T; ++t)
        ts.emplace_back([=, &f] {
            // interleaved 64-path chunks: the cost per path varies along the array
            for (int c0 = t * 64; c0 < n; c0 += T * 64)
                for (int i = c0, e = std::min(n, c0 + 64); i < e; ++i) f(i);
        });
    for (auto& th : ts) th.join();
}

extern "C" {

int oracle_render_pass(const OGeom* geoms, int ngeoms, const OMaterial* mats, int nmats,
                       const OTriangle* tris, int ntris, const ONode* nodes, int nnodes,
                       const OTexture* texs, int ntexs,
                       const OCamera* cam, int depth, const OFlags* fl,
                       int iter_first, int spp, int rank, int world,
                       float* image, uint64_t* bounce_live) {
    Scene sc{geoms, ngeoms, mats, nmats, tris, ntris, nodes, nnodes, texs, ntexs};
    const int W = cam->res[0], H = cam->res[1];
    const int rows = (H - rank + world - 1) / world;
    const int npix = rows * W;
    const int P = npix * spp;
    std::vector<Path> paths((size_t)P);
    par_for(P, [&](int i) {
        const int s = i / npix, lp = i % npix;
        int y = (lp / W) * world + rank, x = lp % W;
        Path& p = paths[(size_t)i];
        raygen(*cam, *fl, iter_first + s, depth, x, y, p);
        p.slot = s * npix + lp;
        p.iter = iter_first + s;
    });
    std::vector<Isect> isect((size_t)P);
    std::vector<int32_t> flags((size_t)P), perm((size_t)P);
    std::vector<Path> tmp((size_t)P);
    int N = P, bounce = 0;
    while (N != 0) {
        if (bounce_live && bounce < depth) bounce_live[bounce] += (uint64_t)N;
        std::memset(isect.data(), 0, sizeof(Isect) * (size_t)P);          // pathtrace.cu:466
        par_for(N, [&](int i) { compute_isect(sc, *fl, paths[i].o, paths[i].d, isect[i]); });
        const bool tap = bounce == g_tap.bounce && N <= g_tap.cap;
        if (tap) {
            g_tap.n = N;
            for (int i = 0; i < N; ++i) g_tap.keys[i] = isect[i].mat;
        }
        if (fl->sort_by_material) {                                          // pathtrace.cu:479-491
            std::vector<int> ord((size_t)N);
            for (int i = 0; i < N; ++i) ord[i] = i;
            // a batched pass sorts each iteration on its own: key (iteration, material)
            std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) {
                return paths[a].iter != paths[b].iter ? paths[a].iter < paths[b].iter : isect[a].mat < isect[b].mat;
            });
            std::vector<Isect> is2((size_t)N);
            for (int i = 0; i < N; ++i) { tmp[i] = paths[ord[i]]; is2[i] = isect[ord[i]]; }
            for (int i = 0; i < N; ++i) { paths[i] = tmp[i]; isect[i] = is2[i]; }
        }
        // RNG key (pathtrace.cu:315): the index within the path's own iteration, i.e. what `spp`
        // sequential pathtrace() calls would use (the array is iteration-major: stable compaction
        // of slot-ordered paths, and the sort above keeps iterations apart)
        {
            std::vector<int32_t> base((size_t)N);
            for (int i = 0, b = 0; i < N; ++i) {
                if (i > 0 && paths[i].iter != paths[i - 1].iter) b = i;
                base[(size_t)i] = b;
            }
            par_for(N, [&](int i) { shade(sc, *fl, paths[i], isect[i], fl->rng_key_pixel ? paths[i].pixel : i - base[(size_t)i]); });
        }
        // relocate_terminated_paths (pathtrace.cu:377-407) == thrust::stable_partition here
        for (int i = 0; i < N; ++i) flags[i] = paths[i].remaining == 0 ? 0 : 1;
        if (tap)
            for (int i = 0; i < N; ++i) g_tap.flags[i] = paths[i].remaining;
        int live = 0;
        {
            std::vector<int32_t> keep(flags.begin(), flags.begin() + N), pos((size_t)N);
            uint32_t acc = 0;
            for (int i = 0; i < N; ++i) { pos[i] = (int32_t)acc; acc += (uint32_t)keep[i]; }
            live = (int)acc;
            for (int i = 0; i < N; ++i) {
                int dst = keep[i] ? pos[i] : live + i - pos[i];
                tmp[dst] = paths[i];
            }
            for (int i = 0; i < N; ++i) paths[i] = tmp[i];
        }
        N = live;
        ++bounce;
    }
    // finalGather (pathtrace.cu:347-356): sum per pixel in sample order.
    std::vector<V3> col((size_t)P);
    for (int i = 0; i < P; ++i) col[(size_t)paths[i].slot] = paths[i].c;
    for (int lp = 0; lp < npix; ++lp) {
        float* px = image + 3 * (size_t)lp;
        for (int s = 0; s < spp; ++s) {
            const V3& c = col[(size_t)s * npix + lp];
            px[0] += c.x; px[1] += c.y; px[2] += c.z;
        }
    }
    return bounce;
}

// Convenience: ITERATIONS passes of spp=1 on the whole image, the reference's render loop
// (main.cpp:140-160).  Returns wall seconds (for the CPU baseline).
double oracle_render(const OGeom* geoms, int ngeoms, const OMaterial* mats, int nmats,
                     const OTriangle* tris, int ntris, const ONode* nodes, int nnodes,
                     const OTexture* texs, int ntexs,
                     const OCamera* cam, int depth, const OFlags* fl,
                     int iter_first, int iters, float* image, uint64_t* bounce_live) {
    auto t0 = std::chrono::high_resolution_clock::now();
    for (int it = 0; it < iters; ++it)
        oracle_render_pass(geoms, ngeoms, mats, nmats, tris, ntris, nodes, nnodes, texs, ntexs,
                           cam, depth, fl, iter_first + it, 1, 0, 1, image, bounce_live);
    auto t1 = std::chrono::high_resolution_clock::now();
    return std::chrono::duration<double>(t1 - t0).count();
}

// Image output: saveImage (main.cpp:88-112) + Image::savePNG (image.cpp:22-42) pixel math.
// Writes W*H*3 bytes, x-mirrored, value = uchar(clamp(sum/spp, 0, 1) * 255).
void oracle_tonemap(const float* image, int W, int H, float samples, uint8_t* out) {
    for (int x = 0; x < W; ++x)
        for (int y = 0; y < H; ++y) {
            const float* p = image + 3 * (size_t)(x + y * W);
            int dx = W - 1 - x;
            for (int k = 0; k < 3; ++k) {
                float v = p[k] / samples;
                v = gmin(gmax(v, 0.0f), 1.0f) * 255.f;
                out[3 * (size_t)(y * W + dx) + k] = (uint8_t)v;
            }
        }
}

// sendImageToPBO (pathtrace.cu:64-86): RGBA8 preview of the accumulator.
void oracle_preview(const float* image, int W, int H, int iter, uint8_t* rgba) {
    for (int i = 0; i < W * H; ++i) {
        for (int k = 0; k < 3; ++k) {
            int v = (int)((double)(image[3 * (size_t)i + k] / iter) * 255.0);
            v = v < 0 ? 0 : (v > 255 ? 255 : v);
            rgba[4 * (size_t)i + k] = (uint8_t)v;
        }
        rgba[4 * (size_t)i + 3] = 0;
    }
}

}  // extern "C"

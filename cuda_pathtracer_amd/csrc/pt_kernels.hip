// MI355X path-tracer hot path: ray generation -> ray/scene intersection -> BSDF shading ->
// stable compaction of terminated paths, one fused kernel per bounce.
//
// Reference: path_tracer/src/pathtrace.cu:183-528 (generateRayFromCamera, computeIntersections,
// shadeMaterials, relocate_terminated_paths, finalGather), intersections.cu, interactions.cu,
// sceneStructs.h.  MI355X design:
//   * path state as three 16-byte planes per path (one dwordx4 per plane, wave-contiguous);
//   * k_bounce, one launch per bounce: [raygen] -> bounded closest hit (conservative bounds pass
//     over all geoms, exact reference tests only for candidates) -> shading -> survivors written
//     in order into this workgroup's segment (wave ballot + mbcnt, 4 wave counts in LDS).  The
//     next launch scans the segment words in LDS, so no workgroup waits on another; no hit-record
//     round trip, no memset of W*H hit records per bounce, no host round trip for the live count;
//   * batched passes: workgroups are dealt to iterations, shading keys are per-iteration
//     compacted indices, so a pass of spp iterations equals spp pathtrace() calls bit for bit;
//   * a path's radiance is added to the framebuffer the moment it terminates (each pixel owns
//     one path per iteration, so this equals finalGather); spp > 1 passes write per-slot colours
//     and a finalize kernel adds them in sample order;
//   * material-sorted shading (flag) = stable counting sort over (iteration, material) keys:
//     one producer per bounce (shade in sorted order, compact by material per tile, intersect,
//     histogram), a three-kernel histogram scan whose last kernel also writes the permutation;
//   * the split pipeline (PT_PIPELINE=split: k_trace + look-back k_compact_paths) is kept for
//     comparison and for the bounded-hit verification mode.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "lookback.h"
#include "pt_device.h"
#include "pt_internal.h"
#include "../../include/sc_amd.h"

using namespace ptd;

namespace {

constexpr int kBlock = 256;

// Path state: three 16-byte planes (one dwordx4 load/store each, a wave moving 1 KiB contiguous
// per instruction): a = (o.xyz, d.x), b = (d.yz, c.rg), c = (c.b, slot, bounces, 0).
typedef float v2f __attribute__((ext_vector_type(2)));
// a = (o, d.x), b = (d.yz, colour.rg), c = (colour.b, slot): every path of a launch has the same
// number of bounces behind it (KArgs::bounce), so it is not stored.
struct PathSoA {
    v4f *a, *b;
    v2f* c;
};
struct HitSoA {   // sorted pipeline, textured scenes: texture coordinates of physical path j
    float* uv;    // [2 * P]
};
struct Ctl {            // per-parity control block (32 B)
    uint32_t ticket;       // claimed tile schedule (look-back kernels)
    uint32_t live;         // path count: after k_compact_paths (split), of this bounce (sorted)
    uint32_t chunk, nseg;  // segment layout written by k_bounce / k_sort_shade
    uint32_t hist_live;    // sorted pipeline: live histogram entries (+1) written by k_sort_produce
    uint32_t pad[3];
};
struct DevStats {
    unsigned long long segments, passes, bounce_live[64];
    uint32_t err, bound_mismatch;
};

struct SceneDev {
    const DGeom* __restrict__ geoms;
    const DGeom* __restrict__ bgeoms;   // the geoms ordered by bkind (DGeom::orig = index in geoms)
    int32_t bk[6];                      // bgeoms[bk[k] .. bk[k+1]) have bkind k
    const DMaterial* __restrict__ mats;
    const DTri* __restrict__ tris;
    const DTriAttr* __restrict__ attrs;
    const DNode* __restrict__ nodes;
    const DTexture* __restrict__ texs;
    int32_t ngeoms, nmats, ntris, nnodes;
    int32_t bvh_depth;     // deepest interior node (root = 0): bounds the traversal stack
    float abs_slack;       // absolute slack of the world-distance lower bounds (bound_geom)
    float wb_tslack;       // the smallest tslack of the world-box cubes (bound_wbox_tagged; DGeom::wback)
    const struct DPair* __restrict__ pairs;   // child-pair layout of the BVH (bvh_walk_pairs)
    int32_t root_code;     // code of the root (see DPair), meaningful when pairs != nullptr
    v4f root_lo, root_hi;  // root box
    const struct DQuad* __restrict__ quads;   // 4-wide collapse of the pair tree (k_traverse4), or null
    int32_t root_qcode;    // root's code in the quad layout (quad index or leaf code)
    const float* __restrict__ tpack;   // the triangles again as packed 36-byte (v0, e1, e2): k_traverse4's task loads
    const uint32_t* __restrict__ qcull;   // exact t-cull margins of the quads' slots (build_qcull), or null: off
};
struct CamDev {
    float pos[3], view[3], up[3], right[3], pl[2];
    int32_t res[2];
};
struct FlagsDev {
    int32_t rr, bvh, bbox, ssaa, dof;
    float aperture, focal;
    int32_t single_albedo;
    int32_t bvh_cull;
    int32_t claimed;   // tile schedule (lookback.h TileSeq)
    int32_t rng_pixel; // shading RNG keyed by global pixel (pt_flags.rng_key_pixel)
    int32_t verify;    // PT_AMD_VERIFY_BOUNDS=1: re-run the plain closest-hit loop, count differences
};
struct TileDev {
    int32_t W, rank, world, npix, spp, P, depth, iter_first;
    uint64_t wdiv;   // ceil(2^40 / W) when npix * W < 2^40 (then lp / W == lp * wdiv >> 40), else 0
};
struct KArgs {
    SceneDev S;
    CamDev cam;
    FlagsDev fl;
    TileDev tile;
    PathSoA in, out;
    HitSoA hit;
    float* image;          // npix * 3 (AoS float3, tile-local)
    v4f* colbuf;           // P (spp > 1): final path colour per slot, one 16-byte store (retire)
    uint8_t* colflag;      // (spp > 1) one byte per slot, pixel-major: [pixel][iteration of the pass]; 1 when
                           // retire stored a (nonzero) colour in the slot this pass — the others are zero colours,
                           // which retire does not store; k_finalize_spp reads and clears them
    int32_t col_spp;       // iterations of the pass (the flag row length), over all lanes
    int32_t col_off;       // this lane's first iteration within the pass
    float inv_npix;        // 1 / tile.npix (retire: a slot's iteration and pixel)
    Ctl* ctl;              // [2]
    uint64_t* status;      // [2][max_tiles] look-back words of k_compact_paths
    int32_t max_tiles;
    int32_t parity;
    int32_t bounce;
    int32_t n_fixed;       // >= 0: path count is known on the host (first bounce)
    int32_t* flags;        // [P] survivor flags of the current bounce
    int32_t* seg;          // [2][kMaxSeg] per-workgroup survivor count | batch iteration << 24 (k_bounce)
    int32_t* ibase;        // [kMaxSpp + 1] split pipeline: first dense index of each iteration
    DevStats* stats;
    unsigned long long* emit_slots;   // [64 bounces][emit_stride]: per-workgroup emissive counts
    int32_t emit_stride;
    int32_t count_pass;    // this launch sequence counts the pass in DevStats::passes (lane 0)
    v4f* mhit;             // [path capacity] k_traverse -> k_bounce<.., kMeshPre>: (t, idx, bx, by)
    uint32_t* tticket;     // k_traverse: this bounce's ray ticket (zeroed at the start of the pass)
    int32_t refill_min;    // k_traverse: idle lanes that trigger a refill (kRefillMin; PT_AMD_REFILL)
    int32_t tchunk;        // k_traverse: largest ray chunk per ticket grab (kTravChunk; PT_AMD_TCHUNK)
    int32_t stack_rows;    // k_traverse: LDS stack entries per thread (HybStack)
    const uint32_t* cmask; // first bounce: per 64 tile pixels, the geoms its camera rays can hit (null: all)
};

// ------------------------------------------------------------------------------------------
// Intersection (computeIntersections, pathtrace.cu:229-298)
// ------------------------------------------------------------------------------------------
struct Hit {
    float t;
    f3 n;
    int32_t mat;
    float u, v;
    int32_t frame = -1;   // cube hits: geom * 6 + slab code (the precomputed tangent frame, DGeom::frm)
};
// The fused first bounce does the same in its own instantiation (k_bounce<true, .., kAnalyticSkip>: 5
// more VGPRs), chosen per context when at least kSkipEmptyMin of the camera-mask blocks are empty
// (build_cmask; config 4's 16:9 view +4.0%, while Cornell at 800x800 lost 1.1% to the registers).
constexpr double kSkipEmptyMin = 0.2;
// What the closest hit returns for a ray that meets nothing (intersect_bounded, computeIntersections'
// t = -1 with materialId 0: pathtrace.cu:466).
__device__ __forceinline__ Hit miss_hit() {
    Hit h;
    h.t = -1.0f;
    h.mat = 0;
    h.n = F3(0, 0, 0);
    h.u = h.v = 0.0f;
    return h;
}

// boxIntersectionTest (intersections.cu:3-58).  The world normal is deferred to the closest
// hit: we keep the slab code (axis*2 + sign, -1 = zero vector) and rebuild n from it.
template <class G>
__device__ __forceinline__ float box_test(const G& g, f3 ro, f3 rd, int& ncode) {
    const f3 qo = xform_point(g.inv, ro);
    const f3 qd = normalize(xform_vector(g.inv, rd));
    float tmin = -1e38f, tmax = 1e38f;
    int nmin = -1, nmax = -1;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float qa = at(qd, a), oa = at(qo, a);
        float t1, t2;
        div2_cr(-0.5f - oa, +0.5f - oa, qa, t1, t2);
        const float ta = gmin(t1, t2), tb = gmax(t1, t2);
        const int code = 2 * a + (t2 < t1 ? 0 : 1);
        if (ta > 0 && ta > tmin) { tmin = ta; nmin = code; }
        if (tb < tmax) { tmax = tb; nmax = code; }
    }
    if (tmax >= tmin && tmax > 0) {
        if (tmin <= 0) { tmin = tmax; nmin = nmax; }
        const f3 ip = xform_point(g.xf, point_on_ray(qo, qd, tmin));
        ncode = nmin;
        return length(ro - ip);
    }
    return -1.0f;
}
// The world normal of slab code `code`: precomputed per cube (DGeom::nrm).  Code -1 (no slab
// bounded the hit: every slab parameter NaN) normalizes the zero vector: 0 * (1 / 0) = NaN.
template <class G>
__device__ __forceinline__ f3 box_normal(const G& g, int code) {
    if (code < 0) return F3(__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""));
    return F3(g.nrm[code][0], g.nrm[code][1], g.nrm[code][2]);
}

// sphereIntersectionTest (intersections.cu:60-115); normal deferred (object-space hit point kept).
template <class G>
__device__ __forceinline__ float sphere_test(const G& g, f3 r_o, f3 r_d, f3& obj, bool& outside) {
    const f3 ro = xform_point(g.inv, r_o);
    const f3 rd = normalize(xform_vector(g.inv, r_d));
    const float vdd = dot(ro, rd);
    const float radicand = vdd * vdd - (dot(ro, ro) - 0.25f);   // powf(0.5f, 2) == 0.25f
    if (radicand < 0) return -1.0f;
    const float sq = sqrt_cr(radicand);
    const float first = -vdd;
    const float t1 = first + sq, t2 = first - sq;
    float t;
    if (t1 < 0 && t2 < 0) return -1.0f;
    if (t1 > 0 && t2 > 0) { t = gmin(t1, t2); outside = true; }
    else { t = gmax(t1, t2); outside = false; }
    obj = point_on_ray(ro, rd, t);
    const f3 ip = xform_point(g.xf, obj);
    return length(r_o - ip);
}
template <class G>
__device__ __forceinline__ f3 sphere_normal(const G& g, f3 obj, bool outside) {
    const f3 n = normalize(xform_vector(g.itr, obj));
    return outside ? n : -n;
}

// glm::intersectRayTriangle (gtx/intersect.inl:37-74) with e1/e2 precomputed on the host.
__device__ __forceinline__ bool ray_tri(const DTri& tr, f3 o, f3 d, float& bx, float& by, float& bz) {
    const f3 v0 = F3(tr.a[0], tr.a[1], tr.a[2]);
    const f3 e1 = F3(tr.b[0], tr.b[1], tr.b[2]);
    const f3 e2 = F3(tr.c[0], tr.c[1], tr.c[2]);
    const f3 p = cross(d, e2);
    const float a = dot(e1, p);
    if (a < kFLT_EPS) return false;
    const float f = div_cr(1.0f, a);
    const f3 s = o - v0;
    bx = f * dot(s, p);
    if (bx < 0.0f || bx > 1.0f) return false;
    const f3 q = cross(s, e1);
    by = f * dot(d, q);
    if (by < 0.0f || by + bx > 1.0f) return false;
    bz = f * dot(e2, q);
    return bz >= 0.0f;
}

// BoundingBox::intersect (boundingbox.h:73-92); `lo` = the entry parameter
__device__ __forceinline__ bool aabb_hit(const float* bmin, const float* bmax, f3 o, f3 inv, float& lo) {
    const float mx = (bmin[0] - o.x) * inv.x, Mx = (bmax[0] - o.x) * inv.x;
    const float my = (bmin[1] - o.y) * inv.y, My = (bmax[1] - o.y) * inv.y;
    const float mz = (bmin[2] - o.z) * inv.z, Mz = (bmax[2] - o.z) * inv.z;
    lo = gmax(gmax(gmin(mx, Mx), gmin(my, My)), gmin(mz, Mz));
    const float hi = gmin(gmin(gmax(mx, Mx), gmax(my, My)), gmax(mz, Mz));
    return !(hi < 0) && !(lo > hi);
}
__device__ __forceinline__ bool aabb_hit(const float* bmin, const float* bmax, f3 o, f3 inv) {
    float lo;
    return aabb_hit(bmin, bmax, o, inv, lo);
}

// The same test for a ray whose o and 1/d are finite: then no slab parameter is NaN (no 0 * inf), and
// fminf/fmaxf (v_min/v_max) give glm's ternary min/max up to the sign of a zero, which neither
// comparison below sees — the same outcome in about 12 fewer instructions.
__device__ __forceinline__ bool aabb_hit_finite(const float* bmin, const float* bmax, f3 o, f3 inv) {
    const float mx = (bmin[0] - o.x) * inv.x, Mx = (bmax[0] - o.x) * inv.x;
    const float my = (bmin[1] - o.y) * inv.y, My = (bmax[1] - o.y) * inv.y;
    const float mz = (bmin[2] - o.z) * inv.z, Mz = (bmax[2] - o.z) * inv.z;
    const float lo = fmaxf(fmaxf(fminf(mx, Mx), fminf(my, My)), fminf(mz, Mz));
    const float hi = fminf(fminf(fmaxf(mx, Mx), fmaxf(my, My)), fmaxf(mz, Mz));
    return !(hi < 0) && !(lo > hi);
}

struct MeshHit {
    bool any;          // BVHIntersectionTest's return value
    int32_t id;        // original triangle id of the closest hit
    int32_t idx;       // index in the BVH-ordered triangle array
    float t, bx, by;
};

// BVHIntersectionTest (intersections.cu:169-224): explicit stack of 64, near child first,
// pops silently on overflow, no t culling; ties keep the first triangle found.
//   The stack lives in LDS (kLdsStack entries per thread, column layout: slot * kBlock + tid, so a
// wave's pushes hit 64 distinct banks) when the tree is shallow enough that the reference's 64
// entries are never reached (pt_create checks the depth: occupancy <= interior depth); deeper trees
// use a 64-entry private array (scratch), which is the reference's exact overflow behaviour.
constexpr int kLdsStack = 32;

template <class Stack>
__device__ __forceinline__ MeshHit bvh_walk(const SceneDev& S, f3 o, f3 d, bool cull, Stack stack) {
    MeshHit r{false, -1, -1, kFLT_MAX, 0.f, 0.f};
    int top = 0, cur = 0;
    const bool neg[3] = {d.x < 0.0f, d.y < 0.0f, d.z < 0.0f};
    const f3 inv = F3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    for (;;) {
        const v4f nlo = S.nodes[cur].lo, nhi = S.nodes[cur].hi;
        const float bmin[3] = {nlo[0], nlo[1], nlo[2]}, bmax[3] = {nhi[0], nhi[1], nhi[2]};
        const int meta = __float_as_int(nlo[3]), link = __float_as_int(nhi[3]);
        float lo;
        // extension (pt_flags.bvh_cull): a node entered beyond the best t (+1e-3 relative) is a miss
        if (aabb_hit(bmin, bmax, o, inv, lo) && !(cull && lo > r.t * 1.001f + 1e-4f)) {
            if (meta > 0) {   // leaf: `meta` triangles from `link`
                for (int k = 0; k < meta; ++k) {
                    const DTri tr = S.tris[link + k];
                    float bx, by, bz;
                    if (ray_tri(tr, o, d, bx, by, bz)) {
                        r.any = true;
                        if (r.t == -1.0f || bz < r.t) {
                            r.t = bz; r.bx = bx; r.by = by; r.id = __float_as_int(tr.a[3]); r.idx = link + k;
                        }
                    }
                }
                if (top == 0) break;
                cur = stack.get(--top);
            } else {          // interior: axis = -meta - 1, right child = link, left child = cur + 1
                if (top == 64) { cur = stack.get(--top); continue; }
                const int axis = -meta - 1;
                const bool ng = axis == 0 ? neg[0] : (axis == 1 ? neg[1] : neg[2]);
                if (ng) { stack.set(top++, cur + 1); cur = link; }
                else { stack.set(top++, link); cur = cur + 1; }
            }
        } else {
            if (top == 0) break;
            cur = stack.get(--top);
        }
    }
    return r;
}

struct LdsStack {
    int* col;   // this thread's column of the block's stack
    __device__ int get(int i) const { return col[i * kBlock]; }
    __device__ void set(int i, int v) const { col[i * kBlock] = v; }
};
// k_traverse: the first `rows` entries in LDS (column layout), the rest of the reference's 64 in a
// private (scratch) array — deep entries are rare, and a short LDS stack keeps more waves resident.
struct HybStack {
    int* col;
    int* priv;   // entries rows .. 63
    int rows;
    __device__ int get(int i) const { return i < rows ? col[i * kBlock] : priv[i - rows]; }
    __device__ void set(int i, int v) const {
        if (i < rows) col[i * kBlock] = v;
        else priv[i - rows] = v;
    }
};
struct PrivStack {
    int* a;
    __device__ int get(int i) const { return a[i]; }
    __device__ void set(int i, int v) const { a[i] = v; }
};

// Child-pair layout of the same tree: one 64-byte entry per INTERIOR node holding both children's
// boxes and codes, so deciding where to go from a node costs one fetch instead of one per child.
//   code >= 0: interior child, entry index * 4 + its split axis;
//   code <  0: leaf child, -(first triangle * 256 + triangle count) - 1.
// The boxes tested, their outcomes (aabb_hit) and the near-first order are those of bvh_walk:
// a child is tested at its parent instead of after being popped, and only passing children are
// pushed, so the triangles tested, their order and the result are the same; used without the
// bvh_cull extension and when the tree is shallow enough for the LDS stack (no overflow case).
struct alignas(16) DPair {
    v4f lmin, lmax, rmin, rmax;   // .w: left code (lmin.w), unused (lmax.w), right code (rmin.w), unused
};

template <class Stack>
__device__ __forceinline__ MeshHit bvh_walk_pairs(const SceneDev& S, f3 o, f3 d, Stack stack) {
    MeshHit r{false, -1, -1, kFLT_MAX, 0.f, 0.f};
    const bool neg[3] = {d.x < 0.0f, d.y < 0.0f, d.z < 0.0f};
    const f3 inv = F3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    {
        const float bmin[3] = {S.root_lo[0], S.root_lo[1], S.root_lo[2]}, bmax[3] = {S.root_hi[0], S.root_hi[1], S.root_hi[2]};
        if (!aabb_hit(bmin, bmax, o, inv)) return r;
    }
    int top = 0, cur = S.root_code;
    for (;;) {
        if (cur < 0) {   // leaf
            const int c = -cur - 1, first = c >> 8, count = c & 255;
            for (int k = 0; k < count; ++k) {
                const DTri tr = S.tris[first + k];
                float bx, by, bz;
                if (ray_tri(tr, o, d, bx, by, bz)) {
                    r.any = true;
                    if (r.t == -1.0f || bz < r.t) {
                        r.t = bz; r.bx = bx; r.by = by; r.id = __float_as_int(tr.a[3]); r.idx = first + k;
                    }
                }
            }
            if (top == 0) break;
            cur = stack.get(--top);
            continue;
        }
        const DPair P = S.pairs[cur >> 2];
        const int axis = cur & 3;
        float lo;
        const float lmn[3] = {P.lmin[0], P.lmin[1], P.lmin[2]}, lmx[3] = {P.lmax[0], P.lmax[1], P.lmax[2]};
        const float rmn[3] = {P.rmin[0], P.rmin[1], P.rmin[2]}, rmx[3] = {P.rmax[0], P.rmax[1], P.rmax[2]};
        const bool hl = aabb_hit(lmn, lmx, o, inv, lo), hr = aabb_hit(rmn, rmx, o, inv, lo);
        const int cl = __float_as_int(P.lmin[3]), cr = __float_as_int(P.rmin[3]);
        const bool ng = axis == 0 ? neg[0] : (axis == 1 ? neg[1] : neg[2]);   // right child first
        const bool h1 = ng ? hr : hl, h2 = ng ? hl : hr;
        const int c1 = ng ? cr : cl, c2 = ng ? cl : cr;
        if (h1) {
            if (h2) stack.set(top++, c2);
            cur = c1;
        } else if (h2) {
            cur = c2;
        } else {
            if (top == 0) break;
            cur = stack.get(--top);
        }
    }
    return r;
}

// 4-wide layout (k_traverse4): the pair entry of interior node N with each interior child X
// replaced by X's own two children when both boxes lie inside X's box (checked on the host, so a
// grandchild box that the ray hits implies a hit on X's box — the slab test is monotone in the box
// bounds for a finite ray: (b - o) * inv is nondecreasing in b for inv > 0 and nonincreasing for
// inv < 0, so X's slab intervals contain the grandchild's).  The leaves reached, and in the
// near-first order below the triangles tested, are BVHIntersectionTest's (intersections.cu:170-224).
//   Slots 0-1: N's left child's group (X's two children, or the child itself in slot 0), slots 2-3
// the right child's.  meta bits: valid slots (0-3) | N's axis << 4 | left group's axis << 6 |
// right group's axis << 8 (3: a one-slot group, never swapped).  Codes as DPair's, with interior
// codes = quad index.  Boxes are SoA (one v4f per bound and axis) so the four slab tests run two
// slots per packed f32 instruction.
// An interior code carries its quad's meta bits above the index (kQuadMetaShift), so a walk learns
// the order of a quad's slots from the code that led to it and loads 112 of the entry's 128 bytes.
struct alignas(16) DQuad {
    v4f lox, hix, loy, hiy, loz, hiz;
    v4f code;   // int bits
    v4f meta;   // [0]: int bits (above; also in the interior codes that point here)
};
constexpr int kQuadMetaShift = 21;                        // interior code = quad index | meta << 21
constexpr int kQuadIdxMask = (1 << kQuadMetaShift) - 1;   // (a layout of more quads is not built)

constexpr int kRecWalkHere = -2;   // k_traverse4 record: not walked (non-finite ray), k_bounce walks it
constexpr int kWalkDone = (int)0x80000000;   // k_traverse: no node left (below every leaf code, first < 2^23)
constexpr int kWalkNone = (int)0x80000001;   // k_traverse: stay (the leaf has triangles left)

#ifdef PT_TRAV_STATS
__device__ unsigned long long g_trav[64 * 8];   // [slot][0 rays, 1 pairs, 2 tris, 3 wave steps, 4 waves]
#endif

__device__ MeshHit bvh_traverse(const SceneDev& S, f3 o, f3 d, bool cull) {
    if (S.nnodes == 0) return MeshHit{false, -1, -1, kFLT_MAX, 0.f, 0.f};
    if (S.bvh_depth < kLdsStack) {
        __shared__ int s_stack[kLdsStack * kBlock];
        if (S.pairs && !cull) return bvh_walk_pairs(S, o, d, LdsStack{s_stack + threadIdx.x});
        return bvh_walk(S, o, d, cull, LdsStack{s_stack + threadIdx.x});
    }
    int stack[64];
    return bvh_walk(S, o, d, cull, PrivStack{stack});
}

// Triangle::intersect's attributes for the closest triangle (sceneStructs.h:151-154).
__device__ __forceinline__ void tri_attrs(const DTriAttr& a, float bx, float by, f3& n, float& u, float& v) {
    const float w = (1.0f - bx) - by;
    u = (a.uv[0][0] * w + a.uv[1][0] * bx) + a.uv[2][0] * by;
    v = (a.uv[0][1] * w + a.uv[1][1] * bx) + a.uv[2][1] * by;
    const f3 n0 = F3(a.n[0][0], a.n[0][1], a.n[0][2]) * bx;
    const f3 n1 = F3(a.n[1][0], a.n[1][1], a.n[1][2]) * by;
    const f3 n2 = F3(a.n[2][0], a.n[2][1], a.n[2][2]) * ((1.0f - bx) - by);
    n = normalize((n0 + n1) + n2);
}

// meshIntersectionTest (intersections.cu:119-167): linear loop, optional world-AABB cull.
template <class G>
__device__ float mesh_linear(const SceneDev& S, const G& g, f3 o, f3 d, bool use_bbox, f3& n, float& u, float& v) {
    if (use_bbox) {
        const f3 inv = F3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
        const float bmin[3] = {g.bmin[0], g.bmin[1], g.bmin[2]}, bmax[3] = {g.bmax[0], g.bmax[1], g.bmax[2]};
        if (!aabb_hit(bmin, bmax, o, inv)) return -1.0f;
    }
    int best = -1;
    float tmin = kFLT_MAX, b0 = 0.f, b1 = 0.f;
    for (int i = g.tri_start; i < g.tri_end; ++i) {
        float bx, by, bz;
        if (ray_tri(S.tris[i], o, d, bx, by, bz) && bz > 0.0f && bz < tmin) { best = i; tmin = bz; b0 = bx; b1 = by; }
    }
    if (best == -1) return -1.0f;
    const float az = (1.0f - b0) - b1;
    const DTriAttr& a = S.attrs[best];
    const f3 s = (az * F3(a.n[0][0], a.n[0][1], a.n[0][2]) + F3(a.n[1][0], a.n[1][1], a.n[1][2])) +
                 F3(a.n[2][0], a.n[2][1], a.n[2][2]);
    n = normalize(s);
    u = (az * a.uv[0][0] + a.uv[1][0]) + a.uv[2][0];
    v = (az * a.uv[0][1] + a.uv[1][1]) + a.uv[2][1];
    return tmin;
}

// `pre`: the BVH closest hit of this ray, already computed by k_traverse (nullptr: traverse here).
template <bool MESH, bool PRE = false>
__device__ __forceinline__ Hit intersect_scene(const SceneDev& S, const FlagsDev& fl, f3 ro, f3 rd,
                                               const MeshHit* pre = nullptr) {
    float t_min = kFLT_MAX;
    int hit_geom = -1, best_code = -1;
    f3 best_obj = F3(0, 0, 0), best_n = F3(0, 0, 0);
    bool best_outside = true;
    float tmp_u = 0.f, tmp_v = 0.f, cu = 0.f, cv = 0.f;
    f3 tmp_n = F3(0, 0, 0);
    MeshHit mh{false, -1, -1, kFLT_MAX, 0.f, 0.f};
    bool traversed = false;
    const auto* G = as_const(S.geoms);   // wave-uniform: scalar loads
    for (int i = 0; i < S.ngeoms; ++i) {
        const auto& g = G[i];
        float t = -1.0f;
        int code = -1;
        f3 obj = F3(0, 0, 0);
        bool outside = true;
        const int type = g.type;
        if (type == PT_GEOM_CUBE) {
            t = box_test(g, ro, rd, code);
        } else if (type == PT_GEOM_SPHERE) {
            t = sphere_test(g, ro, rd, obj, outside);
        } else if (MESH && type == PT_GEOM_MESH) {
            if constexpr (PRE) {   // (PRE kernels run with fl.bvh set)
                if (pre->any && pre->id >= g.tri_start && pre->id < g.tri_end) {
                    t = pre->t;
                    tri_attrs(S.attrs[pre->idx], pre->bx, pre->by, tmp_n, tmp_u, tmp_v);
                }
            } else if (fl.bvh) {
                if (!traversed) { mh = bvh_traverse(S, ro, rd, fl.bvh_cull != 0); traversed = true; }
                if (mh.any && mh.id >= g.tri_start && mh.id < g.tri_end) {
                    t = mh.t;
                    tri_attrs(S.attrs[mh.idx], mh.bx, mh.by, tmp_n, tmp_u, tmp_v);
                }
            } else {
                float u2, v2;
                f3 n2;
                t = mesh_linear(S, g, ro, rd, fl.bbox != 0, n2, u2, v2);
                if (t != -1.0f) { tmp_n = n2; tmp_u = u2; tmp_v = v2; }
            }
        }
        if (t > 0.0f && t_min > t) {
            t_min = t;
            hit_geom = i;
            cu = tmp_u;
            cv = tmp_v;
            best_code = code;
            best_obj = obj;
            best_outside = outside;
            best_n = tmp_n;
        }
    }
    Hit h;
    if (hit_geom < 0) {
        h.t = -1.0f;
        h.mat = 0;
        h.n = F3(0, 0, 0);
        h.u = h.v = 0.f;
        return h;
    }
    const DGeom& g = S.geoms[hit_geom];
    h.t = t_min;
    h.mat = g.material;
    h.u = cu;
    h.v = cv;
    if (g.type == PT_GEOM_CUBE) {
        h.n = box_normal(g, best_code);
        if (best_code >= 0) h.frame = hit_geom * 6 + best_code;
    }
    else if (g.type == PT_GEOM_SPHERE) h.n = sphere_normal(g, best_obj, best_outside);
    else h.n = best_n;
    return h;
}

// ---- bounded closest hit for analytic scenes (cubes + spheres) ------------------------------
// computeIntersections evaluates the exact test of EVERY geom for every ray (≈170 VALU per cube:
// two affine transforms, a correctly rounded normalize, six correctly rounded divisions, the
// back-transform and a length).  Here a cheap pass over all geoms computes, per geom, a LOWER
// BOUND on the reference's world distance (or "surely misses"), from the same inverse transform
// against the unit cube / sphere WIDENED by more than the rounding error of either computation
// (DGeom.slo/shi/r2w, sized on the host from the scene's extent).  Only the geoms whose bound is
// not beyond an exactly evaluated hit are then run through the exact test above — per lane, with
// the geom read from LDS — in increasing-bound order.  A skipped geom either misses exactly or has
// an exact distance strictly larger than an evaluated hit, so the selected hit (minimum t, lowest
// index on ties, pathtrace.cu:284-288) is the reference's bit for bit.  Typically one exact test
// per ray instead of one per geom.  PT_AMD_VERIFY_BOUNDS=1 re-runs the plain loop and counts any
// difference (pt_stats_t.bound_mismatch).

constexpr int kLdsGeoms = 32;
// What the exact tests and the hit normal read: 47 words, padded to a 52-word (208-byte) row so
// the rows of up to 16 geoms start in distinct 4-bank windows — lanes of a wave testing different
// geoms read without LDS bank conflicts (a 48-word row put rows r and r+4 on the same banks:
// SQ_LDS_BANK_CONFLICT 6.8 M cycles per bounce launch).
struct alignas(16) LGeom {
    Affine inv, xf;
    union {
        Affine itr;          // spheres: the hit normal's transform
        float nrm[6][3];     // cubes: the world normal of each slab code (DGeom::nrm)
    };
    int32_t type, material;
    int32_t pad[2];
};
static_assert(sizeof(LGeom) == 208, "LGeom row stride");
constexpr float kInf = __builtin_inff();

// The cubes' tangent frames (DGeom::frm) for shade(): [geom * 6 + code][6] floats.
__device__ __forceinline__ void stage_frames(const SceneDev& S, float* s_frm) {
    if (S.ngeoms > kLdsGeoms) return;
    const auto* G = as_const(S.geoms);
    for (int e = threadIdx.x; e < S.ngeoms * 36; e += blockDim.x) {
        const int gi = e / 36, q = e % 36;
        if (G[gi].type == PT_GEOM_CUBE) s_frm[e] = G[gi].frm[q / 6][q % 6];
    }
}
__device__ __forceinline__ void stage_geoms(const SceneDev& S, LGeom* s_geoms) {
    if (S.ngeoms > kLdsGeoms) return;
    for (int j = threadIdx.x; j < S.ngeoms; j += blockDim.x) {
        const DGeom& g = S.geoms[j];
        s_geoms[j].inv = g.inv;
        s_geoms[j].xf = g.xf;
        if (g.type == PT_GEOM_CUBE)
            for (int q = 0; q < 18; ++q) s_geoms[j].nrm[q / 3][q % 3] = g.nrm[q / 3][q % 3];
        else
            s_geoms[j].itr = g.itr;
        s_geoms[j].type = g.type;
        s_geoms[j].material = g.material;
    }
}

// World-box cubes (bkind 3) in packed f32 operations: both planes of an axis, ((lo - o) * r,
// (hi - o) * r), in one v_pk_add_f32 and one v_pk_mul_f32 (<2 x float> operations; IEEE per
// component, the same bits as two subtractions and two multiplications), the box pair from the
// geom's SGPRs (wbox).  The bound is bound_geom<3>'s (below) up to the rounding of its last step,
// returned TAGGED (tag_bound).
// With E0 = max(E, 0), "E > X || X < 0" is "E0 > X" (NaN slabs included: both are false for a NaN X,
// and a NaN E gives E0 = 0).
__device__ __forceinline__ uint32_t tag_bound(float v, uint32_t i);
// rlt = rl * wb_tslack (per ray): v = E0 * rl * ts - back * ts with the smallest tslack of the world-box
// cubes for every one of them (a smaller slack is still a slack) and wback = back * that, rounded up.
template <class G>
__device__ __forceinline__ uint32_t bound_wbox_tagged(const G& g, f3 o, f3 r, float rlt, uint32_t i) {
    const v2f tx = ((v2f){g.wbox[0], g.wbox[1]} - (v2f){o.x, o.x}) * (v2f){r.x, r.x};
    const v2f ty = ((v2f){g.wbox[2], g.wbox[3]} - (v2f){o.y, o.y}) * (v2f){r.y, r.y};
    const v2f tz = ((v2f){g.wbox[4], g.wbox[5]} - (v2f){o.z, o.z}) * (v2f){r.z, r.z};
    const float E0 = fmaxf(fmaxf(fminf(tx.x, tx.y), fminf(ty.x, ty.y)), fmaxf(fminf(tz.x, tz.y), 0.0f));
    const float X = fminf(fminf(fmaxf(tx.x, tx.y), fmaxf(ty.x, ty.y)), fmaxf(tz.x, tz.y));
    // one fma instead of a product and a difference: a single rounding, so no less a lower bound
    // (tslack's 2^-14 and abs_slack cover both forms).  No clamp at 0: a negative v is a negative
    // int, which tag_bound's integer max turns into the tag of +0, as the clamp did.  (v is never
    // NaN: E0 is a maxNum chain that includes 0, rlt is finite and positive, wback is finite.)
    const float v = fmaf(E0, rlt, -g.wback);
    // a miss ORs in the exponent of +inf: the result is then >= +inf's bits (no candidate) with no
    // branch around the tag, so the geom loop's scalar loads are not split by one
    return tag_bound(v, i) | (E0 > X ? 0x7f800000u : 0u);
}

// The median of three unsigned ints in one v_med3_u32 (the compiler keeps min(c, max(a, b)) as two
// operations even when a <= c is known).
__device__ __forceinline__ uint32_t umed3(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// A bound v >= 0 (or +0 / -0; a negative v counts as +0) with geom index i in its low 5 bits, as
// the bits of a float that is <= v: max(bits, 32) - 32 (as signed ints) with the low 5 bits
// replaced by i (at most 32 ulp below v; +-0 become the denormal i * 2^-149, which is below every
// later comparison's rounding: the scene's absolute slack is subtracted before any use, and
// fl(tag - slack) = fl(0 - slack)).  Non-negative floats order as their bits, so the pass keeps the
// three smallest with integer min / median operations, and the index of a candidate is its low
// bits.  Bits >= +inf's (+inf, or a miss's tag with the exponent ORed in: a NaN pattern, which
// every later comparison rejects) mean no candidate.
__device__ __forceinline__ uint32_t tag_bound(float v, uint32_t i) {
    const uint32_t b = (uint32_t)(max((int32_t)__float_as_uint(v), 32) - 32);
    return (b & ~31u) | i;
}

// Lower bound on the exact test's world distance for geom g (before the scene's absolute slack),
// +inf when the exact test surely misses.  Rounding here is irrelevant: only the widened bounds,
// the relative slack and the comparisons' direction matter (NaNs fall through to "candidate").
// SEL: selects instead of early returns (same value): no branch between one geom's scalar loads and
// the next's — faster for the divergent rays of later bounces, slower for camera rays.
template <int KIND, bool SEL, class G>
__device__ __forceinline__ float bound_geom(const G& g, f3 ro, f3 rd, f3 invd, float rl, float rinf) {
    constexpr int kind = KIND;
    if (kind == 3) {   // world box: t = (plane - o) / d (subtract first: exact zeros in d stay safe)
        float E = -kInf, X = kInf;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float t1 = (g.wlo[k] - at(ro, k)) * at(invd, k), t2 = (g.whi[k] - at(ro, k)) * at(invd, k);
            E = fmaxf(E, fminf(t1, t2));
            X = fminf(X, fmaxf(t1, t2));
        }
        if (!SEL && (E > X || X < 0.0f)) return kInf;
        const float v = fmaxf(fmaxf(E, 0.0f) * rl - g.back, 0.0f) * g.tslack;
        return (E > X || X < 0.0f) ? kInf : v;
    }
    if (kind == 0) return kInf;
    float a, b, q2, lo;
    bool miss;
    f3 qo, qv;
    if (kind == 4) {
        // sphere whose transform is a uniform scale (any rotation): the object-space dot products
        // are rotation invariant, so they come from world space: w = ro - centre, scaled by
        // is2 = |inv v|^2 / |v|^2 (wlo = centre, whi[0] = is2; wider margins, update_bounds)
        const f3 w = F3(ro.x - g.wlo[0], ro.y - g.wlo[1], ro.z - g.wlo[2]);
        a = dot(rd, rd) * g.whi[0];
        b = dot(w, rd) * g.whi[0];
        q2 = dot(w, w) * g.whi[0];
    } else {
        qo = xform_point(g.inv, ro);
        qv = xform_vector(g.inv, rd);   // un-normalized: world parameter = object parameter
        a = dot(qv, qv);
        if (kind == 2) {
            b = dot(qo, qv);
            q2 = dot(qo, qo);
        }
    }
    if (kind == 1) {
        float E = -kInf, X = kInf;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float r = __builtin_amdgcn_rcpf(at(qv, k));
            const float t1 = (g.slo[k] - at(qo, k)) * r, t2 = (g.shi[k] - at(qo, k)) * r;
            E = fmaxf(E, fminf(t1, t2));
            X = fminf(X, fmaxf(t1, t2));
        }
        miss = E > X || X < 0.0f;
        if (!SEL && miss) return kInf;
        lo = fmaxf(E, 0.0f);
    } else {
        const bool departing = b > 0.0f && q2 - 0.25f > (q2 + 1.0f) * (g.kcs * rinf + g.kc3);
        if (!SEL && departing) return kInf;
        const float disc = b * b - a * (q2 - g.r2w);
        if (!SEL && disc < 0.0f) return kInf;
        const float sq = __builtin_amdgcn_sqrtf(disc), ia = __builtin_amdgcn_rcpf(a);
        const float eps = (fabsf(b) + sq) * ia * 0x1p-16f;
        miss = departing || disc < 0.0f || (sq - b) * ia < -eps;
        if (!SEL && miss) return kInf;
        lo = fmaxf((-b - sq) * ia - eps, 0.0f);
    }
    // pointOnRay pulls the hit back by 1e-4 along the NORMALIZED object direction: 1e-4/|qv| here
    const float back = 1.0002e-4f * __builtin_amdgcn_rsqf(a);
    const float v = fmaxf(lo - back, 0.0f) * rl * g.tslack;
    return miss ? kInf : v;
}

// Uniformly scaled spheres (bkind 4) for the select-based pass, returned TAGGED like the world-box
// cubes: bound_geom<4>'s bound with the per-geom transcendentals replaced by per-ray ones and host
// constants — ia = rcp(|d|^2) * (1 / is2) (whi[1]) and the pull-back 1.0002e-4 / sqrt(|d|^2 is2) as
// back (1.0002e-4 / sqrt(is2), rounded up) * rsq(|d|^2): a few ulp from the per-geom forms, inside
// eps (2^-16 relative), the pull-back's 2e-4 margin and tslack — and no clamps at 0 (a negative
// bound is tag_bound's +0; when the sphere is not missed, every term is finite or the bound is -inf).
template <class G>
__device__ __forceinline__ uint32_t bound_sphere_tagged(const G& g, f3 ro, f3 rd, float dd, float rl, float rinf,
                                                       float rdd, float rsdd, uint32_t i) {
    const f3 w = F3(ro.x - g.wlo[0], ro.y - g.wlo[1], ro.z - g.wlo[2]);
    const float a = dd * g.whi[0];
    const float b = dot(w, rd) * g.whi[0];
    const float q2 = dot(w, w) * g.whi[0];
    const bool departing = b > 0.0f && q2 - 0.25f > (q2 + 1.0f) * (g.kcs * rinf + g.kc3);
    const float disc = b * b - a * (q2 - g.r2w);
    const float sq = __builtin_amdgcn_sqrtf(disc), ia = rdd * g.whi[1];
    const float eps = (fabsf(b) + sq) * ia * 0x1p-16f;
    const bool miss = departing || disc < 0.0f || (sq - b) * ia < -eps;
    const float v = (((-b - sq) * ia - eps) - g.back * rsdd) * rl * g.tslack;
    return miss ? 0x7f800000u : tag_bound(v, i);
}

// Oriented cubes (bkind 1) for the select-based pass, returned TAGGED: bound_geom<1>'s slabs, with the
// pull-back bounded per geom instead of per ray — back (update_bounds: 1.0002e-4 * ||inverse of the
// linear part||_F, rounded up) * rsq(|d|^2) >= 1.0002e-4 / |qv| — so no |qv|^2 and no rsq per cube, and
// no clamps at 0 (a negative bound is tag_bound's +0).
template <class G>
__device__ __forceinline__ uint32_t bound_obox_tagged(const G& g, f3 ro, f3 rd, float rl, float rsdd, uint32_t i) {
    const f3 qo = xform_point(g.inv, ro);
    const f3 qv = xform_vector(g.inv, rd);   // un-normalized: world parameter = object parameter
    float E = -kInf, X = kInf;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float r = __builtin_amdgcn_rcpf(at(qv, k));
        const float t1 = (g.slo[k] - at(qo, k)) * r, t2 = (g.shi[k] - at(qo, k)) * r;
        E = fmaxf(E, fminf(t1, t2));
        X = fminf(X, fmaxf(t1, t2));
    }
    const bool miss = E > X || X < 0.0f;
    const float v = (E - g.back * rsdd) * rl * g.tslack;
    return miss ? 0x7f800000u : tag_bound(v, i);
}

// Exact test of one geom from its LDS row: boxIntersectionTest (intersections.cu:3-58) and
// sphereIntersectionTest (:60-115) with their common prologue (object-space ray) and epilogue
// (pointOnRay, back-transform, world length) shared, so a wave whose lanes test different geom
// types runs only the type-specific middle twice.  Same operations, same order: bit-identical.
__device__ __forceinline__ float exact_geom(const LGeom& L, f3 r_o, f3 r_d, int& code, f3& obj, bool& outside) {
    code = -1;
    outside = true;
    const int type = L.type;
    if (type != PT_GEOM_CUBE && type != PT_GEOM_SPHERE) return -1.0f;
    const f3 qo = xform_point(L.inv, r_o);
    const f3 qd = normalize(xform_vector(L.inv, r_d));
    float t;
    bool hit;
    if (type == PT_GEOM_CUBE) {
        float tmin = -1e38f, tmax = 1e38f;
        int nmin = -1, nmax = -1;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float qa = at(qd, a), oa = at(qo, a);
            float t1, t2;
            div2_cr(-0.5f - oa, +0.5f - oa, qa, t1, t2);
            const float ta = gmin(t1, t2), tb = gmax(t1, t2);
            const int c = 2 * a + (t2 < t1 ? 0 : 1);
            if (ta > 0 && ta > tmin) { tmin = ta; nmin = c; }
            if (tb < tmax) { tmax = tb; nmax = c; }
        }
        hit = tmax >= tmin && tmax > 0;
        if (tmin <= 0) { tmin = tmax; nmin = nmax; }
        t = tmin;
        code = nmin;
    } else {
        const float vdd = dot(qo, qd);
        const float radicand = vdd * vdd - (dot(qo, qo) - 0.25f);
        const float sq = sqrt_cr(radicand);
        const float t1 = -vdd + sq, t2 = -vdd - sq;
        hit = !(radicand < 0) && !(t1 < 0 && t2 < 0);
        if (t1 > 0 && t2 > 0) { t = gmin(t1, t2); outside = true; }
        else { t = gmax(t1, t2); outside = false; }
    }
    if (!hit) return -1.0f;
    obj = point_on_ray(qo, qd, t);
    const f3 ip = xform_point(L.xf, obj);
    return length(r_o - ip);
}

// PRE: scenes with meshes whose BVH closest hit `mh` came from k_traverse.  The owning mesh geom
// (the first in index order whose triangle range holds the hit, intersect_scene's rule) enters as an
// exactly evaluated hit before the exact tests; mesh geoms have no bound (bkind 0).
// gmask (wave-uniform): geoms outside it cannot be hit by this wave's rays (the first bounce's
// camera-ray masks, pt_ctx::cmask) and are skipped; a geom no ray can hit is never a candidate
// whose absence changes the result (every geom that can be hit is still bounded and tested).
__device__ __forceinline__ uint32_t ng_all_mask(int n) { return n >= 32 ? ~0u : (1u << n) - 1u; }
#if defined(PT_DUP)
__device__ uint32_t g_dup_sink;
#endif
template <bool SEL, bool PRE = false>
__device__ __forceinline__ Hit intersect_bounded(const SceneDev& S, const FlagsDev& fl, const LGeom* s_geoms, f3 ro,
                                                 f3 rd, const MeshHit* mh = nullptr, uint32_t gmask = ~0u) {
    const float rl = __builtin_amdgcn_sqrtf(dot(rd, rd));
    bool plain = !(rl > 0.5f && rl < 2.0f);   // NaN / degenerate direction: the plain loop
    float t_min = kFLT_MAX;
    int hit_geom = -1, best_code = -1;
    f3 best_obj = F3(0, 0, 0);
    bool best_outside = true;
    int mesh_geom = -1;
    // A NaN direction (glm::refract under total internal reflection, interactions.cu:70) makes
    // every exact test return NaN (box: the NaN slabs leave tmin/tmax at -/+1e38, the hit point is
    // NaN; sphere: NaN radicand passes, NaN t) and `t > 0` rejects it: no hit, without the plain
    // loop over every geom that such a lane would otherwise cost its whole wave.
    if (rd.x != rd.x || rd.y != rd.y || rd.z != rd.z) {
        if (!PRE || !mh->any) {
            Hit h;
            h.t = -1.0f;
            h.mat = 0;
            h.n = F3(0, 0, 0);
            h.u = h.v = 0.f;
            return h;
        }
    }
    if (PRE && mh->any) {
        const auto* G = as_const(S.geoms);
        for (int i = 0; i < S.ngeoms; ++i)
            if (G[i].type == PT_GEOM_MESH && mh->id >= G[i].tri_start && mh->id < G[i].tri_end) { mesh_geom = i; break; }
        if (mesh_geom >= 0 && mh->t > 0.0f) { t_min = mh->t; hit_geom = mesh_geom; }
    }
    float lo1 = kInf, lo2 = kInf, lo3 = kInf;
    int g1 = -1, g2 = -1;
    uint32_t rest = 0u;   // geoms tested after the candidates regardless of bounds
    // A wave whose rays can hit only one geom (the first bounce's camera-ray mask, wave-uniform): that
    // geom's exact test is the closest hit — the bounds pass would make it the only candidate.
    const uint32_t gone = gmask & ng_all_mask(S.ngeoms);
    const bool one = !PRE && !plain && gone != 0u && (gone & (gone - 1u)) == 0u;
    if (one) {
        g1 = __builtin_ctz(gone);
    } else if (!plain) {
        // pass 1: the three smallest lower bounds (scene data wave-uniform: scalar loads)
        const float rinf = fmaxf(fmaxf(fabsf(ro.x), fabsf(ro.y)), fabsf(ro.z));
        const f3 invd = F3(__builtin_amdgcn_rcpf(rd.x), __builtin_amdgcn_rcpf(rd.y), __builtin_amdgcn_rcpf(rd.z));
        // one branch-free loop per bound kind (geoms sorted by kind on the host), so the scalar
        // loads of the next geom need not wait for this one's kind; the candidates' identity and
        // order do not matter to the result (pass 2 below), only the set of bounds
        const auto* B = as_const(S.bgeoms);
        // the three smallest bounds, as tagged bits (tag_bound): u1 <= u2 <= u3, the geoms of the first
        // two in their low bits.  The scene's absolute slack is subtracted from the three after the pass:
        // x - c rounds monotonically, so they are the three smallest slackened bounds; a tie that the
        // subtraction (or the tag) creates between two geoms only swaps which one pass 2 tests first —
        // both are tested (the first hit's t is >= the tied bound), and the selection is order-independent.
        uint32_t u1 = 0x7f800000u, u2 = 0x7f800000u, u3 = 0x7f800000u;
        auto insert_tagged = [&](uint32_t t) {   // (medians: u1 <= u2 <= u3)
            u3 = umed3(u2, t, u3);
            u2 = umed3(u1, t, u2);
            u1 = min(u1, t);
        };
        auto insert = [&](float lo, int i) { insert_tagged(lo == kInf ? 0x7f800000u : tag_bound(lo, (uint32_t)i)); };
        const float rlt = rl * S.wb_tslack;
        for (int j = S.bk[3]; j < S.bk[4]; ++j)   // world-box cubes: packed slabs
            if ((gmask >> B[j].orig) & 1u) insert_tagged(bound_wbox_tagged(B[j], ro, invd, rlt, (uint32_t)B[j].orig));
        if (SEL) {
            const bool spheres = S.bk[4] < S.bk[5], oboxes = S.bk[1] < S.bk[2];
            if (spheres || oboxes) {   // per-ray reciprocals (bound_sphere_tagged, bound_obox_tagged)
                const float dd = dot(rd, rd), rdd = __builtin_amdgcn_rcpf(dd), rsdd = __builtin_amdgcn_rsqf(dd);
                for (int j = S.bk[4]; j < S.bk[5]; ++j)
                    if ((gmask >> B[j].orig) & 1u)
                        insert_tagged(bound_sphere_tagged(B[j], ro, rd, dd, rl, rinf, rdd, rsdd, (uint32_t)B[j].orig));
                for (int j = S.bk[1]; j < S.bk[2]; ++j)
                    if ((gmask >> B[j].orig) & 1u)
                        insert_tagged(bound_obox_tagged(B[j], ro, rd, rl, rsdd, (uint32_t)B[j].orig));
            }
        } else {
            for (int j = S.bk[4]; j < S.bk[5]; ++j)
                if ((gmask >> B[j].orig) & 1u) insert(bound_geom<4, SEL>(B[j], ro, rd, invd, rl, rinf), B[j].orig);
            for (int j = S.bk[1]; j < S.bk[2]; ++j)
                if ((gmask >> B[j].orig) & 1u) insert(bound_geom<1, SEL>(B[j], ro, rd, invd, rl, rinf), B[j].orig);
        }
        for (int j = S.bk[2]; j < S.bk[3]; ++j)
            if ((gmask >> B[j].orig) & 1u) insert(bound_geom<2, SEL>(B[j], ro, rd, invd, rl, rinf), B[j].orig);
        g1 = u1 >= 0x7f800000u ? -1 : (int)(u1 & 31u);
        g2 = u2 >= 0x7f800000u ? -1 : (int)(u2 & 31u);
        lo1 = __uint_as_float(u1) - S.abs_slack;
        lo2 = __uint_as_float(u2) - S.abs_slack;
        lo3 = __uint_as_float(u3) - S.abs_slack;
#if defined(PT_DUP) && PT_DUP == 4   // diagnostic: the bounds pass again on an opaque origin
        if (SEL) {
            f3 r2 = ro;
            asm volatile("" : "+v"(r2.x), "+v"(r2.y), "+v"(r2.z));
            float m1 = kInf, m2 = kInf, m3 = kInf;
            int h1 = -1;
            auto ins2 = [&](float lo, int i) {
                lo -= S.abs_slack;
                const bool c1 = lo < m1, c2 = lo < m2, c3 = lo < m3;
                m3 = c2 ? m2 : (c3 ? lo : m3);
                m2 = c1 ? m1 : (c2 ? lo : m2);
                m1 = c1 ? lo : m1;
                h1 = c1 ? i : h1;
            };
            for (int j = S.bk[3]; j < S.bk[4]; ++j)
                if ((gmask >> B[j].orig) & 1u) ins2(bound_geom<3, SEL>(B[j], r2, rd, invd, rl, rinf), B[j].orig);
            for (int j = S.bk[4]; j < S.bk[5]; ++j)
                if ((gmask >> B[j].orig) & 1u) ins2(bound_geom<4, SEL>(B[j], r2, rd, invd, rl, rinf), B[j].orig);
            for (int j = S.bk[1]; j < S.bk[2]; ++j)
                if ((gmask >> B[j].orig) & 1u) ins2(bound_geom<1, SEL>(B[j], r2, rd, invd, rl, rinf), B[j].orig);
            for (int j = S.bk[2]; j < S.bk[3]; ++j)
                if ((gmask >> B[j].orig) & 1u) ins2(bound_geom<2, SEL>(B[j], r2, rd, invd, rl, rinf), B[j].orig);
            if (__float_as_uint(m1 + m2 + m3) == 0x7f7ffffeu || h1 == 12345) atomicAdd(&g_dup_sink, 1u);
        }
#endif
#if defined(PT_DUP) && PT_DUP == 5   // diagnostic: the first candidate's exact test again
        if (SEL && g1 >= 0) {
            f3 r2 = ro;
            asm volatile("" : "+v"(r2.x), "+v"(r2.y), "+v"(r2.z));
            int code2;
            f3 obj2 = F3(0, 0, 0);
            bool out2;
            const float t2 = exact_geom(s_geoms[g1], r2, rd, code2, obj2, out2);
            if (__float_as_uint(t2) == 0x7f7ffffeu) atomicAdd(&g_dup_sink, 1u);
        }
#endif
    } else if (!PRE) {
        rest = ng_all_mask(S.ngeoms);   // a direction the bounds do not cover: the reference's loop over every geom
    }
    if (PRE && plain) return intersect_scene<PRE, PRE>(S, fl, ro, rd, mh);
    {   // pass 2, one loop over the candidates (so the kernels carry one inlined exact test): the first;
        // the second while its bound does not exceed the best hit; then, if the third-smallest bound does
        // not, every other geom the wave may hit (one with no finite bound misses exactly, so testing it
        // changes nothing; rare: 0 rays on Cornell and config 4).  The selection is order-independent
        // (minimum t, lowest index on ties).
        auto take = [&](int gi) {
            int code;
            f3 obj = F3(0, 0, 0);
            bool outside;
            const float t = exact_geom(s_geoms[gi], ro, rd, code, obj, outside);
            if (t > 0.0f && (t_min > t || (t == t_min && hit_geom >= 0 && gi < hit_geom))) {
                t_min = t; hit_geom = gi; best_code = code; best_obj = obj; best_outside = outside;
            }
        };
        int gi = g1;
        int stage = (one || plain) ? 2 : 0;
        uint32_t m = rest;
        for (;;) {
            if (gi >= 0) take(gi);
            if (stage == 0) {
                stage = 1;
                if (g2 >= 0 && lo2 <= t_min) { gi = g2; continue; }
            }
            if (stage == 1) {
                stage = 2;
                m = lo3 <= t_min ? (ng_all_mask(S.ngeoms) & gmask) & ~(1u << g1) & ~(1u << g2) : 0u;
            }
            if (m == 0u) break;
            gi = __builtin_ctz(m);
            m &= m - 1u;
        }
    }

    Hit h;
    if (hit_geom < 0) {
        h.t = -1.0f;
        h.mat = 0;
        h.n = F3(0, 0, 0);
        h.u = h.v = 0.f;
        return h;
    }
    const LGeom& g = s_geoms[hit_geom];
    h.t = t_min;
    h.mat = g.material;
    h.u = h.v = 0.f;
    if (PRE && hit_geom == mesh_geom) tri_attrs(S.attrs[mh->idx], mh->bx, mh->by, h.n, h.u, h.v);
    else h.n = g.type == PT_GEOM_CUBE ? box_normal(g, best_code) : sphere_normal(g, best_obj, best_outside);
    if (g.type == PT_GEOM_CUBE && best_code >= 0) h.frame = hit_geom * 6 + best_code;
    return h;
}

// The closest hit of the kernels: bounded for analytic scenes that fit the LDS geom table.
// CHECK: compiled-in diagnostic re-run (k_trace and the sorted pipeline only, so the fused
// kernel's code stays small): verify with PT_PIPELINE=split, whose rays are the fused kernel's.
// LDSG: the launch guarantees ngeoms <= kLdsGeoms (the geom table is in LDS), so the plain loop over a
// larger table is not compiled in.
template <bool MESH, bool CHECK, bool SEL = false, bool LDSG = false>
__device__ __forceinline__ Hit closest_hit(const SceneDev& S, const FlagsDev& fl, const LGeom* s_geoms, f3 ro, f3 rd,
                                           uint32_t* mismatch, uint32_t gmask = ~0u) {
    if (MESH || (!LDSG && S.ngeoms > kLdsGeoms)) return intersect_scene<MESH>(S, fl, ro, rd);
    const Hit h = intersect_bounded<SEL>(S, fl, s_geoms, ro, rd, nullptr, gmask);
    if (CHECK && fl.verify) {
        const Hit r = intersect_scene<false>(S, fl, ro, rd);
        if (__float_as_uint(h.t) != __float_as_uint(r.t) || h.mat != r.mat ||
            __float_as_uint(h.n.x) != __float_as_uint(r.n.x) || __float_as_uint(h.n.y) != __float_as_uint(r.n.y) ||
            __float_as_uint(h.n.z) != __float_as_uint(r.n.z))
            atomicAdd(mismatch, 1u);
    }
    return h;
}

// ------------------------------------------------------------------------------------------
// Shading (shadeMaterials pathtrace.cu:300-344, scatterRay interactions.cu:43-85)
// ------------------------------------------------------------------------------------------
struct PathReg {
    f3 o, d, c;
    int32_t slot, bounces;
};

__device__ __forceinline__ f3 tex_color(const DTexture& tx, float u, float v) {   // sceneStructs.h:176-189
    int X = (int)gmin(1.f * tx.width * u, 1.f * tx.width - 1.0f);
    int Y = (int)gmin(1.f * tx.height * (1.0f - v), 1.f * tx.height - 1.0f);
    X = X < 0 ? 0 : X;
    Y = Y < 0 ? 0 : Y;
    const int id = Y * tx.width + X;
    if (tx.components == 3) {
        const uint8_t* p = tx.data + 3 * (size_t)id;
        return 0.003921568627f * F3((float)p[0], (float)p[1], (float)p[2]);
    }
    return F3(0, 0, 0);
}

__device__ __forceinline__ f3 hemisphere(f3 n, Rng& rng, const float* frame = nullptr) {   // interactions.cu:3-41
    const float up = sqrt_cr(rng.u01());
    const float over = sqrt_cr(1 - up * up);
    const float around = rng.u01() * kTWO_PI;
    f3 p1, p2;
    if (frame) {   // a cube's face: the frame of its normal, precomputed (DGeom::frm)
        p1 = F3(frame[0], frame[1], frame[2]);
        p2 = F3(frame[3], frame[4], frame[5]);
    } else {
        f3 dnn;
        if (fabsf(n.x) < kSQRT_1_3) dnn = F3(1, 0, 0);
        else if (fabsf(n.y) < kSQRT_1_3) dnn = F3(0, 1, 0);
        else dnn = F3(0, 0, 1);
        p1 = normalize(cross(n, dnn));
        p2 = normalize(cross(n, p1));
    }
    float sa, ca;
    sincos_c(around, &sa, &ca);
    return (up * n + (ca * over) * p1) + (sa * over) * p2;
}

__device__ __forceinline__ f3 reflect(f3 I, f3 N) { return I - hadamard(N * dot(N, I), F3(2, 2, 2)); }
__device__ __forceinline__ f3 refract(f3 I, f3 N, float eta) {   // glm 0.9.6.3: NaN when k < 0
    const float dv = dot(N, I);
    const float k = 1.0f - eta * eta * (1.0f - dv * dv);
    return (eta * I - (eta * dv + sqrt_cr(k)) * N) * (float)(k >= 0.0f);
}

// Global pixel index of tile slot `slot` (the raygen mapping below): the shading RNG key under
// pt_flags.rng_key_pixel, independent of compaction order and of the shard layout.
__device__ __forceinline__ int slot_pixel(const CamDev& cam, const TileDev& T, int slot) {
    const int lp = slot % T.npix;
    const int row = lp / T.W;
    return (lp - row * T.W) + (row * T.world + T.rank) * cam.res[0];
}

// shade()'s two exits that draw no random numbers (pathtrace.cu:318-330): a miss (colour 0) and an
// emissive hit (colour x material colour x emittance).  True if the path ends there; p.c is then
// its final colour.  The sorted pipeline takes these exits one launch early (k_sort_produce).
template <class MT>
__device__ __forceinline__ bool shade_ends(const Hit& h, const MT* mats, PathReg& p) {
    if (h.t <= 0.0f) { p.c = F3(0, 0, 0); return true; }
    const MT& m = mats[h.mat];
    if (m.emittance > 0.0f) {
        p.c = hadamard(p.c, F3(m.color[0], m.color[1], m.color[2]) * m.emittance);
        return true;
    }
    return false;
}

// Does shade() read the incoming direction for this material (a refractive one, or one that may
// reflect: `rng.u01() < has_reflective` can hold)?  A diffuse bounce only needs the normal.
template <class MT>
__device__ __forceinline__ bool mat_needs_dir(const MT& m) {
    return m.has_refractive != 0.0f || m.has_reflective > 0.0f;
}

// shade() past its two early exits, from the hit point (getPointOnRay, pathtrace.cu:323): the
// material-sorted pipeline stores the hit point instead of the ray's origin and length.
// `frames`: the staged tangent frames of the scene's cubes (LDS, [geom * 6 + code][6]) or null.
template <class MT>
__device__ __forceinline__ bool shade_from(const SceneDev& S, const FlagsDev& fl, int depth, int iter, int idx,
                                           PathReg& p, const Hit& h, f3 hitp, const MT* mats,
                                           const float* frames = nullptr) {
    int remaining = depth - p.bounces;
    Rng rng(iter, idx, remaining);
    const MT& m = mats[h.mat];
    const f3 mcol = F3(m.color[0], m.color[1], m.color[2]);
    const f3 n = h.n;
    p.o = hitp + 0.0001f * n;
    const f3 alb = m.texture_id != -1 ? tex_color(S.texs[m.texture_id], h.u, h.v) : mcol;
    p.c = hadamard(p.c, alb);
    const f3 scol = F3(m.spec_color[0], m.spec_color[1], m.spec_color[2]);
    if (m.has_refractive != 0.0f) {
        const float eta = m.ior;
        const float R0 = ((eta - 1) * (eta - 1)) / ((eta + 1) * (eta + 1));
        const float X = 1 - fabsf(dot(p.d, n));
        const float X2 = X * X;
        const float R = R0 + (1 - R0) * ((X * X2) * X2);
        if (R < rng.u01()) { p.d = refract(p.d, n, eta); p.c = hadamard(p.c, mcol); }
        else { p.d = reflect(p.d, n); p.c = hadamard(p.c, scol); }
    } else if (rng.u01() < m.has_reflective) {
        p.d = reflect(p.d, n);
        p.c = hadamard(p.c, scol);
    } else {
        p.d = hemisphere(n, rng, frames && h.frame >= 0 ? frames + 6 * h.frame : nullptr);
    }
    if (!fl.single_albedo) p.c = hadamard(p.c, mcol);   // interactions.cu:83 (second albedo)
    p.bounces += 1;
    remaining -= 1;
    if (remaining == 0) { p.c = F3(0, 0, 0); return false; }
    if (fl.rr && p.bounces > 3) {
        const f3 luma = F3((float)0.2126, (float)0.7152, (float)0.0722);
        const float l = dot(p.c, luma);
        const float q = gmax(0.05f, 1 - l);
        if (rng.u01() < q) { p.c = F3(0, 0, 0); return false; }
        const float dq = 1.0f - q;   // three divisions by one divisor: its reciprocal step shared
        const float rq = recip_core(dq);
        f3 cq = F3(div_core(p.c.x, dq, rq), div_core(p.c.y, dq, rq), div_core(p.c.z, dq, rq));
        if (__builtin_expect(!(div_ok(dq) && div_ok(p.c.x) && div_ok(p.c.y) && div_ok(p.c.z)), 0)) cq = p.c / dq;
        p.c = cq;
    }
    return true;
}

// Returns true if the path survives.  `idx` is the path's position in the (compacted, possibly
// material-sorted) array — the RNG key of the reference (pathtrace.cu:315).
template <class MT>
__device__ __forceinline__ bool shade(const SceneDev& S, const FlagsDev& fl, int depth, int iter, int idx,
                                      PathReg& p, const Hit& h, const MT* mats, const float* frames = nullptr) {
    if (shade_ends(h, mats, p)) return false;
    return shade_from(S, fl, depth, iter, idx, p, h, point_on_ray(p.o, p.d, h.t), mats, frames);
}

// generateRayFromCamera (pathtrace.cu:183-227) for tile slot `slot`.
// Path `slot` = iteration s of the pass, tile-local pixel lp.
__device__ __forceinline__ void raygen_at(const CamDev& cam, const FlagsDev& fl, const TileDev& T, int slot, int s, int lp,
                                          PathReg& p) {
    const int row = T.wdiv ? (int)(((uint64_t)(uint32_t)lp * T.wdiv) >> 40) : lp / T.W;
    const int x = lp - row * T.W;
    const int y = row * T.world + T.rank;
    const int index = x + y * cam.res[0];
    p.o = F3(cam.pos[0], cam.pos[1], cam.pos[2]);
    p.c = F3(1.0f, 1.0f, 1.0f);
    Rng rng(T.iter_first + s, index, T.depth);
    float ax = (float)x - (float)cam.res[0] * 0.5f;
    float ay = (float)y - (float)cam.res[1] * 0.5f;
    if (fl.ssaa) {
        ax = ax + rng.u01();
        ay = ay + rng.u01();
    }
    const f3 view = F3(cam.view[0], cam.view[1], cam.view[2]);
    const f3 right = F3(cam.right[0], cam.right[1], cam.right[2]);
    const f3 up = F3(cam.up[0], cam.up[1], cam.up[2]);
    p.d = normalize((view - (right * cam.pl[0]) * ax) - (up * cam.pl[1]) * ay);
    if (fl.dof) {
        const float r = rng.u01() * fl.aperture;
        const float th = (rng.u01() * 2) * kPI;
        float sth, cth;
        sincos_c(th, &sth, &cth);
        const f3 lens = F3(r * cth, r * sth, 0.0f);
        const float ft = fl.focal / fabsf(p.d.z);
        const f3 focus = p.o + ft * p.d;
        p.o = p.o + lens;
        p.d = normalize(focus - p.o);
    }
    p.slot = slot;
    p.bounces = 0;
}
__device__ __forceinline__ void raygen(const CamDev& cam, const FlagsDev& fl, const TileDev& T, int slot, PathReg& p) {
    const int s = slot / T.npix;
    raygen_at(cam, fl, T, slot, s, slot - s * T.npix, p);
}

// Path planes stream through HBM once per bounce (GBs per lane, far beyond the Infinity Cache):
// non-temporal loads and stores.
#define PT_LD(p) __builtin_nontemporal_load(p)
#define PT_ST(v, p) __builtin_nontemporal_store((v), (p))
__device__ __forceinline__ void load_path(const PathSoA& B, int i, int bounce, PathReg& p) {
    const v4f a = PT_LD(B.a + i), b = PT_LD(B.b + i);
    const v2f c = PT_LD(B.c + i);
    p.o = F3(a[0], a[1], a[2]);
    p.d = F3(a[3], b[0], b[1]);
    p.c = F3(b[2], b[3], c[0]);
    p.slot = __float_as_int(c[1]);
    p.bounces = bounce;
}
__device__ __forceinline__ void store_path(const PathSoA& B, int i, const PathReg& p) {
    PT_ST((v4f{p.o.x, p.o.y, p.o.z, p.d.x}), B.a + i);
    PT_ST((v4f{p.d.y, p.d.z, p.c.x, p.c.y}), B.b + i);
    PT_ST((v2f{p.c.z, __int_as_float(p.slot)}), B.c + i);
}

// A path that terminated this bounce: its colour is final (finalGather, pathtrace.cu:347-356).
template <bool SPP1>
__device__ __forceinline__ void retire(const KArgs& A, const PathReg& p, int it = -1) {
    if (SPP1) {
        if (p.c.x != 0.0f || p.c.y != 0.0f || p.c.z != 0.0f) {
            float* px = A.image + 3 * (size_t)p.slot;
            px[0] += p.c.x;
            px[1] += p.c.y;
            px[2] += p.c.z;
        }
    } else if (p.c.x != 0.0f || p.c.y != 0.0f || p.c.z != 0.0f) {
        // only nonzero colours are stored (~4% of Cornell's paths: the others miss the light), and
        // flagged in the pass's pixel-major flag row; an unflagged slot is a zero colour (k_finalize_spp)
        // (scattered: plain, so L2 can merge neighbours)
        A.colbuf[p.slot] = v4f{p.c.x, p.c.y, p.c.z, 0.0f};
        // slot = it * npix + pixel within the lane: `it` is the caller's (its workgroup's or tile's
        // iteration, uniform) or, when not known (< 0), derived from the slot
        const int npix = A.tile.npix;
        if (it < 0) {
            it = (int)((float)p.slot * A.inv_npix);
            if (p.slot - it * npix < 0) --it;
            else if (p.slot - it * npix >= npix) ++it;
        }
        const int lp = p.slot - it * npix;
        A.colflag[(size_t)lp * (size_t)A.col_spp + (size_t)(A.col_off + it)] = 1;
    }
}

// The material table is tiny and read at a per-lane (divergent) index by every shaded path:
// staged once per workgroup in LDS so each lookup is a ds_read, not a dependent global round
// trip (measured: bounce 1 of Cornell 120 us -> 41 us with coherent material reads).
constexpr int kLdsMats = 128;
__device__ __forceinline__ void stage_materials(const KArgs& A, DMaterial* s_mats) {
    const int n = A.S.nmats < kLdsMats ? A.S.nmats : kLdsMats;
    const int words = n * (int)(sizeof(DMaterial) / 4);
    const uint32_t* src = reinterpret_cast<const uint32_t*>(A.S.mats);
    uint32_t* dst = reinterpret_cast<uint32_t*>(s_mats);
    for (int j = threadIdx.x; j < words; j += blockDim.x) dst[j] = src[j];
    __syncthreads();
}

// Emissive terminations are counted per wave in a register, reduced per workgroup in LDS and
// added to the workgroup's OWN counter slot with a plain read-modify-write (each blockIdx is
// unique within a launch; launches on a stream are ordered).  No same-address atomics: ~16k of
// them per bounce serialised at the memory-side atomic unit (measured: 120 us -> 41 us).
__device__ __forceinline__ void flush_emissive(const KArgs& A, uint32_t cnt, uint32_t* s_cnt) {
    if (threadIdx.x == 0) *s_cnt = 0u;
    __syncthreads();
    if (cnt && (threadIdx.x & 63) == 0) atomicAdd(s_cnt, cnt);
    __syncthreads();
    if (threadIdx.x == 0 && *s_cnt) {
        unsigned long long* slot = A.emit_slots + (size_t)A.bounce * A.emit_stride + blockIdx.x;
        *slot += *s_cnt;
    }
}

// Two counters: emissions of this launch's bounce and of bounce `b2` (the sorted producer retires
// the emissive hits of the next bounce, k_sort_produce).
__device__ __forceinline__ void flush_emissive2(const KArgs& A, uint32_t cnt, int b2, uint32_t cnt2, uint32_t* s_cnt) {
    if (threadIdx.x == 0) { s_cnt[0] = 0u; s_cnt[1] = 0u; }
    __syncthreads();
    if ((threadIdx.x & 63) == 0) {
        if (cnt) atomicAdd(&s_cnt[0], cnt);
        if (cnt2) atomicAdd(&s_cnt[1], cnt2);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_cnt[0]) A.emit_slots[(size_t)A.bounce * A.emit_stride + blockIdx.x] += s_cnt[0];
        if (s_cnt[1]) A.emit_slots[(size_t)b2 * A.emit_stride + blockIdx.x] += s_cnt[1];
    }
}

__device__ __forceinline__ int live_count(const KArgs& A) {
    return A.n_fixed >= 0 ? A.n_fixed : (int)A.ctl[A.parity].live;
}
__device__ __forceinline__ void count_bounce(const KArgs& A, int N) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(&A.stats->bounce_live[A.bounce], (unsigned long long)N);
        atomicAdd(&A.stats->segments, (unsigned long long)N);
        if (A.bounce == 0 && A.count_pass) atomicAdd(&A.stats->passes, 1ull);   // (no separate ~4 us launch per pass)
    }
}
__device__ __forceinline__ void store_survivor(const PathSoA& B, int i, const PathReg& p, bool with_slot) {
    (void)with_slot;
    B.a[i] = v4f{p.o.x, p.o.y, p.o.z, p.d.x};
    B.b[i] = v4f{p.d.y, p.d.z, p.c.x, p.c.y};
    B.c[i] = v2f{p.c.z, __int_as_float(p.slot)};
}

// A kernel parameter re-read from the kernarg segment (at byte `offset`: parameters are laid out in
// order at their natural alignment; tests/test_kernarg_layout_cpu.py checks the offsets the compiler
// assigned) through a pointer the compiler cannot follow.  (Not through the parameter's own address:
// taking it makes clang copy the parameter to private memory.)  Used at the top of
// a kernel's per-tile loop: the fields are then loaded (scalar loads) in each iteration where they are
// used, instead of being hoisted to the kernel's start and kept live in SGPRs across the loop — at
// 8 waves per SIMD (~80 SGPRs) those spilled to VGPR lanes, and every reload was a v_readlane on the
// VALU (k_bounce<false, false, 0>: 75 SGPRs spilled -> 14, profiles/r06_kernel_resources.txt).
template <class T>
__device__ __forceinline__ const T& fresh_param(uint32_t offset) {
    const char PT_CONST_AS* p = (const char PT_CONST_AS*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(p));
    return *(const T*)(const T PT_CONST_AS*)(p + offset);
}
__device__ __forceinline__ const KArgs& fresh_args() { return fresh_param<KArgs>(0); }

// Trace one bounce: [raygen] -> intersect -> shade, one path per lane, no barriers and no
// inter-workgroup dependency (any grid size is correct).  Survivors are written back IN PLACE
// and flagged; the stable compaction runs in k_compact_paths.  The RNG key of a path is its
// index i in the compacted input (pathtrace.cu:315).
template <bool FIRST, bool SPP1, bool MESH>
__global__ __launch_bounds__(kBlock) void k_trace(const KArgs A) {
    __shared__ DMaterial s_mats[kLdsMats];
    __shared__ LGeom s_geoms[MESH ? 1 : kLdsGeoms];
    __shared__ uint32_t s_cnt;
    const int N = live_count(A);
    if ((int)blockIdx.x * kBlock >= N) return;
    if (!MESH) stage_geoms(A.S, s_geoms);
    stage_materials(A, s_mats);
    const bool lds_mats = A.S.nmats <= kLdsMats;
    count_bounce(A, N);
    uint32_t emit_cnt = 0;
    for (int base = blockIdx.x * kBlock; base < N; base += gridDim.x * kBlock) {
        const KArgs& A = fresh_args();   // (shadows the parameter: its fields are re-read per tile)
        const int i = base + (int)threadIdx.x;
        bool emitted = false;
        if (i < N) {
            PathReg p;
            if (FIRST) raygen(A.cam, A.fl, A.tile, i, p);
            else load_path(A.in, i, A.bounce, p);
            uint32_t gm = ~0u;
            if (FIRST && A.cmask) {   // the wave's 64 consecutive slots: up to two pixel blocks, or four
                const int np = A.tile.npix;   // when they wrap into the next iteration
                const int i0 = __builtin_amdgcn_readfirstlane(i);
                const int l0 = i0 % np, l1 = min(i0 + 63, N - 1) % np;
                gm = A.cmask[l0 >> 6] | A.cmask[(l1 >= l0 ? l1 : np - 1) >> 6];
                if (l1 < l0) gm |= A.cmask[0] | A.cmask[l1 >> 6];
            }
            const Hit h = closest_hit<MESH, true, !FIRST>(A.S, A.fl, s_geoms, p.o, p.d, &A.stats->bound_mismatch, gm);
            const int it = SPP1 ? 0 : p.slot / A.tile.npix;
            const int iter = A.tile.iter_first + it;
            // key: index within the path's own iteration (k_iter_bases; see k_bounce)
            const int key = A.fl.rng_pixel ? slot_pixel(A.cam, A.tile, p.slot)
                                           : i - (SPP1 ? 0 : (FIRST ? it * A.tile.npix : A.ibase[it]));
            const bool alive = lds_mats ? shade(A.S, A.fl, A.tile.depth, iter, key, p, h, s_mats)
                                        : shade(A.S, A.fl, A.tile.depth, iter, key, p, h, A.S.mats);
            if (alive) {
                store_survivor(A.in, i, p, FIRST);
            } else {
                emitted = p.c.x != 0.0f || p.c.y != 0.0f || p.c.z != 0.0f;
                retire<SPP1>(A, p, it);
            }
            A.flags[i] = alive ? 1 : 0;
        }
        emit_cnt += (uint32_t)__popcll(__ballot(emitted));
    }
    flush_emissive(A, emit_cnt, &s_cnt);
}

// Split pipeline, batched passes: the first dense index of every batch iteration present (the
// compacted array is iteration-major because the compaction is stable and slots are too).
__global__ __launch_bounds__(kBlock) void k_iter_bases(const KArgs A) {
    const int N = live_count(A);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
        const int it = __float_as_int(A.in.c[i][1]) / A.tile.npix;
        if (i == 0 || __float_as_int(A.in.c[i - 1][1]) / A.tile.npix != it) A.ibase[it] = i;
    }
}

// ---- fused pipeline: one kernel per bounce ---------------------------------------------------
// Segmented stable compaction, no inter-workgroup dependency.  Workgroup b of a launch owns the
// contiguous LOGICAL path range [b*chunk, (b+1)*chunk) (chunk = whole 256-path tiles) and writes
// its survivors, in order, to the front of PHYSICAL segment b = out[b*chunk ...]; its survivor
// count goes to seg[parity^1][b].  The next launch scans the (<= kMaxSeg) counts in LDS at start:
// logical survivor j lives in the segment s with pre[s] <= j < pre[s+1], at s*chunk + j - pre[s].
// Concatenating the segments in order is exactly the stable compaction of pathtrace.cu:377-407,
// so the logical index is the reference's RNG key (pathtrace.cu:315).
//   Measured before this design (profiles/r01_*): the decoupled look-back per 256-path tile parked
// every wave of a workgroup behind wave 0's cross-CU poll — 57% of wave cycles waiting vs 25% in
// the same trace code without compaction.  Here nothing waits on another workgroup, so the grid
// need not be co-resident and shared GPUs need no claimed schedule.
constexpr int kMaxSeg = 2048;
constexpr int kMaxSpp = kBlock;   // batch iterations per pass (pt_shard.spp): one thread each
constexpr int kMaxLanes = 4;      // lanes of a batched pass (pt_ctx::lanes; PT_AMD_LANES)
constexpr long long kThreeLanePaths = 48ll << 20;   // default: 3 lanes from 48 Mi paths per pass, else 2
// (measured, same box: Cornell 800x800 x 32 (20 M paths): 3 lanes +0.7%, within run-to-run noise,
// while each launch shares the GPU with two others; config 3 (66 M) +1.2%, config 4 (265 M) +3%,
// config 5 (66 M) +2%.  4 lanes + the finalize stream exceed the box's 4 hardware queues: -10%.)
// Iterations of lane l when `spp` are split over `lanes`: the first spp % lanes lanes take one more.
inline int lane_iters(int spp, int lanes, int l) { return spp / lanes + (l < spp % lanes ? 1 : 0); }

// Segment words of k_bounce: survivor count | batch iteration << 24 (pt_create bounds chunk < 2^24).
constexpr int kSegItShift = 24;
constexpr uint32_t kSegCountMask = (1u << kSegItShift) - 1u;

// The launch's workgroup layout from the iteration starts s_ib[0..spp] (see k_bounce), computed
// by the whole workgroup (thread t owns iteration t; spp <= kBlock): s_lay = {tpb, nseg, iteration
// of this workgroup (-1: idle), its chunk index in that iteration}.  s_ib must be visible on entry.
__device__ __forceinline__ void plan_layout(const int32_t* s_ib, int spp, int grid, int b, int32_t* s_lay,
                                            uint32_t* s_tmp, int32_t* s_first = nullptr) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t tl = tid < spp ? (uint32_t)(s_ib[tid + 1] - s_ib[tid] + kBlock - 1) / kBlock : 0u;
    const uint32_t i1 = lb::wave_inclusive_scan(tl);
    if (lane == 63) s_tmp[wave] = i1;
    if (tid == 0) s_lay[2] = -1;
    __syncthreads();
    const int tiles = (int)(s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3]);
    const int tpb = max(1, (tiles + grid - spp - 1) / (grid - spp));
    const uint32_t g = (tl + (uint32_t)tpb - 1u) / (uint32_t)tpb;
    const uint32_t i2 = lb::wave_inclusive_scan(g);
    if (lane == 63) s_tmp[4 + wave] = i2;
    __syncthreads();
    uint32_t pre = i2 - g;
    for (int q = 0; q < wave; ++q) pre += s_tmp[4 + q];
    if (tid < spp && b >= (int)pre && b < (int)(pre + g)) { s_lay[2] = tid; s_lay[3] = b - (int)pre; }
    if (tid == 0) { s_lay[0] = tpb; s_lay[1] = (int)(s_tmp[4] + s_tmp[5] + s_tmp[6] + s_tmp[7]); }
    if (s_first) {   // first workgroup (= output segment) of every iteration, s_first[spp] = nseg
        if (tid < spp) s_first[tid] = (int32_t)pre;
        if (tid == 0) s_first[spp] = (int32_t)(s_tmp[4] + s_tmp[5] + s_tmp[6] + s_tmp[7]);
    }
    __syncthreads();
}

// Exclusive scan of the previous launch's segment counts into s_pre[0..nseg] (s_pre[nseg] = N),
// the logical index where each batch iteration's survivors start into s_ib[0..spp] (s_ib[spp] = N;
// an iteration with no survivor gets the next one's start), and this launch's layout (s_lay).
// s_ib must hold -1 on entry (written before the caller's first barrier).
__device__ __forceinline__ int scan_segments(const uint32_t* __restrict__ words, int nseg, int spp, int32_t* s_pre,
                                             int32_t* s_ib, int32_t* s_lay, uint32_t* s_wsum) {
    constexpr int kPer = kMaxSeg / kBlock;   // 8 counts per thread
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t w[kPer];
    uint32_t sum = 0;
    const int s0 = tid * kPer;
    const uint32_t wprev = (s0 > 0 && s0 - 1 < nseg) ? words[s0 - 1] : 0xffffffffu;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        w[k] = s0 + k < nseg ? words[s0 + k] : 0u;
        sum += w[k] & kSegCountMask;
    }
    const uint32_t incl = lb::wave_inclusive_scan(sum);
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (int q = 0; q < wave; ++q) run += s_wsum[q];
    int prev_it = wprev == 0xffffffffu ? -1 : (int)(wprev >> kSegItShift);
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int s = s0 + k;
        if (s <= nseg) s_pre[s] = (int32_t)run;
        if (s < nseg) {   // first segment of its iteration: that iteration's logical start
            const int it = (int)(w[k] >> kSegItShift);
            if (it != prev_it) s_ib[it] = (int32_t)run;
            prev_it = it;
        }
        run += w[k] & kSegCountMask;
    }
    if (tid == kBlock - 1) s_pre[kMaxSeg] = (int32_t)run;   // nseg == kMaxSeg
    __syncthreads();
    const int N = __builtin_amdgcn_readfirstlane(s_pre[nseg]);
    if (tid == 0) s_ib[spp] = N;
    __syncthreads();
    if (tid < spp && s_ib[tid] < 0) {   // no survivor in iteration tid: the next present start
        int j = tid + 1;                // (a concurrent fill of s_ib[j] writes this same value)
        while (s_ib[j] < 0) ++j;
        s_ib[tid] = s_ib[j];
    }
    __syncthreads();
    plan_layout(s_ib, spp, (int)gridDim.x, (int)blockIdx.x, s_lay, s_wsum + 4);
    return N;
}

// Segment holding logical index i, searching up from `s` (s_pre[s] <= i).
__device__ __forceinline__ int seg_walk(const int32_t* s_pre, int nseg, int s, int i) {
    while (s + 1 < nseg && s_pre[s + 1] <= i) ++s;
    return s;
}

// BVH closest hit of every live path of this bounce, ahead of k_bounce<.., kMeshPre> (which reads it
// at the path's physical index): the divergent, latency-bound walk runs in a lean persistent kernel
// with no barriers in its loop and a depth-sized LDS stack, instead of inside the bounce kernel's tile
// loop (where one wave's walk held its workgroup's other three at every tile barrier, 3 waves/SIMD).
//   Rays per path vary from zero to hundreds of steps, so a wave that walks 64 fixed rays idles most
// lanes behind its longest ray (measured on config 5: 25% of lane slots busy).  Here a lane that
// finishes its ray takes a new one (Aila & Laine 2009, persistent threads + dynamic fetch): when at
// least kRefillMin lanes are idle, they take the next rays of the wave's chunk (kTravChunk rays from
// a per-bounce ticket).  A walk is one while-while round per loop trip: descend interior pairs until
// the lane holds a leaf, test the leaf, pop.  Per ray the sequence of boxes, pushes, pops and
// triangles is bvh_walk_pairs's, so the hit is the reference's whatever the scheduling.
//   Rays: first bounce, camera ray k (raygen, as k_bounce<FIRST> makes it), record k; later bounces,
// the k-th survivor of the previous launch's segments (prefix of the segment words in LDS), record =
// its physical slot.  Record: (t, BVH-order triangle index or -1, bx, by).
constexpr int kMeshInline = 1;   // k_bounce MESH modes: 0 no mesh, 1 traversal inside k_bounce,
constexpr int kMeshPre = 2;      // 2 closest mesh hit precomputed by k_traverse,
constexpr int kAnalyticSkip = 3; // 3 no mesh, first bounce: waves with an empty camera mask skip raygen + hit
constexpr int kAnalyticGM = 4;   // 4 no mesh, more materials or geoms than the LDS tables hold (read from global
                                 //   memory); modes 0 and 3 read both from LDS only (no second inlined shade,
                                 //   no plain per-geom loop for a large table)
constexpr int kTravChunk = 256;  // rays per ticket grab
constexpr int kRefillMin = 16;   // idle lanes that trigger a refill
constexpr int kTravLdsRows = 32; // LDS stack entries per thread (HybStack; the rest in scratch)
constexpr int kTrav4LdsRows = 16;   // k_traverse4: LDS stack entries per thread (5 workgroups per CU)
constexpr int kFoldBatch = 4;      // k_traverse4: task results read per LDS round trip
// k_traverse4 leaf tasks: K = kT4K consecutive triangles of one leaf per lane per trip for walks
// without the exact t-cull; with it, K = 1 (pt_ctx::walk_k).
// Measured (config 5, 64 iterations per pass, same box, two alternations; profiles/r05_walk_ab.txt):
// K = 1 / 2 / 3 / 4: 822 / 929 / 793 / 723 Mray/s.  K = 2 halves the trips the triangle tasks need
// (112 per ray at 64 per trip: they, not the 56 interior steps, bounded a ray's trips) at 122 VGPRs,
// still 4 waves per SIMD; K = 3 and 4 take 132 / 141 VGPRs and drop to 3 waves.  Where the exact t-cull is on
// (the tessellated workload, room.json) the cull leaves few triangles per reached leaf, the trips are
// bound by the interior steps, and the second slot only adds divergent work: K = 2 5,542 vs K = 1
// 5,755 Mray/s on the tessellated workload (same box) — so those walks run K = 1.
constexpr int kT4K = 2;

// Exclusive prefix of the previous launch's segment survivor counts into s_pre[0..nseg]; returns
// the total.  All threads of the block call it (barriers).
__device__ __forceinline__ int seg_prefix(const uint32_t* __restrict__ words, int nseg, int32_t* s_pre, uint32_t* s_wsum) {
    constexpr int kPer = kMaxSeg / kBlock;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t w[kPer], sum = 0;
    const int s0 = tid * kPer;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        w[k] = s0 + k < nseg ? (words[s0 + k] & kSegCountMask) : 0u;
        sum += w[k];
    }
    const uint32_t incl = lb::wave_inclusive_scan(sum);
    if (lane == 63) s_wsum[wave] = incl;
    __syncthreads();
    uint32_t run = incl - sum;
    for (int q = 0; q < wave; ++q) run += s_wsum[q];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (s0 + k <= nseg) s_pre[s0 + k] = (int32_t)run;
        run += w[k];
    }
    if (tid == kBlock - 1) s_pre[kMaxSeg] = (int32_t)run;
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(s_pre[nseg]);
}

template <bool FIRST>
__global__ __launch_bounds__(kBlock) void k_traverse(const KArgs A) {
    extern __shared__ int s_tstack[];   // stack_rows entries per thread, column layout
    __shared__ int32_t s_pre[FIRST ? 1 : kMaxSeg + 1];
    __shared__ uint32_t s_wsum[4];
    const int tid = threadIdx.x, lane = tid & 63;
    const SceneDev& S = A.S;
    int N, nseg = 0, chunk = 0;
    if (FIRST) {
        N = A.tile.P;
    } else {
        const int par = A.parity;
        nseg = (int)A.ctl[par].nseg;
        chunk = (int)A.ctl[par].chunk;
        N = seg_prefix(reinterpret_cast<const uint32_t*>(A.seg) + (size_t)par * kMaxSeg, nseg, s_pre, s_wsum);
    }
    // ray k -> (origin, direction, record slot)
    auto ray = [&](int k, f3& o, f3& d) -> int {
        if (FIRST) {
            PathReg p;
            raygen(A.cam, A.fl, A.tile, k, p);
            o = p.o;
            d = p.d;
            return k;
        }
        int lo = 0, hi = nseg - 1;   // segment holding survivor k: the last s with s_pre[s] <= k
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_pre[mid] <= k) lo = mid; else hi = mid - 1;
        }
        const int q = lo * chunk + (k - s_pre[lo]);
        const v4f a = PT_LD(A.in.a + q), b = PT_LD(A.in.b + q);
        o = F3(a[0], a[1], a[2]);
        d = F3(a[3], b[0], b[1]);
        return q;
    };
    int spill[64];   // stack entries past the LDS rows (HybStack)
    const HybStack st{s_tstack + tid, spill, A.stack_rows};
    // the pair walk pushes only passing children: exact while its stack never reaches the reference's
    // 64 entries (occupancy <= bvh_depth + 1); else, and under bvh_cull, the node-at-a-time walk
    if (!(S.pairs && !A.fl.bvh_cull && S.bvh_depth + 2 <= 64)) {
        for (int k = (int)blockIdx.x * kBlock + tid; k < N; k += (int)gridDim.x * kBlock) {
            f3 o, d;
            const int q = ray(k, o, d);
            const MeshHit r = bvh_walk(S, o, d, A.fl.bvh_cull != 0, st);
            PT_ST((v4f{r.t, __int_as_float(r.any ? r.idx : -1), r.bx, r.by}), A.mhit + q);
        }
        return;
    }
    uint32_t* ticket = A.tticket;
    // chunk size: kTravChunk, smaller when the bounce has few rays (>= 2 chunks per resident wave)
    const int csz = min(A.tchunk, max(64, (N / (int)(gridDim.x * (kBlock / 64) * 2)) & ~63));
    int cnext = 0, cend = 0;   // the wave's chunk of rays (wave-uniform)
    bool exhausted = false;
    bool have = false;         // this lane holds a ray
    // walk state: an interior pair (cur >= 0) or a leaf's triangle range [ti, te) (leaf)
    int q = 0, cur = 0, top = 0, ti = 0, te = 0;
    bool leaf = false, finite = true;   // finite: o and 1/d are finite (aabb_hit_finite)
    f3 o = F3(0, 0, 0), d = F3(0, 0, 0), inv = F3(0, 0, 0);
    uint32_t negm = 0;         // bit a: d[a] < 0
    MeshHit r{false, -1, -1, kFLT_MAX, 0.f, 0.f};
    auto enter = [&](int code) {   // code: interior (>= 0) or leaf (< 0, != kWalkDone)
        leaf = code < 0;
        if (leaf) {
            const int c = -code - 1;
            ti = c >> 8;
            te = ti + (c & 255);
        } else {
            cur = code;
        }
    };
#ifdef PT_TRAV_STATS
    uint32_t n_rays = 0, n_pairs = 0, n_tris = 0, w_trips = 0;
#endif
    for (;;) {
        const uint64_t idle = __ballot(!have);
        const int nidle = __popcll(idle);
        if (nidle >= A.refill_min && !exhausted) {
            if (cnext >= cend) {
                int base = 0;
                if (lane == 0) base = (int)atomicAdd(ticket, (uint32_t)csz);
                base = __shfl(base, 0);
                if (base >= N) exhausted = true;
                else { cnext = base; cend = min(base + csz, N); }
            }
            if (!exhausted) {
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                if (!have && cnext + (int)rank < cend) {
                    q = ray(cnext + (int)rank, o, d);
                    negm = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
                    inv = F3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
                    finite = __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) && __builtin_isfinite(inv.z) &&
                             __builtin_isfinite(o.x) && __builtin_isfinite(o.y) && __builtin_isfinite(o.z);
                    const float bmin[3] = {S.root_lo[0], S.root_lo[1], S.root_lo[2]};
                    const float bmax[3] = {S.root_hi[0], S.root_hi[1], S.root_hi[2]};
                    top = 0;
                    r = MeshHit{false, -1, -1, kFLT_MAX, 0.f, 0.f};
                    if (aabb_hit(bmin, bmax, o, inv)) {
                        enter(S.root_code);
                        have = true;
                    } else {   // misses the whole tree
                        PT_ST((v4f{r.t, __int_as_float(-1), r.bx, r.by}), A.mhit + q);
                    }
#ifdef PT_TRAV_STATS
                    ++n_rays;
#endif
                }
                cnext = min(cnext + nidle, cend);
            }
        }
        if (__ballot(have) == 0) {   // every lane idle: done, or (rays that missed the root) refill
            if (exhausted) break;
            continue;
        }
#ifdef PT_TRAV_STATS
        w_trips += lane == 0 ? 1u : 0u;
#endif
        if (have) {
            // one memory round trip per trip for every lane: a pair (interior) or a triangle (leaf)
            const v4f* src = leaf ? reinterpret_cast<const v4f*>(S.tris + ti) : reinterpret_cast<const v4f*>(S.pairs + (cur >> 2));
            const v4f x0 = src[0], x1 = src[1], x2 = src[2];
            v4f x3 = v4f{0.f, 0.f, 0.f, 0.f};
            if (!leaf) x3 = src[3];
            int next = kWalkNone;
            if (leaf) {
#ifdef PT_TRAV_STATS
                ++n_tris;
#endif
                const DTri tr{x0, x1, x2};
                float bx, by, bz;
                if (ray_tri(tr, o, d, bx, by, bz)) {
                    r.any = true;
                    if (r.t == -1.0f || bz < r.t) {
                        r.t = bz; r.bx = bx; r.by = by; r.idx = ti;
                    }
                }
                if (++ti == te) next = top == 0 ? kWalkDone : st.get(--top);
            } else {
#ifdef PT_TRAV_STATS
                ++n_pairs;
#endif
                const float lmn[3] = {x0[0], x0[1], x0[2]}, lmx[3] = {x1[0], x1[1], x1[2]};
                const float rmn[3] = {x2[0], x2[1], x2[2]}, rmx[3] = {x3[0], x3[1], x3[2]};
                bool hl, hr;
                if (__ballot(!finite) == 0) {   // (wave-uniform)
                    hl = aabb_hit_finite(lmn, lmx, o, inv);
                    hr = aabb_hit_finite(rmn, rmx, o, inv);
                } else {
                    hl = aabb_hit(lmn, lmx, o, inv);
                    hr = aabb_hit(rmn, rmx, o, inv);
                }
                const int cl = __float_as_int(x0[3]), cr = __float_as_int(x2[3]);
                const bool ng = (negm >> (cur & 3)) & 1u;   // split axis: right child first
                const bool h1 = ng ? hr : hl, h2 = ng ? hl : hr;
                const int c1 = ng ? cr : cl, c2 = ng ? cl : cr;
                if (h1 && h2) st.set(top++, c2);
                next = (h1 || h2) ? (h1 ? c1 : c2) : (top == 0 ? kWalkDone : st.get(--top));
            }
            if (next == kWalkDone) {
                PT_ST((v4f{r.t, __int_as_float(r.any ? r.idx : -1), r.bx, r.by}), A.mhit + q);
                have = false;
            } else if (next != kWalkNone) {
                enter(next);
            }
        }
    }
#ifdef PT_TRAV_STATS
    unsigned long long* g = g_trav + (blockIdx.x & 63) * 8;
    atomicAdd(&g[0], (unsigned long long)n_rays);
    atomicAdd(&g[1], (unsigned long long)n_pairs);
    atomicAdd(&g[2], (unsigned long long)n_tris);
    atomicAdd(&g[3], (unsigned long long)w_trips);
    atomicAdd(&g[4], lane == 0 ? 1ull : 0ull);
#endif
}

// The four slab tests of a quad entry for a ray whose o and 1/d are finite (aabb_hit_finite's
// arithmetic per slot: (b - o) * inv, then min/max); bit k set when slot k's box is hit.  The
// subtractions and products run two slots per v_pk_add_f32 / v_pk_mul_f32 (the same correctly
// rounded operations as the scalar forms).
__device__ __forceinline__ uint32_t quad_hits(const v4f& lox, const v4f& hix, const v4f& loy, const v4f& hiy,
                                              const v4f& loz, const v4f& hiz, f3 o, f3 inv) {
    const v4f ox = {o.x, o.x, o.x, o.x}, oy = {o.y, o.y, o.y, o.y}, oz = {o.z, o.z, o.z, o.z};
    const v4f ix = {inv.x, inv.x, inv.x, inv.x}, iy = {inv.y, inv.y, inv.y, inv.y}, iz = {inv.z, inv.z, inv.z, inv.z};
    const v4f mx = (lox - ox) * ix, Mx = (hix - ox) * ix;
    const v4f my = (loy - oy) * iy, My = (hiy - oy) * iy;
    const v4f mz = (loz - oz) * iz, Mz = (hiz - oz) * iz;
    uint32_t h = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float lo = fmaxf(fmaxf(fminf(mx[k], Mx[k]), fminf(my[k], My[k])), fminf(mz[k], Mz[k]));
        const float hi = fminf(fminf(fmaxf(mx[k], Mx[k]), fmaxf(my[k], My[k])), fmaxf(mz[k], Mz[k]));
        h |= (!(hi < 0) && !(lo > hi)) ? (1u << k) : 0u;
    }
    return h;
}

// rocPRIM's wave-level LDS handoff: the stores of one lane are visible to the loads of another
// lane of the same wave after this point.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// k_traverse on the 4-wide layout (DQuad) with leaf work spread over the wave.
//   Round 2's walk (k_traverse above) spent one memory round trip per pair AND per triangle, and
// every trip ran both the box branch and the triangle branch for whichever lanes held a pair or a
// leaf: 111 pair fetches + 112 triangle tests per config-5 ray.  Here, per trip of the wave:
//   * lanes holding an interior node test the four boxes of its quad (128 B, loaded first thing
//     in the trip), push the hit slots in the reference's near-first order (the far group first,
//     within a group the far child first) and continue with the nearest hit;
//   * the REMAINING triangles of every lane holding a leaf are dealt out as tasks, one per lane of
//     the wave (up to 64 per trip, in lane order, by a wave prefix sum of the counts): each owner
//     writes (its ray, the triangle index) into the task slots, each task lane loads its triangle
//     and tests it, and the owner folds its tasks' results in triangle order with the reference's
//     update rule (`r.t == -1 || t < r.t`: the first closest found).  A leaf costs one trip instead
//     of one per triangle, and the triangle tests run with (nearly) every lane busy.  Tasks that do
//     not fit this trip stay with their owner for the next.
// Every lane issues both loads every trip (idle lanes reload a line already cached), so the wait
// counts are static: the quad's loads first, then the triangle's, and the box tests wait for the
// quad only.  The stack is LDS-only in trips where no lane can reach the LDS rows (wave-uniform
// test), else HybStack's LDS/scratch split.
// Per ray the boxes tested and their outcomes, the leaves reached, the triangles tested and their
// order are BVHIntersectionTest's; only the scheduling across lanes differs.  Rays whose o or 1/d
// is not finite (axis-parallel or NaN directions) get the record kRecWalkHere: the bounce kernel
// walks them itself with the node-at-a-time walk (glm's ternary slab test, the reference's stack).
constexpr int kT4Waves = 1; // (minimum waves per SIMD of k_traverse4)
constexpr int kT4WavesFirst = 4; // (minimum waves per SIMD of the camera-ray walk: 138 -> 128 VGPRs, +1%)
template <bool FIRST, int K>
__global__ __launch_bounds__(kBlock, FIRST ? kT4WavesFirst : kT4Waves) void k_traverse4(const KArgs A) {
    extern __shared__ int s_tstack[];   // stack_rows entries per thread, column layout
    __shared__ int32_t s_pre[FIRST ? 1 : kMaxSeg + 1];
    __shared__ uint32_t s_wsum[4];
    // leaf tasks, per task lane j: [2j] = (owner's o, triangle index), [2j + 1] = (owner's d, -),
    // then overwritten by the task's result (t or NaN = no hit, bx, by, -)
    __shared__ v4f s_task[K * kBlock];  // task results only (K per lane)
    __shared__ int32_t s_own[kBlock];   // leaf tasks: tag << 6 | owner lane, at the owner's first task
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const SceneDev& S = A.S;
    int N, nseg = 0, chunk = 0;
    if (FIRST) {
        N = A.tile.P;
    } else {
        const int par = A.parity;
        nseg = (int)A.ctl[par].nseg;
        chunk = (int)A.ctl[par].chunk;
        N = seg_prefix(reinterpret_cast<const uint32_t*>(A.seg) + (size_t)par * kMaxSeg, nseg, s_pre, s_wsum);
    }
    auto seg_of = [&](int k) -> int {   // the last segment starting at or before k (binary search)
        int lo = 0, hi = nseg - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_pre[mid] <= k) lo = mid; else hi = mid - 1;
        }
        return lo;
    };
    int wseg = 0;   // (!FIRST) the segment of the wave's current chunk start
    auto ray = [&](int k, f3& o, f3& d) -> int {   // as k_traverse
        if (FIRST) {
            PathReg p;
            raygen(A.cam, A.fl, A.tile, k, p);
            o = p.o;
            d = p.d;
            return k;
        }
        // a chunk spans a few hundred rays and a segment is a bounce workgroup's survivors: a step
        // or two from the chunk start's segment instead of ~11 dependent LDS reads per refill
        int lo = wseg;
        while (lo + 1 < nseg && s_pre[lo + 1] <= k) ++lo;
        const int q = lo * chunk + (k - s_pre[lo]);
        const v4f a = PT_LD(A.in.a + q), b = PT_LD(A.in.b + q);
        o = F3(a[0], a[1], a[2]);
        d = F3(a[3], b[0], b[1]);
        return q;
    };
    v4f* task = s_task + wave * (64 * K);
#define PT_RES(j) task[(j)]
    int32_t* own = s_own + wave * 64;
    own[lane] = 0;   // tags start at 1
    uint32_t tag = 0;
    int* const col = s_tstack + tid;
    const int rows = A.stack_rows;
    int spill[64];
    const HybStack hst{col, spill, rows};
    uint32_t* ticket = A.tticket;
    const int csz = min(A.tchunk, max(64, (N / (int)(gridDim.x * (kBlock / 64) * 2)) & ~63));
    int cnext = 0, cend = 0;
    bool exhausted = false, have = false, leaf = false;
    int q = 0, cur = 0, top = 0, ti = 0, te = 0;
    f3 o = F3(0, 0, 0), d = F3(0, 0, 0), inv = F3(0, 0, 0);
    uint32_t negm = 0;
    bool cullok = false;   // exact t-cull (S.qcull): the ray's |d|^2 lies in the margins' range
    MeshHit r{false, -1, -1, kFLT_MAX, 0.f, 0.f};
    auto enter = [&](int code) {
        leaf = code < 0;
        if (leaf) {
            const int c = -code - 1;
            ti = c >> 8;
            te = ti + (c & 255);
        } else {
            cur = code;
        }
    };
    auto record = [&]() { PT_ST((v4f{r.t, __int_as_float(r.any ? r.idx : -1), r.bx, r.by}), A.mhit + q); };
    auto fold = [&](const v4f& x, int idx) {   // bvh_walk_pairs's per-triangle update
        if (x[0] == x[0]) {
            r.any = true;
            if (r.t == -1.0f || x[0] < r.t) { r.t = x[0]; r.bx = x[1]; r.by = x[2]; r.idx = idx; }
        }
    };
#ifdef PT_TRAV_STATS
    uint32_t n_rays = 0, n_inner = 0, n_tris = 0, w_trips = 0, n_busy = 0, t_leaf = 0, t_inner = 0;
#endif
    for (;;) {
        // ---- refill: idle lanes take the next rays of the wave's chunk ----
        const uint64_t idle = __ballot(!have);
        const int nidle = __popcll(idle);
        if (nidle >= A.refill_min && !exhausted) {
            if (cnext >= cend) {
                int base = 0;
                if (lane == 0) base = (int)atomicAdd(ticket, (uint32_t)csz);
                base = __shfl(base, 0);
                if (base >= N) exhausted = true;
                else {
                    cnext = base;
                    cend = min(base + csz, N);
                    if (!FIRST) wseg = __builtin_amdgcn_readfirstlane(seg_of(base));
                }
            }
            if (!exhausted) {
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0u));
                if (!have && cnext + (int)rank < cend) {
                    q = ray(cnext + (int)rank, o, d);
                    negm = (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
                    inv = F3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
                    const bool finite = __builtin_isfinite(inv.x) && __builtin_isfinite(inv.y) &&
                                        __builtin_isfinite(inv.z) && __builtin_isfinite(o.x) &&
                                        __builtin_isfinite(o.y) && __builtin_isfinite(o.z);
                    {   // |d|^2 within [1 - 2^-18, 1 + 2^-18] (its float value is within 3 ulp of exact)
                        const float dd = dot(d, d);
                        cullok = dd >= 1.0f - 0x1p-18f + 0x1p-22f && dd <= 1.0f + 0x1p-18f - 0x1p-22f;
                    }
                    top = 0;
                    r = MeshHit{false, -1, -1, kFLT_MAX, 0.f, 0.f};
                    const float bmin[3] = {S.root_lo[0], S.root_lo[1], S.root_lo[2]};
                    const float bmax[3] = {S.root_hi[0], S.root_hi[1], S.root_hi[2]};
                    if (!finite) {   // left to the bounce kernel's node walk (glm's ternary slab test)
                        PT_ST((v4f{0.f, __int_as_float(kRecWalkHere), 0.f, 0.f}), A.mhit + q);
                    } else if (aabb_hit(bmin, bmax, o, inv)) {
                        enter(S.root_qcode);
                        have = true;
                    } else {
                        record();
                    }
#ifdef PT_TRAV_STATS
                    ++n_rays;
#endif
                }
                cnext = min(cnext + nidle, cend);
            }
        }
        const uint64_t busy = __ballot(have);
        if (busy == 0) {
            if (exhausted) break;
            continue;
        }
#ifdef PT_TRAV_STATS
        if (lane == 0) { ++w_trips; n_busy += (uint32_t)__popcll(busy); }
#endif
        // the stack this trip: LDS only unless some lane could reach the LDS rows (3 pushes at most)
        const bool fast = __ballot(top + 4 > rows) == 0;
        auto push = [&](int v) {
            if (fast) col[top * kBlock] = v;
            else hst.set(top, v);
            ++top;
        };
        auto pop = [&]() -> int {
            if (top == 0) return kWalkDone;
            --top;
            return fast ? col[top * kBlock] : hst.get(top);
        };
        // ---- leaf tasks: the remaining triangles of the leaf lanes, one per lane of the wave ----
        const int cnt = (have && leaf) ? te - ti : 0;
        // task slots come in groups of K consecutive triangles of one leaf (one lane tests the
        // group): counted in group units
        const int pcnt = (cnt + K - 1) / K;
        const int incl = (int)lb::wave_inclusive_scan((uint32_t)pcnt);
        const int pre = incl - pcnt;   // first group of this lane's leaf
        const int T = __builtin_amdgcn_readlane(incl, 63);
        const int cov = (pcnt > 0 && pre < 64) ? min(cnt, K * (64 - pre)) : 0;   // triangles covered this trip
        const bool is_task = lane < T;
        bool inner = have && !leaf;
        // A leaf lane whose remaining triangles all go out this trip already takes its next node
        // (everything after the leaf in the walk's order): an interior node is tested in this same
        // trip, beside its leaf's triangle tests, whose results are folded first (the order of the
        // triangles is unchanged: the node's triangles are tested in later trips).
        int after_leaf = kWalkNone;
        if (cov > 0 && cov == cnt) {
            after_leaf = pop();
            if (after_leaf >= 0) {
                cur = after_leaf;
                inner = true;
            }
        }
        // ---- the quad of every interior lane ----
        v4f x0, x1, x2, x3, x4, x5, x6;
        uint32_t meta;
        if (inner) {
            const v4f* qsrc = reinterpret_cast<const v4f*>(S.quads + (cur & kQuadIdxMask));
            x0 = qsrc[0]; x1 = qsrc[1]; x2 = qsrc[2]; x3 = qsrc[3]; x4 = qsrc[4]; x5 = qsrc[5]; x6 = qsrc[6];
        }
        meta = (uint32_t)cur >> kQuadMetaShift;   // (the code that led here carries the quad's meta)
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        v4u cw = {0u, 0u, 0u, 0u};   // the quad's exact t-cull words (one per slot)
        if (S.qcull && inner) cw = *reinterpret_cast<const v4u*>(S.qcull + 4 * (size_t)(cur & kQuadIdxMask));
        f3 to = F3(0, 0, 0), td = F3(0, 0, 0);
        int tidx = 0;
        int ntask = 1;   // (K > 1) triangles tidx .. tidx + ntask - 1 of this task lane
        if (T > 0) {   // (wave-uniform)
            if (tag == (1u << 25)) {   // (never in practice: ~10^5 trips per launch) restart the tags
                own[lane] = 0;
                tag = 0;
                wave_sync();
            }
            ++tag;
            if (cov > 0) own[pre] = (int32_t)((tag << 6) | (uint32_t)lane);
            wave_sync();
            const int v = own[lane];
            const uint64_t heads = __ballot(is_task && ((uint32_t)v >> 6) == tag);
            const uint64_t le = lane == 63 ? ~0ull : ((2ull << lane) - 1ull);
            const int pos = is_task ? 63 - (int)__clzll(heads & le) : lane;   // the owner's first task
            const int ow = __shfl(v, pos) & 63;
            tidx = __shfl(ti, ow) + K * (lane - pos);
            if (K > 1) ntask = min(K, __shfl(te, ow) - tidx);   // (the leaf's triangles left in this group)
            to = F3(__shfl(o.x, ow), __shfl(o.y, ow), __shfl(o.z, ow));
            td = F3(__shfl(d.x, ow), __shfl(d.y, ow), __shfl(d.z, ow));
#ifdef PT_TRAV_STATS
            {   // triangles dealt this trip (K per task lane at most)
                const uint32_t tt = __builtin_amdgcn_readlane(lb::wave_inclusive_scan((uint32_t)cov), 63);
                if (lane == 0) { ++t_leaf; n_tris += tt; }
            }
#endif
        }
        v4f t0, t1, t2;
        v4f u[K > 1 ? K - 1 : 1][3];   // the group's further triangles
        auto load_tri = [&]() {
            // 36 bytes per triangle: a leaf's consecutive triangles cover fewer cache lines
            typedef float v3f __attribute__((ext_vector_type(3)));
            const float* p = S.tpack + 9 * (size_t)tidx;
            if (K == 2) {
                // the group's 72 contiguous bytes in five loads (4 x 16 B + 8 B, dword-aligned) instead
                // of six 12-byte ones: 5.4 instead of 6.4 cache-line accesses per lane on average (the
                // address path's cost); the pack is padded, so a group of one reads a neighbour
                typedef float v4a __attribute__((ext_vector_type(4), aligned(4)));
                typedef float v2a __attribute__((ext_vector_type(2), aligned(4)));
                const v4a q0 = *reinterpret_cast<const v4a*>(p), q1 = *reinterpret_cast<const v4a*>(p + 4),
                          q2 = *reinterpret_cast<const v4a*>(p + 8), q3 = *reinterpret_cast<const v4a*>(p + 12);
                const v2a q4 = *reinterpret_cast<const v2a*>(p + 16);
                t0 = v4f{q0[0], q0[1], q0[2], 0.f}; t1 = v4f{q0[3], q1[0], q1[1], 0.f};
                t2 = v4f{q1[2], q1[3], q2[0], 0.f};
                u[0][0] = v4f{q2[1], q2[2], q2[3], 0.f}; u[0][1] = v4f{q3[0], q3[1], q3[2], 0.f};
                u[0][2] = v4f{q3[3], q4[0], q4[1], 0.f};
                return;
            }
            const v3f a = *reinterpret_cast<const v3f*>(p), b = *reinterpret_cast<const v3f*>(p + 3),
                      c = *reinterpret_cast<const v3f*>(p + 6);
            t0 = v4f{a[0], a[1], a[2], 0.f}; t1 = v4f{b[0], b[1], b[2], 0.f}; t2 = v4f{c[0], c[1], c[2], 0.f};
#pragma unroll
            for (int j = 1; j < K; ++j)
                if (j < ntask) {
                    const float* pj = p + 9 * j;
                    const v3f a2 = *reinterpret_cast<const v3f*>(pj), b2 = *reinterpret_cast<const v3f*>(pj + 3),
                              c2 = *reinterpret_cast<const v3f*>(pj + 6);
                    u[j - 1][0] = v4f{a2[0], a2[1], a2[2], 0.f};
                    u[j - 1][1] = v4f{b2[0], b2[1], b2[2], 0.f};
                    u[j - 1][2] = v4f{c2[0], c2[1], c2[2], 0.f};
                }
        };
        if (is_task) load_tri();
#ifdef PT_TRAV_STATS
        {
            const uint64_t ib = __ballot(inner);
            if (lane == 0 && ib) { ++t_inner; n_inner += (uint32_t)__popcll(ib); }
        }
#endif
        // ---- interior step ----
        int next = kWalkNone;
        if (inner) {
            uint32_t hm = quad_hits(x0, x1, x2, x3, x4, x5, o, inv) & meta & 15u;
            // Exact t-cull: a slot whose box puts a lower bound on glm's computed t of
            // every triangle below it above the best t found so far is not entered — none of them can
            // replace the best or tie it, and the slots entered keep the reference's order.
            if (S.qcull && cullok && r.t < kFLT_MAX) {
                uint32_t cm = 0u;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const float sx = (negm & 1u) ? x1[k] : x0[k];   // the box corner nearest along d
                    const float sy = (negm & 2u) ? x3[k] : x2[k];
                    const float sz = (negm & 4u) ? x5[k] : x4[k];
                    const float tx = (sx - o.x) * d.x, ty = (sy - o.y) * d.y, tz = (sz - o.z) * d.z;
                    const float lo = ((tx + ty) + tz) - ((fabsf(tx) + fabsf(ty)) + fabsf(tz)) * 0x1p-20f;
                    const float A = (float)__builtin_bit_cast(_Float16, (uint16_t)(cw[k] & 0xffffu));
                    const float B = (float)__builtin_bit_cast(_Float16, (uint16_t)(cw[k] >> 16));
                    if (lo > 0.0f && (A * lo) * (1.0f - 0x1p-20f) > (B + r.t) * (1.0f + 0x1p-20f)) cm |= 1u << k;
                }
                hm &= ~cm;
            }
            int c0 = __float_as_int(x6[0]), c1 = __float_as_int(x6[1]);
            int c2 = __float_as_int(x6[2]), c3 = __float_as_int(x6[3]);
            // near-first order: within each group by its axis, then the groups by N's axis
            if ((negm >> ((meta >> 6) & 3u)) & 1u) {
                const int t = c0; c0 = c1; c1 = t;
                hm = (hm & 12u) | ((hm & 1u) << 1) | ((hm >> 1) & 1u);
            }
            if ((negm >> ((meta >> 8) & 3u)) & 1u) {
                const int t = c2; c2 = c3; c3 = t;
                hm = (hm & 3u) | ((hm & 4u) << 1) | ((hm >> 1) & 4u);
            }
            if ((negm >> ((meta >> 4) & 3u)) & 1u) {
                int t = c0; c0 = c2; c2 = t;
                t = c1; c1 = c3; c3 = t;
                hm = ((hm & 3u) << 2) | (hm >> 2);
            }
            // push the later hits (farthest first), continue with the first
            if (fast) {   // (wave-uniform) LDS rows only: the pushes without branches
                // hit slot k after the first hit goes to top + (hit slots above k): the farthest
                // deepest, as the sequential pushes below place them
                const uint32_t m = (uint32_t)__builtin_popcount(hm);
                const int f = __builtin_ctz(hm | 16u);   // first hit (4: none)
                if (((hm >> 1) & 1u) && f < 1) col[(top + __builtin_popcount(hm >> 2)) * kBlock] = c1;
                if (((hm >> 2) & 1u) && f < 2) col[(top + __builtin_popcount(hm >> 3)) * kBlock] = c2;
                if (((hm >> 3) & 1u) && f < 3) col[top * kBlock] = c3;
                const int pn = top > 0 ? col[max(top - 1, 0) * kBlock] : kWalkDone;   // (m == 0: pop)
                next = m == 0 ? pn : (f == 0 ? c0 : (f == 1 ? c1 : (f == 2 ? c2 : c3)));
                top += m > 0 ? (int)m - 1 : (top > 0 ? -1 : 0);
            } else
            {
                int nx = 0;
                bool got = false;
                if (hm & 8u) { nx = c3; got = true; }
                if (hm & 4u) { if (got) push(nx); nx = c2; got = true; }
                if (hm & 2u) { if (got) push(nx); nx = c1; got = true; }
                if (hm & 1u) { if (got) push(nx); nx = c0; got = true; }
                next = got ? nx : pop();
            }
        }
        // ---- triangle tests ----
        if (is_task) {
            float bx = 0.f, by = 0.f, bz = 0.f;
            const bool h = ray_tri(DTri{t0, t1, t2}, to, td, bx, by, bz);
            PT_RES(K * lane) = v4f{h ? bz : __builtin_nanf(""), bx, by, 0.f};
#pragma unroll
            for (int j = 1; j < K; ++j)
                if (j < ntask) {
                    float cx = 0.f, cy = 0.f, cz = 0.f;
                    const bool h2 = ray_tri(DTri{u[j - 1][0], u[j - 1][1], u[j - 1][2]}, to, td, cx, cy, cz);
                    PT_RES(K * lane + j) = v4f{h2 ? cz : __builtin_nanf(""), cx, cy, 0.f};
                }
        }
        if (T > 0) {
            wave_sync();   // the task results
            if (cov > 0) {   // the leaf's triangles in order (bvh_walk_pairs's loop)
                for (int k0 = 0; k0 < cov; k0 += kFoldBatch) {   // reads of a batch issued together
                    v4f x[kFoldBatch];
#pragma unroll
                    for (int k = 0; k < kFoldBatch; ++k)
                        if (k0 + k < cov) x[k] = PT_RES(K * pre + k0 + k);
#pragma unroll
                    for (int k = 0; k < kFoldBatch; ++k)
                        if (k0 + k < cov) fold(x[k], ti + k0 + k);
                }
                ti += cov;
                if (ti == te && !inner) next = after_leaf;   // (inner: the quad step above set `next`)
            }
        }
        if (next == kWalkDone) {
            record();
            have = false;
        } else if (next != kWalkNone) {
            enter(next);
        }
    }
#ifdef PT_TRAV_STATS
    unsigned long long* g = g_trav + (blockIdx.x & 63) * 8;
    atomicAdd(&g[0], (unsigned long long)n_rays);
    atomicAdd(&g[1], (unsigned long long)n_inner);
    atomicAdd(&g[2], (unsigned long long)n_tris);
    atomicAdd(&g[3], (unsigned long long)w_trips);
    atomicAdd(&g[4], lane == 0 ? 1ull : 0ull);
    atomicAdd(&g[5], (unsigned long long)n_busy);
    atomicAdd(&g[6], (unsigned long long)t_leaf);
    atomicAdd(&g[7], (unsigned long long)t_inner);
#endif
}

// [raygen] -> intersect -> shade -> segmented compaction (above).
constexpr int kLaterWaves = 8; // (minimum waves per SIMD of the later-bounce kernels)
// At ~60 VGPRs the later bounces' occupancy is set by their SGPRs: 106 give 7 waves per SIMD (of 800).
// 8 waves (SGPRs capped) lost 0.3% in round 4; after round 5's code-size cuts (LDS-only tables, one
// inlined exact test: 9,473 -> 5,408 ISA lines) they gain: Cornell +0.5%, config 4 +1.5%
// (profiles/r05_later_waves8_ab.txt).
constexpr int kFirstWaves = 8;   // (minimum waves per SIMD of the analytic first-bounce kernels: 8 caps them at 64
                                 // VGPRs, one spilled; Cornell +1.8%, first bounce -11% per launch, profiles/r06_first_waves_ab.txt)
template <bool FIRST, bool SPP1, int MESH>
__global__ __launch_bounds__(kBlock, (MESH != 0 && MESH != kAnalyticSkip) ? 1 : (FIRST ? kFirstWaves : kLaterWaves))
void k_bounce(const KArgs A) {
    // scene tables sized to the scene (dynamic LDS, bounce_lds_bytes): geom rows, then materials
    extern __shared__ __align__(16) uint8_t s_dyn[];
    LGeom* s_geoms = reinterpret_cast<LGeom*>(s_dyn);
    constexpr bool kLdsAll = MESH == 0 || MESH == kAnalyticSkip;   // (launch: materials and geoms fit LDS)
    const int ng_lds = kLdsAll ? A.S.ngeoms : (MESH == kMeshInline || A.S.ngeoms > kLdsGeoms ? 0 : A.S.ngeoms);
    DMaterial* s_mats = reinterpret_cast<DMaterial*>(s_dyn + ng_lds * sizeof(LGeom));
    float* s_frm = reinterpret_cast<float*>(s_mats + min(A.S.nmats, kLdsMats));   // [ng_lds * 6][6]
    __shared__ int32_t s_pre[FIRST ? 1 : kMaxSeg + 1];
    __shared__ int32_t s_ib[kMaxSpp + 1];
    __shared__ uint32_t s_wc[2][4];
    __shared__ uint32_t s_cnt;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int par = A.parity;
    const int spp = A.tile.spp;
    __shared__ int32_t s_lay[4];
    __shared__ uint32_t s_tmp[12];
    int N, nseg_in = 0, chunk_in = 0;
    if (FIRST) {
        N = A.n_fixed;
        for (int j = tid; j <= spp; j += kBlock) s_ib[j] = j * A.tile.npix;   // spp + 1 entries (spp <= kBlock)
        __syncthreads();
        plan_layout(s_ib, spp, (int)gridDim.x, (int)blockIdx.x, s_lay, s_tmp);
    } else {
        for (int j = tid; j <= spp; j += kBlock) s_ib[j] = -1;
        nseg_in = (int)A.ctl[par].nseg;
        chunk_in = (int)A.ctl[par].chunk;
        N = scan_segments(reinterpret_cast<const uint32_t*>(A.seg) + (size_t)par * kMaxSeg, nseg_in, spp, s_pre, s_ib,
                          s_lay, s_tmp);
    }
    // Workgroups are dealt to the batch iterations in order, none spanning two: iteration s gets
    // ceil(tiles_s / tpb) workgroups of tpb whole tiles.  tpb = ceil(tiles / (grid - spp)) keeps the
    // total within the grid.  The survivors of a pass then stay iteration-major, and a path's
    // shading key is its index within ITS iteration's compacted array — pathtrace.cu:315 of the
    // iteration traced alone, so a batched pass equals `spp` sequential pathtrace() calls bit for bit.
    const int tpb = __builtin_amdgcn_readfirstlane(s_lay[0]);
    const int nseg = __builtin_amdgcn_readfirstlane(s_lay[1]);
    const int my_it = __builtin_amdgcn_readfirstlane(s_lay[2]);
    const int my_c = __builtin_amdgcn_readfirstlane(s_lay[3]);
    const int chunk = tpb * kBlock;
    if (blockIdx.x == 0 && tid == 0) {
        A.ctl[par ^ 1].nseg = (uint32_t)nseg;
        A.ctl[par ^ 1].chunk = (uint32_t)chunk;
    }
    if (my_it < 0) return;
    if (MESH != kMeshInline) {
        stage_geoms(A.S, s_geoms);
        stage_frames(A.S, s_frm);
    }
    stage_materials(A, s_mats);   // (its barrier publishes the staged tables)
    // (analytic modes 0 / 3 run only where every material fits the LDS table: launch_bounce)
    const bool lds_mats = (MESH == 0 || MESH == kAnalyticSkip) ? true : (MESH == kAnalyticGM ? false : A.S.nmats <= kLdsMats);
    const float* frames = ng_lds > 0 ? s_frm : nullptr;
    count_bounce(A, N);
    const int it_base = __builtin_amdgcn_readfirstlane(s_ib[my_it]);
    const int first = it_base + my_c * chunk;
    const int last = min(__builtin_amdgcn_readfirstlane(s_ib[my_it + 1]), first + chunk);
    const int iter = A.tile.iter_first + my_it;
    int seg = 0;
    if (!FIRST) {   // segment of this workgroup's first logical path (binary search, uniform)
        int lo = 0, hi = nseg_in - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (s_pre[mid] <= first) lo = mid; else hi = mid - 1;
        }
        seg = lo;
    }
    uint32_t kept = 0, emit_cnt = 0;
    int k = 0;
    for (int base = first; base < last; base += kBlock, ++k) {
        const KArgs& A = fresh_args();   // (shadows the parameter: its fields are re-read per tile)
        const int i = base + tid;
        if (FIRST && (MESH == 0 || MESH == kAnalyticGM) && A.cmask) {
            // a tile whose four camera-mask blocks are all empty: every ray misses — shade's miss exit
            // (colour 0, no random number) without raygen, closest hit or the tile's ballots and
            // barrier (workgroup-uniform; k stays, so the count buffers keep alternating per barrier)
            const int lp0 = base - it_base, nb = ((last - it_base) + 63) >> 6;
            uint32_t any = 0u;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int b = (lp0 >> 6) + w;
                any |= b < nb ? A.cmask[b] : 0u;
            }
            if (any == 0u) {
                if (i < last) {
                    PathReg z;
                    z.c = F3(0.0f, 0.0f, 0.0f);
                    z.slot = i;
                    retire<SPP1>(A, z, my_it);
                }
                --k;
                continue;
            }
        }
        bool alive = false, emitted = false;
        PathReg p;
        // a wave whose camera rays can hit no geom (camera mask 0): no raygen, no closest hit
        // (misses draw no random number)
        bool skip = false;
        if (FIRST && MESH == kAnalyticSkip && A.cmask) {
            const int lp0 = __builtin_amdgcn_readfirstlane(i - it_base);
            skip = lp0 < last - it_base && A.cmask[lp0 >> 6] == 0u;
        }
        if (FIRST && skip) {
            if (i < last) {   // shade's miss exit: colour 0, retired (no record, no random number)
                p.c = F3(0.0f, 0.0f, 0.0f);
                p.slot = i;
                retire<SPP1>(A, p, my_it);
            }
        } else if (i < last) {
            int q = i;   // physical index of the path (and of its k_traverse record)
            if (FIRST) {
                raygen_at(A.cam, A.fl, A.tile, i, my_it, i - it_base, p);   // (a workgroup holds one iteration)
#if defined(PT_DUP) && PT_DUP == 6   // diagnostic: raygen again on an opaque pixel index
                {
                    PathReg p2;
                    int i2 = i;
                    asm volatile("" : "+v"(i2));
                    raygen_at(A.cam, A.fl, A.tile, i2, my_it, i2 - it_base, p2);
                    if (__float_as_uint(p2.d.x + p2.o.y) == 0x7f7ffffeu) atomicAdd(&A.stats->bound_mismatch, 7u);
                }
#endif
            } else {
                const int s = seg_walk(s_pre, nseg_in, seg, i);
                q = s * chunk_in + (i - s_pre[s]);
                load_path(A.in, q, A.bounce, p);
            }
            Hit h;
            if constexpr (MESH == kMeshPre) {
                const v4f m = PT_LD(A.mhit + q);
                MeshHit mh;
                mh.t = m[0];
                mh.idx = __float_as_int(m[1]);
                mh.bx = m[2];
                mh.by = m[3];
                if (mh.idx == kRecWalkHere) {   // a non-finite ray k_traverse4 left to this kernel
                    int wstack[64];
                    const MeshHit w = bvh_walk(A.S, p.o, p.d, false, PrivStack{wstack});
                    mh.t = w.t;
                    mh.idx = w.any ? w.idx : -1;
                    mh.bx = w.bx;
                    mh.by = w.by;
                }
                mh.any = mh.idx >= 0;
                mh.id = mh.any ? __float_as_int(A.S.tris[mh.idx].a[3]) : -1;
                if (A.fl.verify) {   // PT_AMD_VERIFY_BOUNDS=1: the record == the reference's node walk
                    int vstack[64];
                    const MeshHit w = bvh_walk(A.S, p.o, p.d, A.fl.bvh_cull != 0, PrivStack{vstack});
                    const int widx = w.any ? w.idx : -1;
                    if (widx != mh.idx || __float_as_uint(w.t) != __float_as_uint(mh.t) ||
                        __float_as_uint(w.bx) != __float_as_uint(mh.bx) || __float_as_uint(w.by) != __float_as_uint(mh.by))
                        atomicAdd(&A.stats->bound_mismatch, 1u);
                }
                h = intersect_bounded<!FIRST, true>(A.S, A.fl, s_geoms, p.o, p.d, &mh);
            } else {
                uint32_t gm = ~0u;
                if (FIRST && A.cmask) {   // this wave's 64 tile pixels (64-aligned: chunk and tiles are)
                    const int lp0 = __builtin_amdgcn_readfirstlane(i - it_base);
                    gm = A.cmask[lp0 >> 6];
                }
                h = closest_hit<MESH == kMeshInline, false, !FIRST, kLdsAll>(A.S, A.fl, s_geoms, p.o, p.d, &A.stats->bound_mismatch, gm);
#if defined(PT_DUP) && PT_DUP == 7   // diagnostic: the camera ray's closest hit again on an opaque origin
                if (FIRST) {
                    f3 o2 = p.o;
                    asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
                    const Hit h2 = closest_hit<MESH == kMeshInline, false, !FIRST>(A.S, A.fl, s_geoms, o2, p.d, &A.stats->bound_mismatch, gm);
                    if (__float_as_uint(h2.t) == 0x7f7ffffeu) atomicAdd(&A.stats->bound_mismatch, 7u);
                }
#endif
            }
            const int key = A.fl.rng_pixel ? slot_pixel(A.cam, A.tile, p.slot) : i - it_base;
            // every path entering bounce b has b bounces behind it: a wave-uniform value, so the
            // shading RNG's (iteration, remaining depth) hash is computed once per wave on the SALU
            p.bounces = A.bounce;
#if defined(PT_DUP)   // diagnostic builds (scripts/valu_phases.sh): a phase run twice on opaque copies of
            // its inputs, so SQ_INSTS_VALU's increase is that phase's dynamic cost (divergence included)
            if (!FIRST && MESH == 0) {
                f3 o2 = p.o;
                asm volatile("" : "+v"(o2.x), "+v"(o2.y), "+v"(o2.z));
                if (PT_DUP == 1) {
                    const Hit h2 = closest_hit<false, false, true>(A.S, A.fl, s_geoms, o2, p.d, &A.stats->bound_mismatch, ~0u);
                    if (__float_as_uint(h2.t) == 0x7f7ffffeu) atomicAdd(&A.stats->bound_mismatch, 7u);
                } else if (PT_DUP == 2) {
                    PathReg p2 = p;
                    p2.o = o2;
                    Hit hh = h;
                    int key2 = key;
                    asm volatile("" : "+v"(p2.d.x), "+v"(p2.d.y), "+v"(p2.d.z), "+v"(key2));
                    asm volatile("" : "+v"(hh.n.x), "+v"(hh.n.y), "+v"(hh.n.z), "+v"(hh.t), "+v"(hh.mat), "+v"(hh.frame));
                    const bool a2 = lds_mats ? shade(A.S, A.fl, A.tile.depth, iter, key2, p2, hh, s_mats, frames)
                                             : shade(A.S, A.fl, A.tile.depth, iter, key2, p2, hh, A.S.mats, frames);
                    if (a2 && __float_as_uint(p2.c.x) == 0x7f7ffffeu) atomicAdd(&A.stats->bound_mismatch, 7u);
                } else if (PT_DUP == 3) {
                    PathReg p2;
                    int q2 = q;
                    asm volatile("" : "+v"(q2));
                    load_path(A.in, q2, A.bounce, p2);
                    if (__float_as_uint(p2.o.x) == 0x7f7ffffeu) atomicAdd(&A.stats->bound_mismatch, 7u);
                }
            }
#endif
            alive = lds_mats ? shade(A.S, A.fl, A.tile.depth, iter, key, p, h, s_mats, frames)
                             : shade(A.S, A.fl, A.tile.depth, iter, key, p, h, A.S.mats, frames);
            if (!alive) {
                emitted = p.c.x != 0.0f || p.c.y != 0.0f || p.c.z != 0.0f;
                retire<SPP1>(A, p, my_it);
            }
        }
        emit_cnt += (uint32_t)__popcll(__ballot(emitted));
        // in-tile ranks: wave ballot + mbcnt, 4 wave counts through LDS (double-buffered, so
        // one barrier per tile: buffer k&1 was last read two tiles ago, before the last barrier)
        const uint64_t m = __ballot(alive);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (lane == 0) s_wc[k & 1][wave] = (uint32_t)__popcll(m);
        __syncthreads();
        const uint32_t w0 = s_wc[k & 1][0], w1 = s_wc[k & 1][1], w2 = s_wc[k & 1][2], w3 = s_wc[k & 1][3];
        const uint32_t before = (wave > 0 ? w0 : 0u) + (wave > 1 ? w1 : 0u) + (wave > 2 ? w2 : 0u);
        if (alive) store_path(A.out, (int)blockIdx.x * chunk + (int)(kept + before + rank), p);
        kept += (w0 + w1) + (w2 + w3);
        if (!FIRST) seg = seg_walk(s_pre, nseg_in, seg, min(base + kBlock, last - 1));
    }
    if (tid == 0) A.seg[(size_t)(par ^ 1) * kMaxSeg + blockIdx.x] = (int32_t)(kept | ((uint32_t)my_it << kSegItShift));
    flush_emissive(A, emit_cnt, &s_cnt);
}
// Stable compaction of the flagged survivors: tile = 256 threads x 4 paths (path order
// k-major: path = tile*1024 + k*256 + t, so every load/store is wave-contiguous), wave ballot +
// mbcnt ranks, 16 wave counts through LDS, decoupled look-back (lookback.h) over a persistent,
// statically assigned, co-resident grid.  The last tile writes the next bounce's path count.
constexpr int kCompactPer = 4;
constexpr int kCompactTile = kBlock * kCompactPer;

__device__ __forceinline__ void copy_path(const PathSoA& S, const PathSoA& D, int i, int j) {
    D.a[j] = S.a[i];
    D.b[j] = S.b[i];
    D.c[j] = S.c[i];
}

__global__ __launch_bounds__(kBlock) void k_compact_paths(const KArgs A) {
    __shared__ uint32_t s_wc[kCompactPer][4];
    __shared__ uint32_t s_excl;
    __shared__ int s_ring[lb::kRing];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int q = A.parity, nq = q ^ 1;
    uint64_t* st = A.status + (size_t)q * A.max_tiles;
    {   // zero the status words the next compaction launch (other parity) will use
        uint64_t* nst = A.status + (size_t)nq * A.max_tiles;
        for (int j = blockIdx.x * blockDim.x + tid; j < A.max_tiles; j += gridDim.x * blockDim.x) nst[j] = 0ull;
    }
    const int N = live_count(A);
    const int num_tiles = (N + kCompactTile - 1) / kCompactTile;
    if (blockIdx.x == 0 && tid == 0) {
        A.ctl[nq].ticket = 0u;   // the next look-back launch claims from zero
        if (num_tiles == 0) A.ctl[nq].live = 0u;
    }
    if ((int)blockIdx.x >= num_tiles) return;
    lb::TileSeq sq = lb::seq_start(A.fl.claimed != 0, &A.ctl[q].ticket, s_ring, num_tiles);
    while (sq.tile != INT_MAX) {
        lb::seq_step(sq, &A.ctl[q].ticket);
        const int tile = sq.tile;
        bool f[kCompactPer];
        uint32_t rank[kCompactPer];
        uint64_t m[kCompactPer];
#pragma unroll
        for (int k = 0; k < kCompactPer; ++k) {
            const int i = tile * kCompactTile + k * kBlock + tid;
            f[k] = i < N && A.flags[i] != 0;
            m[k] = __ballot(f[k]);
            rank[k] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m[k] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m[k], 0u));
        }
        __syncthreads();   // the previous tile's readers of s_wc / s_excl are done
        if (lane == 0) {
#pragma unroll
            for (int k = 0; k < kCompactPer; ++k) s_wc[k][wave] = (uint32_t)__popcll(m[k]);
        }
        __syncthreads();
        uint32_t off[kCompactPer], run = 0;
#pragma unroll
        for (int k = 0; k < kCompactPer; ++k) {
            uint32_t before = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w) before += (w < wave) ? s_wc[k][w] : 0u;
            off[k] = run + before;
#pragma unroll
            for (int w = 0; w < 4; ++w) run += s_wc[k][w];
        }
        const uint32_t total = run;
        if (wave == 0) {
            uint32_t excl = 0;
            if (tile == 0) {
                if (lane == 0) lb::publish(st, 0, lb::kFlagPre, total);
            } else {
                if (lane == 0) lb::publish(st, tile, lb::kFlagAgg, total);
                excl = lb::lookback(st, tile, lane, &A.stats->err);
                if (lane == 0) lb::publish(st, tile, lb::kFlagPre, excl + total);
            }
            if (lane == 0) {
                s_excl = excl;
                if (tile == num_tiles - 1) A.ctl[nq].live = excl + total;
            }
        }
        __syncthreads();
        const uint32_t excl = s_excl;
#pragma unroll
        for (int k = 0; k < kCompactPer; ++k)
            if (f[k]) copy_path(A.in, A.out, tile * kCompactTile + k * kBlock + tid, (int)(excl + off[k] + rank[k]));
        lb::seq_advance(sq, s_ring);
    }
}

// ---- material-sorted mode (pathtrace.cu:479-491: stable sort_by_key on materialId) ---------
// Material-sorted pipeline (sortbyMaterial): per bounce one producer launch, a histogram scan and
// one scatter.
//   k_sort_produce  shades the paths of bounce b in sorted order (gathered through perm; RNG key =
//                   sorted index within the iteration, pathtrace.cu:315) and INTERSECTS each
//                   survivor's new ray right away (the sort key of bounce b + 1): the survivor's
//                   64-byte record is written once, with its hit.  The first bounce's producer
//                   generates the camera rays instead of shading.
//                   Work unit = TILE: 256 consecutive positions of one iteration's sorted range.
//                   Tile t's survivors go to slots [256 t, 256 t + count_t), grouped by material
//                   (material m's run starts at the tile's exclusive prefix base(t, m) over the
//                   materials, each survivor at base + its rank among the tile's m-survivors), so
//                   the survivors' logical order is the tile order — stable.  Workgroups take
//                   tiles t = b, b + G, b + 2G, ... (G = grid): every workgroup walks the sorted
//                   order in step with the others, so the records being gathered at any moment
//                   belong to one or two iterations (one iteration's records at bounce 1: 20 k tiles
//                   x 16 KiB = 133 MB at 1920x1080, within the 256 MiB Infinity Cache) instead of
//                   every iteration of the pass at once.
//                   Sort keys are counted per tile: hist[iteration][material][tile of that
//                   iteration], and every survivor gets its rank among the same-material survivors
//                   of its tile (one ballot per material present in the wave).  Only the survivors
//                   that go on to be shaded (not ending at the next shade) get a record, and those
//                   are written compacted: material m's at 256 t + kbase(t, m) + their rank among
//                   the tile's m-survivors that go on (kbase: the exclusive prefix of those counts
//                   over the materials), each record carrying its rank among ALL the tile's
//                   m-survivors (the sorted position's offset in its run); hslot holds the first
//                   record slot of each (iteration, material, tile) run, 256 t + kbase(t, m);
//   scan            of the histogram (k_hist_sums / k_hist_scan_sums / k_hist_apply, no co-residency
//                   needed): tiles are in logical order, so hist's flat exclusive scan + the in-tile
//                   rank IS the survivor's position in the stable sort by (iteration, material).
//                   Run e's records are consecutive in both orders, so k_hist_apply, once it has
//                   offs[e] and offs2[e], writes the work list itself: work position offs2[e] + i
//                   gathers record hslot[e] + i (i < hist2[e]) and keys it offs[e] + the record's
//                   rank — whole runs of coalesced stores, no scatter kernel, no per-survivor key.
// Batched passes sort every iteration on its own (stable sort by (iteration, material), as `spp`
// sequential pathtrace() calls would): tiles never span two iterations, and an iteration's tiles
// form one block of the histogram.
// Path j of the sorted pipeline is ONE 32-byte record (only paths that go on to be shaded have one:
// a miss or an emitter ends in the producer), so the gather reads one 32-byte span:
//   r0 = (hit point.xyz, c.r)   r1 = (c.gb, slot, code | rank << 24)
// The hit point (getPointOnRay, as shade computes it) replaces the ray's origin and length.  code
// >= 0: a cube hit, geom * 6 + slab code (Hit::frame): the material is the geom's, the normal its
// precomputed slab normal (box_normal, which is how the hit's normal was made) and the tangent
// frame its precomputed one.  code < 0: -(material + 1), the normal in a side plane (code: 24 bits,
// signed; rank: the record's offset in its run of the sorted order, < 256, rec_code / rec_rank).  The ray's
// direction, which only a refractive or possibly reflective material reads (mat_needs_dir), goes
// to a second side plane for those paths alone.  Block of 4P planes: records in the first two,
// directions in the third, normals in the fourth.  `bounces` is not stored: every path entering
// bounce b has b bounces behind it.  Texture coordinates (textured scenes only) go to a side
// array, double-buffered like the records.
__device__ __forceinline__ v4f* srec(const PathSoA& B, int j) { return B.a + 2 * (size_t)(uint32_t)j; }
__device__ __forceinline__ v4f* sdir(const PathSoA& B, int j) { return B.a + 2 * (B.b - B.a) + (size_t)(uint32_t)j; }
__device__ __forceinline__ v4f* snrm(const PathSoA& B, int j) { return B.a + 3 * (B.b - B.a) + (size_t)(uint32_t)j; }
__device__ __forceinline__ int32_t rec_pack(int code, uint32_t rank) { return (int32_t)((rank << 24) | ((uint32_t)code & 0xffffffu)); }
__device__ __forceinline__ int rec_code(int32_t w) { return (int32_t)((uint32_t)w << 8) >> 8; }
__device__ __forceinline__ uint32_t rec_rank(int32_t w) { return (uint32_t)w >> 24; }

struct SortArgs {
    int32_t* hslot;     // per (iteration, material, tile): first record slot of its run (sort_hidx)
    int32_t* hist;      // per (iteration, material, tile) survivor counts (sort_hidx)
    int32_t* offs;      // its exclusive scan: sorted positions (RNG keys)
    int32_t* hist2;     // per entry: survivors that did not end in the producer (records to shade)
    int32_t* offs2;     // its exclusive scan: the next producer's work positions
    int32_t* perm;      // [P] work position -> record slot
    int32_t* fpos;      // [P] work position -> sorted position of its run's first survivor
    int32_t* itb;       // [2][kMaxSpp + 1] per parity: first tile of each iteration ([spp] = tiles)
    float* uv_out;      // textured scenes: (u, v) of the output records ([2 * cap])
};
// The next producer's work list: per work position, the record it gathers and the sorted position
// of the record's run (+ the record's rank = its sorted position).
// One (slot, position) pair per work position in `perm` (8 bytes: one store
// and one load per path instead of two each); 0: the separate arrays perm / fpos.
typedef int v2i_pf __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void pf_store(int32_t* perm, int32_t* fpos, uint32_t w, int32_t slot, int32_t pos) {
    (void)fpos;
    reinterpret_cast<v2i_pf*>(perm)[w] = v2i_pf{slot, pos};
}

constexpr int kSortMaxMats = 256;  // per-tile material counts in LDS (one thread per material)

// Histogram entry of tile t (iteration tiles [t0, t1)) for material m: [iteration block][material][tile].
__device__ __forceinline__ size_t sort_hidx(int t0, int t1, int nmats, int t, int m) {
    return (size_t)t0 * nmats + (size_t)m * (size_t)(t1 - t0) + (size_t)(t - t0);
}
// Iteration owning tile t: the last it with s_tb[it] <= t (empty iterations own no tile).
__device__ __forceinline__ int tile_iteration(const int32_t* s_tb, int spp, int t) {
    int lo = 0, hi = spp - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (s_tb[mid] <= t) lo = mid; else hi = mid - 1;
    }
    return lo;
}
// The same for a workgroup's increasing tiles t (uniform): from the previous tile's iteration `it`,
// one LDS read when t is still in it (the common case), else a scalar binary search above it.  The
// result and every read are wave-uniform (readfirstlane), so the tile's iteration, its bases and the
// RNG's iteration hash stay on the SALU.
__device__ __forceinline__ int tile_iteration_next(const int32_t* s_tb, int spp, int t, int it) {
    if (it + 1 >= spp || __builtin_amdgcn_readfirstlane(s_tb[it + 1]) > t) return it;
    int lo = it + 1, hi = spp - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (__builtin_amdgcn_readfirstlane(s_tb[mid]) <= t) lo = mid; else hi = mid - 1;
    }
    return __builtin_amdgcn_readfirstlane(lo);
}

__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* s_w, uint32_t* total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t incl = lb::wave_inclusive_scan(v);
    __syncthreads();   // previous users of s_w are done
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (int w = 0; w < wave; ++w) before += s_w[w];
    *total = s_w[0] + s_w[1] + s_w[2] + s_w[3];
    return before + incl - v;
}

constexpr int kProduceWaves = 7; // (minimum waves per SIMD of the analytic producer; 7 caps the
                             // first bounce's producer at 72 VGPRs: config 3 +0.8% on the same box)
constexpr int kProduceWavesFirst = kProduceWaves;
// VERIFY: the PT_AMD_VERIFY_BOUNDS=1 build of the producer (the plain-loop re-run of every closest
// hit compiled in); the default one carries no diagnostic code (round 4: the later producer's 8-byte
// register spill went away with it).
// LDSM: every material and geom is in the LDS tables (launch: nmats <= kLdsMats, ngeoms <= kLdsGeoms), so
// shading reads materials only there (one inlined shade instead of a uniform branch between an LDS and a
// global-memory copy) and the closest hit has no plain loop over a larger geom table.
template <bool FIRST, bool SPP1, bool MESH, bool VERIFY, bool LDSM = false>
__global__ __launch_bounds__(kBlock, MESH ? 1 : (FIRST ? kProduceWavesFirst : kProduceWaves))
void k_sort_produce(const KArgs A, const SortArgs SA) {
    __shared__ DMaterial s_mats[kLdsMats];
    __shared__ LGeom s_geoms[MESH ? 1 : kLdsGeoms];
    __shared__ float s_frm[MESH || FIRST ? 1 : kLdsGeoms * 36];   // the cubes' tangent frames (stage_frames)
    __shared__ int32_t s_sb[kMaxSpp + 1];      // work start of every iteration (first bounce: j * npix)
    __shared__ int32_t s_fb[kMaxSpp + 1];      // sorted start of every iteration (RNG key base)
    __shared__ int32_t s_tb[kMaxSpp + 1];      // first tile of every iteration ([spp] = all tiles)
    __shared__ uint32_t s_tmp[8];
    __shared__ uint32_t s_mw[4];
    __shared__ uint32_t s_base[kSortMaxMats];  // the tile's exclusive prefix over materials: survivors
    __shared__ uint32_t s_kbase[kSortMaxMats]; // ... and records (survivors that go on)
    extern __shared__ uint32_t s_kc[];   // [2][2][4][nmats] (dynamic): per wave, survivors of each material in the tile
#define KC(buf, w, m) s_kc[((buf) * 4 + (w)) * nmats + (m)]
#define KL(buf, w, m) s_kc[(8 + (buf) * 4 + (w)) * nmats + (m)]   // (those that did not end here)
    __shared__ uint32_t s_cnt[2];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int par = A.parity;
    const int spp = A.tile.spp;
    const int nmats = A.S.nmats;
    if (FIRST) {
        for (int j = tid; j <= spp; j += kBlock) s_sb[j] = s_fb[j] = j * A.tile.npix;
    } else {   // the scanned histograms at each iteration's first entry (the previous producer's tiles)
        const int32_t* tb_in = SA.itb + (size_t)par * (kMaxSpp + 1);
        for (int j = tid; j <= spp; j += kBlock) {
            s_sb[j] = SA.offs2[(size_t)tb_in[j] * nmats];
            s_fb[j] = SA.offs[(size_t)tb_in[j] * nmats];
        }
    }
    __syncthreads();
    {   // this launch's tiles: iteration it owns ceil(n_it / 256) of them, from s_tb[it]
        const uint32_t n = tid < spp ? (uint32_t)(s_sb[tid + 1] - s_sb[tid] + kBlock - 1) / kBlock : 0u;
        const uint32_t incl = lb::wave_inclusive_scan(n);
        if (lane == 63) s_tmp[wave] = incl;
        __syncthreads();
        uint32_t pre = incl - n;
        for (int q = 0; q < wave; ++q) pre += s_tmp[q];
        if (tid < spp) s_tb[tid] = (int32_t)pre;
        if (tid == 0) s_tb[spp] = (int32_t)(s_tmp[0] + s_tmp[1] + s_tmp[2] + s_tmp[3]);
        __syncthreads();
    }
    const int T = __builtin_amdgcn_readfirstlane(s_tb[spp]);
    if (blockIdx.x == 0) {
        if (tid == 0) {
            A.ctl[par ^ 1].nseg = (uint32_t)T;   // tiles of the output
            A.ctl[par ^ 1].chunk = (uint32_t)kBlock;
            A.ctl[par ^ 1].hist_live = (uint32_t)(T * nmats + 1);   // entries + the end offset
        }
        int32_t* tb_out = SA.itb + (size_t)(par ^ 1) * (kMaxSpp + 1);
        for (int j = tid; j <= spp; j += kBlock) tb_out[j] = s_tb[j];
        if (!FIRST) count_bounce(A, s_fb[spp]);   // the live paths of bounce b (with those that ended early)
    }
    if ((int)blockIdx.x >= T) return;
    if (!MESH) stage_geoms(A.S, s_geoms);
    if (!MESH && !FIRST) stage_frames(A.S, s_frm);
    stage_materials(A, s_mats);   // (its barrier publishes the staged tables)
    const bool lds_mats = LDSM || nmats <= kLdsMats;
    const bool lds_geoms = !MESH && (LDSM || A.S.ngeoms <= kLdsGeoms);   // (stage_geoms / stage_frames ran)
    const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint32_t emit_cnt = 0, emit_next = 0;
    int k = 0, it = 0;
    for (int t = (int)blockIdx.x; t < T; t += (int)gridDim.x, ++k) {
        const KArgs& A = fresh_args();   // (shadow the parameters: their fields are re-read per tile)
        const SortArgs& SA = fresh_param<SortArgs>((sizeof(KArgs) + alignof(SortArgs) - 1) / alignof(SortArgs) * alignof(SortArgs));
        it = tile_iteration_next(s_tb, spp, t, it);
        const int t0 = __builtin_amdgcn_readfirstlane(s_tb[it]), t1 = __builtin_amdgcn_readfirstlane(s_tb[it + 1]);
        const int it_base = __builtin_amdgcn_readfirstlane(s_sb[it]);
        const int it_end = __builtin_amdgcn_readfirstlane(s_sb[it + 1]);
        const int idx = it_base + (t - t0) * kBlock + tid;   // work position
        const int iter = A.tile.iter_first + it;
        bool alive = false, emitted = false;
        PathReg p;
        Hit h;
        bool ends = false;
        if (FIRST && !VERIFY && A.cmask) {
            // the whole tile's camera-mask blocks empty (workgroup-uniform): every ray misses — colour
            // 0 retired, one run of material 0 holding the tile's paths and no record; the tile's
            // ballots and barriers are skipped (k stays: the count buffers alternate per barrier)
            const int lp0 = idx - tid - it_base, nb = ((it_end - it_base) + 63) >> 6;
            uint32_t any = 0u;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const int b = (lp0 >> 6) + w;
                any |= b < nb ? A.cmask[b] : 0u;
            }
            if (any == 0u) {
                if (idx < it_end) {
                    PathReg z;
                    z.c = F3(0.0f, 0.0f, 0.0f);
                    z.slot = idx;
                    retire<SPP1>(A, z, it);
                }
                if (tid < nmats) {
                    const size_t e = sort_hidx(t0, t1, nmats, t, tid);
                    SA.hist[e] = tid == 0 ? min(kBlock, it_end - (idx - tid)) : 0;
                    SA.hist2[e] = 0;
                    SA.hslot[e] = t * kBlock;
                }
                --k;
                continue;
            }
        }
        bool skip = false;
        if (FIRST && !VERIFY && A.cmask) {
            const int lp0 = __builtin_amdgcn_readfirstlane(idx - it_base);
            skip = lp0 < it_end - it_base && A.cmask[lp0 >> 6] == 0u;
        }
        if (skip) {
            // A wave whose camera rays can hit no geom (mask 0) skips raygen and the closest hit: a
            // miss draws no random number and keeps only its slot and sort key 0 (shade_ends below).
            if (idx < it_end) {
                p.slot = idx;
                h = miss_hit();
                alive = true;
                ends = true;
            }
        } else if (idx < it_end) {
            if (FIRST) {   // (work position idx = iteration it's pixel idx - it * npix: a tile holds one iteration)
                raygen_at(A.cam, A.fl, A.tile, idx, it, idx - it_base, p);
                alive = true;
            } else {
                const v2i_pf pf = reinterpret_cast<const v2i_pf*>(SA.perm)[idx];
                const int j = pf[0], fp = pf[1];
                const v4f* r = srec(A.in, j);
                // (plain loads: a gather of 32-byte records)
                const v4f r0 = r[0], r1 = r[1];
                const f3 hitp = F3(r0[0], r0[1], r0[2]);
                p.c = F3(r0[3], r1[0], r1[1]);
                p.slot = __float_as_int(r1[2]);
                p.bounces = A.bounce;
                const int code = rec_code(__float_as_int(r1[3]));
                const uint32_t rank = rec_rank(__float_as_int(r1[3]));
                if (code >= 0) {   // a cube's slab: the geom's material, normal and frame
                    const int g = code / 6, f = code - 6 * g;
                    if (lds_geoms) {
                        h.mat = s_geoms[g].material;
                        h.n = F3(s_geoms[g].nrm[f][0], s_geoms[g].nrm[f][1], s_geoms[g].nrm[f][2]);
                    } else {
                        h.mat = A.S.geoms[g].material;
                        h.n = F3(A.S.geoms[g].nrm[f][0], A.S.geoms[g].nrm[f][1], A.S.geoms[g].nrm[f][2]);
                    }
                    h.frame = code;
                } else {
                    h.mat = -code - 1;
                    const v4f nv = snrm(A.in, j)[0];
                    h.n = F3(nv[0], nv[1], nv[2]);
                }
                h.u = h.v = 0.0f;
                p.d = F3(0, 0, 0);
                if (lds_mats ? mat_needs_dir(s_mats[h.mat]) : mat_needs_dir(A.S.mats[h.mat])) {
                    const v4f d = sdir(A.in, j)[0];
                    p.d = F3(d[0], d[1], d[2]);
                }
                if (A.S.texs) {
                    const bool tex = lds_mats ? s_mats[h.mat].texture_id != -1 : A.S.mats[h.mat].texture_id != -1;
                    if (tex) {
                        h.u = A.hit.uv[2 * (size_t)j];
                        h.v = A.hit.uv[2 * (size_t)j + 1];
                    }
                }
                // key: sorted index within the path's own iteration (paths that ended in the
                // previous launch hold positions too: fpos)
                const int key = A.fl.rng_pixel ? slot_pixel(A.cam, A.tile, p.slot) : (fp + (int)rank) - __builtin_amdgcn_readfirstlane(s_fb[it]);
                const float* frames = lds_geoms ? s_frm : nullptr;
                alive = lds_mats ? shade_from(A.S, A.fl, A.tile.depth, iter, key, p, h, hitp, s_mats, frames)
                                 : shade_from(A.S, A.fl, A.tile.depth, iter, key, p, h, hitp, A.S.mats, frames);
                if (!alive) {
                    emitted = p.c.x != 0.0f || p.c.y != 0.0f || p.c.z != 0.0f;
                    retire<SPP1>(A, p, it);
                }
            }
            uint32_t gm = ~0u;
            if (FIRST && A.cmask) {   // the wave's 64 pixels of its iteration (tiles are 256-aligned)
                const int lp0 = __builtin_amdgcn_readfirstlane(idx - it_base);
                gm = A.cmask[lp0 >> 6];
            }
            if (alive) {
                h = closest_hit<MESH, VERIFY, !FIRST, LDSM && !MESH>(A.S, A.fl, s_geoms, p.o, p.d, &A.stats->bound_mismatch, gm);
                PathReg e = p;   // (only the verdict here; the colour below)
                ends = lds_mats ? shade_ends(h, s_mats, e) : shade_ends(h, A.S.mats, e);
            }
        }
        const int key = alive ? (h.t == -1.0f ? 0 : h.mat) : -1;   // misses keep materialId 0 (pathtrace.cu:466)
        emit_cnt += (uint32_t)__popcll(__ballot(emitted));
        const uint64_t m = __ballot(alive), me = __ballot(ends);
        // this wave's row of per-material counts: cleared, then one ballot per material present ->
        // in-wave rank (lanes of that key) and the count (written by the first lane of the key).
        // Buffer k&1 was last read two tiles ago, before the previous barrier; a wave's LDS
        // writes land in order.
#pragma unroll
        for (int q = 0; q < kSortMaxMats / 64; ++q)   // (fixed trip count: a dynamic loop here cost 34 VGPRs)
            if (lane + 64 * q < nmats) KC(k & 1, wave, lane + 64 * q) = KL(k & 1, wave, lane + 64 * q) = 0u;
        uint32_t krank = 0, krank2 = 0;
        uint64_t rem = m;
        while (rem) {
            const int src = __builtin_ctzll(rem);
            const int kk = __builtin_amdgcn_readlane(key, src);
            const uint64_t mk = __ballot(key == kk);
            if (key == kk) {
                krank = (uint32_t)__popcll(mk & lt);
                krank2 = (uint32_t)__popcll(mk & ~me & lt);
            }
            if (lane == src) {
                KC(k & 1, wave, kk) = (uint32_t)__popcll(mk);
                KL(k & 1, wave, kk) = (uint32_t)__popcll(mk & ~me);
            }
            rem &= ~mk;
        }
        __syncthreads();
        {   // material mm = tid: the tile's survivor and record counts and their exclusive prefixes over
            // the materials (one scan of both, 16 bits each: counts <= 256); the histogram entries
            const int mm = tid;
            const uint32_t cm = mm < nmats ? (KC(k & 1, 0, mm) + KC(k & 1, 1, mm)) + (KC(k & 1, 2, mm) + KC(k & 1, 3, mm)) : 0u;
            const uint32_t cl = mm < nmats ? (KL(k & 1, 0, mm) + KL(k & 1, 1, mm)) + (KL(k & 1, 2, mm) + KL(k & 1, 3, mm)) : 0u;
            uint32_t tot;
            const uint32_t bb = block_excl_scan(cm | (cl << 16), s_mw, &tot);   // (its barriers: s_base's readers are done)
            if (mm < nmats) {
                s_base[mm] = bb & 0xffffu;
                s_kbase[mm] = bb >> 16;
                const size_t e = sort_hidx(t0, t1, nmats, t, mm);
                SA.hist[e] = (int32_t)cm;
                SA.hist2[e] = (int32_t)cl;
                SA.hslot[e] = t * kBlock + (int32_t)(bb >> 16);
            }
        }
        __syncthreads();
        bool em_next = false;
        if (alive) {
            // kb: the survivor's rank among the tile's same-material survivors (its sorted position
            // is its run's + kb); kb2: among those that go on (its record's place in the run)
            uint32_t kb = krank, kb2 = krank2;
            for (int w = 0; w < wave; ++w) {
                kb += KC(k & 1, w, key);
                kb2 += KL(k & 1, w, key);
            }
            // A path whose new ray misses or meets an emitter ends at the next shade without drawing
            // a random number (shade_ends): it keeps its sorted position (hist counts it, so the
            // next launch's RNG keys do), but ends here — retired with the colour that shade would
            // give it, no record written, and no work position in the next launch (hist2 leaves it out).
            if (ends) {
                PathReg e = p;
                (void)(lds_mats ? shade_ends(h, s_mats, e) : shade_ends(h, A.S.mats, e));
                em_next = e.c.x != 0.0f || e.c.y != 0.0f || e.c.z != 0.0f;
                retire<SPP1>(A, e, it);
            } else {
                const int q = t * kBlock + (int)(s_kbase[key] + kb2);
                v4f* r = srec(A.out, q);
                // (plain stores: each store instruction covers 16 of every 32 bytes, and L2 merges the
                // two into whole lines; non-temporal ones halved config 3's rate)
                const f3 hitp = point_on_ray(p.o, p.d, h.t);
                const int code = h.frame >= 0 ? h.frame : -(h.mat + 1);
                r[0] = v4f{hitp.x, hitp.y, hitp.z, p.c.x};
                r[1] = v4f{p.c.y, p.c.z, __int_as_float(p.slot), __int_as_float(rec_pack(code, kb))};
                if (code < 0) snrm(A.out, q)[0] = v4f{h.n.x, h.n.y, h.n.z, 0.0f};
                if (lds_mats ? mat_needs_dir(s_mats[h.mat]) : mat_needs_dir(A.S.mats[h.mat]))
                    sdir(A.out, q)[0] = v4f{p.d.x, p.d.y, p.d.z, 0.0f};
                if (A.S.texs) {
                    SA.uv_out[2 * (size_t)q] = h.u;
                    SA.uv_out[2 * (size_t)q + 1] = h.v;
                }
            }
        }
        emit_next += (uint32_t)__popcll(__ballot(em_next));
    }
    // (the camera rays' ends are bounce 0's; a later producer's are the next bounce's)
    flush_emissive2(A, emit_cnt, FIRST ? A.bounce : A.bounce + 1, emit_next, s_cnt);
#undef KC
#undef KL
}

// Exclusive scan of the sorted pipeline's histogram when two lanes share the GPU: reduce, scan of
// the tile sums (one workgroup), rescan.  No workgroup waits on another, so unlike the library's
// single-pass scan (whose static schedule needs its whole grid co-resident) two of these can run
// side by side.  The histogram is small (nmats x paths / 64 ints) and cache-resident.
constexpr int kHistPer = 4;                        // ints per thread (one 16-byte load)
constexpr int kHistTile = kBlock * kHistPer;       // 1024: 4x the workgroups of 4096 (latency-bound scan)

typedef int v4i_h __attribute__((ext_vector_type(4)));
// this thread's kHistPer consecutive ints (16-byte loads; guarded at the end of the array)
__device__ __forceinline__ void hist_load(const int32_t* __restrict__ in, int64_t n, int64_t base, uint32_t (&x)[kHistPer]) {
    if (base + kHistPer <= n) {
#pragma unroll
        for (int q = 0; q < kHistPer / 4; ++q) {
            const v4i_h v = *reinterpret_cast<const v4i_h*>(in + base + 4 * q);
#pragma unroll
            for (int e = 0; e < 4; ++e) x[4 * q + e] = (uint32_t)v[e];
        }
    } else {
#pragma unroll
        for (int k = 0; k < kHistPer; ++k) x[k] = base + k < n ? (uint32_t)in[base + k] : 0u;
    }
}

// n: capacity; *nlive (if given): the live entry count (<= n), written by the producer.
__device__ __forceinline__ int64_t hist_n(int64_t n, const uint32_t* nlive) {
    return nlive ? (int64_t)min((uint64_t)n, (uint64_t)*nlive) : n;
}
// The two histograms (hist: every survivor, the sorted positions; hist2: those that did not end in
// the producer, the next producer's work positions) are scanned side by side: sums[2 b] and
// sums[2 b + 1] are workgroup b's totals.
__global__ __launch_bounds__(kBlock) void k_hist_sums(const int32_t* __restrict__ in, const int32_t* __restrict__ in2,
                                                      int64_t n, const uint32_t* nlive, uint32_t* __restrict__ sums) {
    __shared__ uint32_t s_w[4], s_w2[4];
    n = hist_n(n, nlive);
    // (a grid-stride loop over blocks of kHistTile entries: the grid is sized for the capacity, the
    // live length is read here, and later bounces use a few blocks)
    for (int64_t blk = blockIdx.x; blk * kHistTile < n; blk += gridDim.x) {
        const int64_t base = blk * kHistTile + (int64_t)threadIdx.x * kHistPer;
        uint32_t x[kHistPer], y[kHistPer], v = 0, v2 = 0;
        hist_load(in, n, base, x);
        hist_load(in2, n, base, y);
#pragma unroll
        for (int k = 0; k < kHistPer; ++k) { v += x[k]; v2 += y[k]; }
        uint32_t total, total2;
        (void)block_excl_scan(v, s_w, &total);
        (void)block_excl_scan(v2, s_w2, &total2);
        if (threadIdx.x == 0) { sums[2 * blk] = total; sums[2 * blk + 1] = total2; }
    }
}

__global__ __launch_bounds__(kBlock) void k_hist_scan_sums(uint32_t* __restrict__ sums, int64_t n, const uint32_t* nlive) {
    __shared__ uint32_t s_w[4], s_w2[4];
    const int tiles = (int)((hist_n(n, nlive) + kHistTile - 1) / kHistTile);
    const int per = (tiles + kBlock - 1) / kBlock;
    const int j0 = (int)threadIdx.x * per;
    uint32_t v = 0, v2 = 0;
    for (int j = j0; j < j0 + per && j < tiles; ++j) { v += sums[2 * j]; v2 += sums[2 * j + 1]; }
    uint32_t total, total2;
    uint32_t run = block_excl_scan(v, s_w, &total), run2 = block_excl_scan(v2, s_w2, &total2);
    for (int j = j0; j < j0 + per && j < tiles; ++j) {
        const uint32_t a = sums[2 * j], b = sums[2 * j + 1];
        sums[2 * j] = run;
        sums[2 * j + 1] = run2;
        run += a;
        run2 += b;
    }
}

__device__ __forceinline__ void hist_store(int32_t* __restrict__ out, int64_t n, int64_t base, uint32_t run,
                                           const uint32_t (&x)[kHistPer]) {
    if (base + kHistPer <= n) {
#pragma unroll
        for (int q = 0; q < kHistPer / 4; ++q) {
            v4i_h o;
#pragma unroll
            for (int e = 0; e < 4; ++e) { o[e] = (int32_t)run; run += x[4 * q + e]; }
            *reinterpret_cast<v4i_h*>(out + base + 4 * q) = o;
        }
    } else {
#pragma unroll
        for (int k = 0; k < kHistPer; ++k) {
            if (base + k < n) out[base + k] = (int32_t)run;
            run += x[k];
        }
    }
}

// The scans (out: sorted positions, out2: work positions) and the next producer's work list: for
// the live entries but the last (the end offset, whose count is not written), run e's records
// hslot[e] + i (i < in2[e]: the survivors that go on, stored consecutively by the producer) at work
// positions out2[e] + i, each with its run's sorted position out[e] (the record adds its rank).
__global__ __launch_bounds__(kBlock) void k_hist_apply(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                       const int32_t* __restrict__ in2, int32_t* __restrict__ out2,
                                                       int64_t n, const uint32_t* nlive, const uint32_t* __restrict__ sums,
                                                       const int32_t* __restrict__ hslot, int32_t* __restrict__ perm,
                                                       int32_t* __restrict__ fpos) {
    __shared__ uint32_t s_w[4], s_w2[4];
    n = hist_n(n, nlive);
    const int lane = (int)threadIdx.x & 63;
    for (int64_t blk = blockIdx.x; blk * kHistTile < n; blk += gridDim.x) {   // (as k_hist_sums)
        const int64_t base = blk * kHistTile + (int64_t)threadIdx.x * kHistPer;
        uint32_t x[kHistPer], y[kHistPer], v = 0, v2 = 0;
        hist_load(in, n, base, x);
        hist_load(in2, n, base, y);
#pragma unroll
        for (int k = 0; k < kHistPer; ++k) { v += x[k]; v2 += y[k]; }
        uint32_t total, total2;
        const uint32_t run = block_excl_scan(v, s_w, &total) + sums[2 * blk];
        const uint32_t run2 = block_excl_scan(v2, s_w2, &total2) + sums[2 * blk + 1];
        int32_t s0[kHistPer];
#pragma unroll
        for (int k = 0; k < kHistPer; ++k) s0[k] = (base + k < n - 1 && y[k] != 0u) ? hslot[base + k] : 0;
        uint32_t o = run, o2 = run2;
#pragma unroll
        for (int k = 0; k < kHistPer; ++k) {   // the wave writes its entries' runs one after the other
            uint64_t rem = __ballot(base + k < n - 1 && y[k] != 0u);
            while (rem) {
                const int src = __builtin_ctzll(rem);
                const uint32_t ro = __builtin_amdgcn_readlane(o, src), ro2 = __builtin_amdgcn_readlane(o2, src);
                const uint32_t rl = __builtin_amdgcn_readlane(y[k], src);
                const int32_t rs = __builtin_amdgcn_readlane(s0[k], src);
                for (uint32_t r = (uint32_t)lane; r < rl; r += 64)   // 64 consecutive positions per store
                    pf_store(perm, fpos, ro2 + r, rs + (int32_t)r, (int32_t)ro);
                rem &= rem - 1;
            }
            o += x[k];
            o2 += y[k];
        }
        hist_store(out, n, base, run, x);
        hist_store(out2, n, base, run2, y);
    }
}

// spp > 1: add the per-slot colours in sample order (finalGather as `spp` sequential iterations).
constexpr int kFinBatch = 16;
// finalGather of a batched pass: each pixel's colours added in sample order.  Only flagged slots hold
// a colour (retire); the others are zero colours, whose additions are identities once the sum is not
// -0 — colours are never -0 (products and sums of non-negative factors, or +0), so one +0 added first
// (turning an accumulator of -0, which only pt_set_accum can give, into +0) and the flagged colours in
// order give the bits that adding every slot's colour gave.  The flags are cleared for the next pass.
__global__ void k_finalize_spp(float* __restrict__ image, const v4f* __restrict__ col, uint8_t* __restrict__ flag,
                               int npix, int spp) {
    for (int lp = blockIdx.x * blockDim.x + threadIdx.x; lp < npix; lp += gridDim.x * blockDim.x) {
        float r = image[3 * (size_t)lp] + 0.0f, g = image[3 * (size_t)lp + 1] + 0.0f, b = image[3 * (size_t)lp + 2] + 0.0f;
        uint8_t* row = flag + (size_t)lp * (size_t)spp;
        int s = 0;
        if ((spp & 15) == 0 && (((size_t)row) & 15) == 0) {   // 16 flags per load (row starts 16-byte aligned)
            for (; s < spp; s += 16) {
                uint4 f = *reinterpret_cast<const uint4*>(row + s);
                if ((f.x | f.y | f.z | f.w) == 0u) continue;
                *reinterpret_cast<uint4*>(row + s) = make_uint4(0u, 0u, 0u, 0u);
                const uint32_t w[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    for (uint32_t m = w[q]; m != 0u; m &= m - 1u) {   // flagged bytes (each holds 1) in sample order
                        const int k = 4 * q + (__builtin_ctz(m) >> 3);
                        const v4f c = PT_LD(col + (size_t)(s + k) * npix + lp);
                        r += c[0]; g += c[1]; b += c[2];
                    }
            }
        } else {
            for (; s < spp; ++s)
                if (row[s]) {
                    row[s] = 0;
                    const v4f c = PT_LD(col + (size_t)s * npix + lp);
                    r += c[0]; g += c[1]; b += c[2];
                }
        }
        image[3 * (size_t)lp] = r; image[3 * (size_t)lp + 1] = g; image[3 * (size_t)lp + 2] = b;
    }
}

// Render-ahead claim (add != 0: the iteration's colours into the image — k_finalize_spp with one
// sample — and its counts into the context's) or drop (add == 0: the counts zeroed, device errors
// kept).  Emissive counts: `rows` bounces of `stride` per-workgroup slots.
__global__ void k_ahead_settle(float* __restrict__ image, const v4f* __restrict__ col, uint8_t* __restrict__ flag, int npix,
                               DevStats* __restrict__ st, DevStats* __restrict__ ast, unsigned long long* __restrict__ emit,
                               unsigned long long* __restrict__ aemit, int nemit, int add) {
    const int gid = blockIdx.x * blockDim.x + threadIdx.x, gsz = gridDim.x * blockDim.x;
    for (int lp = gid; lp < npix; lp += gsz) {   // (a dropped iteration's flags are cleared too)
        const bool f = flag[lp] != 0;
        if (f) flag[lp] = 0;
        if (add) {
            // the flagged colour, else the zero colour retire did not store (k_finalize_spp)
            const v4f c = f ? PT_LD(col + lp) : v4f{0.0f, 0.0f, 0.0f, 0.0f};
            image[3 * (size_t)lp] += c[0]; image[3 * (size_t)lp + 1] += c[1]; image[3 * (size_t)lp + 2] += c[2];
        }
    }
    for (int j = gid; j < nemit; j += gsz) {
        const unsigned long long v = aemit[j];
        if (v) {
            if (add) emit[j] += v;
            aemit[j] = 0ull;
        }
    }
    if (gid < 66) {   // segments, passes, bounce_live[64]
        unsigned long long* a = gid == 0 ? &ast->segments : (gid == 1 ? &ast->passes : &ast->bounce_live[gid - 2]);
        unsigned long long* b = gid == 0 ? &st->segments : (gid == 1 ? &st->passes : &st->bounce_live[gid - 2]);
        if (add) *b += *a;
        *a = 0ull;
    } else if (gid == 66) {
        st->err |= ast->err;
        st->bound_mismatch += ast->bound_mismatch;
        ast->err = 0u;
        ast->bound_mismatch = 0u;
    }
}

// sendImageToPBO (pathtrace.cu:64-86)
__global__ void k_preview(const float* __restrict__ image, uint8_t* __restrict__ rgba, int npix, int iter) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < npix; i += gridDim.x * blockDim.x) {
        for (int k = 0; k < 3; ++k) {
            int v = (int)((double)(image[3 * (size_t)i + k] / iter) * 255.0);
            v = v < 0 ? 0 : (v > 255 ? 255 : v);
            rgba[4 * (size_t)i + k] = (uint8_t)v;
        }
        rgba[4 * (size_t)i + 3] = 0;
    }
}

// pt_selftest_math: the range-gated cores of pt_device.h against the library sqrtf and '/'.
__device__ __forceinline__ bool same_bits(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}
__device__ __forceinline__ float selftest_operand(uint32_t h, uint64_t i, int slot) {
    const uint32_t kind = (uint32_t)(i >> 2) % 16u;
    if ((i & 3) == 0) return __uint_as_float((h & 0x807fffffu) | ((0x70u + ((h >> 23) & 0x1fu)) << 23));   // |x| in [2^-15, 2^17)
    if (kind == 0 && slot == 0) {   // edge operands
        const float e[8] = {0.0f, -0.0f, 1e-45f, -3e-39f, __builtin_inff(), -__builtin_inff(), __builtin_nanf(""), 0x1p-40f};
        return e[(h >> 3) & 7];
    }
    return __uint_as_float(h);
}
__global__ void k_selftest_math(uint64_t n, uint32_t seed, unsigned long long* bad) {
    unsigned long long e = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t h1 = utilhash((uint32_t)i ^ seed ^ (uint32_t)(i >> 32) * 0x9e3779b9u);
        const uint32_t h2 = utilhash(h1 + 0x7f4a7c15u), h3 = utilhash(h2 ^ 0x85ebca6bu);
        const float x = selftest_operand(h1, i, 0), y = selftest_operand(h2, i, 1), z = selftest_operand(h3, i, 2);
        e += same_bits(sqrt_cr(fabsf(x)), sqrtf(fabsf(x))) ? 0 : 1;
        e += same_bits(sqrt_cr(x), sqrtf(x)) ? 0 : 1;
        e += same_bits(div_cr(x, y), x / y) ? 0 : 1;
        e += same_bits(div_cr(1.0f, y), 1.0f / y) ? 0 : 1;
        float q1, q2;
        div2_cr(x, z, y, q1, q2);
        e += same_bits(q1, x / y) ? 0 : 1;
        e += same_bits(q2, z / y) ? 0 : 1;
        const f3 v = F3(x, y, z), nv = normalize(v), rv = v * (1.0f / sqrtf(dot(v, v)));
        e += (same_bits(nv.x, rv.x) && same_bits(nv.y, rv.y) && same_bits(nv.z, rv.z)) ? 0 : 1;
        e += same_bits(length(v), sqrtf(dot(v, v))) ? 0 : 1;
    }
    if (e) atomicAdd(bad, e);
}

// ------------------------------------------------------------------------------------------
// Host context
// ------------------------------------------------------------------------------------------
#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return pt::fail(PT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e)); \
    } while (0)

struct ProfEv {
    hipEvent_t a, b;
    int kind;
};

}  // namespace

// Compute streams held by the live contexts of this process (pt_ctx::busy_streams), against the
// hardware queues HIP gives one priority level of a process (GPU_MAX_HW_QUEUES, default 4).
static std::atomic<int> g_busy_streams{0};
static int stream_budget() {
    const char* q = std::getenv("GPU_MAX_HW_QUEUES");
    const int n = q ? std::atoi(q) : 0;
    return n > 0 ? n : 4;
}

struct pt_ctx {
    int device = 0;
    int depth = 8;
    int nmats = 0;
    pt_flags flags{};
    KArgs args{};
    int max_tiles = 0, max_t64 = 0;
    int grid_trace = 0, grid_compact = 0;
    int grid_bounce[2] = {};   // k_bounce (later, first bounce): one full wave of workgroups
    bool fused = true;   // pipeline: fused bounce kernel (default) or trace + compact
    uint64_t compact_launches = 0;   // parity of the look-back status / live-count words
    uint64_t n_cmask_builds = 0, n_flag_syncs = 0;   // pt_ctx_counters
    double cmask_empty = 0.0;    // share of the camera-mask blocks whose mask is empty (build_cmask)
    bool cmask_skip = false;     // the fused first bounce's empty-wave instantiation is in use
    // owned device allocations
    std::vector<void*> allocs;
    PathSoA buf[2]{};
    int cur = 0;
    DevStats* stats = nullptr;
    bool profiling = false;
    std::vector<ProfEv> events;   // pool; the first `ev_used` are recorded and unread
    size_t ev_used = 0;
    size_t path_cap = 0;          // entries per path buffer (>= P, see pt_create)
    std::vector<DGeom> hgeoms;    // host copy of the geom table (bounds re-derived by pt_set_flags)
    uint32_t* d_cmask = nullptr;  // first-bounce geom masks, one per 64 tile pixels (build_cmask)
    DGeom* d_geoms = nullptr;
    DGeom* d_bgeoms = nullptr;    // the same geoms ordered by bound kind (SceneDev::bgeoms)
    double scene_ext = 0.0;       // max |coordinate| over every surface and the camera position
    // Batched passes (spp > 1): pass p's path colours go to colbuf half h = p & 1 and are added
    // into the image by k_finalize_spp on fin_stream, concurrently with the next pass's bounces
    // on the caller's stream (memory-bound finalize beside the VALU-bound first bounce).  A pass
    // waits for the finalize still reading its half; image readers wait for the last one.
    v4f* colbuf = nullptr;        // 2 x P
    // Lanes (fused pipeline, spp >= 2): a pass's iterations are split in two; lane 0 traces the
    // first ceil(spp/2) on the caller's stream with the buffers above, lane 1 the rest on
    // lane_stream with its own path buffers and control words.  The lanes are independent (every
    // path's RNG keys and colour slot depend only on its iteration), so one lane's first bounce,
    // short tail bounces and launch gaps overlap the other's work.  PT_AMD_LANES=1 disables.
    // The caller's stream does not wait for lanes 1.. at the end of a pass (async_lanes): only the
    // pass's finalize does, so the next pass's lane 0 starts while their tail bounces still run;
    // lanes 1.. of the next pass wait for the caller's stream (lane 0 of this pass, the colour half).
    // PT_AMD_SYNC_LANES=1 joins every lane into the caller's stream instead.
    int lanes = 1;                       // lanes 1.. use the arrays below; lane 0 the context's own
    bool async_lanes = true;
    PathSoA lbuf[kMaxLanes][2]{};
    Ctl* lctl[kMaxLanes] = {};
    int32_t* lseg[kMaxLanes] = {};
    unsigned long long* lemit[kMaxLanes] = {};
    uint64_t llaunches[kMaxLanes] = {};
    hipStream_t lane_stream[kMaxLanes] = {};
    hipEvent_t ev_fork = nullptr, ev_join[kMaxLanes] = {};
    struct SortSet {   // material-sort buffers of one lane (k_sort_produce / k_hist_*)
        int32_t *hslot = nullptr, *hist = nullptr, *offs = nullptr, *perm = nullptr, *itb = nullptr;
        int32_t *hist2 = nullptr, *offs2 = nullptr, *fpos = nullptr;
        float* uv[2] = {nullptr, nullptr};   // (u, v) of the records in buf[0] / buf[1]
        uint32_t* sums = nullptr;            // histogram scan: tile sums
        int64_t hist_cap = 0;                // histogram entries allocated (+ the end offset)
    } sset[kMaxLanes];
    // Mesh scenes: the BVH walk runs in k_traverse ahead of k_bounce<.., kMeshPre> (mesh_mode 2) when
    // the BVH is on and the geom table fits LDS; otherwise inside k_bounce (kMeshInline).
    v4f* mhit[kMaxLanes] = {};           // per lane, indexed by physical path slot
    size_t lcap[kMaxLanes] = {};         // path capacity of each lane's buffers
    bool mesh_inline = false;            // PT_AMD_MESH_INLINE=1 at pt_create: always kMeshInline
    uint32_t* tq = nullptr;              // k_traverse ray tickets: [lane][bounce], zeroed per pass
    int grid_traverse = 0;               // k_traverse: one resident wave of workgroups
    int grid_traverse4 = 0;              // k_traverse4 (4-wide layout): the same for its footprint
    int cus = 256;                       // compute units of the device
    int quad_occ = 0;                    // k_traverse4: bound on its stack occupancy (build_quads)
    double tcull_frac = 0.0;             // share of quad slots whose exact t-cull margin can pay (build_qcull)
    bool trav_quads = false;             // mesh mode 2 walks the 4-wide layout (PT_AMD_TRAV=pairs: off)
    int walk_k = kT4K;                   // k_traverse4's triangle tasks per lane: kT4K, 1 with the exact t-cull
    hipStream_t fin_stream = nullptr;
    hipEvent_t ev_pass[2] = {}, ev_fin[2] = {};
    bool fin_out[2] = {false, false};
    int col_half = 0, last_fin = -1;
    // Context-scoped synchronisation (no hipDeviceSynchronize, no synchronous copy on the legacy
    // default stream): ev_done is recorded after the last work this context enqueued (a pass ends
    // with it on the stream that finishes the pass: the caller's, or the finalize stream, which the
    // lanes join); the synchronous entry points wait for that event alone and move data on io_stream,
    // a non-blocking stream of their own.  So reading one context's image does not wait for another
    // context's passes, nor for unrelated work elsewhere on the GPU.
    hipStream_t io_stream = nullptr;
    hipEvent_t ev_done = nullptr;
    bool done_recorded = false;
    hipStream_t done_stream = nullptr;   // the stream ev_done was last recorded on
    int busy_streams = 0;                // compute streams this context holds (stream budget, below)
    bool lanes_capped = false;           // pt_create gave it fewer lanes than it would alone
    hipStream_t pass_stream = nullptr;   // the caller's stream of the last pass or render-ahead
    // Render-ahead (one-iteration contexts, pt_render_ahead): the bounces of iteration ahead_iter,
    // queued before the call that asks for it, keep their colours in ahead_col and their counts in
    // ahead_stats / ahead_emit until pt_render_pass claims them (the same iteration and flags: the
    // colours are added into the image then, as finalGather would) or drops them (anything else).
    // Ordering, on any mix of streams: an ahead pass first waits for the context's last work
    // (ev_done: the last pass, claim settle or image call) when that was on another stream, and every
    // later pass — and the next ahead pass, whose drop settle rewrites ahead_col — waits for ev_ahead.
    v4f* ahead_col = nullptr;
    DevStats* ahead_stats = nullptr;
    unsigned long long* ahead_emit = nullptr;
    hipEvent_t ev_ahead = nullptr;
    bool ahead_recorded = false, ahead_valid = false;
    int32_t ahead_iter = 0;
    pt_flags ahead_flags{};
    uint8_t* colflag = nullptr;   // 2 x P flag bytes (KArgs::colflag), pass halves like colbuf; zero between passes
    uint8_t* ahead_flag = nullptr;   // npix flag bytes of the render-ahead colours

    ~pt_ctx() {
        g_busy_streams.fetch_sub(busy_streams);
        for (auto& e : events) { (void)hipEventDestroy(e.a); (void)hipEventDestroy(e.b); }
        for (int h = 0; h < 2; ++h) {
            if (ev_pass[h]) (void)hipEventDestroy(ev_pass[h]);
            if (ev_fin[h]) (void)hipEventDestroy(ev_fin[h]);
        }
        if (fin_stream) (void)hipStreamDestroy(fin_stream);
        if (io_stream) (void)hipStreamDestroy(io_stream);
        if (ev_done) (void)hipEventDestroy(ev_done);
        if (ev_ahead) (void)hipEventDestroy(ev_ahead);
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        for (int l = 0; l < kMaxLanes; ++l) {
            if (ev_join[l]) (void)hipEventDestroy(ev_join[l]);
            if (lane_stream[l]) (void)hipStreamDestroy(lane_stream[l]);
        }
        for (void* p : allocs) (void)hipFree(p);
    }
    template <typename T>
    int alloc(T** p, size_t count) {
        void* q = nullptr;
        const size_t bytes_ = std::max<size_t>(count * sizeof(T), 16);
        hipError_t e = hipMalloc(&q, bytes_);
        if (e != hipSuccess) return pt::fail(PT_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        allocs.push_back(q);
        *p = static_cast<T*>(q);
        return PT_OK;
    }
};

namespace {

// Synchronous copy on the context's own non-blocking stream (pt_ctx::io_stream): unlike hipMemcpy,
// which runs on the legacy default stream, it waits for nothing but itself.
hipError_t io_copy(pt_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
    if (!c->io_stream) return hipMemcpy(dst, src, bytes, kind);   // (pt_create, before the stream exists)
    hipError_t e = hipMemcpyAsync(dst, src, bytes, kind, c->io_stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->io_stream);
    return e;
}

// Wait for everything this context has enqueued so far (pt_ctx::ev_done).
int wait_ctx(pt_ctx* c) {
    if (c->done_recorded) HIP_TRY(hipEventSynchronize(c->ev_done));
    return PT_OK;
}
int mark_ctx(pt_ctx* c, hipStream_t s) {
    HIP_TRY(hipEventRecord(c->ev_done, s));
    c->done_recorded = true;
    c->done_stream = s;
    return PT_OK;
}
// Work about to be queued on st that shares the context's path buffers, control words or ahead
// buffers waits for everything the context queued before, when that went to another stream (on
// the same stream, stream order already holds).
int order_after_ctx(pt_ctx* c, hipStream_t st) {
    if (c->done_recorded && c->done_stream != st) HIP_TRY(hipStreamWaitEvent(st, c->ev_done, 0));
    return PT_OK;
}

void set_flags_dev(pt_ctx* c, const pt_flags& f) {
    c->flags = f;
    c->args.fl.rr = f.russian_roulette;
    c->args.fl.bvh = f.use_bvh;
    c->args.fl.bbox = f.use_bbox;
    c->args.fl.ssaa = f.ssaa;
    c->args.fl.dof = f.dof;
    c->args.fl.aperture = f.aperture;
    c->args.fl.focal = f.focal_dist;
    c->args.fl.single_albedo = f.single_albedo;
    c->args.fl.bvh_cull = f.bvh_cull;
    c->args.fl.claimed = f.shared_gpu;
    c->args.fl.rng_pixel = f.rng_key_pixel;
    const char* vb = std::getenv("PT_AMD_VERIFY_BOUNDS");
    c->args.fl.verify = vb && std::strcmp(vb, "1") == 0;
}

float bits_to_float(int32_t v) {
    float f;
    std::memcpy(&f, &v, 4);
    return f;
}
int32_t __float_as_int_host(float f) {
    int32_t v;
    std::memcpy(&v, &f, 4);
    return v;
}

Affine to_affine(const float* m) {   // glm column-major 4x4 -> 3x4 + the exact w=0 terms
    Affine a;
    for (int col = 0; col < 4; ++col)
        for (int r = 0; r < 3; ++r) a.c[col][r] = m[4 * col + r];
    for (int r = 0; r < 3; ++r) a.z3[r] = m[12 + r] * 0.0f;
    return a;
}

// Widened bounds of the bounded closest-hit pass (bound_geom), sized from R = the largest
// |coordinate| any ray origin can have: a surface point (+1e-4 offsets) or the camera lens.
//   qo = inv * ro is computed with <= 4 ulp of S_a = sum_i |inv_ia| R + |inv_3a| absolute error by
// either side (exact test, bounds test), the exact slab parameters add <= 5 ulp of (S_a + 0.5):
// mu_a = 2^-18 (S_a + 1) is >= 10x that.  The sphere's b^2 - a c cancels to <= 2^-20 (S + 1)^2:
// kappa = 2^-16 (S + 1)^2.  tslack covers the back-transform (transform * inverse != I in float)
// and the rounding of the reference's length(); abs_slack its absolute part.
void update_bounds(pt_ctx* c, float aperture) {
    const double R = c->scene_ext + std::fabs((double)aperture) + 1e-2;
    for (DGeom& d : c->hgeoms) {
        double smax = 0.0;
        for (int a = 0; a < 3; ++a) {
            double S = std::fabs((double)d.inv.c[3][a]);
            for (int i = 0; i < 3; ++i) S += std::fabs((double)d.inv.c[i][a]) * R;
            const double mu = std::ldexp(S + 1.0, -18);
            d.slo[a] = (float)(-0.5 - mu);
            d.shi[a] = (float)(0.5 + mu);
            smax = std::max(smax, S);
        }
        d.r2w = (float)(0.25 + std::ldexp((smax + 1.0) * (smax + 1.0), -16));
        // departing-ray test: |qo_exact - qo_bound| <= 2^-21 S_ray (S_ray <= cs |ro|_inf + c3) moves
        // |qo|^2 by <= 2^-20 |qo| S_ray; the dot products add <= 2^-21 |qo|^2.  kappa_ray is >= 6x that.
        double cs = 0.0, c3 = 0.0;
        for (int a = 0; a < 3; ++a) {
            cs = std::max(cs, std::fabs((double)d.inv.c[0][a]) + std::fabs((double)d.inv.c[1][a]) +
                                  std::fabs((double)d.inv.c[2][a]));
            c3 = std::max(c3, std::fabs((double)d.inv.c[3][a]));
        }
        d.kcs = (float)std::ldexp(cs, -18);
        d.kc3 = (float)std::ldexp(c3 + 2.0, -18);
        d.bkind = d.type == PT_GEOM_CUBE ? 1 : (d.type == PT_GEOM_SPHERE ? 2 : 0);
        if (d.type == PT_GEOM_SPHERE) {
            // uniform scale (x rotation): G = L^T L = sigma^2 I up to delta, L = the linear part of inv
            double G[3][3], tr = 0.0, dev = 0.0;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) {
                    G[i][j] = 0.0;
                    for (int a = 0; a < 3; ++a) G[i][j] += (double)d.inv.c[i][a] * (double)d.inv.c[j][a];
                }
            for (int i = 0; i < 3; ++i) tr += G[i][i];
            const double s2 = tr / 3.0;
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) dev = std::max(dev, std::fabs(G[i][j] - (i == j ? s2 : 0.0)));
            if (s2 > 0.0 && dev <= std::ldexp(s2, -20)) {
                // the world-space dot products differ from the object-space ones by the
                // non-uniformity (<= 2^-20 relative) and the rounding of w = ro - centre (within the
                // 4 ulp of S_a assumed above): margins doubled
                for (int k = 0; k < 3; ++k) d.wlo[k] = d.xf.c[3][k];
                d.whi[0] = (float)s2;
                // bound_sphere_tagged's per-geom constants: 1 / is2 and the pull-back factor
                // 1.0002e-4 / sqrt(is2), rounded up (is2 as the device reads it, a float)
                d.whi[1] = (float)(1.0 / (double)d.whi[0]);
                d.back = std::nextafter((float)(1.0002e-4 / std::sqrt((double)d.whi[0])), HUGE_VALF);
                d.r2w = (float)(0.25 + std::ldexp((smax + 1.0) * (smax + 1.0), -15));
                d.kcs *= 2.0f;
                d.kc3 *= 2.0f;
                d.bkind = 4;
            }
        }
        if (d.type == PT_GEOM_CUBE) {   // world box of the widened cube, if the transform is axis-aligned
            double M[3][3], X[3][3];
            for (int r = 0; r < 3; ++r)
                for (int k = 0; k < 3; ++k) M[r][k] = d.inv.c[k][r];   // q = M p + t
            const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                               M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
                               M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
            bool aligned = std::fabs(det) > 0.0;
            if (aligned) {
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k) {
                        const int r1 = (k + 1) % 3, r2 = (k + 2) % 3, k1 = (r + 1) % 3, k2 = (r + 2) % 3;
                        X[r][k] = (M[r1][k1] * M[r2][k2] - M[r1][k2] * M[r2][k1]) / det;   // adjugate / det
                    }
                for (int r = 0; r < 3 && aligned; ++r) {
                    double big = 0.0;
                    for (int k = 0; k < 3; ++k) big = std::max(big, std::fabs(X[r][k]));
                    int n = 0;
                    for (int k = 0; k < 3; ++k) n += std::fabs(X[r][k]) > 1e-6 * big;
                    aligned = n == 1;
                }
            }
            if (aligned) {
                double stretch = 0.0, lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
                for (int corner = 0; corner < 8; ++corner) {
                    double q[3];
                    for (int k = 0; k < 3; ++k) q[k] = ((corner >> k) & 1 ? d.shi[k] : d.slo[k]) - d.inv.c[3][k];
                    for (int r = 0; r < 3; ++r) {
                        const double v = X[r][0] * q[0] + X[r][1] * q[1] + X[r][2] * q[2];
                        lo[r] = std::min(lo[r], v);
                        hi[r] = std::max(hi[r], v);
                    }
                }
                for (int r = 0; r < 3; ++r)
                    for (int k = 0; k < 3; ++k) stretch = std::max(stretch, std::fabs(X[r][k]));
                const double pad = std::ldexp(R + 1.0, -18);
                for (int r = 0; r < 3; ++r) {
                    d.wlo[r] = (float)(lo[r] - pad - std::ldexp(std::fabs(lo[r]), -18));
                    d.whi[r] = (float)(hi[r] + pad + std::ldexp(std::fabs(hi[r]), -18));
                }
                d.back = (float)(1.0002e-4 * stretch * (1.0 + 1e-5));
                for (int r = 0; r < 3; ++r) {
                    d.wbox[2 * r] = d.wlo[r];
                    d.wbox[2 * r + 1] = d.whi[r];
                }
                d.bkind = 3;
            } else {
                // oriented cube (bkind 1): bound_obox_tagged's pull-back factor, 1.0002e-4 / sigma_min(L)
                // bounded by the Frobenius norm of X = L^-1 (a singular L: +inf, the bound is then 0)
                double fro = HUGE_VAL;
                if (std::fabs(det) > 0.0) {   // (X is computed above exactly then)
                    fro = 0.0;
                    for (int r = 0; r < 3; ++r)
                        for (int k = 0; k < 3; ++k) fro += X[r][k] * X[r][k];
                }
                d.back = std::isfinite(fro) ? std::nextafter((float)(1.0002e-4 * std::sqrt(fro) * (1.0 + 1e-5)), HUGE_VALF)
                                            : HUGE_VALF;
            }
        }
        double dev = 0.0;   // Frobenius norm of xf_lin * inv_lin - I
        for (int r = 0; r < 3; ++r)
            for (int col = 0; col < 3; ++col) {
                double m = 0.0;
                for (int k = 0; k < 3; ++k) m += (double)d.xf.c[k][r] * (double)d.inv.c[col][k];
                m -= r == col ? 1.0 : 0.0;
                dev += m * m;
            }
        d.tslack = (float)(1.0 - 4.0 * std::sqrt(dev) - std::ldexp(1.0, -14));
    }
    c->args.S.abs_slack = (float)std::ldexp(R + 1.0, -17);
    // bound_wbox_tagged: one tslack for every world-box cube (their smallest), folded into the pull-back
    float ts = 1.0f;
    for (const DGeom& d : c->hgeoms)
        if (d.bkind == 3) ts = std::min(ts, d.tslack);
    c->args.S.wb_tslack = ts;
    for (DGeom& d : c->hgeoms)
        d.wback = d.bkind == 3 ? std::nextafter((float)((double)d.back * (double)ts), HUGE_VALF) : 0.0f;
}

// ---- first-bounce geom masks ----------------------------------------------------------------
// A wave of the first bounce traces 64 consecutive tile pixels of one iteration.  Every camera
// ray of those pixels (any SSAA jitter in [0, 1) pixel, any lens sample within the aperture) is
//   o + s (F - o), s >= 0,   o in cam.pos + [-a, a]^2 x {0},   F in the focal-plane image of the
// pixels' rectangle (DoF; raygen's focus point, pathtrace.cu:203-224), or
//   cam.pos + s v,           v in the span of the rectangle's view vectors (no DoF).
// Bounding o and F - o (or v) by boxes and asking, axis by axis, for a common s >= 0 at which the
// ray box meets a geom's world box gives a conservative "can hit" test (never false for a ray that
// hits).  The geom's box is its test region [slo, shi]^3 (already wider than the exact test's
// rounding, update_bounds) mapped by the exact inverse of `inv`, padded again.  A geom outside the
// mask is skipped by the bounds pass of those rays: the closest hit is unchanged (intersect_bounded).
static bool beam_meets_box(const double olo[3], const double ohi[3], const double dlo[3], const double dhi[3],
                           const double blo[3], const double bhi[3]) {
    double smin = 0.0, smax = HUGE_VAL;
    for (int k = 0; k < 3; ++k) {
        // o_lo + s d_lo <= b_hi  and  o_hi + s d_hi >= b_lo  (the ray box's extent along axis k at s)
        const double c1 = bhi[k] - olo[k], c2 = blo[k] - ohi[k];
        if (dlo[k] > 0.0) smax = std::min(smax, c1 / dlo[k]);
        else if (dlo[k] < 0.0) smin = std::max(smin, c1 / dlo[k]);
        else if (c1 < 0.0) return false;
        if (dhi[k] > 0.0) smin = std::max(smin, c2 / dhi[k]);
        else if (dhi[k] < 0.0) smax = std::min(smax, c2 / dhi[k]);
        else if (c2 > 0.0) return false;
    }
    return smin <= smax * (1.0 + 1e-9) + 1e-12;
}

int build_cmask(pt_ctx* c) {
    KArgs& A = c->args;
    A.cmask = nullptr;
    ++c->n_cmask_builds;
    c->cmask_empty = 0.0;
    c->cmask_skip = false;
    const int ng = A.S.ngeoms;
    const char* off = std::getenv("PT_AMD_NO_CMASK");
    if ((off && std::strcmp(off, "1") == 0) || ng <= 0 || ng > kLdsGeoms || A.S.ntris > 0) return PT_OK;
    const TileDev& T = A.tile;
    const CamDev& cam = A.cam;
    const size_t nblk = ((size_t)T.npix + 63) / 64;
    if (!c->d_cmask)
        if (int rc = c->alloc(&c->d_cmask, nblk)) return rc;
    // world boxes of the geoms' test regions
    std::vector<std::array<double, 6>> gb((size_t)ng);
    std::vector<bool> always((size_t)ng, false);
    for (int g = 0; g < ng; ++g) {
        const DGeom& d = c->hgeoms[(size_t)g];
        if (d.type != PT_GEOM_CUBE && d.type != PT_GEOM_SPHERE) { always[(size_t)g] = true; continue; }
        double M[3][3], X[3][3];
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) M[r][k] = d.inv.c[k][r];   // q = M p + t
        const double det = M[0][0] * (M[1][1] * M[2][2] - M[1][2] * M[2][1]) -
                           M[0][1] * (M[1][0] * M[2][2] - M[1][2] * M[2][0]) +
                           M[0][2] * (M[1][0] * M[2][1] - M[1][1] * M[2][0]);
        if (!(std::fabs(det) > 0.0) || !std::isfinite(det)) { always[(size_t)g] = true; continue; }
        for (int r = 0; r < 3; ++r)
            for (int k = 0; k < 3; ++k) {
                const int r1 = (k + 1) % 3, r2 = (k + 2) % 3, k1 = (r + 1) % 3, k2 = (r + 2) % 3;
                X[r][k] = (M[r1][k1] * M[r2][k2] - M[r1][k2] * M[r2][k1]) / det;
            }
        const double rs = d.type == PT_GEOM_SPHERE ? std::sqrt(std::max(0.0, (double)d.r2w)) : 0.0;
        double lo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, hi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
        for (int corner = 0; corner < 8; ++corner) {
            double q[3];
            for (int k = 0; k < 3; ++k) {
                const double a = std::min((double)d.slo[k], -rs), b = std::max((double)d.shi[k], rs);
                q[k] = ((corner >> k) & 1 ? b : a) * (1.0 + 1e-4) - d.inv.c[3][k];
            }
            for (int r = 0; r < 3; ++r) {
                const double v = X[r][0] * q[0] + X[r][1] * q[1] + X[r][2] * q[2];
                lo[r] = std::min(lo[r], v);
                hi[r] = std::max(hi[r], v);
            }
        }
        for (int r = 0; r < 3; ++r) {
            const double pad = 1e-3 + 1e-5 * std::max(std::fabs(lo[r]), std::fabs(hi[r]));
            gb[(size_t)g][r] = lo[r] - pad;
            gb[(size_t)g][3 + r] = hi[r] + pad;
        }
        if (!std::isfinite(gb[(size_t)g][0] + gb[(size_t)g][1] + gb[(size_t)g][2] + gb[(size_t)g][3] +
                           gb[(size_t)g][4] + gb[(size_t)g][5]))
            always[(size_t)g] = true;
    }
    const double pos[3] = {cam.pos[0], cam.pos[1], cam.pos[2]};
    const double jit = A.fl.ssaa ? 1.0 : 0.0, eps = 0.01;   // pixel units
    const bool dof = A.fl.dof != 0;
    const double ap = std::fabs((double)A.fl.aperture), focal = A.fl.focal;
    // rays of tile row `row`, tile columns [x0, x1]: their geoms
    auto row_mask = [&](int row, int x0, int x1) -> uint32_t {
        const int y = row * T.world + T.rank;
        const double ax0 = x0 - cam.res[0] * 0.5 - eps, ax1 = x1 - cam.res[0] * 0.5 + jit + eps;
        const double ay0 = y - cam.res[1] * 0.5 - eps, ay1 = y - cam.res[1] * 0.5 + jit + eps;
        double v[4][3];
        for (int q = 0; q < 4; ++q) {
            const double ax = q & 1 ? ax1 : ax0, ay = q & 2 ? ay1 : ay0;
            for (int k = 0; k < 3; ++k)
                v[q][k] = (double)cam.view[k] - (double)cam.right[k] * cam.pl[0] * ax - (double)cam.up[k] * cam.pl[1] * ay;
        }
        double olo[3], ohi[3], dlo[3], dhi[3];
        if (!dof) {
            for (int k = 0; k < 3; ++k) {
                olo[k] = pos[k] - 1e-4 * (1.0 + std::fabs(pos[k]));
                ohi[k] = pos[k] + 1e-4 * (1.0 + std::fabs(pos[k]));
                dlo[k] = std::min({v[0][k], v[1][k], v[2][k], v[3][k]});
                dhi[k] = std::max({v[0][k], v[1][k], v[2][k], v[3][k]});
                const double m = 1e-5 * (std::fabs(dlo[k]) + std::fabs(dhi[k]) + 1e-3);
                dlo[k] -= m;
                dhi[k] += m;
            }
        } else {
            double flo[3] = {HUGE_VAL, HUGE_VAL, HUGE_VAL}, fhi[3] = {-HUGE_VAL, -HUGE_VAL, -HUGE_VAL};
            int sign = 0;
            for (int q = 0; q < 4; ++q) {
                const double n = std::sqrt(v[q][0] * v[q][0] + v[q][1] * v[q][1] + v[q][2] * v[q][2]);
                const int sg = v[q][2] > 0.0 ? 1 : -1;
                if (!(std::fabs(v[q][2]) > 1e-3 * n) || (sign != 0 && sg != sign)) return ~0u;   // focus plane unbounded
                sign = sg;
                for (int k = 0; k < 3; ++k) {
                    const double f = pos[k] + focal * v[q][k] / std::fabs(v[q][2]);
                    flo[k] = std::min(flo[k], f);
                    fhi[k] = std::max(fhi[k], f);
                }
            }
            for (int k = 0; k < 3; ++k) {
                const double fp = 1e-4 * (1.0 + std::fabs(flo[k]) + std::fabs(fhi[k]));
                const double a = k < 2 ? ap * (1.0 + 1e-4) + 1e-6 : 1e-6;
                olo[k] = pos[k] - a - 1e-4 * (1.0 + std::fabs(pos[k]));
                ohi[k] = pos[k] + a + 1e-4 * (1.0 + std::fabs(pos[k]));
                dlo[k] = (flo[k] - fp) - ohi[k];
                dhi[k] = (fhi[k] + fp) - olo[k];
            }
        }
        uint32_t m = 0u;
        for (int g = 0; g < ng; ++g)
            if (always[(size_t)g] || beam_meets_box(olo, ohi, dlo, dhi, &gb[(size_t)g][0], &gb[(size_t)g][3]))
                m |= 1u << g;
        return m;
    };
    std::vector<uint32_t> mask(nblk, 0u);
    for (size_t b = 0; b < nblk; ++b) {
        const int lp0 = (int)(b * 64), lp1 = std::min(T.npix - 1, lp0 + 63);
        const int r0 = lp0 / T.W, r1 = lp1 / T.W;
        uint32_t m = 0u;
        for (int r = r0; r <= r1; ++r)
            m |= row_mask(r, r == r0 ? lp0 - r * T.W : 0, r == r1 ? lp1 - r * T.W : T.W - 1);
        mask[b] = m;
    }
    if (const char* st = std::getenv("PT_AMD_CMASK_STATS")) {
        if (std::strcmp(st, "1") == 0) {
            double tot = 0.0;
            for (uint32_t m : mask) tot += __builtin_popcount(m);
            std::fprintf(stderr, "[pt_amd] camera masks: %zu blocks, %.2f of %d geoms per block\n", nblk, tot / (double)nblk, ng);
        }
    }
    hipError_t e = io_copy(c, c->d_cmask, mask.data(), nblk * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) return pt::fail(PT_ERR_HIP, std::string("camera masks: ") + hipGetErrorString(e));
    A.cmask = c->d_cmask;
    size_t empty = 0;
    for (uint32_t m : mask) empty += m == 0u;
    c->cmask_empty = nblk ? (double)empty / (double)nblk : 0.0;
    c->cmask_skip = c->cmask_empty >= kSkipEmptyMin;
    if (const char* sk = std::getenv("PT_AMD_SKIP_EMPTY")) {   // A/B and tests: 0 never, 1 always
        if (std::strcmp(sk, "0") == 0) c->cmask_skip = false;
        if (std::strcmp(sk, "1") == 0) c->cmask_skip = true;
    }
    return PT_OK;
}

// One block of 4P planes per parity: the fused / split pipelines use the first three as the
// a, b, c planes; the sorted pipeline uses the first two as P 32-byte records (srec), the third
// for the ray directions of specular hits (sdir) and the fourth for normals not held by a code.
int alloc_paths(pt_ctx* c, PathSoA& B, size_t P) {
    if (int rc = c->alloc(&B.a, 4 * P)) return rc;
    B.b = B.a + P;
    B.c = reinterpret_cast<v2f*>(B.a + 2 * P);
    return PT_OK;
}

int prof_begin(pt_ctx* c, hipStream_t st, int kind, ProfEv** out) {
    *out = nullptr;
    if (!c->profiling) return PT_OK;
    if (c->ev_used == c->events.size()) {
        ProfEv ev{};
        HIP_TRY(hipEventCreate(&ev.a));
        HIP_TRY(hipEventCreate(&ev.b));
        c->events.push_back(ev);
    }
    ProfEv* ev = &c->events[c->ev_used++];
    ev->kind = kind;
    HIP_TRY(hipEventRecord(ev->a, st));
    *out = ev;
    return PT_OK;
}
int prof_end(ProfEv* ev, hipStream_t st) {
    if (ev) HIP_TRY(hipEventRecord(ev->b, st));
    return PT_OK;
}

// Workgroups per CU that are guaranteed co-resident for a persistent look-back kernel: the
// occupancy API's answer, lowered while LDS or VGPRs would be filled (almost) exactly.  Measured:
// five 32 KiB-LDS workgroups per CU are not all resident (scripts/probes/residency.hip), and a
// k_bounce variant at 7 x 72 VGPRs per SIMD stalled its look-back; 2 x 176 VGPRs and 3 x 48 KiB
// LDS are fine.  Budget: <= 448 of 512 VGPRs per SIMD lane, <= 152 KiB of 160 KiB LDS per CU.
int resident_per_cu(const void* kernel) {
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0) != hipSuccess || per_cu <= 0)
        return 1;
    per_cu = std::min(per_cu, 8);
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, kernel) != hipSuccess) return std::max(1, per_cu - 1);
    const int vgpr = ((fa.numRegs + 7) / 8) * 8;
    const size_t lds = fa.sharedSizeBytes;
    while (per_cu > 1 && ((size_t)per_cu * lds > (size_t)(152 * 1024) || per_cu * vgpr > 448)) --per_cu;
    return per_cu;
}

// Dynamic LDS of k_bounce: the scene's geom rows (analytic scenes of <= kLdsGeoms geoms) and
// materials (<= kLdsMats); Cornell needs 1.6 KiB instead of a fixed 12 KiB.
size_t bounce_lds_bytes(const SceneDev& S, int mesh) {
    const int g = (mesh == kMeshInline || S.ngeoms > kLdsGeoms) ? 0 : S.ngeoms;
    const int m = std::min(S.nmats, kLdsMats);
    return (size_t)g * sizeof(LGeom) + (size_t)m * sizeof(DMaterial) + (size_t)g * 36 * sizeof(float);
}

// k_bounce's mesh mode for the current flags (see pt_ctx::mhit).
int mesh_mode(const pt_ctx* c) {
    const SceneDev& S = c->args.S;
    if (S.ntris == 0) return 0;
    return (c->args.fl.bvh && S.nnodes > 0 && S.ngeoms <= kLdsGeoms && c->mhit[0] && !c->mesh_inline) ? kMeshPre
                                                                                                     : kMeshInline;
}

using KernelFn = void (*)(const KArgs);
KernelFn bounce_kernel(bool first, bool spp1, int mesh, bool skip = false, bool gmats = false) {   // mesh: 0, kMeshInline, kMeshPre
    if (mesh == 0 && gmats) {   // (more materials than kLdsMats)
        static const KernelFn gm[4] = {k_bounce<false, false, kAnalyticGM>, k_bounce<false, true, kAnalyticGM>,
                                       k_bounce<true, false, kAnalyticGM>, k_bounce<true, true, kAnalyticGM>};
        return gm[(first ? 2 : 0) + (spp1 ? 1 : 0)];
    }
    if (first && skip && mesh == 0) return spp1 ? k_bounce<true, true, kAnalyticSkip> : k_bounce<true, false, kAnalyticSkip>;
    static const KernelFn table[12] = {
        k_bounce<false, false, 0>, k_bounce<false, false, 1>, k_bounce<false, false, 2>,
        k_bounce<false, true, 0>,  k_bounce<false, true, 1>,  k_bounce<false, true, 2>,
        k_bounce<true, false, 0>,  k_bounce<true, false, 1>,  k_bounce<true, false, 2>,
        k_bounce<true, true, 0>,   k_bounce<true, true, 1>,   k_bounce<true, true, 2>};
    return table[(first ? 6 : 0) + (spp1 ? 3 : 0) + mesh];
}
KernelFn trace_kernel(bool first, bool spp1, bool mesh) {
    static const KernelFn table[8] = {
        k_trace<false, false, false>, k_trace<false, false, true>, k_trace<false, true, false>,
        k_trace<false, true, true>,   k_trace<true, false, false>, k_trace<true, false, true>,
        k_trace<true, true, false>,   k_trace<true, true, true>};
    return table[(first ? 4 : 0) + (spp1 ? 2 : 0) + (mesh ? 1 : 0)];
}

using SortKernelFn = void (*)(const KArgs, const SortArgs);
SortKernelFn produce_kernel(bool first, bool spp1, bool mesh, bool verify, bool ldsm = false) {
    if (ldsm && !verify) {
        static const SortKernelFn lt[8] = {
            k_sort_produce<false, false, false, false, true>, k_sort_produce<false, false, true, false, true>,
            k_sort_produce<false, true, false, false, true>,  k_sort_produce<false, true, true, false, true>,
            k_sort_produce<true, false, false, false, true>,  k_sort_produce<true, false, true, false, true>,
            k_sort_produce<true, true, false, false, true>,   k_sort_produce<true, true, true, false, true>};
        return lt[(first ? 4 : 0) + (spp1 ? 2 : 0) + (mesh ? 1 : 0)];
    }
    static const SortKernelFn table[16] = {
        k_sort_produce<false, false, false, false>, k_sort_produce<false, false, true, false>,
        k_sort_produce<false, true, false, false>,  k_sort_produce<false, true, true, false>,
        k_sort_produce<true, false, false, false>,  k_sort_produce<true, false, true, false>,
        k_sort_produce<true, true, false, false>,   k_sort_produce<true, true, true, false>,
        k_sort_produce<false, false, false, true>,  k_sort_produce<false, false, true, true>,
        k_sort_produce<false, true, false, true>,   k_sort_produce<false, true, true, true>,
        k_sort_produce<true, false, false, true>,   k_sort_produce<true, false, true, true>,
        k_sort_produce<true, true, false, true>,    k_sort_produce<true, true, true, true>};
    return table[(verify ? 8 : 0) + (first ? 4 : 0) + (spp1 ? 2 : 0) + (mesh ? 1 : 0)];
}

template <typename K>
int launch_k(pt_ctx* c, K kernel, int grid, hipStream_t st, int kind, const KArgs& a, size_t lds = 0) {
    ProfEv* ev;
    if (int rc = prof_begin(c, st, kind, &ev)) return rc;
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(kBlock), lds, st, a);
    HIP_TRY(hipGetLastError());
    return prof_end(ev, st);
}

// One bounce of the fused pipeline: [k_traverse (mesh mode 2)] + k_bounce.  Profiled as two kinds:
// the walk (PT_KIND_TRAVERSE / PT_KIND_FIRST_TRAVERSE) and the bounce kernel (PT_KIND_BOUNCE /
// PT_KIND_FIRST_BOUNCE), each bracketed by its own events on the launch stream.
// `cap`: path capacity of the lane's buffers (k_traverse's later-bounce grid covers every slot).
int launch_bounce(pt_ctx* c, bool first, bool spp1, int mesh, hipStream_t st, const KArgs& a, size_t cap) {
    ProfEv* ev;
    (void)cap;
    if (mesh == kMeshPre) {
        if (int rc = prof_begin(c, st, first ? PT_KIND_FIRST_TRAVERSE : PT_KIND_TRAVERSE, &ev)) return rc;
        const size_t lds = (size_t)a.stack_rows * kBlock * sizeof(int);
        const bool quad = c->trav_quads && !a.fl.bvh_cull;
        if (quad && c->walk_k == 1) {
            if (first) hipLaunchKernelGGL((k_traverse4<true, 1>), dim3(c->grid_traverse4), dim3(kBlock), lds, st, a);
            else hipLaunchKernelGGL((k_traverse4<false, 1>), dim3(c->grid_traverse4), dim3(kBlock), lds, st, a);
        } else if (quad && first) hipLaunchKernelGGL((k_traverse4<true, kT4K>), dim3(c->grid_traverse4), dim3(kBlock), lds, st, a);
        else if (quad) hipLaunchKernelGGL((k_traverse4<false, kT4K>), dim3(c->grid_traverse4), dim3(kBlock), lds, st, a);
        else if (first) hipLaunchKernelGGL(k_traverse<true>, dim3(c->grid_traverse), dim3(kBlock), lds, st, a);
        else hipLaunchKernelGGL(k_traverse<false>, dim3(c->grid_traverse), dim3(kBlock), lds, st, a);
        HIP_TRY(hipGetLastError());
        if (int rc = prof_end(ev, st)) return rc;
    }
    if (int rc = prof_begin(c, st, first ? PT_KIND_FIRST_BOUNCE : PT_KIND_BOUNCE, &ev)) return rc;
    hipLaunchKernelGGL(bounce_kernel(first, spp1, mesh, first && c->cmask_skip, a.S.nmats > kLdsMats || a.S.ngeoms > kLdsGeoms),
                       dim3(c->grid_bounce[first]), dim3(kBlock),
                       bounce_lds_bytes(a.S, mesh), st, a);
    HIP_TRY(hipGetLastError());
    return prof_end(ev, st);
}

// The 4-wide layout (DQuad) of the flattened tree `nodes` (DNode encoding: left child = i + 1).
// An interior child X of a quad's node is replaced by its two children when both boxes lie inside
// X's box as floats (the nesting k_traverse4's exactness rests on); otherwise it keeps one slot.
// Also bounds the walk's stack: per quad (valid slots - 1) pushes, summed along the worst path.
// Leaves of zero triangles (never built by the SAH builder) or a bound beyond the stack's capacity
// leave the quad layout off (k_traverse's pair walk runs instead).
// The flattened reference tree (BVH_tree.h:54-61) in the device encoding (DNode).
std::vector<DNode> to_dnodes(const std::vector<pt_bvh_node>& bvh) {
    std::vector<DNode> nodes(bvh.size());
    for (size_t i = 0; i < bvh.size(); ++i) {
        const pt_bvh_node& b = bvh[i];
        const int32_t meta = b.sub_areas > 0 ? b.sub_areas : -(b.axis + 1);
        const int32_t link = b.sub_areas > 0 ? b.first_area_idx : b.rchild_idx;
        for (int k = 0; k < 3; ++k) { nodes[i].lo[k] = b.bmin[k]; nodes[i].hi[k] = b.bmax[k]; }
        nodes[i].lo[3] = bits_to_float(meta);
        nodes[i].hi[3] = bits_to_float(link);
    }
    return nodes;
}

// Host part: fills `quads`, the root's code and the stack bound; false = no quad layout.
bool make_quads(const std::vector<DNode>& nodes, std::vector<DQuad>& quads, int32_t& root_code, int32_t& root_occ,
                std::vector<int32_t>* slot_node = nullptr) {
    const size_t n = nodes.size();
    quads.clear();
    if (slot_node) slot_node->clear();
    if (n == 0) return false;
    auto meta = [&](size_t i) { return __float_as_int_host(nodes[i].lo[3]); };
    auto link = [&](size_t i) { return __float_as_int_host(nodes[i].hi[3]); };
    for (size_t i = 0; i < n; ++i)
        if (meta(i) == 0 || (meta(i) < 0 && (link(i) <= (int32_t)i + 1 || (size_t)link(i) >= n)))
            return false;   // (a zero-triangle leaf is indistinguishable here; malformed links)
    auto inside = [&](size_t in, size_t out) {
        for (int k = 0; k < 3; ++k)
            if (!(nodes[in].lo[k] >= nodes[out].lo[k] && nodes[in].hi[k] <= nodes[out].hi[k])) return false;
        return true;
    };
    std::vector<int32_t> occ;   // stack bound of the walk below each quad
    std::vector<int32_t> qid(n, -1);
    auto leaf_code = [&](size_t i) { return -(link(i) * 256 + meta(i)) - 1; };
    // first pass: assign quad ids in DFS order
    std::vector<size_t> order;
    {
        std::vector<size_t> stk{0};
        if (meta(0) > 0) stk.clear();
        while (!stk.empty()) {
            const size_t i = stk.back();
            stk.pop_back();
            qid[i] = (int32_t)order.size();
            order.push_back(i);
            const size_t ch[2] = {i + 1, (size_t)link(i)};
            std::vector<size_t> kids;
            for (size_t x : ch) {
                if (meta(x) > 0) continue;
                const size_t g[2] = {x + 1, (size_t)link(x)};
                if (inside(g[0], x) && inside(g[1], x)) {
                    for (size_t y : g)
                        if (meta(y) <= 0) kids.push_back(y);
                } else {
                    kids.push_back(x);
                }
            }
            for (auto it = kids.rbegin(); it != kids.rend(); ++it) stk.push_back(*it);
        }
    }
    if (order.size() > (size_t)kQuadIdxMask) return false;
    quads.resize(std::max<size_t>(order.size(), 1));
    if (slot_node) slot_node->assign(4 * quads.size(), -1);
    occ.assign(order.size(), 0);
    // each quad's meta first: the interior codes pointing at a quad carry it
    std::vector<uint32_t> qmeta(order.size(), 0);
    for (size_t qi = 0; qi < order.size(); ++qi) {
        const size_t i = order[qi];
        uint32_t valid = 0, axes[2] = {3u, 3u};
        const size_t ch[2] = {i + 1, (size_t)link(i)};
        for (int g = 0; g < 2; ++g) {
            const size_t x = ch[g];
            if (meta(x) <= 0 && inside(x + 1, x) && inside((size_t)link(x), x)) {
                valid |= 3u << (2 * g);
                axes[g] = (uint32_t)(-meta(x) - 1);
            } else {
                valid |= 1u << (2 * g);
            }
        }
        qmeta[qi] = valid | ((uint32_t)(-meta(i) - 1) << 4) | (axes[0] << 6) | (axes[1] << 8);
    }
    auto qcode = [&](size_t y) { return (int32_t)((uint32_t)qid[y] | (qmeta[(size_t)qid[y]] << kQuadMetaShift)); };
    for (size_t qi = 0; qi < order.size(); ++qi) {
        const size_t i = order[qi];
        DQuad& Q = quads[qi];
        std::memset(&Q, 0, sizeof Q);
        uint32_t valid = 0, axes[2] = {3u, 3u};
        int32_t codes[4] = {0, 0, 0, 0};
        size_t box[4] = {0, 0, 0, 0};
        const size_t ch[2] = {i + 1, (size_t)link(i)};
        for (int g = 0; g < 2; ++g) {
            const size_t x = ch[g];
            auto slot = [&](int s, size_t y) {
                valid |= 1u << s;
                box[s] = y;
                codes[s] = meta(y) > 0 ? leaf_code(y) : qcode(y);
                if (slot_node) (*slot_node)[4 * qi + (size_t)s] = (int32_t)y;
            };
            if (meta(x) <= 0 && inside(x + 1, x) && inside((size_t)link(x), x)) {
                slot(2 * g, x + 1);
                slot(2 * g + 1, (size_t)link(x));
                axes[g] = (uint32_t)(-meta(x) - 1);
            } else {
                slot(2 * g, x);
            }
        }
        for (int s = 0; s < 4; ++s) {
            const DNode& b = nodes[box[s]];
            Q.lox[s] = b.lo[0]; Q.hix[s] = b.hi[0];
            Q.loy[s] = b.lo[1]; Q.hiy[s] = b.hi[1];
            Q.loz[s] = b.lo[2]; Q.hiz[s] = b.hi[2];
            Q.code[s] = bits_to_float(codes[s]);
        }
        const uint32_t m = valid | ((uint32_t)(-meta(i) - 1) << 4) | (axes[0] << 6) | (axes[1] << 8);
        Q.meta[0] = bits_to_float((int32_t)m);
    }
    // stack bound: children quads come later in DFS order, so a reverse sweep sees them first
    root_occ = 0;
    for (size_t qi = order.size(); qi-- > 0;) {
        const DQuad& Q = quads[qi];
        const uint32_t m = (uint32_t)__float_as_int_host(Q.meta[0]);
        int32_t deepest = 0, nv = 0;
        for (int s = 0; s < 4; ++s) {
            if (!((m >> s) & 1u)) continue;
            ++nv;
            const int32_t cd = __float_as_int_host(Q.code[s]);
            if (cd >= 0) deepest = std::max(deepest, occ[(size_t)(cd & kQuadIdxMask)]);
        }
        occ[qi] = nv - 1 + deepest;
        root_occ = occ[qi];
    }
    if (order.empty()) root_occ = 0;
    root_code = meta(0) > 0 ? leaf_code(0) : qcode(0);
    return root_occ <= 64;   // HybStack holds rows + 64 >= 64 entries
}

// IEEE binary16 bits of x >= 0 rounded down (toward 0) or up (toward +inf; +inf past the range).
uint16_t half_dir(double x, bool up) {
    if (!(x >= 0.0)) return up ? (uint16_t)0x7c00 : (uint16_t)0;
    auto val = [](uint16_t bits) {
        _Float16 t;
        std::memcpy(&t, &bits, 2);
        return (double)t;
    };
    const _Float16 h = (_Float16)(float)x;
    uint16_t b;
    std::memcpy(&b, &h, 2);
    if (up) {
        while (b < 0x7c00 && val(b) < x) ++b;
    } else {
        while (b > 0 && val(b) > x) --b;
    }
    return b;
}

// Exact t-cull margins of the 4-wide walk (DESIGN.md §4.3 "exact t-cull").  For a triangle with
// float edges e1, e2 that glm::intersectRayTriangle reports hit (gtx/intersect.inl:37-74: the
// determinant a >= FLT_EPSILON, barycentrics in range), its computed t satisfies
//     t >= (tau_min(B) - (g lambda + 4.8 u) diam / |d|) / (1 + g),   g = c (1 + u) / (1 - c),
//     c = (1 + u)(9 |e1||e2| |d| + 1.74 u),  lambda = 1 + 3.01 u,  diam = max(|e1|, |e2|),
// for every box B that holds the triangle, tau_min(B) = min over B of (X - o).d / |d|^2 (u = 2^-24).
// Per quad slot (a node of the reference tree) with the maxima of |e1||e2| and diam over its
// subtree: the slot's children are culled when A tau_lo > B + best (with relative slack), where
// A = 1 / ((1 + g)(1 + 2^-18)) (|d|^2 in [1 - 2^-18, 1 + 2^-18], checked per ray) rounded down and
// B = (g lambda + 4.8 u) diam / ((1 - 2^-19)(1 + g)) rounded up, both as binary16: one 32-bit word
// per slot, A | B << 16.  c >= 1 (large triangles): A = 0, B = inf, never culled.
// Returns the fraction of valid slots with A >= 1/2 (the share where the cull can pay).
double build_qcull(const std::vector<DNode>& nodes, const std::vector<pt_triangle>& tris,
                   const std::vector<int32_t>& slot_node, std::vector<uint32_t>& qcull) {
    const size_t n = nodes.size();
    std::vector<double> mmax(n, 0.0), dmax(n, 0.0);
    for (size_t i = n; i-- > 0;) {
        const int32_t meta = __float_as_int_host(nodes[i].lo[3]), link = __float_as_int_host(nodes[i].hi[3]);
        if (meta > 0) {
            for (int32_t k = link; k < link + meta && (size_t)k < tris.size(); ++k) {
                const pt_triangle& t = tris[(size_t)k];
                double l1 = 0.0, l2 = 0.0;
                for (int a = 0; a < 3; ++a) {
                    const float e1 = t.v[1][a] - t.v[0][a], e2 = t.v[2][a] - t.v[0][a];   // the device's e1, e2
                    l1 += (double)e1 * e1;
                    l2 += (double)e2 * e2;
                }
                l1 = std::sqrt(l1) * (1.0 + 1e-12);
                l2 = std::sqrt(l2) * (1.0 + 1e-12);
                mmax[i] = std::max(mmax[i], l1 * l2 * (1.0 + 1e-12));
                dmax[i] = std::max(dmax[i], std::max(l1, l2));
                if (!std::isfinite(l1 * l2)) mmax[i] = HUGE_VAL;
            }
        } else if ((size_t)link < n && i + 1 < n) {
            mmax[i] = std::max(mmax[i + 1], mmax[(size_t)link]);
            dmax[i] = std::max(dmax[i + 1], dmax[(size_t)link]);
        }
    }
    const double u = std::ldexp(1.0, -24), lam = 1.0 + 3.01 * u;
    const double dhi = 1.0 + std::ldexp(1.0, -19), dlo = 1.0 - std::ldexp(1.0, -19);
    qcull.assign(slot_node.size(), 0x7c000000u);   // A = 0, B = inf
    size_t valid = 0, good = 0;
    for (size_t k = 0; k < slot_node.size(); ++k) {
        const int32_t y = slot_node[k];
        if (y < 0) continue;
        ++valid;
        const double c = (1.0 + u) * (9.0 * mmax[(size_t)y] * dhi + 1.74 * u);
        if (!(c < 1.0)) continue;
        const double g = c * (1.0 + u) / (1.0 - c);
        const double A = 1.0 / ((1.0 + g) * (1.0 + std::ldexp(1.0, -18))) * (1.0 - 1e-12);
        const double B = (g * lam + 4.8 * u) * dmax[(size_t)y] / (dlo * (1.0 + g)) * (1.0 + 1e-12);
        qcull[k] = (uint32_t)half_dir(A, false) | ((uint32_t)half_dir(B, true) << 16);
        if (A >= 0.5) ++good;
    }
    return valid ? (double)good / (double)valid : 0.0;
}

int build_quads(pt_ctx* c, const std::vector<DNode>& nodes, const std::vector<pt_triangle>& tris) {
    std::vector<DQuad> quads;
    std::vector<int32_t> slot_node;
    int32_t root_code = 0, occ = 0;
    if (!make_quads(nodes, quads, root_code, occ, &slot_node)) return PT_OK;
    DQuad* d_quads;
    if (int rc = c->alloc(&d_quads, quads.size())) return rc;
    HIP_TRY(hipMemcpy(d_quads, quads.data(), quads.size() * sizeof(DQuad), hipMemcpyHostToDevice));
    c->args.S.quads = d_quads;
    c->args.S.root_qcode = root_code;
    c->quad_occ = occ;
    // exact t-cull: on when at least a quarter of the slots can cull (A >= 1/2), PT_AMD_TCULL=0/1 forces
    std::vector<uint32_t> qcull;
    c->tcull_frac = build_qcull(nodes, tris, slot_node, qcull);
    bool on = c->tcull_frac >= 0.25;
    if (const char* e = std::getenv("PT_AMD_TCULL")) on = std::strcmp(e, "1") == 0;
    c->args.S.qcull = nullptr;
    if (on) {
        uint32_t* d_q;
        if (int rc = c->alloc(&d_q, qcull.size())) return rc;
        HIP_TRY(hipMemcpy(d_q, qcull.data(), qcull.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
        c->args.S.qcull = d_q;
    }
    // triangle tasks per lane: kT4K, or 1 where the t-cull leaves few triangles per reached leaf
    // (PT_AMD_WALK_TASKS=1/2 forces one; the results are the same bits)
    c->walk_k = on ? 1 : kT4K;
    if (const char* wt = std::getenv("PT_AMD_WALK_TASKS")) c->walk_k = std::atoi(wt) == 1 ? 1 : kT4K;
    return PT_OK;
}

// SceneDev::bgeoms: the geom table stably ordered by bkind, each row keeping its index in `orig`.
int upload_bound_order(pt_ctx* c) {
    std::vector<DGeom> b;
    int32_t bk[6] = {0, 0, 0, 0, 0, 0};
    for (int k = 0; k < 5; ++k) {
        bk[k] = (int32_t)b.size();
        for (size_t i = 0; i < c->hgeoms.size(); ++i)
            if (c->hgeoms[i].bkind == k) {
                b.push_back(c->hgeoms[i]);
                b.back().orig = (int32_t)i;
            }
    }
    bk[5] = (int32_t)b.size();
    if (b.size() != c->hgeoms.size()) return pt::fail(PT_ERR_ARG, "geom with an unknown bound kind");
    HIP_TRY(io_copy(c, c->d_bgeoms, b.data(), b.size() * sizeof(DGeom), hipMemcpyHostToDevice));
    c->args.S.bgeoms = c->d_bgeoms;
    for (int k = 0; k < 6; ++k) c->args.S.bk[k] = bk[k];
    return PT_OK;
}

}  // namespace

extern "C" {

int pt_create(const pt_scene* scene, const pt_flags* flags, const pt_shard* shard, pt_ctx** out) {
    if (!scene || !out) return pt::fail(PT_ERR_ARG, "null argument");
    const auto& S = *reinterpret_cast<const pt::Scene*>(scene);
    if (!S.finalized) return pt::fail(PT_ERR_ARG, "scene not finalized (pt_scene_finalize)");
    if (S.materials.empty() || S.geoms.empty()) return pt::fail(PT_ERR_ARG, "scene has no geometry/materials");
    pt_shard sh{0, 1, 1, 0};
    if (shard) sh = *shard;
    if (sh.world < 1 || sh.rank < 0 || sh.rank >= sh.world || sh.spp < 1 || sh.spp > kMaxSpp)
        return pt::fail(PT_ERR_ARG, "bad shard (rank/world, or spp outside 1..256)");
    const int W = S.camera.res[0], H = S.camera.res[1];
    const int rows = (H - sh.rank + sh.world - 1) / sh.world;
    if (rows <= 0) return pt::fail(PT_ERR_ARG, "empty tile");
    const long long npix = (long long)rows * W;
    const long long P = npix * sh.spp;
    if (P > 0x7fffffffLL - 4096) return pt::fail(PT_ERR_ARG, "too many paths per pass");
    for (const auto& t : S.textures)
        if (t.pixels.empty()) return pt::fail(PT_ERR_ARG, "texture without pixels: " + t.path);

    auto* c = new pt_ctx();
    auto bail = [&](int rc) { delete c; return rc; };
    hipError_t e = hipGetDevice(&c->device);
    if (e != hipSuccess) return bail(pt::fail(PT_ERR_HIP, std::string("hipGetDevice: ") + hipGetErrorString(e)));
    c->depth = S.depth;
    c->nmats = (int)S.materials.size();
    KArgs& A = c->args;
    std::memset(&A, 0, sizeof A);
    set_flags_dev(c, flags ? *flags : [] { pt_flags f; pt_flags_default(&f); return f; }());

    // ---- scene upload ----
    std::vector<DGeom> dg(S.geoms.size());
    for (size_t i = 0; i < S.geoms.size(); ++i) {
        const pt_geom& g = S.geoms[i];
        DGeom& d = dg[i];
        std::memset(&d, 0, sizeof d);
        d.type = g.type;
        d.material = g.material_id;
        d.tri_start = g.tri_start;
        d.tri_end = g.tri_end;
        d.inv = to_affine(g.inverse_transform);
        d.xf = to_affine(g.transform);
        d.itr = to_affine(g.inv_transpose);
        if (d.type == PT_GEOM_CUBE)   // DGeom::nrm: glm's multiplyMV + normalize of each unit axis, in float32
            for (int code = 0; code < 6; ++code) {
                const float sg = (code & 1) ? -1.0f : 1.0f;
                const int a = code >> 1;
                const float n[3] = {a == 0 ? sg : 0.0f, a == 1 ? sg : 0.0f, a == 2 ? sg : 0.0f};
                float v[3];
                for (int r = 0; r < 3; ++r)
                    v[r] = (d.itr.c[0][r] * n[0] + d.itr.c[1][r] * n[1]) + (d.itr.c[2][r] * n[2] + d.itr.z3[r]);
                const float inv = 1.0f / std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
                for (int r = 0; r < 3; ++r) d.nrm[code][r] = v[r] * inv;
                // DGeom::frm: the hemisphere frame of that normal (float32, the device's cross/normalize)
                const float* nn = d.nrm[code];
                float dnn[3] = {0.0f, 0.0f, 1.0f};
                if (std::fabs(nn[0]) < ptd::kSQRT_1_3) { dnn[0] = 1.0f; dnn[2] = 0.0f; }
                else if (std::fabs(nn[1]) < ptd::kSQRT_1_3) { dnn[1] = 1.0f; dnn[2] = 0.0f; }
                auto crs = [](const float* a, const float* b, float* o) {
                    o[0] = a[1] * b[2] - b[1] * a[2];
                    o[1] = a[2] * b[0] - b[2] * a[0];
                    o[2] = a[0] * b[1] - b[0] * a[1];
                };
                auto nrmz = [](float* x) {
                    const float iv = 1.0f / std::sqrt((x[0] * x[0] + x[1] * x[1]) + x[2] * x[2]);
                    for (int r = 0; r < 3; ++r) x[r] = x[r] * iv;
                };
                float p1[3], p2[3];
                crs(nn, dnn, p1);
                nrmz(p1);
                crs(nn, p1, p2);
                nrmz(p2);
                for (int r = 0; r < 3; ++r) { d.frm[code][r] = p1[r]; d.frm[code][3 + r] = p2[r]; }
            }
        for (int k = 0; k < 3; ++k) { d.bmin[k] = g.min_bound[k]; d.bmax[k] = g.max_bound[k]; }
    }
    {   // scene extent: every surface point (cube/sphere corners, mesh vertices) and the camera
        double ext = 0.0;
        for (int k = 0; k < 3; ++k) ext = std::max(ext, std::fabs((double)S.camera.position[k]));
        for (const pt_geom& g : S.geoms) {
            if (g.type != PT_GEOM_CUBE && g.type != PT_GEOM_SPHERE) continue;
            for (int corner = 0; corner < 8; ++corner) {
                const double p[3] = {corner & 1 ? 0.5 : -0.5, corner & 2 ? 0.5 : -0.5, corner & 4 ? 0.5 : -0.5};
                for (int r = 0; r < 3; ++r) {
                    double v = g.transform[12 + r];
                    for (int k = 0; k < 3; ++k) v += (double)g.transform[4 * k + r] * p[k];
                    ext = std::max(ext, std::fabs(v));
                }
            }
        }
        for (const pt_triangle& t : S.triangles)
            for (int v = 0; v < 3; ++v)
                for (int k = 0; k < 3; ++k) ext = std::max(ext, std::fabs((double)t.v[v][k]));
        c->scene_ext = ext;
    }
    c->hgeoms = dg;
    update_bounds(c, c->flags.aperture);
    dg = c->hgeoms;
    DGeom* d_geoms;
    DMaterial* d_mats;
    if (int rc = c->alloc(&d_geoms, dg.size())) return bail(rc);
    c->d_geoms = d_geoms;
    if (int rc = c->alloc(&c->d_bgeoms, dg.size())) return bail(rc);
    if (int rc = c->alloc(&d_mats, S.materials.size())) return bail(rc);
    if ((e = hipMemcpy(d_geoms, dg.data(), dg.size() * sizeof(DGeom), hipMemcpyHostToDevice)) != hipSuccess ||
        (e = hipMemcpy(d_mats, S.materials.data(), S.materials.size() * sizeof(DMaterial), hipMemcpyHostToDevice)) != hipSuccess)
        return bail(pt::fail(PT_ERR_HIP, std::string("scene upload: ") + hipGetErrorString(e)));
    static_assert(sizeof(DMaterial) == sizeof(pt_material), "material layout");
    static_assert(sizeof(DNode) == 32 && sizeof(DTri) == 48, "packed device layouts");
    A.S.geoms = d_geoms;
    if (int rc = upload_bound_order(c)) return bail(rc);
    A.S.mats = d_mats;
    A.S.ngeoms = (int)dg.size();
    A.S.nmats = (int)S.materials.size();
    if (!S.triangles.empty()) {
        std::vector<DTri> tr(S.triangles.size());
        std::vector<DTriAttr> at(S.triangles.size());
        for (size_t i = 0; i < S.triangles.size(); ++i) {
            const pt_triangle& t = S.triangles[i];
            for (int k = 0; k < 3; ++k) {
                tr[i].a[k] = t.v[0][k];
                tr[i].b[k] = t.v[1][k] - t.v[0][k];
                tr[i].c[k] = t.v[2][k] - t.v[0][k];
            }
            int32_t id = t.id;
            tr[i].a[3] = bits_to_float(id);
            tr[i].b[3] = tr[i].c[3] = 0.0f;
            std::memcpy(at[i].n, t.n, sizeof at[i].n);
            std::memcpy(at[i].uv, t.uv, sizeof at[i].uv);
        }
        std::vector<float> pack(9 * tr.size() + 16);   // (+16: k_traverse4's group loads may read past the last)
        for (size_t i = 0; i < tr.size(); ++i)
            for (int k = 0; k < 3; ++k) {
                pack[9 * i + k] = tr[i].a[k];
                pack[9 * i + 3 + k] = tr[i].b[k];
                pack[9 * i + 6 + k] = tr[i].c[k];
            }
        DTri* d_tr;
        DTriAttr* d_at;
        float* d_pack;
        if (int rc = c->alloc(&d_pack, pack.size())) return bail(rc);
        if ((e = hipMemcpy(d_pack, pack.data(), pack.size() * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(pt::fail(PT_ERR_HIP, std::string("triangle upload: ") + hipGetErrorString(e)));
        A.S.tpack = d_pack;
        if (int rc = c->alloc(&d_tr, tr.size())) return bail(rc);
        if (int rc = c->alloc(&d_at, at.size())) return bail(rc);
        if ((e = hipMemcpy(d_tr, tr.data(), tr.size() * sizeof(DTri), hipMemcpyHostToDevice)) != hipSuccess ||
            (e = hipMemcpy(d_at, at.data(), at.size() * sizeof(DTriAttr), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(pt::fail(PT_ERR_HIP, std::string("triangle upload: ") + hipGetErrorString(e)));
        A.S.tris = d_tr;
        A.S.attrs = d_at;
        A.S.ntris = (int)tr.size();
    }
    if (!S.bvh.empty()) {
        const std::vector<DNode> nodes = to_dnodes(S.bvh);
        DNode* d_nodes;
        if (int rc = c->alloc(&d_nodes, nodes.size())) return bail(rc);
        if ((e = hipMemcpy(d_nodes, nodes.data(), nodes.size() * sizeof(DNode), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(pt::fail(PT_ERR_HIP, std::string("bvh upload: ") + hipGetErrorString(e)));
        A.S.nodes = d_nodes;
        A.S.nnodes = (int)S.bvh.size();
        std::vector<int32_t> depth(S.bvh.size(), 0);
        int32_t deepest = 0;
        for (size_t i = 0; i < S.bvh.size(); ++i)
            if (S.bvh[i].sub_areas == 0) {
                deepest = std::max(deepest, depth[i]);
                if (i + 1 < depth.size()) depth[i + 1] = depth[i] + 1;
                if (S.bvh[i].rchild_idx > 0 && (size_t)S.bvh[i].rchild_idx < depth.size())
                    depth[(size_t)S.bvh[i].rchild_idx] = depth[i] + 1;
            }
        A.S.bvh_depth = deepest;
        // child-pair layout (bvh_walk_pairs): leaves of <= 255 triangles, triangle ids < 2^23
        bool fits = S.triangles.size() < (1u << 23);
        for (const DNode& n : nodes)
            if (__float_as_int_host(n.lo[3]) > 255) fits = false;
        if (fits) {
            std::vector<int32_t> pid(nodes.size(), -1);
            int32_t np = 0;
            for (size_t i = 0; i < nodes.size(); ++i)
                if (__float_as_int_host(nodes[i].lo[3]) <= 0) pid[i] = np++;
            auto code = [&](size_t i) -> int32_t {
                const int32_t meta = __float_as_int_host(nodes[i].lo[3]), link = __float_as_int_host(nodes[i].hi[3]);
                if (meta > 0) return -(link * 256 + meta) - 1;
                return pid[i] * 4 + (-meta - 1);
            };
            std::vector<DPair> pairs((size_t)std::max(np, 1));
            for (size_t i = 0; i < nodes.size(); ++i) {
                if (pid[i] < 0) continue;
                const size_t L = i + 1, R = (size_t)__float_as_int_host(nodes[i].hi[3]);
                DPair& q = pairs[(size_t)pid[i]];
                for (int k = 0; k < 3; ++k) {
                    q.lmin[k] = nodes[L].lo[k]; q.lmax[k] = nodes[L].hi[k];
                    q.rmin[k] = nodes[R].lo[k]; q.rmax[k] = nodes[R].hi[k];
                }
                q.lmin[3] = bits_to_float(code(L));
                q.rmin[3] = bits_to_float(code(R));
                q.lmax[3] = q.rmax[3] = 0.0f;
            }
            DPair* d_pairs;
            if (int rc = c->alloc(&d_pairs, pairs.size())) return bail(rc);
            if ((e = hipMemcpy(d_pairs, pairs.data(), pairs.size() * sizeof(DPair), hipMemcpyHostToDevice)) != hipSuccess)
                return bail(pt::fail(PT_ERR_HIP, std::string("bvh pair upload: ") + hipGetErrorString(e)));
            A.S.pairs = d_pairs;
            A.S.root_code = code(0);
            for (int k = 0; k < 4; ++k) { A.S.root_lo[k] = nodes[0].lo[k]; A.S.root_hi[k] = nodes[0].hi[k]; }
            if (int rc = build_quads(c, nodes, S.triangles)) return bail(rc);
        }
    }
    if (!S.textures.empty()) {
        std::vector<DTexture> tx(S.textures.size());
        for (size_t i = 0; i < S.textures.size(); ++i) {
            const auto& t = S.textures[i];
            uint8_t* d_px;
            if (int rc = c->alloc(&d_px, t.pixels.size())) return bail(rc);
            if ((e = hipMemcpy(d_px, t.pixels.data(), t.pixels.size(), hipMemcpyHostToDevice)) != hipSuccess)
                return bail(pt::fail(PT_ERR_HIP, std::string("texture upload: ") + hipGetErrorString(e)));
            tx[i] = DTexture{t.width, t.height, t.components, 0, d_px};
        }
        DTexture* d_tx;
        if (int rc = c->alloc(&d_tx, tx.size())) return bail(rc);
        if ((e = hipMemcpy(d_tx, tx.data(), tx.size() * sizeof(DTexture), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(pt::fail(PT_ERR_HIP, std::string("texture table upload: ") + hipGetErrorString(e)));
        A.S.texs = d_tx;
    }

    // ---- camera / tile ----
    const pt_camera& cam = S.camera;
    for (int k = 0; k < 3; ++k) {
        A.cam.pos[k] = cam.position[k];
        A.cam.view[k] = cam.view[k];
        A.cam.up[k] = cam.up[k];
        A.cam.right[k] = cam.right[k];
    }
    A.cam.pl[0] = cam.pixel_length[0];
    A.cam.pl[1] = cam.pixel_length[1];
    A.cam.res[0] = W;
    A.cam.res[1] = H;
    A.tile = TileDev{W, sh.rank, sh.world, (int)npix, sh.spp, (int)P, S.depth, 1, 0};
    if ((double)npix * (double)W < 0x1p40) A.tile.wdiv = ((1ull << 40) + (uint64_t)W - 1) / (uint64_t)W;
    A.inv_npix = 1.0f / (float)std::max<int64_t>((int64_t)npix, 1);   // (retire's estimate, corrected by one step)

    A.emit_stride = 256 * 8;   // >= any grid_trace (cus * 8) / grid_bounce
    // k_trace has no inter-workgroup dependency: 8 workgroups per CU, grid-stride beyond that.
    // k_compact_paths is persistent + look-back: co-resident grid (one block/CU below the
    // occupancy API's answer, which can over-report by one for SGPR-heavy kernels).
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    c->cus = cus;
    c->grid_trace = std::max(1, std::min({(int)((P + kBlock - 1) / kBlock), cus * 8, A.emit_stride}));
    c->grid_compact = std::max(1, std::min((int)((P + kCompactTile - 1) / kCompactTile), cus * resident_per_cu((const void*)k_compact_paths)));
    for (int f = 0; f < 2; ++f) {   // k_bounce: any grid is correct; one full wave of equal-work
        int per_cu = 0;              // workgroups avoids a half-empty second wave
        const int mm = A.S.ntris > 0 ? kMeshPre : 0;   // (any grid is correct for either mesh mode)
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bounce_kernel(f, sh.spp == 1, mm, false, A.S.nmats > kLdsMats || A.S.ngeoms > kLdsGeoms), kBlock,
                                                         bounce_lds_bytes(A.S, mm)) != hipSuccess || per_cu <= 0)
            per_cu = 4;
        // > 2 spp workgroups: the per-iteration layout of k_bounce needs grid - spp >= spp
        // the first bounce (raygen, 5 waves/SIMD) balances better over two waves of workgroups
        // (measured: 393 -> 379 us per 10.24 M paths); later bounces over one (131 vs 134 us)
        c->grid_bounce[f] = std::max(2 * sh.spp + 1, std::min({cus * per_cu * (f ? 2 : 1), kMaxSeg, A.emit_stride}));
    }
    // ---- path state, image, control ----
    // k_bounce writes workgroup b's survivors at b * chunk: with the per-iteration layout the last
    // segment can end past P by < spp chunks (tiles <= P/256 + spp, tpb <= ceil(tiles / (grid - spp))).
    auto path_cap = [&](long long paths, long long spp, size_t* cap) {
        const long long g = std::min(c->grid_bounce[0], c->grid_bounce[1]);
        const long long tiles = (paths + kBlock - 1) / kBlock + spp;
        const long long tpb = (tiles + g - spp - 1) / (g - spp);
        *cap = (size_t)kBlock * (size_t)(tiles + spp * tpb);
        if (tpb * kBlock > (long long)kSegCountMask)
            return pt::fail(PT_ERR_ARG, "pass too large for the bounce kernel's segment words (chunk >= 2^24)");
        if (*cap > (size_t)0x7fffffff) return pt::fail(PT_ERR_ARG, "pass too large: path buffer index exceeds int32");
        return (int)PT_OK;
    };
    if (int rc = path_cap(P, sh.spp, &c->path_cap)) return bail(rc);
    for (int b = 0; b < 2; ++b)
        if (int rc = alloc_paths(c, c->buf[b], c->path_cap)) return bail(rc);
    c->lcap[0] = c->path_cap;
    if (const char* mi = std::getenv("PT_AMD_MESH_INLINE")) c->mesh_inline = std::strcmp(mi, "1") == 0;
    if (const char* sl = std::getenv("PT_AMD_SYNC_LANES")) c->async_lanes = std::strcmp(sl, "1") != 0;
    if (A.S.nnodes > 0) {   // k_traverse records (mesh mode 2), tickets, stack depth and grid
        if (int rc = c->alloc(&c->mhit[0], c->path_cap)) return bail(rc);
        if (int rc = c->alloc(&c->tq, (size_t)kMaxLanes * 64)) return bail(rc);
        const char* tv = std::getenv("PT_AMD_TRAV");
        c->trav_quads = A.S.quads != nullptr && !(tv && std::strcmp(tv, "pairs") == 0);
        A.stack_rows = c->trav_quads ? std::max(1, std::min(c->quad_occ, kTrav4LdsRows))
                                     : std::min(A.S.bvh_depth + 2, kTravLdsRows);
        if (const char* sr = std::getenv("PT_AMD_STACK_ROWS")) A.stack_rows = std::max(1, std::min(64, std::atoi(sr)));
        const size_t slds = (size_t)A.stack_rows * kBlock * sizeof(int);
        int per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_traverse<false>, kBlock, slds) != hipSuccess ||
            per_cu <= 0)
            per_cu = 4;
        c->grid_traverse = cus * per_cu;
        per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, c->walk_k == 1 ? k_traverse4<false, 1> : k_traverse4<false, kT4K>,
                                                         kBlock, slds) != hipSuccess ||
            per_cu <= 0)
            per_cu = 4;
        c->grid_traverse4 = cus * per_cu;
        A.refill_min = kRefillMin;
        A.tchunk = kTravChunk;
        if (const char* tc = std::getenv("PT_AMD_TCHUNK")) A.tchunk = std::max(64, std::min(4096, std::atoi(tc)));
        if (const char* rf = std::getenv("PT_AMD_REFILL")) A.refill_min = std::max(1, std::min(64, std::atoi(rf)));
    }
    if (int rc = c->alloc(&A.image, (size_t)npix * 3)) return bail(rc);
    if ((e = hipEventCreateWithFlags(&c->ev_done, hipEventDisableTiming)) != hipSuccess)
        return bail(pt::fail(PT_ERR_HIP, std::string("context event: ") + hipGetErrorString(e)));
    if (sh.spp > 1) {
        if (int rc = c->alloc(&c->colbuf, 2 * (size_t)P)) return bail(rc);
        A.colbuf = c->colbuf;
        if (int rc = c->alloc(&c->colflag, 2 * (size_t)P)) return bail(rc);   // (every pass's finalize clears its half)
        if ((e = hipMemset(c->colflag, 0, 2 * (size_t)P)) != hipSuccess)
            return bail(pt::fail(PT_ERR_HIP, std::string("hipMemset: ") + hipGetErrorString(e)));
        if ((e = hipStreamCreateWithFlags(&c->fin_stream, hipStreamNonBlocking)) != hipSuccess)
            return bail(pt::fail(PT_ERR_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e)));
        for (int h = 0; h < 2; ++h)
            if ((e = hipEventCreateWithFlags(&c->ev_pass[h], hipEventDisableTiming)) != hipSuccess ||
                (e = hipEventCreateWithFlags(&c->ev_fin[h], hipEventDisableTiming)) != hipSuccess)
                return bail(pt::fail(PT_ERR_HIP, std::string("hipEventCreate: ") + hipGetErrorString(e)));
    }
    // The synchronous entry points' copies run on a stream of their own at the greatest priority.
    // HIP maps the streams of a process onto GPU_MAX_HW_QUEUES (4) hardware queues PER PRIORITY, and
    // streams beyond that share a queue and run in submission order: a fifth normal-priority stream
    // made two of config 3's three lanes share one (35.6k vs 39.6k Mray/s), and a copy stream that
    // shares a queue with another context's busy stream waits behind its passes.  The high-priority
    // pool holds only these copy streams, so they take no queue from the compute streams and no
    // compute stream can sit in front of them.
    {
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) greatest = 0;
        if ((e = hipStreamCreateWithPriority(&c->io_stream, hipStreamNonBlocking, greatest)) != hipSuccess)
            return bail(pt::fail(PT_ERR_HIP, std::string("context stream: ") + hipGetErrorString(e)));
    }
    c->max_tiles = (int)((P + kCompactTile - 1) / kCompactTile);   // k_compact_paths tiles
    if (int rc = c->alloc(&A.flags, (size_t)P)) return bail(rc);
    if (int rc = c->alloc(&A.ctl, 2)) return bail(rc);
    if (int rc = c->alloc(&A.seg, (size_t)2 * kMaxSeg)) return bail(rc);
    if (int rc = c->alloc(&A.ibase, (size_t)kMaxSpp + 1)) return bail(rc);
    if (int rc = c->alloc(&A.status, (size_t)2 * c->max_tiles)) return bail(rc);
    if (int rc = c->alloc(&c->stats, 1)) return bail(rc);
    A.stats = c->stats;
    if (int rc = c->alloc(&A.emit_slots, (size_t)64 * A.emit_stride)) return bail(rc);
    if ((e = hipMemset(A.emit_slots, 0, (size_t)64 * A.emit_stride * sizeof(unsigned long long))) != hipSuccess)
        return bail(pt::fail(PT_ERR_HIP, std::string("hipMemset: ") + hipGetErrorString(e)));
    A.max_tiles = c->max_tiles;
    A.count_pass = 1;
    {   // lanes 1..L-1: each its own path buffers, control words, emissive slots and stream
        const char* lv = std::getenv("PT_AMD_LANES");
        // (async lanes: two lanes match three on the fused pipeline at every pass size; the sorted
        // pipeline's five launches per bounce still gain from a third lane on large passes)
        const bool three = c->flags.sort_by_material != 0 && P >= kThreeLanePaths;
        // (the BVH walk's persistent grid fills the GPU, so a second lane's bounce kernel only waits
        // for it: config 5 at one lane 794.6 vs 784.8 Mray/s, same box, two alternations)
        const bool walk = c->flags.sort_by_material == 0 && mesh_mode(c) == kMeshPre && c->trav_quads &&
                          c->flags.bvh_cull == 0;   // (the pair walk with bvh_cull: 790 at two lanes vs 730 at one)
        const int want = lv ? std::max(1, std::min(kMaxLanes, std::atoi(lv))) : (three ? 3 : (walk ? 1 : 2));
        int L = std::min(want, sh.spp);
        // Stream budget: a batched context keeps the caller's stream, L - 1 lane streams and the
        // finalize stream busy.  Unless PT_AMD_LANES asks for a count, the lanes are capped so that the
        // busy streams of all live contexts stay within the hardware queues (stream_budget()): lanes
        // beyond it would share queues with other contexts' streams and serialise behind them.
        if (!lv && L > 1) {
            const int room = stream_budget() - g_busy_streams.load() - 2;   // - caller - finalize
            const int capped = std::max(1, std::min(L, room + 1));
            c->lanes_capped = capped < L;
            L = capped;
        }
        if (L >= 2) {
            if ((e = hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming)) != hipSuccess)
                return bail(pt::fail(PT_ERR_HIP, std::string("lane setup: ") + hipGetErrorString(e)));
            for (int l = 1; l < L; ++l) {
                const int n_l = lane_iters(sh.spp, L, l);
                size_t cap_l = 0;
                if (int rc = path_cap((long long)n_l * (long long)npix, n_l, &cap_l)) return bail(rc);
                for (int b = 0; b < 2; ++b)
                    if (int rc = alloc_paths(c, c->lbuf[l][b], cap_l)) return bail(rc);
                c->lcap[l] = cap_l;
                if (c->mhit[0])
                    if (int rc = c->alloc(&c->mhit[l], cap_l)) return bail(rc);
                if (int rc = c->alloc(&c->lctl[l], 2)) return bail(rc);
                if (int rc = c->alloc(&c->lseg[l], (size_t)2 * kMaxSeg)) return bail(rc);
                if (int rc = c->alloc(&c->lemit[l], (size_t)64 * A.emit_stride)) return bail(rc);
                if ((e = hipMemset(c->lctl[l], 0, 2 * sizeof(Ctl))) != hipSuccess ||
                    (e = hipMemset(c->lseg[l], 0, (size_t)2 * kMaxSeg * sizeof(int32_t))) != hipSuccess ||
                    (e = hipMemset(c->lemit[l], 0, (size_t)64 * A.emit_stride * sizeof(unsigned long long))) != hipSuccess ||
                    (e = hipStreamCreateWithFlags(&c->lane_stream[l], hipStreamNonBlocking)) != hipSuccess ||
                    (e = hipEventCreateWithFlags(&c->ev_join[l], hipEventDisableTiming)) != hipSuccess)
                    return bail(pt::fail(PT_ERR_HIP, std::string("lane setup: ") + hipGetErrorString(e)));
            }
            c->lanes = L;
        }
    }
    c->busy_streams = 1 + (c->lanes - 1) + (c->fin_stream ? 1 : 0);   // caller + lanes + finalize
    g_busy_streams.fetch_add(c->busy_streams);
    if ((e = hipMemset(A.image, 0, (size_t)npix * 3 * sizeof(float))) != hipSuccess ||
        (e = hipMemset(A.ctl, 0, 2 * sizeof(Ctl))) != hipSuccess ||
        (e = hipMemset(A.seg, 0, (size_t)2 * kMaxSeg * sizeof(int32_t))) != hipSuccess ||
        (e = hipMemset(A.status, 0, (size_t)2 * c->max_tiles * sizeof(uint64_t))) != hipSuccess ||
        (e = hipMemset(c->stats, 0, sizeof(DevStats))) != hipSuccess)
        return bail(pt::fail(PT_ERR_HIP, std::string("hipMemset: ") + hipGetErrorString(e)));
    // material-sort buffers, per lane: uv by physical slot (< cap), perm by sorted position
    // (< the lane's paths), the histogram by (producer tile, material) (cap / 256 tiles at most)
    for (int l = 0; l < c->lanes; ++l) {
        auto& ss = c->sset[l];
        const int n_l = lane_iters(sh.spp, c->lanes, l);
        const size_t paths = (size_t)n_l * (size_t)npix, cap = c->lcap[l];
        ss.hist_cap = (int64_t)((size_t)c->nmats * (cap / kBlock + 1) + 2);
        const size_t tiles = ((size_t)ss.hist_cap + kHistTile - 1) / kHistTile;
        if (int rc = c->alloc(&ss.hslot, (size_t)ss.hist_cap)) return bail(rc);
        if (int rc = c->alloc(&ss.perm, 2 * paths)) return bail(rc);   // (pf_store)
        if (int rc = c->alloc(&ss.fpos, 1)) return bail(rc);
        if (int rc = c->alloc(&ss.hist2, (size_t)ss.hist_cap)) return bail(rc);
        if (int rc = c->alloc(&ss.offs2, (size_t)ss.hist_cap)) return bail(rc);
        if (int rc = c->alloc(&ss.hist, (size_t)ss.hist_cap)) return bail(rc);
        if (int rc = c->alloc(&ss.offs, (size_t)ss.hist_cap)) return bail(rc);
        if (int rc = c->alloc(&ss.itb, 2 * ((size_t)kMaxSpp + 1))) return bail(rc);
        if (int rc = c->alloc(&ss.sums, 2 * tiles)) return bail(rc);
        if (!S.textures.empty())
            for (int h = 0; h < 2; ++h)
                if (int rc = c->alloc(&ss.uv[h], 2 * cap)) return bail(rc);
    }
    if (const char* pl = std::getenv("PT_PIPELINE")) c->fused = std::string(pl) != "split";
    if (int rc = build_cmask(c)) return bail(rc);
    *out = c;
    return PT_OK;
}

int pt_destroy(pt_ctx* c) {
    if (c) {   // the context's own queued work only (its streams, and the last pass on the caller's)
        (void)wait_ctx(c);
        if (c->ahead_recorded) (void)hipEventSynchronize(c->ev_ahead);
        if (c->fin_stream) (void)hipStreamSynchronize(c->fin_stream);
        for (int l = 1; l < kMaxLanes; ++l)
            if (c->lane_stream[l]) (void)hipStreamSynchronize(c->lane_stream[l]);
        if (c->io_stream) (void)hipStreamSynchronize(c->io_stream);
        delete c;
    }
    return PT_OK;
}

// The reference re-reads its GUI flags on every pathtrace() call (pathtrace.cu:438-463), so this is
// called once per iteration by a drop-in caller (host/pathtrace.cpp).  Only the lens (aperture) and
// the camera-ray shape (SSAA, DoF, aperture, focal distance) reach device data — the widened geom
// bounds and the first-bounce camera masks; every other flag is copied into the launch arguments
// by value at pt_render_pass.  So a call that changes none of those four returns without a device
// synchronisation and without rebuilding the masks (pt_ctx_counters counts both).
int pt_set_flags(pt_ctx* c, const pt_flags* f) {
    if (!c || !f) return pt::fail(PT_ERR_ARG, "null argument");
    auto same = [](float a, float b) { return std::memcmp(&a, &b, sizeof a) == 0; };
    const bool lens = !same(f->aperture, c->flags.aperture);
    const bool rays = lens || f->ssaa != c->flags.ssaa || f->dof != c->flags.dof ||
                      !same(f->focal_dist, c->flags.focal_dist);
    set_flags_dev(c, *f);
    if (!rays) return PT_OK;
    ++c->n_flag_syncs;
    // (this context's queued passes still read the old bounds and masks; nothing else is waited for)
    if (int rc = wait_ctx(c)) return rc;
    if (c->ahead_recorded) HIP_TRY(hipEventSynchronize(c->ev_ahead));   // (and is dropped: flags differ)
    if (lens) {   // the camera lens bounds the ray origins: re-derive the widened bounds
        update_bounds(c, f->aperture);
        HIP_TRY(io_copy(c, c->d_geoms, c->hgeoms.data(), c->hgeoms.size() * sizeof(DGeom), hipMemcpyHostToDevice));
        if (int rc = upload_bound_order(c)) return rc;
    }
    return build_cmask(c);   // SSAA / DoF / aperture / focal distance bound the camera rays
}

int pt_ctx_walk_info(const pt_ctx* c, int32_t* quad_walk, int32_t* tcull_on, double* tcull_frac) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    if (quad_walk) *quad_walk = c->trav_quads ? 1 : 0;
    if (tcull_on) *tcull_on = c->args.S.qcull != nullptr ? 1 : 0;
    if (tcull_frac) *tcull_frac = c->tcull_frac;
    return PT_OK;
}

int pt_ctx_cmask_info(const pt_ctx* c, int32_t* on, double* empty_frac, int32_t* skip_fused) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    if (on) *on = c->args.cmask != nullptr ? 1 : 0;
    if (empty_frac) *empty_frac = c->cmask_empty;
    if (skip_fused) *skip_fused = c->cmask_skip ? 1 : 0;
    return PT_OK;
}

int pt_ctx_stream_info(const pt_ctx* c, int32_t* lanes, int32_t* busy_streams, int32_t* process_busy,
                       int32_t* hw_queues, int32_t* lanes_capped) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    if (lanes) *lanes = c->lanes;
    if (busy_streams) *busy_streams = c->busy_streams;
    if (process_busy) *process_busy = g_busy_streams.load();
    if (hw_queues) *hw_queues = stream_budget();
    if (lanes_capped) *lanes_capped = c->lanes_capped ? 1 : 0;
    return PT_OK;
}

int pt_ctx_counters(const pt_ctx* c, uint64_t* mask_builds, uint64_t* flag_syncs) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    if (mask_builds) *mask_builds = c->n_cmask_builds;
    if (flag_syncs) *flag_syncs = c->n_flag_syncs;
    return PT_OK;
}

static int wait_finalize(pt_ctx* c, hipStream_t st);

// One pass on st; ahead: a render-ahead pass (one-iteration context) whose colours and counts go to
// the ahead buffers and that neither finalizes nor marks the context (pt_render_ahead).
static int render_pass(pt_ctx* c, int32_t iter_first, hipStream_t st, bool ahead) {
    KArgs A = c->args;
    A.tile.iter_first = iter_first;
    const bool spp1 = A.tile.spp == 1 && !ahead;
    const bool sorted = c->flags.sort_by_material != 0;
    const bool mesh = A.S.ntris > 0;
    const int mmode = mesh_mode(c);   // k_bounce's mesh mode (fused pipeline)
    int cur = 0;   // paths start in buf[0]
    const int h = c->col_half;
    A.col_spp = A.tile.spp;
    A.col_off = 0;
    if (ahead) {
        A.colbuf = c->ahead_col;
        A.colflag = c->ahead_flag;
        A.stats = c->ahead_stats;
        A.emit_slots = c->ahead_emit;
    } else if (!spp1) {
        A.colbuf = c->colbuf + (size_t)h * (size_t)A.tile.P;
        A.colflag = c->colflag + (size_t)h * (size_t)A.tile.P;
        if (c->fin_out[h]) HIP_TRY(hipStreamWaitEvent(st, c->ev_fin[h], 0));   // pass p-2's finalize
    }
    const bool laned = (sorted || c->fused) && c->lanes >= 2 && !spp1 && !ahead;
    // One bounce b of the material-sorted pipeline on stream s, for the lane whose buffers are `bufs`
    // (current one: lcur), launch counter `lc` and sort buffers `ss`: [the first bounce's producer],
    // histogram scan, scatter, producer (shade b + intersect b + 1).  Every producer flips the buffers.
    auto sort_bounce = [&](KArgs& a, pt_ctx::SortSet& ss, hipStream_t s, int b, int& lcur, uint64_t& lc,
                           const PathSoA* bufs) -> int {
        ProfEv* ev;
        auto produce = [&](bool first) -> int {
            a.parity = (int)(lc & 1);
            a.in = bufs[lcur];
            a.out = bufs[lcur ^ 1];
            a.hit.uv = ss.uv[lcur];
            const SortArgs sa{ss.hslot, ss.hist, ss.offs, ss.hist2, ss.offs2, ss.perm, ss.fpos, ss.itb, ss.uv[lcur ^ 1]};
            hipLaunchKernelGGL(produce_kernel(first, spp1, mesh, a.fl.verify != 0,
                                              c->nmats <= kLdsMats && a.S.ngeoms <= kLdsGeoms),
                               dim3(c->grid_bounce[0]), dim3(kBlock),
                               (size_t)16 * c->nmats * sizeof(uint32_t), s, a, sa);
            HIP_TRY(hipGetLastError());
            ++lc;
            lcur ^= 1;
            return PT_OK;
        };
        if (b == 0) {   // raygen + intersection of the camera rays: profiled as the first bounce
            if (int rc = prof_begin(c, s, PT_KIND_FIRST_BOUNCE, &ev)) return rc;
            if (int rc = produce(true)) return rc;
            if (int rc = prof_end(ev, s)) return rc;
        }
        if (int rc = prof_begin(c, s, PT_KIND_SORT, &ev)) return rc;
        a.parity = (int)(lc & 1);
        const uint32_t* nlive = &a.ctl[a.parity].hist_live;
        const int tiles = (int)((ss.hist_cap + kHistTile - 1) / kHistTile);
        constexpr int kHistGrid = 4; // (histogram-scan workgroups per CU)
        const int hgrid = std::min(tiles, kHistGrid * c->cus);   // (grid-stride over the live blocks)
        hipLaunchKernelGGL(k_hist_sums, dim3(hgrid), dim3(kBlock), 0, s, (const int32_t*)ss.hist, (const int32_t*)ss.hist2,
                           ss.hist_cap, nlive, ss.sums);
        hipLaunchKernelGGL(k_hist_scan_sums, dim3(1), dim3(kBlock), 0, s, ss.sums, ss.hist_cap, nlive);
        hipLaunchKernelGGL(k_hist_apply, dim3(hgrid), dim3(kBlock), 0, s,
                           (const int32_t*)ss.hist, ss.offs, (const int32_t*)ss.hist2, ss.offs2, ss.hist_cap, nlive,
                           (const uint32_t*)ss.sums, (const int32_t*)ss.hslot, ss.perm, ss.fpos);
        HIP_TRY(hipGetLastError());
        if (int rc = produce(false)) return rc;
        return prof_end(ev, s);
    };
    if (sorted && c->nmats > kSortMaxMats)
        return pt::fail(PT_ERR_ARG, "material-sorted shading supports at most 256 materials");
    const bool tickets = !sorted && c->fused && mmode == kMeshPre;   // k_traverse's per-bounce ray tickets
    if (tickets && !laned) HIP_TRY(hipMemsetAsync(c->tq, 0, (size_t)kMaxLanes * 64 * sizeof(uint32_t), st));
    if (laned) {
        const int npix = A.tile.npix, nl = c->lanes;
        KArgs L[kMaxLanes];
        hipStream_t ls[kMaxLanes];
        const PathSoA* bufs[kMaxLanes];
        uint64_t* cnt[kMaxLanes];
        for (int l = 0, off = 0; l < nl; ++l) {
            const int n_l = lane_iters(A.tile.spp, nl, l);
            L[l] = A;
            L[l].tile.spp = n_l;
            L[l].tile.P = n_l * npix;
            L[l].tile.iter_first = iter_first + off;
            L[l].colbuf = A.colbuf + (size_t)off * (size_t)npix;
            L[l].col_off = off;   // (the flag rows are the whole pass's, pixel-major)
            if (l > 0) {
                L[l].ctl = c->lctl[l];
                L[l].seg = c->lseg[l];
                L[l].emit_slots = c->lemit[l];
                L[l].count_pass = 0;
            }
            ls[l] = l == 0 ? st : c->lane_stream[l];
            bufs[l] = l == 0 ? c->buf : c->lbuf[l];
            cnt[l] = l == 0 ? &c->compact_launches : &c->llaunches[l];
            off += n_l;
        }
        HIP_TRY(hipEventRecord(c->ev_fork, st));   // after the wait for this colour half above
        for (int l = 1; l < nl; ++l) HIP_TRY(hipStreamWaitEvent(c->lane_stream[l], c->ev_fork, 0));
        // each lane zeroes its own tickets: its previous pass's tail may still be running
        for (int l = 0; tickets && l < nl; ++l)
            HIP_TRY(hipMemsetAsync(c->tq + 64 * l, 0, 64 * sizeof(uint32_t), ls[l]));
        // every exit, the error returns included, orders the lanes' queued work before the pass's
        // finalize (async_lanes) or before later work on st
        struct Join {
            pt_ctx* c;
            hipStream_t st;
            ~Join() {
                for (int l = 1; l < c->lanes; ++l) {
                    (void)hipEventRecord(c->ev_join[l], c->lane_stream[l]);
                    (void)hipStreamWaitEvent(c->async_lanes ? c->fin_stream : st, c->ev_join[l], 0);
                }
            }
        } join{c, st};
        int lcur[kMaxLanes] = {};
        for (int b = 0; b < c->depth; ++b)
            for (int l = 0; l < nl; ++l) {
                KArgs& a = L[l];
                a.bounce = b;
                if (sorted) {
                    if (int rc = sort_bounce(a, c->sset[l], ls[l], b, lcur[l], *cnt[l], bufs[l])) return rc;
                    continue;
                }
                a.parity = (int)(*cnt[l] & 1);
                a.n_fixed = b == 0 ? a.tile.P : -1;
                a.in = bufs[l][lcur[l]];
                a.out = bufs[l][lcur[l] ^ 1];
                a.mhit = c->mhit[l];
                a.tticket = c->tq ? c->tq + 64 * l + b : nullptr;
                if (int rc = launch_bounce(c, b == 0, false, mmode, ls[l], a, c->lcap[l])) return rc;
                ++*cnt[l];
                lcur[l] ^= 1;
            }
    }
    for (int b = 0; b < c->depth && !laned; ++b) {
        const bool last = b == c->depth - 1;   // every path is dead after the last bounce
        A.parity = (int)(c->compact_launches & 1);
        A.bounce = b;
        A.n_fixed = b == 0 ? A.tile.P : -1;
        A.in = c->buf[cur];
        A.out = c->buf[cur ^ 1];
        int rc;
        if (!sorted && c->fused) {
            A.mhit = c->mhit[0];
            A.tticket = c->tq ? c->tq + b : nullptr;
            rc = launch_bounce(c, b == 0, spp1, mmode, st, A, c->lcap[0]);
            if (rc) return rc;
            ++c->compact_launches;
            cur ^= 1;
        } else if (!sorted) {
            if (b > 0 && !spp1 && (rc = launch_k(c, k_iter_bases, c->grid_trace, st, PT_KIND_COMPACT, A))) return rc;
            rc = launch_k(c, trace_kernel(b == 0, spp1, mesh), c->grid_trace, st,
                          b == 0 ? PT_KIND_FIRST_BOUNCE : PT_KIND_BOUNCE, A);
            if (rc) return rc;
            if (!last) {
                // batched passes: the previous pass's finalize (side stream) may hold CUs while this
                // look-back runs, so its static co-resident schedule is not guaranteed — tiles are
                // claimed instead (lookback.h; the split pipeline is the diagnostic one)
                KArgs Ac = A;
                if (!spp1) Ac.fl.claimed = 1;
                if ((rc = launch_k(c, k_compact_paths, c->grid_compact, st, PT_KIND_COMPACT, Ac))) return rc;
                ++c->compact_launches;
                cur ^= 1;
            }
        } else if ((rc = sort_bounce(A, c->sset[0], st, b, cur, c->compact_launches, c->buf))) {
            return rc;
        }
    }

    if (ahead) return PT_OK;
    if (!spp1) {
        const int npix = A.tile.npix;
        HIP_TRY(hipEventRecord(c->ev_pass[h], st));
        HIP_TRY(hipStreamWaitEvent(c->fin_stream, c->ev_pass[h], 0));
        hipLaunchKernelGGL(k_finalize_spp, dim3(std::min((npix + 255) / 256, 4096)), dim3(256), 0, c->fin_stream,
                           A.image, (const v4f*)A.colbuf, A.colflag, npix, A.tile.spp);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ev_fin[h], c->fin_stream));
        c->fin_out[h] = true;
        c->last_fin = h;
        c->col_half = h ^ 1;
        return mark_ctx(c, c->fin_stream);   // (the finalize waited for every lane of the pass)
    }
    return mark_ctx(c, st);
}

static int settle_ahead(pt_ctx* c, hipStream_t st, bool add) {
    const int npix = c->args.tile.npix;
    const int nemit = std::min(c->depth, 64) * c->args.emit_stride;
    hipLaunchKernelGGL(k_ahead_settle, dim3(add ? std::min((npix + 255) / 256, 4096) : 64), dim3(256), 0, st,
                       c->args.image, (const v4f*)c->ahead_col, c->ahead_flag, npix, c->stats, c->ahead_stats,
                       c->args.emit_slots, c->ahead_emit, nemit, add ? 1 : 0);
    HIP_TRY(hipGetLastError());
    c->ahead_valid = false;
    return PT_OK;
}

int pt_render_pass(pt_ctx* c, int32_t iter_first, void* stream) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    if (iter_first < 0) return pt::fail(PT_ERR_ARG, "iteration index must be >= 0");
    hipStream_t st = (hipStream_t)stream;
    // A pass on another stream than the previous one first waits for all of the context's queued
    // work (its lanes and finalize included); consecutive passes on one stream keep their overlap
    // (the next pass starts during the previous one's finalize tail).
    if (c->pass_stream && c->pass_stream != st)
        if (int rc = order_after_ctx(c, st)) return rc;
    c->pass_stream = st;
    if (c->ahead_recorded) {
        HIP_TRY(hipStreamWaitEvent(st, c->ev_ahead, 0));   // its path buffers, counts and colours
        if (c->ahead_valid) {
            if (iter_first == c->ahead_iter && c->args.tile.spp == 1 &&
                std::memcmp(&c->flags, &c->ahead_flags, sizeof c->flags) == 0) {
                // the iteration was traced ahead with these flags: only its colours are left to add
                if (int rc = wait_finalize(c, st)) return rc;
                if (int rc = settle_ahead(c, st, true)) return rc;
                return mark_ctx(c, st);
            }
            if (int rc = settle_ahead(c, st, false)) return rc;
        }
    }
    return render_pass(c, iter_first, st, false);
}

// The bounces of iteration `iter` queued now, for the pt_render_pass(iter) that follows (pt_amd.h).
static int render_ahead(pt_ctx* c, int32_t iter, hipStream_t st);
int pt_render_ahead(pt_ctx* c, int32_t iter, void* stream) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    if (iter < 0) return pt::fail(PT_ERR_ARG, "iteration index must be >= 0");
    if (c->args.tile.spp != 1) return pt::fail(PT_ERR_ARG, "render-ahead needs a context of one iteration per pass");
    const int rc = render_ahead(c, iter, (hipStream_t)stream);
    if (rc != PT_OK) {
        // A caller may treat a failed render-ahead as a lost overlap only (host/pathtrace.cpp): nothing
        // is left to claim, later passes still order after whatever was queued, and the HIP last-error
        // is cleared so the next pass's launch check does not report this failure.
        c->ahead_valid = false;
        if (c->ev_ahead && hipEventRecord(c->ev_ahead, (hipStream_t)stream) == hipSuccess) c->ahead_recorded = true;
        (void)hipGetLastError();
    }
    return rc;
}

static int render_ahead(pt_ctx* c, int32_t iter, hipStream_t st) {
    if (!c->ev_ahead) {   // first use: the ahead buffers
        const size_t nemit = (size_t)64 * c->args.emit_stride;
        if (int rc = c->alloc(&c->ahead_col, (size_t)c->args.tile.P)) return rc;
        if (int rc = c->alloc(&c->ahead_flag, (size_t)c->args.tile.P)) return rc;
        if (int rc = c->alloc(&c->ahead_stats, 1)) return rc;
        if (int rc = c->alloc(&c->ahead_emit, nemit)) return rc;
        HIP_TRY(hipMemsetAsync(c->ahead_flag, 0, (size_t)c->args.tile.P, c->io_stream));
        HIP_TRY(hipMemsetAsync(c->ahead_stats, 0, sizeof(DevStats), c->io_stream));
        HIP_TRY(hipMemsetAsync(c->ahead_emit, 0, nemit * sizeof(unsigned long long), c->io_stream));
        HIP_TRY(hipStreamSynchronize(c->io_stream));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_ahead, hipEventDisableTiming));
    }
    // the context's last pass (its path buffers, control and segment words, tickets) and the last
    // claim's settle (which reads ahead_col) may still run on another stream
    if (int rc = order_after_ctx(c, st)) return rc;
    c->pass_stream = st;
    if (c->ahead_recorded) {
        HIP_TRY(hipStreamWaitEvent(st, c->ev_ahead, 0));
        if (c->ahead_valid)
            if (int rc = settle_ahead(c, st, false)) return rc;   // never claimed: dropped
    }
    if (int rc = render_pass(c, iter, st, true)) return rc;
    HIP_TRY(hipEventRecord(c->ev_ahead, st));
    c->ahead_recorded = c->ahead_valid = true;
    c->ahead_iter = iter;
    c->ahead_flags = c->flags;
    return PT_OK;
}

// Work on `st` that reads or writes the image first waits for this context's last enqueued work
// (the last deferred finalize of a batched pass, or an image call on another stream), and is then
// itself the work the synchronous entry points wait for (mark_ctx).
static int wait_finalize(pt_ctx* c, hipStream_t st) {
    if (c->done_recorded) HIP_TRY(hipStreamWaitEvent(st, c->ev_done, 0));
    else if (c->last_fin >= 0) HIP_TRY(hipStreamWaitEvent(st, c->ev_fin[c->last_fin], 0));
    return PT_OK;
}

int pt_preview_rgba(pt_ctx* c, int32_t iter, uint8_t* d_rgba, void* stream) {
    if (!c || !d_rgba || iter <= 0) return pt::fail(PT_ERR_ARG, "bad argument");
    const int npix = c->args.tile.npix;
    if (int rc = wait_finalize(c, (hipStream_t)stream)) return rc;
    hipLaunchKernelGGL(k_preview, dim3(std::min((npix + 255) / 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)c->args.image, d_rgba, npix, iter);
    HIP_TRY(hipGetLastError());
    return mark_ctx(c, (hipStream_t)stream);
}

int pt_render_iteration(pt_ctx* c, int32_t iter, uint8_t* d_rgba, void* stream) {
    if (!c || iter <= 0) return pt::fail(PT_ERR_ARG, "bad argument");
    const int rc = pt_render_pass(c, iter, stream);
    if (rc || !d_rgba) return rc;
    return pt_preview_rgba(c, iter + c->args.tile.spp - 1, d_rgba, stream);
}

int pt_tile_info(const pt_ctx* c, int32_t* width, int32_t* rows, int32_t* npix, int32_t* npaths) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    const TileDev& T = c->args.tile;
    if (width) *width = T.W;
    if (rows) *rows = T.npix / T.W;
    if (npix) *npix = T.npix;
    if (npaths) *npaths = T.P;
    return PT_OK;
}

int pt_get_image(pt_ctx* c, float* host_rgb) {
    if (!c || !host_rgb) return pt::fail(PT_ERR_ARG, "null argument");
    if (int rc = wait_ctx(c)) return rc;   // this context's passes only (pathtrace.cu:524's copy)
    HIP_TRY(io_copy(c, host_rgb, c->args.image, (size_t)c->args.tile.npix * 3 * sizeof(float), hipMemcpyDeviceToHost));
    return PT_OK;
}

int pt_get_accum(pt_ctx* c, float* host_rgb) { return pt_get_image(c, host_rgb); }

int pt_host_register(void* host, uint64_t bytes) {
    if (!host || !bytes) return pt::fail(PT_ERR_ARG, "null argument");
    const hipError_t e = hipHostRegister(host, (size_t)bytes, hipHostRegisterDefault);
    if (e != hipSuccess) {
        // a caller may go on without the page lock (the copies still work, staged): leave no sticky
        // last-error behind for the next launch's hipGetLastError check to report
        (void)hipGetLastError();
        return pt::fail(PT_ERR_DEVICE, std::string("hipHostRegister: ") + hipGetErrorString(e));
    }
    return PT_OK;
}

int pt_host_unregister(void* host) {
    if (!host) return pt::fail(PT_ERR_ARG, "null argument");
    HIP_TRY(hipHostUnregister(host));
    return PT_OK;
}

int pt_stream_create(void** stream) {
    if (!stream) return pt::fail(PT_ERR_ARG, "null argument");
    hipStream_t s = nullptr;
    HIP_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return PT_OK;
}

int pt_stream_destroy(void* stream) {
    if (stream) HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return PT_OK;
}

// The accumulator is loaded with every -0 replaced by +0.  The reference adds every iteration's colour
// (zero or not) into every pixel, so after any pass its image holds no -0 (-0 + 0 = +0); the passes here
// skip the additions of zero colours (retire, k_finalize_spp), which are identities on every value but -0.
// A +0 loaded in place of -0 makes the two agree bit for bit from the first pass on.
int pt_set_accum(pt_ctx* c, const float* host_rgb) {
    if (!c || !host_rgb) return pt::fail(PT_ERR_ARG, "null argument");
    if (int rc = wait_ctx(c)) return rc;
    const size_t n = (size_t)c->args.tile.npix * 3;
    std::vector<float> img(host_rgb, host_rgb + n);
    for (float& v : img)
        if (v == 0.0f) v = 0.0f;   // (-0 == 0: both zeros become +0)
    HIP_TRY(io_copy(c, c->args.image, img.data(), n * sizeof(float), hipMemcpyHostToDevice));
    return PT_OK;
}

int pt_copy_image(pt_ctx* c, float* d_rgb, void* stream) {
    if (!c || !d_rgb) return pt::fail(PT_ERR_ARG, "null argument");
    if (int rc = wait_finalize(c, (hipStream_t)stream)) return rc;
    HIP_TRY(hipMemcpyAsync(d_rgb, c->args.image, (size_t)c->args.tile.npix * 3 * sizeof(float),
                           hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return mark_ctx(c, (hipStream_t)stream);
}

int pt_reset_image(pt_ctx* c, void* stream) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    if (int rc = wait_finalize(c, (hipStream_t)stream)) return rc;
    HIP_TRY(hipMemsetAsync(c->args.image, 0, (size_t)c->args.tile.npix * 3 * sizeof(float), (hipStream_t)stream));
    return mark_ctx(c, (hipStream_t)stream);
}

int pt_stats(pt_ctx* c, pt_stats_t* out) {
    if (!c || !out) return pt::fail(PT_ERR_ARG, "null argument");
    if (int rc = wait_ctx(c)) return rc;
    DevStats s;
    HIP_TRY(io_copy(c, &s, c->stats, sizeof s, hipMemcpyDeviceToHost));
    std::vector<unsigned long long> slots((size_t)64 * c->args.emit_stride);
    HIP_TRY(io_copy(c, slots.data(), c->args.emit_slots, slots.size() * sizeof(unsigned long long),
                    hipMemcpyDeviceToHost));
    for (int l = 1; l < c->lanes; ++l) {   // the other lanes' per-workgroup counts
        std::vector<unsigned long long> l1(slots.size());
        HIP_TRY(io_copy(c, l1.data(), c->lemit[l], l1.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        for (size_t j = 0; j < slots.size(); ++j) slots[j] += l1[j];
    }
    std::memset(out, 0, sizeof *out);
    out->segments = s.segments;
    out->passes = s.passes;
    for (int k = 0; k < 64; ++k) {
        out->bounce_live[k] = s.bounce_live[k];
        unsigned long long e = 0;
        for (int j = 0; j < c->args.emit_stride; ++j) e += slots[(size_t)k * c->args.emit_stride + j];
        out->bounce_emit[k] = e;
        out->emissive_hits += e;
    }
    out->device_error = s.err;
    out->bound_mismatch = s.bound_mismatch;
    return s.err ? pt::fail(PT_ERR_DEVICE, (s.err & 2u) ? "material scan hit its look-back spin bound (GPU shared? set "
                                                         "pt_flags.shared_gpu)"
                                                       : "device-side look-back spin bound was hit")
                 : PT_OK;
}


#ifdef PT_TRAV_STATS
// Diagnostic build only (scripts/trav_stats.py): k_traverse[4]'s counters summed over their slots:
// out[0] rays, [1] interior fetches (pairs, or quads), [2] triangle tests, [3] wave trips (loop
// iterations with a busy lane), [4] waves; k_traverse4 only: [5] busy lane-trips, [6] trips with
// leaf tasks, [7] trips with an interior lane.
int pt_debug_trav(unsigned long long* out8, int32_t reset) {
    HIP_TRY(hipDeviceSynchronize());
    static unsigned long long h[64 * 8];
    HIP_TRY(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_trav), sizeof h));
    for (int k = 0; k < 8; ++k) {
        out8[k] = 0;
        for (int q = 0; q < 64; ++q) out8[k] += h[q * 8 + k];
    }
    if (reset) {
        std::memset(h, 0, sizeof h);
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_trav), h, sizeof h));
    }
    return PT_OK;
}
#endif

int pt_scene_bvh_quads(const pt_scene* scene, void* out, int32_t cap, int32_t* root_code, int32_t* stack_bound) {
    if (!scene) return -PT_ERR_ARG;
    const auto& S = *reinterpret_cast<const pt::Scene*>(scene);
    std::vector<DQuad> quads;
    int32_t rc = 0, occ = 0;
    if (!make_quads(to_dnodes(S.bvh), quads, rc, occ)) return 0;
    if (root_code) *root_code = rc;
    if (stack_bound) *stack_bound = occ;
    if (out && cap > 0) std::memcpy(out, quads.data(), std::min<size_t>((size_t)cap, quads.size()) * sizeof(DQuad));
    return (int)quads.size();
}

int pt_scene_bvh_tcull(const pt_scene* scene, uint32_t* words, int32_t cap, double* cullable_frac) {
    if (!scene) return -PT_ERR_ARG;
    const auto& S = *reinterpret_cast<const pt::Scene*>(scene);
    std::vector<DQuad> quads;
    std::vector<int32_t> slot_node;
    int32_t rc = 0, occ = 0;
    const std::vector<DNode> nodes = to_dnodes(S.bvh);
    if (!make_quads(nodes, quads, rc, occ, &slot_node)) return 0;
    std::vector<uint32_t> q;
    const double frac = build_qcull(nodes, S.triangles, slot_node, q);
    if (cullable_frac) *cullable_frac = frac;
    if (words && cap > 0) std::memcpy(words, q.data(), std::min<size_t>((size_t)cap, q.size()) * sizeof(uint32_t));
    return (int)q.size();
}

int pt_selftest_math(uint64_t n, uint32_t seed, uint64_t* mismatches) {
    if (!mismatches) return pt::fail(PT_ERR_ARG, "null argument");
    unsigned long long* d = nullptr;
    HIP_TRY(hipMalloc(&d, sizeof *d));
    hipError_t e = hipMemset(d, 0, sizeof *d);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_selftest_math, dim3(2048), dim3(256), 0, nullptr, n, seed, d);
        e = hipGetLastError();
    }
    unsigned long long h = 0;
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);   // (synchronises)
    (void)hipFree(d);
    if (e != hipSuccess) return pt::fail(PT_ERR_HIP, std::string("selftest: ") + hipGetErrorString(e));
    *mismatches = h;
    return PT_OK;
}

int pt_profile_enable(pt_ctx* c, int32_t on) {
    if (!c) return pt::fail(PT_ERR_ARG, "null context");
    c->profiling = on != 0;
    return PT_OK;
}

namespace {
int profile_read(pt_ctx* c, int32_t nkinds, double* ms, double* busy_ms, uint64_t* launches, bool fold_walk);
}

int pt_profile_read_kinds(pt_ctx* c, int32_t nkinds, double* ms, double* busy_ms, uint64_t* launches) {
    return profile_read(c, nkinds, ms, busy_ms, launches, false);
}

int pt_profile_read_busy(pt_ctx* c, double ms[4], double busy_ms[4], uint64_t launches[4]) {
    return profile_read(c, 4, ms, busy_ms, launches, true);
}

int pt_profile_read(pt_ctx* c, double ms[4], uint64_t launches[4]) {
    return profile_read(c, 4, ms, nullptr, launches, true);
}

}  // extern "C"

namespace {
// fold_walk: the four-kind calls count the BVH walk in the bounce kinds, as they did before the walk
// had kinds of its own (TRAVERSE -> BOUNCE, FIRST_TRAVERSE -> FIRST_BOUNCE; busy = the union of both)
int profile_read(pt_ctx* c, int32_t nkinds, double* ms, double* busy_ms, uint64_t* launches, bool fold_walk) {
    if (!c || !ms || !launches || nkinds < 0) return pt::fail(PT_ERR_ARG, "bad argument");
    std::vector<std::pair<double, double>> iv[PT_KIND_COUNT];   // per kind: [start, end) after the first event
    double m[PT_KIND_COUNT] = {}, busy[PT_KIND_COUNT] = {};
    uint64_t n[PT_KIND_COUNT] = {};
    for (size_t i = 0; i < c->ev_used; ++i) {
        ProfEv& ev = c->events[i];
        HIP_TRY(hipEventSynchronize(ev.b));
        float t = 0.f, t0 = 0.f;
        HIP_TRY(hipEventElapsedTime(&t, ev.a, ev.b));
        HIP_TRY(hipEventElapsedTime(&t0, c->events[0].a, ev.a));
        const int k = !fold_walk ? ev.kind : ev.kind == PT_KIND_TRAVERSE ? PT_KIND_BOUNCE
                                             : ev.kind == PT_KIND_FIRST_TRAVERSE ? PT_KIND_FIRST_BOUNCE : ev.kind;
        m[k] += t;
        n[k] += 1;
        iv[k].push_back({(double)t0, (double)t0 + (double)t});
    }
    // union of each kind's launch intervals: lanes run kernels of one kind concurrently
    for (int k = 0; k < PT_KIND_COUNT; ++k) {
        std::sort(iv[k].begin(), iv[k].end());
        double end = -1e300;
        for (const auto& x : iv[k]) {
            if (x.first > end) { busy[k] += x.second - x.first; end = x.second; }
            else if (x.second > end) { busy[k] += x.second - end; end = x.second; }
        }
    }
    for (int k = 0; k < nkinds; ++k) {
        ms[k] = k < PT_KIND_COUNT ? m[k] : 0.0;
        launches[k] = k < PT_KIND_COUNT ? n[k] : 0;
        if (busy_ms) busy_ms[k] = k < PT_KIND_COUNT ? busy[k] : 0.0;
    }
    c->ev_used = 0;
    return PT_OK;
}

}  // namespace

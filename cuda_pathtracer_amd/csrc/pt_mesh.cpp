// Mesh objects: OBJ loading (scene.cpp:94-173 with tinyobjloader 1.0.6 semantics) and the SAH BVH
// (BVH_tree.cpp:27-181, boundingbox.h), restated so the device sees exactly the triangles, the
// triangle order and the flattened node array the reference host would have produced.
//
// Reference behaviour kept on purpose:
//   * OBJ numbers are parsed with tinyobjloader's own decimal routine (digit accumulation in
//     double, 10^-k from a table, ldexp(m * 5^e, e)) and then rounded to float, not strtof;
//   * polygons become triangle fans (v0, v[k-1], v[k]); relative (negative) indices are resolved
//     against the counts seen so far; a missing normal / uv stays (0,0,0) / (0,0);
//   * vertices go to world space as glm::vec3(transform * vec4(v, 1)), normals as
//     glm::vec3(invTranspose * vec4(n, 0)) (not renormalised);
//   * a mesh geom's bound starts from (FLT_MAX, FLT_MIN) — so its max is never below FLT_MIN —
//     and is only used by the linear (non-BVH) path;
//   * ONE BVH spans all mesh triangles of the scene; the triangle array is reordered into leaf
//     order while each triangle keeps its load-order id and each geom its load-order id range;
//   * BoundingBox::operator|| treats an all-zero box as empty, including a real degenerate box
//     at the origin;
//   * 2-triangle splits order by centroid like libstdc++'s nth_element on two elements; larger
//     ranges bin centroids into 7 regions, cost split i from regions < i and > i (region i is
//     in neither side), and partition with libstdc++'s (unstable) bidirectional std::partition.
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include "pt_internal.h"

namespace pt {
namespace {

// ---- OBJ --------------------------------------------------------------------------------
bool is_digit(char c) { return (unsigned)(c - '0') < 10u; }

// tinyobjloader 1.0.6 tryParseDouble: [sign] digits [. digits] [e[sign]digits], in [s, end).
bool obj_parse_double(const char* s, const char* end, double* out) {
    if (s >= end) return false;
    double m = 0.0;
    int exponent = 0;
    bool neg = false, exp_neg = false;
    const char* c = s;
    if (*c == '+' || *c == '-') {
        neg = *c == '-';
        ++c;
    } else if (!is_digit(*c)) {
        return false;
    }
    int read = 0;
    while (c != end && is_digit(*c)) {
        m *= 10;
        m += (int)(*c - '0');
        ++c;
        ++read;
    }
    if (read == 0) return false;
    if (c != end) {
        bool more = true;
        if (*c == '.') {
            ++c;
            static const double kPow10Neg[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            int k = 1;
            while (c != end && is_digit(*c)) {
                m += (int)(*c - '0') * (k < 8 ? kPow10Neg[k] : std::pow(10.0, -k));
                ++k;
                ++c;
            }
            more = c != end;
        } else if (*c != 'e' && *c != 'E') {
            more = false;
        }
        if (more && (*c == 'e' || *c == 'E')) {
            ++c;
            if (c != end && (*c == '+' || *c == '-')) {
                exp_neg = *c == '-';
                ++c;
            } else if (!is_digit(*c)) {
                return false;
            }
            int digits = 0;
            while (c != end && is_digit(*c)) {
                exponent = exponent * 10 + (int)(*c - '0');
                ++c;
                ++digits;
            }
            if (exp_neg) exponent = -exponent;
            if (digits == 0) return false;
        }
    }
    *out = (neg ? -1 : 1) * (exponent ? std::ldexp(m * std::pow(5.0, exponent), exponent) : m);
    return true;
}

// parseReal: skip blanks, take the token up to a blank, default 0 when it does not parse.
float obj_real(const char*& p) {
    p += std::strspn(p, " \t");
    const char* end = p + std::strcspn(p, " \t\r");
    double v = 0.0;
    obj_parse_double(p, end, &v);
    p = end;
    return (float)v;
}

int obj_fix_index(int idx, int n) {   // 1-based, 0 stays 0, negative = relative
    if (idx > 0) return idx - 1;
    if (idx == 0) return 0;
    return n + idx;
}

struct ObjCorner {
    int v = -1, vt = -1, vn = -1;
};

// parseTriple: v, v/vt, v//vn, v/vt/vn
ObjCorner obj_corner(const char*& p, int nv, int nvn, int nvt) {
    ObjCorner c;
    c.v = obj_fix_index(std::atoi(p), nv);
    p += std::strcspn(p, "/ \t\r");
    if (*p != '/') return c;
    ++p;
    if (*p == '/') {
        ++p;
        c.vn = obj_fix_index(std::atoi(p), nvn);
        p += std::strcspn(p, "/ \t\r");
        return c;
    }
    c.vt = obj_fix_index(std::atoi(p), nvt);
    p += std::strcspn(p, "/ \t\r");
    if (*p != '/') return c;
    ++p;
    c.vn = obj_fix_index(std::atoi(p), nvn);
    p += std::strcspn(p, "/ \t\r");
    return c;
}

struct ObjData {
    std::vector<float> v, vn, vt;
    std::vector<int32_t> face_sizes;
    std::vector<ObjCorner> corners;   // per face-vertex, faces in file order
};

int parse_obj(const std::string& path, ObjData& d) {
    std::ifstream f(path, std::ios::binary);
    if (!f) return fail(PT_ERR_IO, "cannot open OBJ file " + path);
    std::string line;
    while (std::getline(f, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const char* p = line.c_str();
        p += std::strspn(p, " \t");
        if (*p == '\0' || *p == '#') continue;
        const auto blank = [](char c) { return c == ' ' || c == '\t'; };
        if (p[0] == 'v' && blank(p[1])) {
            p += 2;
            for (int k = 0; k < 3; ++k) d.v.push_back(obj_real(p));
        } else if (p[0] == 'v' && p[1] == 'n' && blank(p[2])) {
            p += 3;
            for (int k = 0; k < 3; ++k) d.vn.push_back(obj_real(p));
        } else if (p[0] == 'v' && p[1] == 't' && blank(p[2])) {
            p += 3;
            for (int k = 0; k < 2; ++k) d.vt.push_back(obj_real(p));
        } else if (p[0] == 'f' && blank(p[1])) {
            p += 2;
            p += std::strspn(p, " \t");
            int n = 0;
            while (*p != '\0' && *p != '\r' && *p != '\n') {
                d.corners.push_back(obj_corner(p, (int)d.v.size() / 3, (int)d.vn.size() / 3, (int)d.vt.size() / 2));
                ++n;
                p += std::strspn(p, " \t\r");
            }
            d.face_sizes.push_back(n);
        }
        // mtllib / usemtl / g / o / s: groups only split shapes, the face order is unchanged
    }
    return PT_OK;
}

// glm::vec3(M * vec4(x, y, z, w)) with glm's (m0 v0 + m1 v1) + (m2 v2 + m3 v3) association
void xform4(const float* m, float x, float y, float z, float w, float* out) {
    for (int r = 0; r < 3; ++r) out[r] = (m[r] * x + m[4 + r] * y) + (m[8 + r] * z + m[12 + r] * w);
}

void tri_bounds(const pt_triangle& t, float* mn, float* mx) {   // Triangle::calculate_boundaries
    for (int a = 0; a < 3; ++a) {
        const float x = t.v[0][a], y = t.v[1][a], z = t.v[2][a];
        const float lo = x < y ? x : y, hi = x > y ? x : y;   // glm::min / glm::max
        mn[a] = lo < z ? lo : z;
        mx[a] = hi > z ? hi : z;
    }
}

// Fan-triangulate faces into world-space triangles of a new mesh geom.  Returns the geom id, or
// a negated PT_ERR_* code (the scene is left unchanged on error).  World vertices must be finite
// and below 2^126 in magnitude: beyond, the SAH build (BVH_tree.cpp:27-126) meets NaN or infinite
// centres or extents, puts every triangle in one bucket and recurses on the same range without end
// (the reference's behaviour there is undefined: an unbounded recursion); tinyobj reads no NaN, so
// only a programmatic mesh or an extreme transform gets here.
int append_mesh_impl(Scene& S, int32_t mat, const float* t, const float* r, const float* s, const float* pos, int32_t npos,
                const float* nrm, int32_t nnrm, const float* uv, int32_t nuv, const int32_t* face_sizes, int32_t nfaces,
                const ObjCorner* corners, int64_t ncorners) {
    const int gid = scene_add_geom(S, PT_GEOM_MESH, mat, t, r, s);
    pt_geom& g = S.geoms[(size_t)gid];
    g.tri_start = (int32_t)S.tris_load.size();
    g.bbox_idx = 0;
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {FLT_MIN, FLT_MIN, FLT_MIN};
    int64_t base = 0;
    for (int32_t f = 0; f < nfaces; ++f) {
        const int n = face_sizes[f];
        if (n < 0 || base + n > ncorners) return -fail(PT_ERR_ARG, "mesh face indices out of range");
        for (int k = 2; k < n; ++k) {
            const ObjCorner* c[3] = {&corners[base], &corners[base + k - 1], &corners[base + k]};
            pt_triangle tri;
            std::memset(&tri, 0, sizeof tri);
            for (int j = 0; j < 3; ++j) {
                if (c[j]->v < 0 || c[j]->v >= npos) return -fail(PT_ERR_ARG, "mesh vertex index out of range");
                const float* p = pos + 3 * (size_t)c[j]->v;
                xform4(g.transform, p[0], p[1], p[2], 1.0f, tri.v[j]);
                if (c[j]->vn >= 0) {
                    if (c[j]->vn >= nnrm) return -fail(PT_ERR_ARG, "mesh normal index out of range");
                    const float* q = nrm + 3 * (size_t)c[j]->vn;
                    xform4(g.inv_transpose, q[0], q[1], q[2], 0.0f, tri.n[j]);
                }
                if (c[j]->vt >= 0) {
                    if (c[j]->vt >= nuv) return -fail(PT_ERR_ARG, "mesh uv index out of range");
                    tri.uv[j][0] = uv[2 * (size_t)c[j]->vt];
                    tri.uv[j][1] = uv[2 * (size_t)c[j]->vt + 1];
                }
            }
            for (int j = 0; j < 3; ++j)   // (see below)
                for (int a = 0; a < 3; ++a)
                    if (!(std::fabs(tri.v[j][a]) < 0x1p126f))
                        return -fail(PT_ERR_ARG, "mesh vertex not finite, or beyond 2^126, after the transform");
            tri_bounds(tri, tri.bmin, tri.bmax);
            for (int a = 0; a < 3; ++a) {   // std::min / std::max (scene.cpp:146-160)
                mn[a] = mn[a] < tri.bmin[a] ? mn[a] : tri.bmin[a];
                mx[a] = tri.bmax[a] < mx[a] ? mx[a] : tri.bmax[a];
            }
            tri.id = (int32_t)S.tris_load.size();
            S.tris_load.push_back(tri);
        }
        base += n;
    }
    S.geoms[(size_t)gid].tri_end = (int32_t)S.tris_load.size();
    for (int a = 0; a < 3; ++a) {
        S.geoms[(size_t)gid].min_bound[a] = mn[a];
        S.geoms[(size_t)gid].max_bound[a] = mx[a];
    }
    S.bvh_built = false;
    return gid;
}

int append_mesh(Scene& S, int32_t mat, const float* t, const float* r, const float* s, const float* pos, int32_t npos,
                const float* nrm, int32_t nnrm, const float* uv, int32_t nuv, const int32_t* face_sizes, int32_t nfaces,
                const ObjCorner* corners, int64_t ncorners) {
    const size_t ng = S.geoms.size(), nt = S.tris_load.size();
    const int rc = append_mesh_impl(S, mat, t, r, s, pos, npos, nrm, nnrm, uv, nuv, face_sizes, nfaces, corners,
                                    ncorners);
    if (rc < 0) {
        S.geoms.resize(ng);
        S.tris_load.resize(nt);
    }
    return rc;
}

// ---- BVH --------------------------------------------------------------------------------
struct Box {
    float mn[3], mx[3];
};
bool is_zero(const Box& b) {
    return b.mn[0] == 0.0f && b.mn[1] == 0.0f && b.mn[2] == 0.0f && b.mx[0] == 0.0f && b.mx[1] == 0.0f &&
           b.mx[2] == 0.0f;
}
Box box_union(const Box& self, const Box& o) {   // self || o
    if (is_zero(self)) return o;
    Box r;
    for (int a = 0; a < 3; ++a) {
        r.mn[a] = o.mn[a] < self.mn[a] ? o.mn[a] : self.mn[a];
        r.mx[a] = o.mx[a] > self.mx[a] ? o.mx[a] : self.mx[a];
    }
    return r;
}
Box box_union_point(const Box& self, const float* p) {
    Box r;
    for (int a = 0; a < 3; ++a) {
        r.mn[a] = p[a] < self.mn[a] ? p[a] : self.mn[a];
        r.mx[a] = p[a] > self.mx[a] ? p[a] : self.mx[a];
    }
    return r;
}
float box_area(const Box& b) {
    const float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return 2.0f * ((dx * dy + dx * dz) + dy * dz);
}
int longest_axis(const Box& b) {
    const float dx = b.mx[0] - b.mn[0], dy = b.mx[1] - b.mn[1], dz = b.mx[2] - b.mn[2];
    return (dx > dy && dx > dz) ? 0 : (dy > dz) ? 1 : 2;
}
float box_offset(const Box& b, const float* p, int axis) {   // getOffsetBoxes(p)[axis]
    float o = p[axis] - b.mn[axis];
    if (b.mx[axis] > b.mn[axis]) o /= (b.mx[axis] - b.mn[axis]);
    return o;
}

struct Prim {
    int index;
    Box bounds;
    float center[3];
};

struct BuildNode {
    Box box;
    int left = -1, right = -1;   // indices into the node pool
    int axis = -1, count = 0, first = 0;
};

constexpr int kRegions = 7;   // MAX_AREAS - 1

// getOffsetBoxes -> bucket (BVH_tree.cpp:75-84): (int)(7 * offset), 7 -> 6.  Offsets outside
// [0, 7] — where the reference's int conversion is undefined (NaN or infinite centres) or indexes
// outside its buckets — are clamped; every defined case is unchanged (bvh_build.hip: the same).
int region_of(const Box& cb, const Prim& p, int axis) {
    const float f = kRegions * box_offset(cb, p.center, axis);
    return !(f >= 0.0f) ? 0 : (f >= (float)kRegions ? kRegions - 1 : (int)f);
}

struct Builder {
    std::vector<Prim>& prims;
    const std::vector<pt_triangle>& tris;
    std::vector<pt_triangle>& ordered;
    std::vector<BuildNode> pool;

    int leaf(int start, int end, const Box& bounds) {
        BuildNode n;
        n.box = bounds;
        n.first = (int)ordered.size();
        n.count = end - start;
        for (int i = start; i < end; ++i) ordered.push_back(tris[(size_t)prims[(size_t)i].index]);
        pool.push_back(n);
        return (int)pool.size() - 1;
    }
    int inner(int axis, int l, int r) {
        BuildNode n;
        n.axis = axis;
        n.left = l;
        n.right = r;
        n.box = box_union(pool[(size_t)l].box, pool[(size_t)r].box);
        pool.push_back(n);
        return (int)pool.size() - 1;
    }

    // build_bvh (BVH_tree.cpp:27-126); the node pool is post-order, flattened afterwards
    int build(int start, int end) {
        Box bounds = prims[(size_t)start].bounds;
        for (int i = start; i < end; ++i) bounds = box_union(bounds, prims[(size_t)i].bounds);
        const int n = end - start;
        if (n == 1) return leaf(start, end, bounds);
        Box cb;
        for (int a = 0; a < 3; ++a) cb.mn[a] = cb.mx[a] = prims[(size_t)start].center[a];
        for (int i = start; i < end; ++i) cb = box_union_point(cb, prims[(size_t)i].center);
        const int axis = longest_axis(cb);
        if (cb.mn[axis] == cb.mx[axis]) return leaf(start, end, bounds);
        if (n == 2) {
            // nth_element on two elements == insertion sort: swap when second < first
            if (prims[(size_t)start + 1].center[axis] < prims[(size_t)start].center[axis])
                std::swap(prims[(size_t)start], prims[(size_t)start + 1]);
            const int mid = (int)(1.0f * (float)(start + end) / 2.0f);
            const int l = build(start, mid);
            const int r = build(mid, end);
            return inner(axis, l, r);
        }
        int count[kRegions] = {};
        Box rb[kRegions];
        std::memset(rb, 0, sizeof rb);
        for (int i = start; i < end; ++i) {
            const int idx = region_of(cb, prims[(size_t)i], axis);
            count[idx] += 1;
            rb[idx] = box_union(rb[idx], prims[(size_t)i].bounds);
        }
        float cost[kRegions - 1];
        const float total_area = box_area(bounds);
        for (int i = 0; i < kRegions - 1; ++i) {
            int c0 = 0, c1 = 0;
            Box a0, a1;
            std::memset(&a0, 0, sizeof a0);
            std::memset(&a1, 0, sizeof a1);
            for (int j = 0; j < i; ++j) { c0 += count[j]; a0 = box_union(a0, rb[j]); }
            for (int j = i + 1; j < kRegions; ++j) { c1 += count[j]; a1 = box_union(a1, rb[j]); }
            cost[i] = 1.0f * ((float)c0 * box_area(a0) + (float)c1 * box_area(a1)) / total_area;
        }
        float min_cost = FLT_MAX;
        int split = 0;
        for (int i = 0; i < kRegions - 1; ++i)
            if (cost[i] < min_cost) { min_cost = cost[i]; split = i; }
        if (min_cost >= (float)n && n <= kRegions + 1) return leaf(start, end, bounds);
        // libstdc++ std::partition (bidirectional form)
        int first = start, last = end;
        const auto pred = [&](int i) { return region_of(cb, prims[(size_t)i], axis) <= split; };
        for (;;) {
            for (;;) {
                if (first == last) goto done;
                if (pred(first)) ++first;
                else break;
            }
            --last;
            for (;;) {
                if (first == last) goto done;
                if (!pred(last)) --last;
                else break;
            }
            std::swap(prims[(size_t)first], prims[(size_t)last]);
            ++first;
        }
    done:
        const int mid = (int)(float)first;   // the reference keeps the split index in a float
        const int l = build(start, mid);
        const int r = build(mid, end);
        return inner(axis, l, r);
    }
};

// traverse_bvh (BVH_tree.cpp:128-147): depth-first, left child at index + 1.
int flatten(const std::vector<BuildNode>& pool, int node, std::vector<pt_bvh_node>& out) {
    const BuildNode& b = pool[(size_t)node];
    const int me = (int)out.size();
    pt_bvh_node f;
    std::memset(&f, 0, sizeof f);
    for (int a = 0; a < 3; ++a) { f.bmin[a] = b.box.mn[a]; f.bmax[a] = b.box.mx[a]; }
    out.push_back(f);
    if (b.count > 0) {
        out[(size_t)me].sub_areas = b.count;
        out[(size_t)me].first_area_idx = b.first;
        out[(size_t)me].axis = -1;
        out[(size_t)me].rchild_idx = -1;
        return me;
    }
    out[(size_t)me].sub_areas = 0;
    out[(size_t)me].axis = b.axis;
    out[(size_t)me].first_area_idx = 0;
    flatten(pool, b.left, out);
    const int r = flatten(pool, b.right, out);
    out[(size_t)me].rchild_idx = r;
    return me;
}

}  // namespace

int load_obj_mesh(Scene& S, const std::string& path, int32_t mat, const float* t, const float* r, const float* s) {
    ObjData d;
    if (int rc = parse_obj(path, d)) return rc;
    const int gid = append_mesh(S, mat, t, r, s, d.v.data(), (int32_t)d.v.size() / 3, d.vn.data(),
                                (int32_t)d.vn.size() / 3, d.vt.data(), (int32_t)d.vt.size() / 2, d.face_sizes.data(),
                                (int32_t)d.face_sizes.size(), d.corners.data(), (int64_t)d.corners.size());
    return gid < 0 ? -gid : PT_OK;
}

int add_mesh(Scene& S, int32_t mat, const float* t, const float* r, const float* s, const float* pos, int32_t npos,
             const float* nrm, int32_t nnrm, const float* uv, int32_t nuv, const int32_t* face_sizes, int32_t nfaces,
             const int32_t* ip, const int32_t* in, const int32_t* it, int32_t* id_out) {
    if (!t || !r || !s || (nfaces > 0 && (!face_sizes || !ip)) || (npos > 0 && !pos))
        return fail(PT_ERR_ARG, "null mesh argument");
    int64_t ncorners = 0;
    for (int32_t f = 0; f < nfaces; ++f) ncorners += face_sizes[f] > 0 ? face_sizes[f] : 0;
    std::vector<ObjCorner> corners((size_t)ncorners);
    for (int64_t k = 0; k < ncorners; ++k) {
        corners[(size_t)k].v = ip[k];
        corners[(size_t)k].vn = in ? in[k] : -1;
        corners[(size_t)k].vt = it ? it[k] : -1;
    }
    const int gid = append_mesh(S, mat, t, r, s, pos, npos, nrm, nrm ? nnrm : 0, uv, uv ? nuv : 0, face_sizes, nfaces,
                                corners.data(), ncorners);
    if (gid < 0) return -gid;
    if (id_out) *id_out = gid;
    return PT_OK;
}

// build_bvh_tree (BVH_tree.cpp:149-181): one tree over every mesh triangle of the scene, always
// from the load order (finalize may run more than once).
int build_bvh(Scene& S) {
    S.bvh.clear();
    S.triangles.clear();
    if (!S.tris_load.empty()) {
        std::vector<Prim> prims(S.tris_load.size());
        for (size_t i = 0; i < S.tris_load.size(); ++i) {
            Prim& p = prims[i];
            p.index = (int)i;
            tri_bounds(S.tris_load[i], p.bounds.mn, p.bounds.mx);
            for (int a = 0; a < 3; ++a) p.center[a] = 0.5f * (p.bounds.mn[a] + p.bounds.mx[a]);
        }
        S.triangles.reserve(S.tris_load.size());
        Builder b{prims, S.tris_load, S.triangles, {}};
        b.pool.reserve(2 * prims.size());
        const int root = b.build(0, (int)prims.size());
        flatten(b.pool, root, S.bvh);
    }
    S.bvh_built = true;
    return PT_OK;
}

}  // namespace pt

extern "C" int pt_scene_add_mesh(pt_scene* s, int32_t mat, const float* t, const float* r, const float* sc,
                                 const float* pos, int32_t npos, const float* nrm, int32_t nnrm, const float* uv,
                                 int32_t nuv, const int32_t* fs, int32_t nf, const int32_t* ip, const int32_t* in,
                                 const int32_t* it, int32_t* id_out) {
    if (!s) return pt::fail(PT_ERR_ARG, "null scene");
    return pt::add_mesh(*reinterpret_cast<pt::Scene*>(s), mat, t, r, sc, pos, npos, nrm, nnrm, uv, nuv, fs, nf, ip, in,
                        it, id_out);
}

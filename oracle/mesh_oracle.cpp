// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/binding.py).  Serial CPU restatement of the
// reference's mesh path, written literally from the reference sources so the product's own
// restatement (cuda_pathtracer_amd/csrc/pt_mesh.cpp, structured differently) can be checked
// against it:
//   * tinyobjloader 1.0.6 (path_tracer/src/tiny_obj_loader.h, vendored in the reference):
//     tryParseDouble :474-578, parseReal :580, fixIndex :425, parseTriple :692-723, the 'v' /
//     'vn' / 'vt' / 'f' line handling of LoadObj and exportFaceGroupToShape's triangle fan :890-944;
//   * Scene::loadFromJSON's mesh branch (scene.cpp:94-173): world-space vertices and normals,
//     Triangle::calculate_boundaries, the geom bound starting at (FLT_MAX, FLT_MIN);
//   * BVH_tree.cpp:27-181 + boundingbox.h: recursive build with BVHTreeNode objects, the real
//     std::nth_element / std::partition of this toolchain's libstdc++, DFS flattening.
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <fstream>
#include <string>
#include <vector>

extern "C" {
struct MTriangle {             // == OTriangle / pt_triangle (124 bytes)
    int32_t id;
    float v[3][3];
    float uv[3][2];
    float n[3][3];
    float bmin[3], bmax[3];
};
struct MNode {                 // == ONode / pt_bvh_node (40 bytes)
    float bmin[3], bmax[3];
    int32_t sub_areas, axis, first_area_idx, rchild_idx;
};
}

namespace {

#define M_IS_DIGIT(x) (static_cast<unsigned int>((x) - '0') < static_cast<unsigned int>(10))

bool tryParseDouble(const char* s, const char* s_end, double* result) {
    if (s >= s_end) return false;
    double mantissa = 0.0;
    int exponent = 0;
    char sign = '+';
    char exp_sign = '+';
    char const* curr = s;
    int read = 0;
    bool end_not_reached = false;
    if (*curr == '+' || *curr == '-') {
        sign = *curr;
        curr++;
    } else if (M_IS_DIGIT(*curr)) {
    } else {
        goto fail;
    }
    end_not_reached = (curr != s_end);
    while (end_not_reached && M_IS_DIGIT(*curr)) {
        mantissa *= 10;
        mantissa += static_cast<int>(*curr - 0x30);
        curr++;
        read++;
        end_not_reached = (curr != s_end);
    }
    if (read == 0) goto fail;
    if (!end_not_reached) goto assemble;
    if (*curr == '.') {
        curr++;
        read = 1;
        end_not_reached = (curr != s_end);
        while (end_not_reached && M_IS_DIGIT(*curr)) {
            static const double pow_lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            const int lut_entries = sizeof pow_lut / sizeof pow_lut[0];
            mantissa += static_cast<int>(*curr - 0x30) * (read < lut_entries ? pow_lut[read] : std::pow(10.0, -read));
            read++;
            curr++;
            end_not_reached = (curr != s_end);
        }
    } else if (*curr == 'e' || *curr == 'E') {
    } else {
        goto assemble;
    }
    if (!end_not_reached) goto assemble;
    if (*curr == 'e' || *curr == 'E') {
        curr++;
        end_not_reached = (curr != s_end);
        if (end_not_reached && (*curr == '+' || *curr == '-')) {
            exp_sign = *curr;
            curr++;
        } else if (M_IS_DIGIT(*curr)) {
        } else {
            goto fail;
        }
        read = 0;
        end_not_reached = (curr != s_end);
        while (end_not_reached && M_IS_DIGIT(*curr)) {
            exponent *= 10;
            exponent += static_cast<int>(*curr - 0x30);
            curr++;
            read++;
            end_not_reached = (curr != s_end);
        }
        exponent *= (exp_sign == '+' ? 1 : -1);
        if (read == 0) goto fail;
    }
assemble:
    *result = (sign == '+' ? 1 : -1) * (exponent ? std::ldexp(mantissa * std::pow(5.0, exponent), exponent) : mantissa);
    return true;
fail:
    return false;
}

float parseReal(const char** token, double default_value = 0.0) {
    (*token) += strspn((*token), " \t");
    const char* end = (*token) + strcspn((*token), " \t\r");
    double val = default_value;
    tryParseDouble((*token), end, &val);
    float f = static_cast<float>(val);
    (*token) = end;
    return f;
}

int fixIndex(int idx, int n) {
    if (idx > 0) return idx - 1;
    if (idx == 0) return 0;
    return n + idx;
}

struct vertex_index { int v_idx, vt_idx, vn_idx; };

vertex_index parseTriple(const char** token, int vsize, int vnsize, int vtsize) {
    vertex_index vi{-1, -1, -1};
    vi.v_idx = fixIndex(atoi((*token)), vsize);
    (*token) += strcspn((*token), "/ \t\r");
    if ((*token)[0] != '/') return vi;
    (*token)++;
    if ((*token)[0] == '/') {
        (*token)++;
        vi.vn_idx = fixIndex(atoi((*token)), vnsize);
        (*token) += strcspn((*token), "/ \t\r");
        return vi;
    }
    vi.vt_idx = fixIndex(atoi((*token)), vtsize);
    (*token) += strcspn((*token), "/ \t\r");
    if ((*token)[0] != '/') return vi;
    (*token)++;
    vi.vn_idx = fixIndex(atoi((*token)), vnsize);
    (*token) += strcspn((*token), "/ \t\r");
    return vi;
}

#define M_IS_SPACE(x) (((x) == ' ') || ((x) == '\t'))
#define M_IS_NEW_LINE(x) (((x) == '\r') || ((x) == '\n') || ((x) == '\0'))

struct Obj {
    std::vector<float> v, vn, vt;
    std::vector<vertex_index> tri_corners;   // after the fan conversion, 3 per triangle
};

bool load_obj(const char* path, Obj& o) {
    std::ifstream f(path);
    if (!f) return false;
    std::string linebuf;
    while (std::getline(f, linebuf)) {
        if (!linebuf.empty() && linebuf[linebuf.size() - 1] == '\r') linebuf.erase(linebuf.size() - 1);
        if (linebuf.empty()) continue;
        const char* token = linebuf.c_str();
        token += strspn(token, " \t");
        if (token[0] == '\0' || token[0] == '#') continue;
        if (token[0] == 'v' && M_IS_SPACE(token[1])) {
            token += 2;
            float x = parseReal(&token), y = parseReal(&token), z = parseReal(&token);
            o.v.push_back(x); o.v.push_back(y); o.v.push_back(z);
            continue;
        }
        if (token[0] == 'v' && token[1] == 'n' && M_IS_SPACE(token[2])) {
            token += 3;
            float x = parseReal(&token), y = parseReal(&token), z = parseReal(&token);
            o.vn.push_back(x); o.vn.push_back(y); o.vn.push_back(z);
            continue;
        }
        if (token[0] == 'v' && token[1] == 't' && M_IS_SPACE(token[2])) {
            token += 3;
            float x = parseReal(&token), y = parseReal(&token);
            o.vt.push_back(x); o.vt.push_back(y);
            continue;
        }
        if (token[0] == 'f' && M_IS_SPACE(token[1])) {
            token += 2;
            token += strspn(token, " \t");
            std::vector<vertex_index> face;
            while (!M_IS_NEW_LINE(token[0])) {
                face.push_back(parseTriple(&token, (int)(o.v.size() / 3), (int)(o.vn.size() / 3), (int)(o.vt.size() / 2)));
                size_t n = strspn(token, " \t\r");
                token += n;
            }
            if (face.empty()) continue;
            vertex_index i0 = face[0], i1{-1, -1, -1}, i2 = face[1 < face.size() ? 1 : 0];
            for (size_t k = 2; k < face.size(); k++) {   // polygon -> triangle fan
                i1 = i2;
                i2 = face[k];
                o.tri_corners.push_back(i0);
                o.tri_corners.push_back(i1);
                o.tri_corners.push_back(i2);
            }
        }
    }
    return true;
}

// ---- BoundingBox / BVH (boundingbox.h, BVH_tree.{h,cpp}) ----------------------------------
struct BoundingBox {
    float mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
    BoundingBox() {}
    BoundingBox(const float* a, const float* b) { for (int i = 0; i < 3; ++i) { mn[i] = a[i]; mx[i] = b[i]; } }
    int longest_axis() const {
        float d[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        return (d[0] > d[1] && d[0] > d[2]) ? 0 : (d[1] > d[2]) ? 1 : 2;
    }
    float area() const {
        float d[3] = {mx[0] - mn[0], mx[1] - mn[1], mx[2] - mn[2]};
        return 2.0f * (d[0] * d[1] + d[0] * d[2] + d[1] * d[2]);
    }
    BoundingBox operator||(const BoundingBox& b) const {
        if (mn[0] == 0.0f && mn[1] == 0.0f && mn[2] == 0.0f && mx[0] == 0.0f && mx[1] == 0.0f && mx[2] == 0.0f) return b;
        BoundingBox r;
        for (int i = 0; i < 3; ++i) {
            r.mn[i] = b.mn[i] < mn[i] ? b.mn[i] : mn[i];   // glm::min(b, this)
            r.mx[i] = b.mx[i] > mx[i] ? b.mx[i] : mx[i];   // glm::max(b, this)
        }
        return r;
    }
    BoundingBox point_union(const float* p) const {
        BoundingBox r;
        for (int i = 0; i < 3; ++i) {
            r.mn[i] = p[i] < mn[i] ? p[i] : mn[i];
            r.mx[i] = p[i] > mx[i] ? p[i] : mx[i];
        }
        return r;
    }
    void offset(const float* p, float* o) const {
        for (int i = 0; i < 3; ++i) {
            o[i] = p[i] - mn[i];
            if (mx[i] > mn[i]) o[i] /= (mx[i] - mn[i]);
        }
    }
};

struct BVH_BBox {
    int index;
    BoundingBox bounds;
    float center[3];
};

struct BVHTreeNode {
    BoundingBox bbox;
    BVHTreeNode* L = nullptr;
    BVHTreeNode* R = nullptr;
    int Axis = -1, sub_areas = 0, first_area_idx = 0;
};

int CMP_AXIS = 0;
bool compare_bbox(const BVH_BBox& a, const BVH_BBox& b) { return a.center[CMP_AXIS] < b.center[CMP_AXIS]; }

BVHTreeNode* build_bvh(std::vector<BVH_BBox>& bb, std::vector<MTriangle>& ordered, const std::vector<MTriangle>& tris,
                       int start, int end, int& n_nodes) {
    BVHTreeNode* node = new BVHTreeNode();
    n_nodes += 1;
    BoundingBox bounds = bb[start].bounds;
    for (int i = start; i < end; ++i) bounds = bounds || bb[i].bounds;
    const int n_tris = end - start;
    auto make_leaf = [&]() {
        node->first_area_idx = (int)ordered.size();
        for (int i = start; i < end; ++i) ordered.push_back(tris[bb[i].index]);
        node->sub_areas = n_tris;
        node->bbox = bounds;
        node->Axis = -1;
        return node;
    };
    if (n_tris == 1) return make_leaf();
    BoundingBox central(bb[start].center, bb[start].center);
    for (int i = start; i < end; ++i) central = central.point_union(bb[i].center);
    const int axis = central.longest_axis();
    if (central.mn[axis] == central.mx[axis]) return make_leaf();
    float mid;
    if (n_tris == 2) {
        mid = 1.0f * (start + end) / 2.0f;
        CMP_AXIS = axis;
        std::nth_element(&bb[start], &bb[(int)mid], &bb[end - 1] + 1, compare_bbox);
    } else {
        constexpr int n_regions = 7;
        int count[n_regions] = {};
        BoundingBox rb[n_regions];
        float off[3];
        for (int i = start; i < end; ++i) {
            central.offset(bb[i].center, off);
            int idx = n_regions * off[axis];
            if (idx == n_regions) idx = n_regions - 1;
            count[idx] += 1;
            rb[idx] = rb[idx] || bb[i].bounds;
        }
        float cost[n_regions - 1];
        for (int i = 0; i < n_regions - 1; ++i) {
            int c0 = 0, c1 = 0;
            BoundingBox a0, a1;
            for (int j = 0; j < i; ++j) { c0 += count[j]; a0 = a0 || rb[j]; }
            for (int j = i + 1; j < n_regions; ++j) { c1 += count[j]; a1 = a1 || rb[j]; }
            cost[i] = 1.0f * (c0 * a0.area() + c1 * a1.area()) / bounds.area();
        }
        float min_cost = FLT_MAX;
        int split_idx = 0;
        for (int i = 0; i < n_regions - 1; ++i)
            if (cost[i] < min_cost) { min_cost = cost[i]; split_idx = i; }
        if (min_cost >= n_tris && n_tris <= 8) return make_leaf();
        BVH_BBox* mid_ptr = std::partition(&bb[start], &bb[end - 1] + 1, [&](const BVH_BBox& b) {
            float o[3];
            central.offset(b.center, o);
            int idx = n_regions * o[axis];
            if (idx == n_regions) idx = n_regions - 1;
            return idx <= split_idx;
        });
        mid = mid_ptr - &bb[0];
    }
    node->L = build_bvh(bb, ordered, tris, start, (int)mid, n_nodes);
    node->R = build_bvh(bb, ordered, tris, (int)mid, end, n_nodes);
    node->Axis = axis;
    node->bbox = node->L->bbox || node->R->bbox;
    node->sub_areas = 0;
    return node;
}

int traverse_bvh(BVHTreeNode* node, MNode* tree, int& offset) {
    MNode* t = &tree[offset];
    for (int i = 0; i < 3; ++i) { t->bmin[i] = node->bbox.mn[i]; t->bmax[i] = node->bbox.mx[i]; }
    int next_offset = offset++;
    if (node->sub_areas > 0) {
        t->first_area_idx = node->first_area_idx;
        t->sub_areas = node->sub_areas;
        t->axis = -1;
        t->rchild_idx = -1;
        return next_offset;
    }
    t->sub_areas = 0;
    t->axis = node->Axis;
    t->first_area_idx = 0;
    traverse_bvh(node->L, tree, offset);
    t->rchild_idx = traverse_bvh(node->R, tree, offset);
    return next_offset;
}

void delete_tree(BVHTreeNode* n) {
    if (!n) return;
    delete_tree(n->L);
    delete_tree(n->R);
    delete n;
}

}  // namespace

extern "C" {

// Loads an OBJ as world-space triangles of one mesh geom (ids id_base, id_base+1, ...).  Returns
// the triangle count (writes at most `cap`), or -1 if the file cannot be read.  T / IT: the
// geom's transform and inverse-transpose, glm column-major.  bmin/bmax: the geom bound.
int oracle_load_obj(const char* path, const float* T, const float* IT, int id_base, MTriangle* out, int cap,
                    float* bmin, float* bmax) {
    Obj o;
    if (!load_obj(path, o)) return -1;
    const int ntri = (int)(o.tri_corners.size() / 3);
    float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {FLT_MIN, FLT_MIN, FLT_MIN};
    for (int t = 0; t < ntri; ++t) {
        MTriangle tri;
        std::memset(&tri, 0, sizeof tri);
        for (int k = 0; k < 3; ++k) {
            const vertex_index& c = o.tri_corners[3 * t + k];
            const float vx = o.v[3 * c.v_idx], vy = o.v[3 * c.v_idx + 1], vz = o.v[3 * c.v_idx + 2];
            for (int r = 0; r < 3; ++r)   // glm::vec3(transform * vec4(v, 1))
                tri.v[k][r] = (T[r] * vx + T[4 + r] * vy) + (T[8 + r] * vz + T[12 + r] * 1.0f);
            if (c.vn_idx >= 0) {
                const float nx = o.vn[3 * c.vn_idx], ny = o.vn[3 * c.vn_idx + 1], nz = o.vn[3 * c.vn_idx + 2];
                for (int r = 0; r < 3; ++r)   // glm::vec3(invTranspose * vec4(n, 0))
                    tri.n[k][r] = (IT[r] * nx + IT[4 + r] * ny) + (IT[8 + r] * nz + IT[12 + r] * 0.0f);
            }
            if (c.vt_idx >= 0) {
                tri.uv[k][0] = o.vt[2 * c.vt_idx];
                tri.uv[k][1] = o.vt[2 * c.vt_idx + 1];
            }
        }
        for (int a = 0; a < 3; ++a) {   // calculate_boundaries: glm::min(glm::min(v0, v1), v2)
            const float m01 = tri.v[0][a] < tri.v[1][a] ? tri.v[0][a] : tri.v[1][a];
            const float M01 = tri.v[0][a] > tri.v[1][a] ? tri.v[0][a] : tri.v[1][a];
            tri.bmin[a] = m01 < tri.v[2][a] ? m01 : tri.v[2][a];
            tri.bmax[a] = M01 > tri.v[2][a] ? M01 : tri.v[2][a];
            mn[a] = std::min(tri.bmin[a], mn[a]);
            mx[a] = std::max(tri.bmax[a], mx[a]);
        }
        tri.id = id_base + t;
        if (t < cap) out[t] = tri;
    }
    for (int a = 0; a < 3; ++a) { bmin[a] = mn[a]; bmax[a] = mx[a]; }
    return ntri;
}

// build_bvh_tree: reorders tris[0..n) into leaf order in place; writes the flattened nodes
// (at most cap) and returns the node count.
int oracle_build_bvh(MTriangle* tris, int n, MNode* nodes, int cap) {
    if (n <= 0) return 0;
    std::vector<MTriangle> orig(tris, tris + n);
    std::vector<BVH_BBox> bb((size_t)n);
    for (int i = 0; i < n; ++i) {
        bb[i].index = i;
        bb[i].bounds = BoundingBox(orig[i].bmin, orig[i].bmax);
        for (int a = 0; a < 3; ++a) bb[i].center[a] = 0.5f * (orig[i].bmin[a] + orig[i].bmax[a]);
    }
    std::vector<MTriangle> ordered;
    ordered.reserve((size_t)n);
    int n_nodes = 0;
    BVHTreeNode* root = build_bvh(bb, ordered, orig, 0, n, n_nodes);
    std::vector<MNode> flat((size_t)n_nodes);
    int offset = 0;
    traverse_bvh(root, flat.data(), offset);
    delete_tree(root);
    for (int i = 0; i < n; ++i) tris[i] = ordered[(size_t)i];
    for (int i = 0; i < n_nodes && i < cap; ++i) nodes[i] = flat[(size_t)i];
    return n_nodes;
}

}  // extern "C"

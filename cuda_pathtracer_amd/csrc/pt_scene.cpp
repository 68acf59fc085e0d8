// Host-side scene model for the MI355X path tracer: JSON scene loading, object transforms,
// camera set-up, OBJ meshes and the SAH BVH.  Replaces path_tracer/src/scene.{h,cpp},
// utilities.cpp:84-92 (buildTransformationMatrix), the first-frame camera of main.cpp:59-136 and
// BVH_tree.cpp.  Matrix and camera arithmetic follow glm 0.9.6.3's association so the GPU
// renders from exactly the numbers the reference host would have produced.
#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "json_lite.h"
#include "pt_internal.h"

namespace pt {

thread_local std::string g_err;
int fail(int code, const std::string& msg) { g_err = msg; return code; }

namespace {

constexpr float kPI = 3.1415926535897932384626422832795028841971f;   // utilities.h:12

struct Mat4 {
    float c[4][4];   // c[column][row], glm layout
};
Mat4 identity() {
    Mat4 m;
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) m.c[a][b] = a == b ? 1.0f : 0.0f;
    return m;
}
// glm mat4*mat4: column j = ((A0*B[j][0] + A1*B[j][1]) + A2*B[j][2]) + A3*B[j][3]
Mat4 mul(const Mat4& A, const Mat4& B) {
    Mat4 R;
    for (int j = 0; j < 4; ++j)
        for (int r = 0; r < 4; ++r) {
            float acc = A.c[0][r] * B.c[j][0] + A.c[1][r] * B.c[j][1];
            acc = acc + A.c[2][r] * B.c[j][2];
            R.c[j][r] = acc + A.c[3][r] * B.c[j][3];
        }
    return R;
}
Mat4 translate(const float* v) {                 // glm::translate(mat4(), v)
    Mat4 I = identity(), R = I;
    for (int r = 0; r < 4; ++r) {
        float acc = I.c[0][r] * v[0] + I.c[1][r] * v[1];
        acc = acc + I.c[2][r] * v[2];
        R.c[3][r] = acc + I.c[3][r];
    }
    return R;
}
Mat4 rotate(float angle, float ax, float ay, float az) {   // glm::rotate(mat4(), angle, axis)
    const float co = cosf(angle), si = sinf(angle);
    const float inv_len = 1.0f / sqrtf((ax * ax + ay * ay) + az * az);
    const float a[3] = {ax * inv_len, ay * inv_len, az * inv_len};
    const float t[3] = {(1.0f - co) * a[0], (1.0f - co) * a[1], (1.0f - co) * a[2]};
    float Rm[3][3];
    Rm[0][0] = co + t[0] * a[0];
    Rm[0][1] = (0.0f + t[0] * a[1]) + si * a[2];
    Rm[0][2] = (0.0f + t[0] * a[2]) - si * a[1];
    Rm[1][0] = (0.0f + t[1] * a[0]) - si * a[2];
    Rm[1][1] = co + t[1] * a[1];
    Rm[1][2] = (0.0f + t[1] * a[2]) + si * a[0];
    Rm[2][0] = (0.0f + t[2] * a[0]) + si * a[1];
    Rm[2][1] = (0.0f + t[2] * a[1]) - si * a[0];
    Rm[2][2] = co + t[2] * a[2];
    const Mat4 I = identity();
    Mat4 R;
    for (int j = 0; j < 3; ++j)
        for (int r = 0; r < 4; ++r)
            R.c[j][r] = (I.c[0][r] * Rm[j][0] + I.c[1][r] * Rm[j][1]) + I.c[2][r] * Rm[j][2];
    for (int r = 0; r < 4; ++r) R.c[3][r] = I.c[3][r];
    return R;
}
Mat4 scale(const float* v) {                     // glm::scale(mat4(), v)
    const Mat4 I = identity();
    Mat4 R;
    for (int j = 0; j < 3; ++j)
        for (int r = 0; r < 4; ++r) R.c[j][r] = I.c[j][r] * v[j];
    for (int r = 0; r < 4; ++r) R.c[3][r] = I.c[3][r];
    return R;
}
// glm::inverse (detail/type_mat4x4.inl compute_inverse): cofactor pairs, sign vectors, 1/det.
Mat4 inverse(const Mat4& M) {
    auto m = [&](int a, int b) { return M.c[a][b]; };
    const float k00 = m(2,2) * m(3,3) - m(3,2) * m(2,3), k02 = m(1,2) * m(3,3) - m(3,2) * m(1,3), k03 = m(1,2) * m(2,3) - m(2,2) * m(1,3);
    const float k04 = m(2,1) * m(3,3) - m(3,1) * m(2,3), k06 = m(1,1) * m(3,3) - m(3,1) * m(1,3), k07 = m(1,1) * m(2,3) - m(2,1) * m(1,3);
    const float k08 = m(2,1) * m(3,2) - m(3,1) * m(2,2), k10 = m(1,1) * m(3,2) - m(3,1) * m(1,2), k11 = m(1,1) * m(2,2) - m(2,1) * m(1,2);
    const float k12 = m(2,0) * m(3,3) - m(3,0) * m(2,3), k14 = m(1,0) * m(3,3) - m(3,0) * m(1,3), k15 = m(1,0) * m(2,3) - m(2,0) * m(1,3);
    const float k16 = m(2,0) * m(3,2) - m(3,0) * m(2,2), k18 = m(1,0) * m(3,2) - m(3,0) * m(1,2), k19 = m(1,0) * m(2,2) - m(2,0) * m(1,2);
    const float k20 = m(2,0) * m(3,1) - m(3,0) * m(2,1), k22 = m(1,0) * m(3,1) - m(3,0) * m(1,1), k23 = m(1,0) * m(2,1) - m(2,0) * m(1,1);
    const float f[6][4] = {{k00, k00, k02, k03}, {k04, k04, k06, k07}, {k08, k08, k10, k11},
                           {k12, k12, k14, k15}, {k16, k16, k18, k19}, {k20, k20, k22, k23}};
    const float v[4][4] = {{m(1,0), m(0,0), m(0,0), m(0,0)}, {m(1,1), m(0,1), m(0,1), m(0,1)},
                           {m(1,2), m(0,2), m(0,2), m(0,2)}, {m(1,3), m(0,3), m(0,3), m(0,3)}};
    // Inv_c = (v_a * f_p - v_b * f_q + v_c * f_s) * sign
    static const int use[4][6] = {{1, 0, 2, 1, 3, 2}, {0, 0, 2, 3, 3, 4}, {0, 1, 1, 3, 3, 5}, {0, 2, 1, 4, 2, 5}};
    Mat4 R;
    for (int col = 0; col < 4; ++col)
        for (int k = 0; k < 4; ++k) {
            const int* u = use[col];
            float x = v[u[0]][k] * f[u[1]][k] - v[u[2]][k] * f[u[3]][k];
            x = x + v[u[4]][k] * f[u[5]][k];
            const float sign = ((col + k) & 1) ? -1.0f : 1.0f;
            R.c[col][k] = x * sign;
        }
    float d[4];
    for (int k = 0; k < 4; ++k) d[k] = M.c[0][k] * R.c[k][0];
    const float det = (d[0] + d[1]) + (d[2] + d[3]);
    const float inv_det = 1.0f / det;
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) R.c[a][b] = R.c[a][b] * inv_det;
    return R;
}
// glm::inverseTranspose (gtc/matrix_inverse.inl:95-147): adjugate via 19 2x2 sub-factors, / det.
Mat4 inverse_transpose(const Mat4& M) {
    auto m = [&](int a, int b) { return M.c[a][b]; };
    auto sf = [&](int a, int b, int c, int d) { return m(a / 10, a % 10) * m(b / 10, b % 10) - m(c / 10, c % 10) * m(d / 10, d % 10); };
    const float S[19] = {
        sf(22, 33, 32, 23), sf(21, 33, 31, 23), sf(21, 32, 31, 22), sf(20, 33, 30, 23), sf(20, 32, 30, 22),
        sf(20, 31, 30, 21), sf(12, 33, 32, 13), sf(11, 33, 31, 13), sf(11, 32, 31, 12), sf(10, 33, 30, 13),
        sf(10, 32, 30, 12), sf(11, 33, 31, 13), sf(10, 31, 30, 11), sf(12, 23, 22, 13), sf(11, 23, 21, 13),
        sf(11, 22, 21, 12), sf(10, 23, 20, 13), sf(10, 22, 20, 12), sf(10, 21, 20, 11)};
    // entry (c, r) = sign * ((m(p, a) * S[x] - m(p, b) * S[y]) + m(p, e) * S[z])
    struct Term { int p, a, x, b, y, e, z; float sign; };
    static const Term T[16] = {
        {1, 1, 0, 2, 1, 3, 2, +1}, {1, 0, 0, 2, 3, 3, 4, -1}, {1, 0, 1, 1, 3, 3, 5, +1}, {1, 0, 2, 1, 4, 2, 5, -1},
        {0, 1, 0, 2, 1, 3, 2, -1}, {0, 0, 0, 2, 3, 3, 4, +1}, {0, 0, 1, 1, 3, 3, 5, -1}, {0, 0, 2, 1, 4, 2, 5, +1},
        {0, 1, 6, 2, 7, 3, 8, +1}, {0, 0, 6, 2, 9, 3, 10, -1}, {0, 0, 11, 1, 9, 3, 12, +1}, {0, 0, 8, 1, 10, 2, 12, -1},
        {0, 1, 13, 2, 14, 3, 15, -1}, {0, 0, 13, 2, 16, 3, 17, +1}, {0, 0, 14, 1, 16, 3, 18, -1}, {0, 0, 15, 1, 17, 2, 18, +1}};
    Mat4 R;
    for (int i = 0; i < 16; ++i) {
        const Term& t = T[i];
        float x = m(t.p, t.a) * S[t.x] - m(t.p, t.b) * S[t.y];
        x = x + m(t.p, t.e) * S[t.z];
        R.c[i / 4][i % 4] = t.sign > 0 ? +x : -x;
    }
    float det = m(0, 0) * R.c[0][0] + m(0, 1) * R.c[0][1];
    det = det + m(0, 2) * R.c[0][2];
    det = det + m(0, 3) * R.c[0][3];
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) R.c[a][b] = R.c[a][b] / det;
    return R;
}
void store(const Mat4& m, float* out) {
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) out[4 * a + b] = m.c[a][b];
}

// utilityCore::buildTransformationMatrix (utilities.cpp:84-92): T * Rx * Ry * Rz * S, degrees.
void build_transforms(pt_geom& g) {
    const Mat4 T = translate(g.translation);
    Mat4 R = rotate(g.rotation[0] * kPI / 180, 1, 0, 0);
    R = mul(R, rotate(g.rotation[1] * kPI / 180, 0, 1, 0));
    R = mul(R, rotate(g.rotation[2] * kPI / 180, 0, 0, 1));
    const Mat4 S = scale(g.scale);
    const Mat4 X = mul(mul(T, R), S);
    store(X, g.transform);
    store(inverse(X), g.inverse_transform);
    store(inverse_transpose(X), g.inv_transpose);
}

struct V { float x, y, z; };
inline V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline float dotv(V a, V b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
inline V normv(V a) { const float s = 1.0f / sqrtf(dotv(a, a)); return {a.x * s, a.y * s, a.z * s}; }
inline V crossv(V a, V b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }

std::string read_file(const std::string& path, bool* ok) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { *ok = false; return {}; }
    std::stringstream ss;
    ss << f.rdbuf();
    *ok = true;
    return ss.str();
}

std::string parent_dir(const std::string& p) {
    const size_t k = p.find_last_of('/');
    return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

void read3(const jl::Value& a, float* out) {
    for (int i = 0; i < 3; ++i) out[i] = (float)a[i].number();
}

}  // namespace

// ---- camera (scene.cpp:185-211 + main.cpp:59-73 + main.cpp:117-136) ----------------------
// runCuda's camchanged block (main.cpp:117-136): the position on the orbit (zoom, phi, theta) about
// look_at, view towards it, right = view x (0,1,0) (not normalised), up = right x view.
static void apply_orbit(Scene& S, float phi, float theta, float zoom, const float* la_in) {
    pt_camera& cam = S.camera;
    const V la{la_in[0], la_in[1], la_in[2]};
    const V cp{(zoom * sinf(phi)) * sinf(theta), zoom * cosf(theta), (zoom * cosf(phi)) * sinf(theta)};
    const V nv = normv(cp);
    const V v{-nv.x, -nv.y, -nv.z};
    const V r = crossv(v, V{0, 1, 0});
    const V u = crossv(r, v);
    const float p[3] = {cp.x + la.x, cp.y + la.y, cp.z + la.z};
    for (int i = 0; i < 3; ++i) {
        cam.position[i] = p[i];
        cam.look_at[i] = la_in[i];
    }
    cam.view[0] = v.x; cam.view[1] = v.y; cam.view[2] = v.z;
    cam.up[0] = u.x; cam.up[1] = u.y; cam.up[2] = u.z;
    cam.right[0] = r.x; cam.right[1] = r.y; cam.right[2] = r.z;
}

static void finalize_camera(Scene& S) {
    pt_camera& cam = S.camera;
    const V pos{S.eye[0], S.eye[1], S.eye[2]}, la{S.look_at[0], S.look_at[1], S.look_at[2]};
    const float fovy = S.fovy;
    const float yscaled = tanf(fovy * (kPI / 180));
    const float xscaled = (yscaled * cam.res[0]) / cam.res[1];
    const float fovx = (atanf(xscaled) * 180) / kPI;
    cam.fov[0] = fovx;
    cam.fov[1] = fovy;
    cam.pixel_length[0] = 2 * xscaled / (float)cam.res[0];
    cam.pixel_length[1] = 2 * yscaled / (float)cam.res[1];
    // main.cpp:59-73: the orbit angles of the loaded view and its distance to the look-at point
    const V view = normv(sub(la, pos));
    const V vxz{view.x, 0.0f, view.z}, vzy{0.0f, view.y, view.z};
    const float phi = acosf(dotv(normv(vxz), V{0, 0, -1}));
    const float theta = acosf(dotv(normv(vzy), V{0, 1, 0}));
    const float zoom = sqrtf(dotv(sub(pos, la), sub(pos, la)));
    S.orbit[0] = phi;
    S.orbit[1] = theta;
    S.orbit[2] = zoom;
    apply_orbit(S, phi, theta, zoom, S.look_at);   // the first frame (camchanged starts true)
}

int scene_add_geom(Scene& S, int32_t type, int32_t mat, const float* t, const float* r, const float* s) {
    pt_geom g;
    std::memset(&g, 0, sizeof g);
    g.type = type;
    g.material_id = mat;
    for (int i = 0; i < 3; ++i) { g.translation[i] = t[i]; g.rotation[i] = r[i]; g.scale[i] = s[i]; }
    build_transforms(g);
    g.tri_start = g.tri_end = 0;
    g.bbox_idx = -1;
    S.geoms.push_back(g);
    S.finalized = false;
    return (int)S.geoms.size() - 1;
}

// Does the file opt in to the refraction extension?  Top-level "Extensions": {"REFRACTION": true}
// (or a list holding "REFRACTION"); the reference loader ignores unknown top-level keys.
static bool file_wants_refraction(const jl::Value& root) {
    if (!root.has("Extensions")) return false;
    const jl::Value& e = root["Extensions"];
    if (e.kind == jl::Value::Object) return e.has("REFRACTION") && e["REFRACTION"].kind == jl::Value::Bool && e["REFRACTION"].b;
    if (e.kind == jl::Value::Array)
        for (const auto& x : e.arr)
            if (x.kind == jl::Value::String && x.str == "REFRACTION") return true;
    return false;
}

// Scene::loadFromJSON (scene.cpp:33-219).  `options`: PT_LOAD_* bits (pt_amd.h).
static int load_json(Scene& S, const std::string& path, uint32_t options) {
    bool ok = false;
    const std::string text = read_file(path, &ok);
    if (!ok) return fail(PT_ERR_IO, "cannot read scene file " + path);
    jl::Value root;
    try {
        root = jl::parse(text);
    } catch (const std::exception& e) {
        return fail(PT_ERR_PARSE, e.what());
    }
    try {
        const std::string dir = parent_dir(path);
        // The reference reads neither REFRACTIVE nor IOR (scene.cpp:46-56: hasRefractive and
        // indexOfRefraction stay 0), so by default neither do we; the
        // extension is on only when the caller asks (PT_LOAD_REFRACTION) or the file opts in.
        const bool refraction = (options & PT_LOAD_REFRACTION) != 0 || file_wants_refraction(root);
        // Materials: std::map iteration order == sorted names (scene.cpp:42-74).
        std::map<std::string, int> name_to_id;
        const jl::Value& mats = root["Materials"];
        for (const auto& kv : mats.obj) {
            const jl::Value& p = kv.second;
            pt_material m;
            std::memset(&m, 0, sizeof m);
            float rgb[3] = {0, 0, 0};
            if (p.has("RGB")) read3(p["RGB"], rgb);
            float spec[3] = {rgb[0], rgb[1], rgb[2]};
            if (p.has("SPECRGB")) read3(p["SPECRGB"], spec);
            m.spec_exponent = p.has("SPECEX") ? (float)p["SPECEX"].number() : 1.0f;
            m.has_reflective = p.has("REFLECTIVE") ? (float)p["REFLECTIVE"].number() : 0.0f;
            m.emittance = p.has("EMITTANCE") ? (float)p["EMITTANCE"].number() : 0.0f;
            for (int i = 0; i < 3; ++i) { m.color[i] = rgb[i]; m.spec_color[i] = spec[i]; }
            // Extension (north-star config 4; off by default, see above): REFRACTIVE / IOR.  Absent
            // keys keep the reference's zeros.
            if (refraction && p.has("REFRACTIVE")) m.has_refractive = (float)p["REFRACTIVE"].number();
            if (refraction && p.has("IOR")) m.ior = (float)p["IOR"].number();
            m.texture_id = -1;
            name_to_id[kv.first] = (int)S.materials.size();
            if (p.has("TEXTURE_FILE") && !p["TEXTURE_FILE"].string().empty()) {
                m.texture_id = (int)S.textures.size();
                TextureHost th;
                th.path = dir + "/Textures/" + p["TEXTURE_FILE"].string();
                // Texture::load (scene.cpp:61-71): decoded here; a failure ends the load
                if (int rc = load_texture_file(th)) return rc;
                S.textures.push_back(std::move(th));
            }
            S.materials.push_back(m);
        }
        const jl::Value& objs = root["Objects"];
        for (const auto& o : objs.arr) {
            const std::string mname = o["MATERIAL"].string();
            auto it = name_to_id.find(mname);
            int mat_id = 0;
            if (it == name_to_id.end()) name_to_id[mname] = 0;   // std::map operator[] inserts 0
            else mat_id = it->second;
            float t[3], r[3], s[3];
            read3(o["TRANS"], t);
            read3(o["ROTAT"], r);
            read3(o["SCALE"], s);
            const std::string type = o["TYPE"].string();
            if (type == "mesh") {
                const std::string obj = dir + "/Models/" + o["OBJ_FILE"].string();
                const int rc = load_obj_mesh(S, obj, mat_id, t, r, s);
                if (rc) return rc;
            } else if (type == "cube") {
                scene_add_geom(S, PT_GEOM_CUBE, mat_id, t, r, s);
            } else if (type == "sphere") {
                scene_add_geom(S, PT_GEOM_SPHERE, mat_id, t, r, s);
            } else {
                return fail(PT_ERR_PARSE, "unknown object TYPE '" + type + "'");
            }
        }
        const jl::Value& cam = root["Camera"];
        S.camera.res[0] = (int)cam["RES"][0].number();
        S.camera.res[1] = (int)cam["RES"][1].number();
        S.fovy = (float)cam["FOVY"].number();
        S.iterations = (int)cam["ITERATIONS"].number();
        S.depth = (int)cam["DEPTH"].number();
        S.file = cam["FILE"].string();
        read3(cam["EYE"], S.eye);
        read3(cam["LOOKAT"], S.look_at);
        read3(cam["UP"], S.up);
        S.camera_set = true;
    } catch (const std::exception& e) {
        return fail(PT_ERR_PARSE, std::string("scene: ") + e.what());
    }
    return PT_OK;
}

int scene_finalize(Scene& S) {
    if (!S.camera_set) return fail(PT_ERR_ARG, "camera not set");
    if (S.camera.res[0] <= 0 || S.camera.res[1] <= 0) return fail(PT_ERR_ARG, "bad resolution");
    if (S.depth < 1 || S.depth > 64) return fail(PT_ERR_ARG, "DEPTH must be in [1, 64]");
    for (const auto& g : S.geoms)
        if (g.material_id < 0 || g.material_id >= (int)S.materials.size())
            return fail(PT_ERR_ARG, "geom references a missing material");
    finalize_camera(S);
    // BVH (scene.cpp:218 -> BVH_tree.cpp:156): the host restatement, or the same tree built on the
    // current HIP device (falls back to the host for the cases bvh_build.hip leaves to it)
    S.bvh_on_device = 0;
    int rc = 1;
    if (S.bvh_builder == 1) {
        rc = build_bvh_device(S, &S.bvh_ms);
        if (rc == PT_OK) S.bvh_on_device = 1;
        else if (rc != 1) return rc;
    }
    if (rc == 1) {
        const auto t0 = std::chrono::steady_clock::now();
        rc = build_bvh(S);
        S.bvh_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    if (rc) return rc;
    S.finalized = true;
    return PT_OK;
}

}  // namespace pt

using pt::fail;

extern "C" {

const char* pt_last_error(void) { return pt::g_err.c_str(); }

void pt_flags_default(pt_flags* f) {   // utilities.h:23-33
    if (!f) return;
    f->russian_roulette = 1;
    f->use_bvh = 1;
    f->use_bbox = 1;
    f->sort_by_material = 0;
    f->use_thrust_partition = 0;
    f->ssaa = 1;
    f->dof = 1;
    f->single_albedo = 0;
    f->rng_key_pixel = 0;
    f->bvh_cull = 0;
    const char* sched = std::getenv("PT_AMD_SCHEDULE");
    f->shared_gpu = sched && std::strcmp(sched, "claim") == 0;
    f->aperture = 0.1f;
    f->focal_dist = 10.0f;
}

int pt_scene_create(pt_scene** out) {
    if (!out) return fail(PT_ERR_ARG, "null out");
    *out = reinterpret_cast<pt_scene*>(new pt::Scene());
    return PT_OK;
}

void pt_scene_free(pt_scene* s) { delete reinterpret_cast<pt::Scene*>(s); }

int pt_scene_load_json(const char* path, pt_scene** out) { return pt_scene_load_json_ex(path, 0u, out); }

int pt_scene_load_json_ex(const char* path, uint32_t options, pt_scene** out) {
    if (!path || !out) return fail(PT_ERR_ARG, "null argument");
    if (options & ~(uint32_t)(PT_LOAD_REFRACTION | PT_LOAD_DEVICE_BVH)) return fail(PT_ERR_ARG, "unknown PT_LOAD_* option");
    auto* S = new pt::Scene();
    S->bvh_builder = (options & PT_LOAD_DEVICE_BVH) ? 1 : 0;
    int rc = pt::load_json(*S, path, options);
    if (!rc) rc = pt::scene_finalize(*S);
    if (rc) { delete S; return rc; }
    *out = reinterpret_cast<pt_scene*>(S);
    return PT_OK;
}

int pt_scene_set_bvh_builder(pt_scene* s, int32_t device) {
    if (!s || (device != 0 && device != 1)) return fail(PT_ERR_ARG, "bad argument");
    auto& S = *reinterpret_cast<pt::Scene*>(s);
    S.bvh_builder = device;
    return PT_OK;
}

int pt_scene_bvh_build_info(const pt_scene* s, int32_t* on_device, double* ms) {
    if (!s) return fail(PT_ERR_ARG, "null scene");
    const auto& S = *reinterpret_cast<const pt::Scene*>(s);
    if (on_device) *on_device = S.bvh_on_device;
    if (ms) *ms = S.bvh_ms;
    return PT_OK;
}

int pt_scene_add_material(pt_scene* s, const pt_material* m, int32_t* id_out) {
    if (!s || !m) return fail(PT_ERR_ARG, "null argument");
    auto& S = *reinterpret_cast<pt::Scene*>(s);
    if (m->texture_id >= (int)S.textures.size()) return fail(PT_ERR_ARG, "texture_id out of range");
    S.materials.push_back(*m);
    if (id_out) *id_out = (int)S.materials.size() - 1;
    return PT_OK;
}

int pt_scene_add_texture(pt_scene* s, int32_t w, int32_t h, int32_t comps, const uint8_t* px, int32_t* id_out) {
    if (!s || !px || w <= 0 || h <= 0 || comps <= 0) return fail(PT_ERR_ARG, "bad texture");
    auto& S = *reinterpret_cast<pt::Scene*>(s);
    pt::TextureHost th;
    th.width = w; th.height = h; th.components = comps;
    th.pixels.assign(px, px + (size_t)w * h * comps);
    S.textures.push_back(std::move(th));
    if (id_out) *id_out = (int)S.textures.size() - 1;
    return PT_OK;
}

int pt_scene_set_texture_pixels(pt_scene* s, int32_t id, int32_t w, int32_t h, int32_t comps, const uint8_t* px) {
    if (!s || !px || w <= 0 || h <= 0 || comps <= 0) return fail(PT_ERR_ARG, "bad texture");
    auto& S = *reinterpret_cast<pt::Scene*>(s);
    if (id < 0 || id >= (int)S.textures.size()) return fail(PT_ERR_ARG, "texture id out of range");
    auto& th = S.textures[(size_t)id];
    th.width = w; th.height = h; th.components = comps;
    th.pixels.assign(px, px + (size_t)w * h * comps);
    return PT_OK;
}

int pt_scene_texture_path(const pt_scene* s, int32_t id, char* buf, int32_t cap) {
    if (!s || !buf || cap <= 0) return fail(PT_ERR_ARG, "bad argument");
    const auto& S = *reinterpret_cast<const pt::Scene*>(s);
    if (id < 0 || id >= (int)S.textures.size()) return fail(PT_ERR_ARG, "texture id out of range");
    std::snprintf(buf, (size_t)cap, "%s", S.textures[(size_t)id].path.c_str());
    return PT_OK;
}

int pt_scene_add_geom(pt_scene* s, int32_t type, int32_t mat, const float* t, const float* r, const float* sc,
                      int32_t* id_out) {
    if (!s || !t || !r || !sc) return fail(PT_ERR_ARG, "null argument");
    if (type != PT_GEOM_CUBE && type != PT_GEOM_SPHERE) return fail(PT_ERR_ARG, "type must be cube or sphere");
    const int id = pt::scene_add_geom(*reinterpret_cast<pt::Scene*>(s), type, mat, t, r, sc);
    if (id_out) *id_out = id;
    return PT_OK;
}

int pt_scene_set_camera(pt_scene* s, int32_t rx, int32_t ry, float fovy, const float* eye, const float* la,
                        const float* up) {
    if (!s || !eye || !la || !up) return fail(PT_ERR_ARG, "null argument");
    if (rx <= 0 || ry <= 0) return fail(PT_ERR_ARG, "bad resolution");
    auto& S = *reinterpret_cast<pt::Scene*>(s);
    S.camera.res[0] = rx;
    S.camera.res[1] = ry;
    S.fovy = fovy;
    for (int i = 0; i < 3; ++i) { S.eye[i] = eye[i]; S.look_at[i] = la[i]; S.up[i] = up[i]; }
    S.camera_set = true;
    S.finalized = false;
    return PT_OK;
}

int pt_scene_set_render(pt_scene* s, int32_t iterations, int32_t depth, const char* file) {
    if (!s) return fail(PT_ERR_ARG, "null scene");
    auto& S = *reinterpret_cast<pt::Scene*>(s);
    S.iterations = iterations;
    S.depth = depth;
    S.file = file ? file : "";
    S.finalized = false;
    return PT_OK;
}

int pt_scene_finalize(pt_scene* s) {
    if (!s) return fail(PT_ERR_ARG, "null scene");
    return pt::scene_finalize(*reinterpret_cast<pt::Scene*>(s));
}

int pt_scene_counts(const pt_scene* s, int32_t* ng, int32_t* nm, int32_t* nt, int32_t* nn, int32_t* ntex) {
    if (!s) return fail(PT_ERR_ARG, "null scene");
    const auto& S = *reinterpret_cast<const pt::Scene*>(s);
    if (ng) *ng = (int)S.geoms.size();
    if (nm) *nm = (int)S.materials.size();
    if (nt) *nt = (int)S.triangles.size();
    if (nn) *nn = (int)S.bvh.size();
    if (ntex) *ntex = (int)S.textures.size();
    return PT_OK;
}

int pt_scene_get_camera(const pt_scene* s, pt_camera* out) {
    if (!s || !out) return fail(PT_ERR_ARG, "null argument");
    *out = reinterpret_cast<const pt::Scene*>(s)->camera;
    return PT_OK;
}

int pt_scene_get_orbit(const pt_scene* s, float* phi, float* theta, float* zoom) {
    if (!s) return fail(PT_ERR_ARG, "null scene");
    const auto& S = *reinterpret_cast<const pt::Scene*>(s);
    if (!S.finalized) return fail(PT_ERR_ARG, "scene not finalized (pt_scene_finalize)");
    if (phi) *phi = S.orbit[0];
    if (theta) *theta = S.orbit[1];
    if (zoom) *zoom = S.orbit[2];
    return PT_OK;
}

int pt_scene_set_orbit(pt_scene* s, float phi, float theta, float zoom, const float* look_at) {
    if (!s || !look_at) return fail(PT_ERR_ARG, "null argument");
    auto& S = *reinterpret_cast<pt::Scene*>(s);
    if (!S.finalized) return fail(PT_ERR_ARG, "scene not finalized (pt_scene_finalize)");
    pt::apply_orbit(S, phi, theta, zoom, look_at);   // geometry unchanged: the scene stays finalized
    return PT_OK;
}

int pt_scene_get_render(const pt_scene* s, int32_t* iterations, int32_t* depth, char* file, int32_t cap) {
    if (!s) return fail(PT_ERR_ARG, "null scene");
    const auto& S = *reinterpret_cast<const pt::Scene*>(s);
    if (iterations) *iterations = S.iterations;
    if (depth) *depth = S.depth;
    if (file && cap > 0) std::snprintf(file, (size_t)cap, "%s", S.file.c_str());
    return PT_OK;
}

#define PT_COPY_OUT(field)                                                             \
    if (!s || (!out && cap > 0)) return -fail(PT_ERR_ARG, "null argument");            \
    const auto& S = *reinterpret_cast<const pt::Scene*>(s);                            \
    const int n = (int)S.field.size() < cap ? (int)S.field.size() : cap;               \
    for (int i = 0; i < n; ++i) out[i] = S.field[(size_t)i];                           \
    return n;

int pt_scene_get_geoms(const pt_scene* s, pt_geom* out, int32_t cap) { PT_COPY_OUT(geoms) }
int pt_scene_get_materials(const pt_scene* s, pt_material* out, int32_t cap) { PT_COPY_OUT(materials) }
int pt_scene_get_triangles(const pt_scene* s, pt_triangle* out, int32_t cap) { PT_COPY_OUT(triangles) }
int pt_scene_get_bvh(const pt_scene* s, pt_bvh_node* out, int32_t cap) { PT_COPY_OUT(bvh) }
#undef PT_COPY_OUT

}  // extern "C"

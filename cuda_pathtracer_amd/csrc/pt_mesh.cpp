// Mesh loading and BVH construction (scene.cpp:94-173, BVH_tree.cpp).  First slice: analytic
// scenes only; meshes are rejected with a clear error until the OBJ + SAH-BVH restatement lands.
#include "pt_internal.h"

namespace pt {

int load_obj_mesh(Scene&, const std::string& path, int32_t, const float*, const float*, const float*) {
    return fail(PT_ERR_ARG, "mesh objects are not supported yet (" + path + ")");
}

int add_mesh(Scene&, int32_t, const float*, const float*, const float*, const float*, int32_t, const float*,
             int32_t, const float*, int32_t, const int32_t*, int32_t, const int32_t*, const int32_t*,
             const int32_t*) {
    return fail(PT_ERR_ARG, "mesh objects are not supported yet");
}

int build_bvh(Scene& S) {
    S.bvh.clear();
    S.bvh_built = true;
    return PT_OK;
}

}  // namespace pt

extern "C" int pt_scene_add_mesh(pt_scene* s, int32_t mat, const float* t, const float* r, const float* sc,
                                 const float* pos, int32_t npos, const float* nrm, int32_t nnrm, const float* uv,
                                 int32_t nuv, const int32_t* fs, int32_t nf, const int32_t* ip, const int32_t* in,
                                 const int32_t* it, int32_t* id_out) {
    if (!s) return pt::fail(PT_ERR_ARG, "null scene");
    const int rc = pt::add_mesh(*reinterpret_cast<pt::Scene*>(s), mat, t, r, sc, pos, npos, nrm, nnrm, uv, nuv, fs,
                                nf, ip, in, it);
    if (rc < 0) return -rc;
    if (id_out) *id_out = rc;
    return rc > 0 ? PT_OK : PT_OK;
}

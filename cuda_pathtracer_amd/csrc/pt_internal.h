// Internal host-side types shared by the scene loader, mesh/BVH builder and render context.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/pt_amd.h"

namespace pt {

extern thread_local std::string g_err;
int fail(int code, const std::string& msg);

struct TextureHost {
    std::string path;            // TEXTURE_FILE of a JSON scene (decoded by the loader, pt_jpeg.cpp)
    int32_t width = 0, height = 0, components = 0;
    std::vector<uint8_t> pixels;
};

struct Scene {
    std::vector<pt_geom> geoms;
    std::vector<pt_material> materials;
    std::vector<pt_triangle> tris_load;     // mesh triangles in load order (ids = index here)
    std::vector<pt_triangle> triangles;     // BVH leaf order, built from tris_load by finalize
    std::vector<pt_bvh_node> bvh;
    std::vector<TextureHost> textures;
    pt_camera camera{};
    float fovy = 45.0f;
    float eye[3] = {0, 0, 0}, look_at[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    float orbit[3] = {0, 0, 0};   // phi, theta, zoom of the loaded camera (main.cpp:59-73), set by finalize
    int32_t iterations = 1, depth = 8;
    std::string file = "render";
    bool camera_set = false;
    bool finalized = false;
    bool bvh_built = false;
    int32_t bvh_builder = 0;     // requested: 0 host (pt_mesh.cpp), 1 device (bvh_build.hip)
    int32_t bvh_on_device = 0;   // the last build ran on the device
    double bvh_ms = 0.0;         // the last build's wall time (host clock)
};

int scene_add_geom(Scene& S, int32_t type, int32_t mat, const float* t, const float* r, const float* s);
int scene_finalize(Scene& S);
// Mesh / BVH (pt_mesh.cpp)
int load_obj_mesh(Scene& S, const std::string& path, int32_t mat, const float* t, const float* r, const float* s);
int add_mesh(Scene& S, int32_t mat, const float* t, const float* r, const float* s, const float* pos, int32_t npos,
             const float* nrm, int32_t nnrm, const float* uv, int32_t nuv, const int32_t* face_sizes, int32_t nfaces,
             const int32_t* ip, const int32_t* in, const int32_t* it, int32_t* id_out);
int build_bvh(Scene& S);
// Device SAH build (bvh_build.hip): PT_OK, 1 = not on the device (the caller builds on the host), or an error.
int build_bvh_device(Scene& S, double* ms);
// JPEG textures (pt_jpeg.cpp): stbi_load(path, ..., req_comp = 0) restated
int decode_jpeg(const uint8_t* data, size_t size, int32_t* width, int32_t* height, int32_t* components,
                std::vector<uint8_t>* pixels);
int load_texture_file(TextureHost& t);

}  // namespace pt

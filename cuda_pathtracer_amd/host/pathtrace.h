// C++ host mirror of the reference's render boundary, backed by the C ABI in include/pt_amd.h.
// Same names, argument meaning and error behaviour as
//   path_tracer/src/pathtrace.h:6-9       InitDataContainer / pathtraceInit / pathtraceFree / pathtrace
//   path_tracer/src/utilities.h:17-34     GuiDataContainer (runtime flags, reference defaults)
//   path_tracer/src/scene.h:17-35         Scene(filename): geoms, materials, triangles, state
//   path_tracer/src/sceneStructs.h:71-78  RenderState (camera, iterations, traceDepth, image, imageName)
// Like the reference, the four pathtrace functions drive ONE implicit global render and copy the
// accumulated image into scene->state.image after every iteration (pathtrace.cu:524); errors print
// a message and exit(EXIT_FAILURE) like checkCUDAError.  Code that wants several renders, streams,
// pixel shards or no per-iteration copy uses the pt_* C ABI directly.
#pragma once

#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "pt_amd.h"

class GuiDataContainer {
public:
    GuiDataContainer() : TracedDepth(0) {}
    int TracedDepth;
    bool russianRoulette{true};
    bool useBVHtree{true};
    bool useBBox{true};
    bool sortbyMaterial{false};
    bool useThrustPartition{false};
    bool SSAA{true};
    bool DoF{true};
    float aperture{0.1f};
    float focal_len{10.0f};
    bool singleAlbedo{false};   // extension (include/pt_amd.h pt_flags.single_albedo)
    bool bvhCull{false};        // extension (include/pt_amd.h pt_flags.bvh_cull)
    bool sharedGPU{false};      // extension (include/pt_amd.h pt_flags.shared_gpu); see flags_of()
    bool rngKeyPixel{false};    // extension (include/pt_amd.h pt_flags.rng_key_pixel)
};

struct vec3f {
    float x, y, z;
};

struct RenderState {
    pt_camera camera;
    unsigned int iterations;
    int traceDepth;
    std::vector<vec3f> image;
    std::string imageName;
};

class Scene {
public:
    explicit Scene(std::string filename);   // loadFromJSON + first-frame camera + BVH
    ~Scene();
    Scene(const Scene&) = delete;
    Scene& operator=(const Scene&) = delete;

    std::vector<pt_geom> geoms;
    std::vector<pt_material> materials;
    std::vector<pt_triangle> triangles;
    RenderState state;

    pt_scene* handle() const { return h_; }

private:
    pt_scene* h_ = nullptr;
};

void InitDataContainer(GuiDataContainer* guiData);
void pathtraceInit(Scene* scene);
void pathtraceFree();
void pathtrace(uchar4* pbo, int frame, int iteration);

// Extension (no reference counterpart): the context the four functions above drive (null before
// pathtraceInit), for callers that also want pt_stats / pt_ctx_counters of the global render.
pt_ctx* pathtraceContext();

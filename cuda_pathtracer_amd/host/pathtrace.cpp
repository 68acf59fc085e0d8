// pathtrace.h mirror over the pt_* C ABI (see pathtrace.h for the reference citations).
#include "pathtrace.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace {

GuiDataContainer* g_gui = nullptr;
Scene* g_scene = nullptr;
pt_ctx* g_ctx = nullptr;
// The context's passes run on a non-blocking stream of its own, and the host image is page-locked
// while the context lives: pathtrace()'s per-iteration image copy (pathtrace.cu:524) then waits for
// this context alone and runs at the link's DMA rate (pt_host_register).
void* g_stream = nullptr;
void* g_pinned = nullptr;
// Render-ahead (pt_render_ahead): each call queues the next iteration's bounces before its image copy,
// so they run during the copy; the next call claims them (same iteration and flags: the same image
// bits) or they are dropped.  Not past the scene's last iteration.  PT_AMD_AHEAD=0 turns it off.
bool g_ahead = true;

// checkCUDAError (utilities / common.cu:3-15 pattern): print and exit.
void check(int rc, const char* what) {
    if (rc == PT_OK) return;
    std::fprintf(stderr, "pathtracer error: %s: %s\n", what, pt_last_error());
    std::exit(EXIT_FAILURE);
}

pt_flags flags_of(const GuiDataContainer* g) {
    pt_flags f;
    pt_flags_default(&f);
    if (g) {
        f.russian_roulette = g->russianRoulette;
        f.use_bvh = g->useBVHtree;
        f.use_bbox = g->useBBox;
        f.sort_by_material = g->sortbyMaterial;
        f.use_thrust_partition = g->useThrustPartition;
        f.ssaa = g->SSAA;
        f.dof = g->DoF;
        f.aperture = g->aperture;
        f.focal_dist = g->focal_len;
        f.single_albedo = g->singleAlbedo;
        f.bvh_cull = g->bvhCull;
        f.shared_gpu = g->sharedGPU || f.shared_gpu;   // PT_AMD_SCHEDULE=claim also selects it
        f.rng_key_pixel = g->rngKeyPixel;
    }
    return f;
}

}  // namespace

Scene::Scene(std::string filename) {
    std::printf("Reading scene from %s ...\n", filename.c_str());
    // textures are decoded by the loader (pt_decode_jpeg: stb_image 2.06's JPEG path restated)
    check(pt_scene_load_json(filename.c_str(), &h_), "loadFromJSON");
    int32_t ng = 0, nm = 0, nt = 0, nn = 0, ntex = 0;
    check(pt_scene_counts(h_, &ng, &nm, &nt, &nn, &ntex), "counts");
    geoms.resize(ng);
    materials.resize(nm);
    triangles.resize(nt);
    if (pt_scene_get_geoms(h_, geoms.data(), ng) != ng) check(PT_ERR_ARG, "geoms");
    if (pt_scene_get_materials(h_, materials.data(), nm) != nm) check(PT_ERR_ARG, "materials");
    if (pt_scene_get_triangles(h_, triangles.data(), nt) != nt) check(PT_ERR_ARG, "triangles");
    check(pt_scene_get_camera(h_, &state.camera), "camera");
    int32_t it = 0, depth = 0;
    char name[1024];
    check(pt_scene_get_render(h_, &it, &depth, name, sizeof name), "render state");
    state.iterations = (unsigned)it;
    state.traceDepth = depth;
    state.imageName = name;
    state.image.assign((size_t)state.camera.res[0] * state.camera.res[1], vec3f{0.f, 0.f, 0.f});
}

Scene::~Scene() {
    if (g_scene == this) pathtraceFree();
    pt_scene_free(h_);
}

void InitDataContainer(GuiDataContainer* guiData) {
    g_gui = guiData;
    if (g_ctx) {
        const pt_flags f = flags_of(g_gui);
        check(pt_set_flags(g_ctx, &f), "InitDataContainer");
    }
}

void pathtraceInit(Scene* scene) {
    pathtraceFree();
    g_scene = scene;
    const pt_flags f = flags_of(g_gui);
    check(pt_create(scene->handle(), &f, nullptr, &g_ctx), "pathtraceInit");
    check(pt_stream_create(&g_stream), "pathtraceInit stream");
    const char* ah = std::getenv("PT_AMD_AHEAD");
    g_ahead = !(ah && ah[0] == '0');
    std::fill(scene->state.image.begin(), scene->state.image.end(), vec3f{0.f, 0.f, 0.f});
    if (!scene->state.image.empty() &&
        pt_host_register(scene->state.image.data(), scene->state.image.size() * sizeof(vec3f)) == PT_OK)
        g_pinned = scene->state.image.data();   // (not page-locked: the copy still works, staged)
}

void pathtraceFree() {
    if (g_ctx) check(pt_destroy(g_ctx), "pathtraceFree");
    g_ctx = nullptr;
    if (g_stream) (void)pt_stream_destroy(g_stream);
    g_stream = nullptr;
    if (g_pinned) (void)pt_host_unregister(g_pinned);
    g_pinned = nullptr;
}

pt_ctx* pathtraceContext() { return g_ctx; }

void pathtrace(uchar4* pbo, int frame, int iteration) {
    (void)frame;
    if (!g_ctx || !g_scene) {
        std::fprintf(stderr, "pathtracer error: pathtrace() before pathtraceInit()\n");
        std::exit(EXIT_FAILURE);
    }
    const pt_flags f = flags_of(g_gui);   // the reference re-reads the GUI flags every call
    check(pt_set_flags(g_ctx, &f), "flags");
    check(pt_render_pass(g_ctx, iteration, g_stream), "pathtrace");
    if (pbo) check(pt_preview_rgba(g_ctx, iteration, reinterpret_cast<uint8_t*>(pbo), g_stream), "sendImageToPBO");
    if (g_gui) g_gui->TracedDepth = g_scene->state.traceDepth;
    if (g_ahead && iteration >= 1 && (unsigned)iteration < g_scene->state.iterations)
        (void)pt_render_ahead(g_ctx, iteration + 1, g_stream);   // (a failure only costs the overlap)
    check(pt_get_image(g_ctx, reinterpret_cast<float*>(g_scene->state.image.data())), "image copy");
}

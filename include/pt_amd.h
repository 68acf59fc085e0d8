/* pt_amd.h — C ABI of the MI355X path tracer (libpt_amd.so).
 *
 * Replaces the reference's render boundary path_tracer/src/pathtrace.h:6-9
 *     void InitDataContainer(GuiDataContainer*);   -> pt_set_flags
 *     void pathtraceInit(Scene*);                  -> pt_create
 *     void pathtraceFree();                        -> pt_destroy
 *     void pathtrace(uchar4* pbo, int frame, int iteration);
 *                                                  -> pt_render_pass (+ pt_preview_rgba for the PBO)
 * the scene loader path_tracer/src/scene.h:17-35 / scene.cpp:16-219 (Scene::Scene, loadFromJSON)
 *                                                  -> pt_scene_load_json / pt_scene_* builders
 * the first-frame camera recompute of main.cpp:59-73,117-136           -> pt_scene_finalize
 * and the image output main.cpp:88-112 + image.cpp:22-42 (saveImage, Image::savePNG)
 *                                                  -> pt_save_png / pt_tonemap
 *
 * Differences from the reference, by design:
 *   - no file-static globals: every render owns a pt_ctx; any number can coexist;
 *   - status codes (PT_OK / PT_ERR_*) instead of exit(); pt_last_error() gives the message;
 *   - explicit stream (hipStream_t passed as void*; NULL = the legacy default stream);
 *   - no per-iteration device->host copy of the image: pt_get_image / pt_copy_image on demand;
 *   - the context renders a pixel TILE (rows y with y % world == rank) and may trace `spp`
 *     consecutive iterations per pass; world == 1, spp == 1 is exactly the reference's
 *     pathtrace() (same RNG keys, same stable compaction order, same accumulation).
 * All structs are plain C with the reference's field order (sceneStructs.h).
 */
#ifndef PT_AMD_H
#define PT_AMD_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PT_OK 0
#define PT_ERR_ARG 1
#define PT_ERR_HIP 2
#define PT_ERR_NOMEM 3
#define PT_ERR_IO 4
#define PT_ERR_PARSE 5
#define PT_ERR_DEVICE 6   /* a device-side check failed (e.g. look-back spin bound hit) */

#define PT_GEOM_SPHERE 0  /* sceneStructs.h:12-17 */
#define PT_GEOM_CUBE 1
#define PT_GEOM_MESH 2

/* Runtime flags: GuiDataContainer (utilities.h:17-34), mirrored into Settings (pathtrace.cu:31-55). */
typedef struct pt_flags {
    int32_t russian_roulette;     /* default 1 */
    int32_t use_bvh;              /* default 1 */
    int32_t use_bbox;             /* default 1 (linear mesh path only) */
    int32_t sort_by_material;     /* default 0: stable material sort before shading */
    int32_t use_thrust_partition; /* default 0: same stable partition either way */
    int32_t ssaa;                 /* default 1 */
    int32_t dof;                  /* default 1 */
    float aperture;               /* default 0.1 */
    float focal_dist;             /* default 10 */
    /* Extension (default 0 = the reference): apply the surface albedo once.  The reference
     * multiplies the path colour by the albedo at interactions.cu:60 AND :83; its own course
     * image (img/REFERENCE_cornell.5000samp.png) matches the single-albedo model. */
    int32_t single_albedo;
    /* Extension (default 0 = the reference): skip BVH nodes whose entry distance exceeds the
     * closest triangle found so far by a 1e-3 relative margin.  BVHIntersectionTest
     * (intersections.cu:170-224) visits every node the ray line crosses.  The closest hit is
     * unchanged unless rounding moves a triangle's computed t by more than the margin
     * (DESIGN.md §4). */
    int32_t bvh_cull;
    /* Another context, stream or process shares the GPU (0 = no).  1 makes every inter-workgroup
     * wait of a render pass safe without co-residency: the split pipeline's look-back compaction
     * claims tiles in order from a ticket (lookback.h), and the material-sorted pipeline scans its
     * histogram with the three-kernel reduce/scan/apply path instead of the single-pass library
     * scan.  With 0, a static-schedule wait that cannot get the whole GPU hits its spin bound and
     * pt_stats reports PT_ERR_DEVICE.  pt_flags_default: 1 if PT_AMD_SCHEDULE=claim, else 0. */
    int32_t shared_gpu;
    /* Extension (default 0 = the reference): key the shading RNG by the path's global pixel index
     * instead of its position in the compacted path array (pathtrace.cu:315).  The image then
     * no longer depends on how pixels are sharded across GPUs or sorted by material: N-GPU output
     * is bitwise equal to 1-GPU output (SURVEY.md §8e's rng_key=pixel mode). */
    int32_t rng_key_pixel;
} pt_flags;

/* Material (sceneStructs.h:43-57), 48 bytes. */
typedef struct pt_material {
    float color[3];
    float spec_exponent;
    float spec_color[3];
    float has_reflective;
    float has_refractive;
    float ior;
    float emittance;
    int32_t texture_id;           /* -1: none */
} pt_material;

/* Geom (sceneStructs.h:25-41), 272 bytes.  Matrices are glm column-major: m[c][r] = a[4c+r]. */
typedef struct pt_geom {
    int32_t type;
    int32_t material_id;
    float translation[3];
    float rotation[3];            /* degrees */
    float scale[3];
    float transform[16];
    float inverse_transform[16];
    float inv_transpose[16];
    int32_t tri_start, tri_end, bbox_idx;
    float min_bound[3], max_bound[3];
} pt_geom;

/* Camera (sceneStructs.h:59-69). */
typedef struct pt_camera {
    int32_t res[2];
    float position[3], look_at[3], view[3], up[3], right[3];
    float fov[2];
    float pixel_length[2];
} pt_camera;

/* Triangle (sceneStructs.h:103-161), 124 bytes, world space. */
typedef struct pt_triangle {
    int32_t id;                   /* original (load-order) index */
    float v[3][3];
    float uv[3][2];
    float n[3][3];
    float bmin[3], bmax[3];
} pt_triangle;

/* Flattened BVH node (BVH_tree.h:54-61), 40 bytes. */
typedef struct pt_bvh_node {
    float bmin[3], bmax[3];
    int32_t sub_areas, axis, first_area_idx, rchild_idx;
} pt_bvh_node;

typedef struct pt_scene pt_scene;
typedef struct pt_ctx pt_ctx;

/* Tile / batching of one context.  rank/world: this context owns image rows y % world == rank.
 * spp: iterations traced together per pass (1 = the reference). */
typedef struct pt_shard {
    int32_t rank, world, spp, reserved;
} pt_shard;

/* Per-context counters (device-side, read back by pt_stats). */
typedef struct pt_stats_t {
    uint64_t segments;            /* sum over bounces of live paths entering intersection */
    uint64_t passes;
    uint64_t bounce_live[64];     /* live paths entering bounce k (k < depth) */
    uint64_t emissive_hits;       /* paths that terminated with non-zero radiance (framebuffer adds) */
    uint64_t bounce_emit[64];     /* of those, per bounce */
    uint32_t device_error;        /* nonzero: a device-side bound was hit */
    uint32_t bound_mismatch;      /* PT_AMD_VERIFY_BOUNDS=1 only: closest hits where the bounded
                                     pass differed from the plain per-geom loop (must stay 0) */
} pt_stats_t;

const char* pt_last_error(void);
void pt_flags_default(pt_flags* f);

/* ---- scene ---------------------------------------------------------------------------- */
int pt_scene_load_json(const char* path, pt_scene** out);   /* Scene::Scene(filename) incl. pt_scene_finalize */
/* Loader extensions, all off by default (pt_scene_load_json == options 0 == the reference's loader).
 * PT_LOAD_REFRACTION: read the material keys REFRACTIVE and IOR, which the reference's
 * Scene::loadFromJSON never reads (scene.cpp:46-56; refraction is unreachable from its files).  A
 * file can also opt in itself with the top-level key "Extensions": {"REFRACTION": true}, which the
 * reference ignores; a reference scene file therefore loads exactly as the reference loads it. */
#define PT_LOAD_REFRACTION 1u
/* PT_LOAD_DEVICE_BVH: build the scene's BVH on the current HIP device (pt_scene_set_bvh_builder). */
#define PT_LOAD_DEVICE_BVH 2u
int pt_scene_load_json_ex(const char* path, uint32_t options, pt_scene** out);
int pt_scene_create(pt_scene** out);
void pt_scene_free(pt_scene* s);
int pt_scene_add_material(pt_scene* s, const pt_material* m, int32_t* id_out);
/* Texture pixels (row-major, `components` bytes per texel; only 3 is shaded, like the reference). */
int pt_scene_add_texture(pt_scene* s, int32_t width, int32_t height, int32_t components,
                         const uint8_t* pixels, int32_t* id_out);
/* JSON scenes reference textures by file (scene.cpp:61-71).  pt_scene_load_json decodes JPEG files
 * with pt_decode_jpeg (below) and fails with PT_ERR_IO where the reference prints "Texture load
 * error!" and exits (missing file, corrupt JPEG).  Files that are not JPEG (no SOI marker: PNG, BMP,
 * TGA, ... which the reference's stbi_load also reads) are NOT decoded here: the texture keeps its
 * path and no pixels, the host fills it with pt_scene_set_texture_pixels (the Python Scene does so
 * for lossless formats, whose texels any decoder reproduces), and pt_create refuses a scene with a
 * texture left unfilled.  pt_scene_set_texture_pixels also replaces a decoded texture's pixels. */
int pt_scene_texture_path(const pt_scene* s, int32_t id, char* buf, int32_t cap);
int pt_scene_set_texture_pixels(pt_scene* s, int32_t id, int32_t width, int32_t height,
                                int32_t components, const uint8_t* pixels);
/* Cube / sphere: builds transform, inverse, inverse-transpose like scene.cpp:80-91. */
int pt_scene_add_geom(pt_scene* s, int32_t type, int32_t material_id, const float t[3],
                      const float r[3], const float sc[3], int32_t* id_out);
/* Mesh: object-space polygon soup, fan-triangulated (tinyobj triangulate=true), pre-transformed
 * to world space (scene.cpp:94-173).  face_sizes[f] vertices per face; idx_* per face-vertex
 * (-1 = absent), positions/normals (xyz), uvs (uv).  PT_ERR_ARG for a world vertex that is not
 * finite or beyond 2^126 in magnitude (the SAH build would recurse without end on it). */
int pt_scene_add_mesh(pt_scene* s, int32_t material_id, const float t[3], const float r[3],
                      const float sc[3], const float* positions, int32_t npos,
                      const float* normals, int32_t nnorm, const float* uvs, int32_t nuv,
                      const int32_t* face_sizes, int32_t nfaces, const int32_t* idx_pos,
                      const int32_t* idx_norm, const int32_t* idx_uv, int32_t* id_out);
int pt_scene_set_camera(pt_scene* s, int32_t res_x, int32_t res_y, float fovy, const float eye[3],
                        const float look_at[3], const float up[3]);
int pt_scene_set_render(pt_scene* s, int32_t iterations, int32_t depth, const char* file);
/* Camera orbit recompute of the first frame (main.cpp:59-73,117-136) + BVH build (scene.cpp:218). */
int pt_scene_finalize(pt_scene* s);
/* Where pt_scene_finalize builds the BVH (BVH_tree.cpp:27-181's SAH tree): 0 (default) on the host,
 * 1 on the current HIP device — the same nodes, byte for byte, and the same triangle order
 * (bvh_build.hip); a tree the device builder leaves to the host (NaN vertex coordinates) is built
 * there.  pt_scene_bvh_build_info: where the last build ran and its wall time in ms. */
int pt_scene_set_bvh_builder(pt_scene* s, int32_t device);
int pt_scene_bvh_build_info(const pt_scene* s, int32_t* on_device, double* ms);
int pt_scene_counts(const pt_scene* s, int32_t* ngeoms, int32_t* nmats, int32_t* ntris,
                    int32_t* nnodes, int32_t* ntex);
int pt_scene_get_camera(const pt_scene* s, pt_camera* out);
int pt_scene_get_render(const pt_scene* s, int32_t* iterations, int32_t* depth, char* file, int32_t cap);
/* The interactive camera of the preview (main.cpp).  pt_scene_get_orbit: the orbit of the loaded
 * camera, phi / theta / zoom as main.cpp:59-73 derives them (pt_scene_finalize computes them).
 * pt_scene_set_orbit: runCuda's camchanged recompute (main.cpp:117-136) for the orbit (phi, theta,
 * zoom) about look_at — position, view, right (= view x (0,1,0), unnormalised) and up; the scene stays
 * finalized, and contexts created after the call render the new camera (the reference re-runs
 * pathtraceInit at iteration 0).  Both need a finalized scene (PT_ERR_ARG otherwise). */
int pt_scene_get_orbit(const pt_scene* s, float* phi, float* theta, float* zoom);
int pt_scene_set_orbit(pt_scene* s, float phi, float theta, float zoom, const float look_at[3]);
/* Getters copy min(count, cap) records and return that number (>= 0), or -PT_ERR_ARG. */
int pt_scene_get_geoms(const pt_scene* s, pt_geom* out, int32_t cap);
int pt_scene_get_materials(const pt_scene* s, pt_material* out, int32_t cap);
int pt_scene_get_triangles(const pt_scene* s, pt_triangle* out, int32_t cap);
int pt_scene_get_bvh(const pt_scene* s, pt_bvh_node* out, int32_t cap);
/* Inspection (host only, used by the tests): the 4-wide layout the BVH walk of mesh scenes runs on
 * (128-byte entries: lo.x, hi.x, lo.y, hi.y, lo.z, hi.z, codes, meta — each 4 slots; layout and
 * codes in pt_kernels.hip DQuad).  Returns the entry count (0: no 4-wide layout for this tree; the
 * pair walk runs) and copies min(count, cap) entries; *root_code / *stack_bound as pt_create uses. */
int pt_scene_bvh_quads(const pt_scene* s, void* out, int32_t cap, int32_t* root_code, int32_t* stack_bound);
/* Inspection (host only): the 4-wide walk's exact t-cull words, 4 per quad in pt_scene_bvh_quads's
 * order (slot k: binary16 A in bits 0-15, binary16 B in bits 16-31; a slot's children are not entered
 * when A * tau_lo > B + best), and the share of slots with A >= 1/2.  Returns the word
 * count (0: no 4-wide layout) and copies min(count, cap) words. */
int pt_scene_bvh_tcull(const pt_scene* s, uint32_t* words, int32_t cap, double* cullable_frac);

/* ---- render context -------------------------------------------------------------------- */
/* pathtraceInit: uploads the scene to the current HIP device, allocates SoA path buffers for
 * rows_in_tile * width * spp paths.  shard may be NULL (= {0, 1, 1}). */
int pt_create(const pt_scene* s, const pt_flags* flags, const pt_shard* shard, pt_ctx** out);
int pt_destroy(pt_ctx* c);                                  /* pathtraceFree */
/* InitDataContainer / Settings.  Cheap when called every iteration with unchanged camera-ray flags:
 * only a change of ssaa, dof, aperture or focal_dist synchronises the device and rebuilds the
 * first-bounce camera masks (and, for the aperture, the widened geom bounds). */
int pt_set_flags(pt_ctx* c, const pt_flags* flags);
/* Host-side counters of a context: first-bounce camera-mask builds (pt_create builds one) and the
 * pt_set_flags calls that synchronised the device. */
int pt_ctx_counters(const pt_ctx* c, uint64_t* mask_builds, uint64_t* flag_syncs);
/* Inspection: the first-bounce camera masks of a context — built (on), the share of 64-pixel blocks
 * whose mask is empty (no geom reachable: those waves skip raygen and the closest hit), and whether
 * the fused first bounce runs its empty-wave instantiation (chosen when that share is >= 0.2;
 * PT_AMD_SKIP_EMPTY=0/1 forces it).  Results are the same bits either way. */
int pt_ctx_cmask_info(const pt_ctx* c, int32_t* on, double* empty_frac, int32_t* skip_fused);
/* Mesh scenes: whether the BVH walk runs on the 4-wide layout, whether its exact t-cull is on, and
 * the share of the layout's slots whose cull margin can pay.  The cull is on when
 * that share is >= 1/4 (PT_AMD_TCULL=0/1 forces it); it never changes a result. */
int pt_ctx_walk_info(const pt_ctx* c, int32_t* quad_walk, int32_t* tcull_on, double* tcull_frac);
/* Stream budget.  HIP maps a process's streams of one priority onto GPU_MAX_HW_QUEUES (default 4)
 * hardware queues; streams beyond that share queues and their work runs in submission order.  A
 * context keeps busy: the caller's stream, one stream per extra lane of a batched pass, and the
 * finalize stream of a batched pass.  pt_create caps the lanes it picks by itself so that the busy
 * streams of all live contexts stay within GPU_MAX_HW_QUEUES (PT_AMD_LANES overrides the choice and
 * the cap).  The synchronous entry points copy on a high-priority stream of the context's own, a
 * pool of queues apart from the compute streams.  So one context's passes never wait for another's,
 * and its synchronous reads never queue behind another's passes, while the process's busy
 * normal-priority streams — the library's and the caller's own (torch's stream pool, say) — are at
 * most GPU_MAX_HW_QUEUES; past that, contexts share queues and may serialise (still correct).
 * pt_ctx_stream_info: the context's lanes, its busy streams, the sum over the live contexts, the
 * budget, and whether its lanes were capped. */
int pt_ctx_stream_info(const pt_ctx* c, int32_t* lanes, int32_t* busy_streams, int32_t* process_busy,
                       int32_t* hw_queues, int32_t* lanes_capped);
/* One pass: iterations [iter_first, iter_first + spp) for this tile, accumulated into the tile
 * image.  Asynchronous on `stream`; no host synchronisation inside.  A batched pass (spp > 1)
 * runs its iterations in lanes on internal streams and adds their colours into the image on a
 * finalize stream; `stream` itself is not made to wait for every lane (the next pass starts during
 * this one's tail).  Read the image through pt_copy_image / pt_preview_rgba / pt_reset_image (they
 * wait for the last finalize on their stream) or the synchronising calls.  Passes of one context
 * may go to different streams: a pass on another stream than the previous pass first waits (on the
 * device) for all of the context's queued work; passes on one stream keep their overlap. */
int pt_render_pass(pt_ctx* c, int32_t iter_first, void* stream);
/* Render-ahead for a one-iteration context (spp 1; the drop-in pathtrace() loop): queues the bounces
 * of iteration `iter` on `stream` now, without touching the image, so they run while the caller
 * copies the previous image to the host (pathtrace.cu:524's copy).  A later pt_render_pass(c, iter)
 * with the same flags claims them and only adds their colours into the image (the same bits as
 * rendering then); any other pass — another iteration, changed flags — drops them first.  Counts
 * (pt_stats) include an iteration once it is claimed.  Not synchronising; pt_get_image and the
 * other synchronising calls do not wait for unclaimed ahead work.  Ordering on any streams: the
 * ahead work waits (on the device) for the context's last pass, claim or image call when that went
 * to another stream, and every later pass or ahead waits for the ahead work.  On failure nothing is
 * left to claim and the HIP last-error is cleared (the caller may go on without the overlap). */
int pt_render_ahead(pt_ctx* c, int32_t iter, void* stream);
/* sendImageToPBO (pathtrace.cu:64-86) for the tile: d_rgba = npix * 4 bytes on the device. */
int pt_preview_rgba(pt_ctx* c, int32_t iter, uint8_t* d_rgba, void* stream);
/* pathtrace(pbo, frame, iteration) (pathtrace.h:9, pathtrace.cu:437-525) as one call, under the
 * name SURVEY.md §8b gives it: pt_render_pass for iterations [iter, iter + spp), then, when d_rgba
 * is non-NULL, pt_preview_rgba of the accumulated iter + spp - 1 samples (iterations counted from 1). */
int pt_render_iteration(pt_ctx* c, int32_t iter, uint8_t* d_rgba, void* stream);
int pt_tile_info(const pt_ctx* c, int32_t* width, int32_t* rows, int32_t* npix, int32_t* npaths);
int pt_get_image(pt_ctx* c, float* host_rgb);               /* tile accumulator, npix*3 floats (sync) */
int pt_get_accum(pt_ctx* c, float* host_rgb);               /* §8b name of pt_get_image (pathtrace.cu:524) */
int pt_copy_image(pt_ctx* c, float* d_rgb, void* stream);   /* device-to-device copy */
int pt_reset_image(pt_ctx* c, void* stream);
/* Resume (extension; the reference has none): load a previously saved float accumulator of this
 * context's tile (npix x float3, as pt_get_accum returns it).  Continuing with the next iteration
 * indices reproduces an uninterrupted render bit for bit.  Any -0 is loaded as +0 (the reference's
 * image holds no -0 after a pass: every iteration adds a colour, zero or not, into every pixel). */
int pt_set_accum(pt_ctx* c, const float* host_rgb);
int pt_stats(pt_ctx* c, pt_stats_t* out);                   /* synchronises the context stream */
/* The synchronous calls above (pt_get_image, pt_get_accum, pt_set_accum, pt_stats, and pt_set_flags
 * when it rebuilds device data) and pt_destroy wait for THIS context's enqueued work only — an event
 * recorded after its last pass or image call — and move data on a non-blocking stream of the
 * context's own: another context's passes, or other work on the GPU, are not waited for.
 *
 * Drop-in helpers (host/pathtrace.cpp, the pathtrace.h mirror): page-lock a host buffer that
 * pt_get_image copies into every iteration (the reference's Scene::state.image, pathtrace.cu:524),
 * so the copy runs at the link's DMA rate; and a non-blocking stream for a context's passes, so they
 * neither wait for nor hold up the legacy default stream. */
int pt_host_register(void* host, uint64_t bytes);
int pt_host_unregister(void* host);
int pt_stream_create(void** stream);
int pt_stream_destroy(void* stream);
/* Per-kernel device timing with hipEvents recorded on the launch stream (for the roofline).  When
 * enabled, pt_render_pass brackets every launch with pooled events; pt_profile_read synchronises
 * and returns, per kernel kind, the summed milliseconds and launch counts since the last read. */
#define PT_KIND_FIRST_BOUNCE 0   /* bounce 0: k_bounce<FIRST> (fused), k_trace<FIRST> (split), or the
                                    first k_sort_produce (sorted: raygen + intersection)           */
#define PT_KIND_BOUNCE 1         /* bounces >= 1: k_bounce (fused) or k_trace (split)          */
#define PT_KIND_COMPACT 2        /* split pipeline only: k_compact_paths                        */
#define PT_KIND_SORT 3           /* material-sorted mode, per bounce: histogram scan + producer
                                    (shade bounce b, compact, intersect bounce b + 1)              */
#define PT_KIND_TRAVERSE 4       /* mesh scenes, bounces >= 1: the BVH walk k_traverse[4]       */
#define PT_KIND_FIRST_TRAVERSE 5 /* mesh scenes, bounce 0: the BVH walk of the camera rays       */
#define PT_KIND_COUNT 6
int pt_profile_enable(pt_ctx* c, int32_t on);
/* The first four kinds (pt_profile_read_kinds returns all of them).  These two calls count the BVH
 * walk (kinds 4 and 5) in BOUNCE and FIRST_BOUNCE, as before the walk had kinds of its own.  In the
 * material-sorted pipeline the camera-ray producer counts as FIRST_BOUNCE, not SORT (since round 3). */
int pt_profile_read(pt_ctx* c, double ms[4], uint64_t launches[4]);
/* Same, plus busy_ms[kind]: the length of the union of that kind's launch intervals.  Batched
 * passes of the fused pipeline run two lanes of iterations concurrently (pt_render_pass), so
 * launches of one kind overlap and busy_ms < ms. */
int pt_profile_read_busy(pt_ctx* c, double ms[4], double busy_ms[4], uint64_t launches[4]);
/* Every kind: arrays of nkinds entries (kinds >= PT_KIND_COUNT read 0).  busy_ms may be NULL. */
int pt_profile_read_kinds(pt_ctx* c, int32_t nkinds, double* ms, double* busy_ms, uint64_t* launches);

/* Device self-check of the range-gated correctly rounded sqrt / division cores the kernels use
 * (pt_device.h) against hipcc's library sqrtf and '/': n operand sets from `seed` (random bit
 * patterns over every exponent, a quarter near 1, plus zeros, denormals, infinities and NaNs).
 * *mismatches = operations whose bits differ (NaN == NaN).  Synchronous. */
int pt_selftest_math(uint64_t n, uint32_t seed, uint64_t* mismatches);

/* ---- texture input --------------------------------------------------------------------- */
/* Texture::load (sceneStructs.h:171-175) = stbi_load(file, &w, &h, &comp, 0) for JPEG data:
 * stb_image 2.06's JPEG decoder restated (baseline + progressive, its integer IDCT, triangle-filter
 * chroma upsampling and fixed-point YCbCr->RGB), so texels equal the reference's.  Writes width,
 * height, components (1 or 3); with out != NULL also the w*h*components interleaved bytes (top row
 * first; cap = size of out).  out == NULL: header only. */
int pt_decode_jpeg(const uint8_t* data, int64_t size, int32_t* width, int32_t* height, int32_t* components,
                   uint8_t* out, int64_t cap);

/* ---- image output ---------------------------------------------------------------------- */
/* saveImage + Image::savePNG pixel math: out[3*(y*W + (W-1-x)) + k] = uchar(clamp(rgb/spp,0,1)*255). */
int pt_tonemap(const float* rgb, int32_t width, int32_t height, float samples, uint8_t* out);
/* Writes `path` as an 8-bit RGB PNG of the tonemapped image. */
int pt_save_png(const char* path, const float* rgb, int32_t width, int32_t height, float samples);
/* Image::saveHDR (image.cpp:44-49) via stb_image_write's Radiance RGBE writer (vendored by the
 * reference: external/include/stb_image_write.h:246-387), pixels as saveImage (x-mirrored,
 * accumulated / samples).  pt_encode_hdr writes the file bytes to `out` (NULL: size only). */
int pt_save_hdr(const char* path, const float* rgb, int32_t width, int32_t height, float samples);
int pt_encode_hdr(const float* rgb, int32_t width, int32_t height, float samples, uint8_t* out, int64_t cap,
                  int64_t* size);

#ifdef __cplusplus
}
#endif
#endif /* PT_AMD_H */

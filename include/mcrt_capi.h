/*
 * mcrt_capi.h -- C ABI of the MI355X-native Monte-Carlo path-tracing core.
 *
 * This is the drop-in boundary for the reference's hot path
 * (compix/Monte-Carlo-Raytracer).  Every entry point names the reference
 * interface it replaces (paths relative to the reference repo root):
 *
 *   RR  = third_party/RadeonRays/RadeonRays
 *   APP = source/application/PathTracer
 *   KRN = assets/kernels
 *
 * Plain C: opaque handles, plain pointers and sizes, no C++ or torch types.
 * Every call returns an mcrt_status; mcrt_last_error() gives the message
 * (the reference threw std::exception / Calc::Exception and the passes caught
 * them: APP/raytracing/renderPasses/RTPathTracingPass.cpp:89-104).
 *
 * All structs below are byte-identical to the OpenCL device structs of
 * KRN/kernel_data.h (sizes/offsets: SURVEY.md Appendix B), so the scene
 * arrays the reference's RTScene builds (APP/raytracing/scene/RTScene.cpp)
 * can be passed unchanged.
 */
#ifndef MCRT_CAPI_H
#define MCRT_CAPI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MCRT_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* Status codes                                                             */
/* ------------------------------------------------------------------------ */
typedef int mcrt_status;
#define MCRT_OK                   0
#define MCRT_ERROR_INVALID_ARG    1
#define MCRT_ERROR_OUT_OF_MEMORY  2
#define MCRT_ERROR_DEVICE         3
#define MCRT_ERROR_NOT_READY      4  /* e.g. trace before mcrt_accel_build */
#define MCRT_ERROR_NO_DEVICE      5

/* ------------------------------------------------------------------------ */
/* Device-layout value types (OpenCL float3 = 16 B, float2 = 8 B)           */
/* ------------------------------------------------------------------------ */
typedef struct __attribute__((aligned(16))) { float x, y, z, w; } mcrt_float4;
typedef mcrt_float4 mcrt_float3;                      /* OpenCL float3: 16 B */
typedef struct __attribute__((aligned(8))) { float x, y; } mcrt_float2;
typedef struct __attribute__((aligned(16))) { mcrt_float4 m0, m1, m2, m3; } mcrt_mat4; /* row major, KRN/matrix.cl:4-11 */

/* RTShape, KRN/kernel_data.h:36-52 (160 B) */
typedef struct __attribute__((aligned(16))) {
    mcrt_mat4 toWorldTransform;
    mcrt_mat4 toWorldInverseTranspose;
    uint32_t  startIdx;
    uint32_t  startVertex;
    uint32_t  numTriangles;
    int32_t   materialId;   /* -1 = none */
    int32_t   lightID;      /* -1 = not an emitter */
    float     area;
    int32_t   pad[2];
} mcrt_shape;

/* RTMaterial (uber material), KRN/kernel_data.h:87-113 (128 B) */
typedef struct __attribute__((aligned(16))) {
    mcrt_float3 uber_kd;
    mcrt_float3 uber_ks;
    mcrt_float3 uber_kr;
    mcrt_float4 uber_kt;        /* w >= 0.5: glossy, else perfect specular transmission */
    mcrt_float3 uber_opacity;
    mcrt_float2 uber_roughness;
    float       uber_eta;
    int32_t     type;           /* 0 = RT_UBER_MATERIAL */
    int32_t     uber_normalMapId;
    int32_t     uber_diffuseTexId;
    int32_t     uber_glossyTexId;
    int32_t     uber_specReflectionTexId;
    int32_t     uber_transmissionTexId;
    int32_t     uber_opacityTexId;
    int32_t     uber_roughnessTexId;
    int32_t     uber_iorTexId;
} mcrt_material;

/* RTLight, KRN/kernel_data.h:137-152 (80 B) */
#define MCRT_DIRECTIONAL_LIGHT        0
#define MCRT_POINT_LIGHT              1
#define MCRT_DISK_AREA_LIGHT          2
#define MCRT_TRIANGLE_MESH_AREA_LIGHT 3
#define MCRT_LIGHT_FLAG_DELTA_POSITION  (1 << 1)
#define MCRT_LIGHT_FLAG_DELTA_DIRECTION (1 << 2)
#define MCRT_LIGHT_FLAG_AREA            (1 << 3)
typedef struct __attribute__((aligned(16))) {
    mcrt_float3 d;
    mcrt_float3 p;
    mcrt_float3 intensity;
    float   radius;
    float   area;
    float   choicePdf;
    int32_t shapeId;
    int32_t type;
    int32_t flags;
    int32_t pad[2];
} mcrt_light;

/* RTPinholeCamera, KRN/kernel_data.h:246-264 (176 B) */
typedef struct __attribute__((aligned(16))) {
    mcrt_mat4   worldToClip;
    mcrt_float3 r00, r10, r11, r01;   /* corner directions, APP/.../RTPrimaryRaysPass.cpp:96-99 */
    mcrt_float3 pos;
    mcrt_float3 direction;
    uint32_t    width;
    uint32_t    height;
    float       area;
    int32_t     padding;
} mcrt_camera;

/* TextureDesc2D, KRN/kernel_data.h:317-326 (16 B); texels are RGBA8 */
typedef struct {
    uint16_t width, height, numMipLevels, format, wrap, pad;
    uint32_t memOffset;       /* byte offset into tex_data */
} mcrt_texture_desc;

/* RadeonRays ray, RR/src/kernels/CL/common.cl:53-60 and KRN/kernel_data.h:407-417 (48 B) */
typedef struct __attribute__((aligned(16))) {
    mcrt_float4 o;            /* xyz origin, w = max range */
    mcrt_float4 d;            /* xyz direction, w = time (unused) */
    int32_t extra[2];         /* [0] = mask (-1: all shapes), [1] = active flag (0: inactive) */
    int32_t doBackfaceCulling;
    int32_t padding;
} mcrt_ray;

/* RadeonRays Intersection, RR/src/kernels/CL/common.cl:63-70 (32 B) */
typedef struct __attribute__((aligned(16))) {
    int32_t shapeid;          /* -1 on miss */
    int32_t primid;           /* -1 on miss */
    int32_t padding[2];
    mcrt_float4 uvwt;         /* (u, v, 0, t); left untouched on miss */
} mcrt_intersection;

/* RTFilterProperties with the DEVICE layout (56 B): KRN/kernel_data.h:63-80.
 * The reference host struct is 48 B (RadeonRays::float2 is 4-byte aligned),
 * so the reference device read shifted fields; this ABI
 * uses the explicit, correctly laid-out device struct. */
#define MCRT_BOX_FILTER          0
#define MCRT_TRIANGLE_FILTER     1
#define MCRT_GAUSSIAN_FILTER     2
#define MCRT_MITCHELL_FILTER     3
#define MCRT_LANCZOS_SINC_FILTER 4
typedef struct __attribute__((aligned(8))) {
    int32_t     filterType;
    int32_t     _align0;
    mcrt_float2 radius;
    float       mitchellB;
    float       mitchellC;
    float       lanczosSincTau;
    float       gaussianAlpha;
    float       gaussianExpX;
    float       gaussianExpY;
    mcrt_float2 pixelOffset;
    float       pad;
    int32_t     _align1;
} mcrt_filter;

/* ------------------------------------------------------------------------ */
/* Scene description = the 15 SCENE_PARAMS arrays (KRN/kernel_data.h:338-352,
 * filled by RTScene::setSceneArgs, APP/raytracing/scene/RTScene.cpp:178-197).
 * Host pointers; they are COPIED to HBM and may be freed after the call.     */
/* ------------------------------------------------------------------------ */
typedef struct {
    const mcrt_shape*        shapes;        uint32_t num_shapes;
    const uint32_t*          indices;       uint32_t num_indices;   /* per-shape local vertex indices */
    const mcrt_float3*       positions;     uint32_t num_vertices;  /* all per-vertex arrays have num_vertices */
    const mcrt_float2*       uvs;
    const mcrt_float3*       normals;
    const mcrt_float3*       tangents;
    const mcrt_float3*       binormals;
    const mcrt_float3*       colors;        /* may be NULL */
    const mcrt_texture_desc* textures;      uint32_t num_textures;
    const uint8_t*           tex_data;      uint64_t tex_data_bytes;
    const uint32_t*          sobol_matrices; uint32_t num_sobol_words; /* 1024 x 52 (APP/raytracing/sampling/sobol.h:34); may be NULL for the random sampler */
    const mcrt_light*        lights;        uint32_t num_lights;
    const mcrt_material*     materials;     uint32_t num_materials;
} mcrt_scene_desc;

/* BVH build options: RTScene::commit SetOption calls (APP/raytracing/scene/RTScene.cpp:203-238)
 * and IntersectorLDS::Process (RR/src/intersector/intersector_lds.cpp:176-196). */
typedef struct {
    float traversal_cost;   /* "bvh.sah.traversal_cost", default 10 */
    int   num_bins;         /* "bvh.sah.num_bins", default 64 */
    int   use_sah;          /* "bvh.builder" == "sah", default 1 */
    /* Which builder makes the flat structure.  0 (default) / 2: RadeonRays' Bvh2 node for node
     * (bit-exact parity), built on the device (mcrt_sahbuild.hip: the reference's split
     * arithmetic incl. this host's _mm_rcp_ps, its partition order in closed form; ~0.2 s for
     * 10 M triangles); falls back to 3 for num_bins > 64.  3: the same tree built on the host
     * (mcrt_bvh.cpp; ~2 s for 10 M triangles).  1: on-device linear BVH (Morton order, rocPRIM
     * radix sort), same record format and triangle data, different tree (equal-t hit ties may
     * resolve differently from the reference); ignores the three SAH fields.  4: perf tree (A/B
     * option, not the parity default): host binned SAH over all three axes, the cheapest split
     * wins (RR bins the largest centroid axis only); same records and traversal, another tree. */
    int   device_build;
    /* Two-level (instanced) structure: RadeonRays' IntersectorTwoLevel, which RR selects when a
     * shape is an instance (RTScene::attachMesh -> CreateInstance for every further entity that
     * shares a mesh, APP/raytracing/scene/RTScene.cpp:572-596) unless "bvh.forceflat"; forced by
     * "bvh.force2level" (RR/src/device/calc_intersection_device.cpp:68-105, defaults off,
     * PathTracingSettings.h:239-240).  Shapes with equal (startIdx, startVertex, numTriangles)
     * are instances of the first one; each keeps its own transform, shape id and material.
     * Host-built (device_build applies to the flat structure only). */
    int   force_2level;
    int   force_flat;
    /* Per-shape world-to-local matrices (Shape::SetTransform's minv, RR/include/radeon_rays.h;
     * the reference passes Transform::getWorldToLocalMatrix).  NULL: the transpose of each
     * shape's toWorldInverseTranspose.  Used by the two-level structure only. */
    const mcrt_mat4* world_to_local;
} mcrt_accel_opts;

#define MCRT_SAMPLER_SOBOL  0   /* KRN/samplers.cl:16 */
#define MCRT_SAMPLER_RANDOM 1   /* KRN/samplers.cl:17 (reference default) */

/* Integrators: RTPathTracingPass (KRN/PathTracing.cl) and RTBDPTPass (KRN/BDPT.cl). */
#define MCRT_INTEGRATOR_PT   0
#define MCRT_INTEGRATOR_BDPT 1

/* One frame = one sample per pixel (RTPathTracingPass::update, APP/.../RTPathTracingPass.cpp:40-114). */
typedef struct {
    int32_t frame_index;        /* integrator_frameNum */
    int32_t max_depth;          /* PathTracerSettings::GI.maxDepth (default 2) */
    int32_t sampler;            /* MCRT_SAMPLER_* */
    int32_t russian_roulette;   /* 0 = off (parity mode; the reference has none) */
    int32_t rr_start_depth;     /* first bounce at which RR may terminate */
    /* Tile split for multi-GPU: rows y with (y / band_rows) % num_bands == band_index
     * are rendered; others are left untouched.  num_bands = 1 renders everything. */
    int32_t band_rows;
    int32_t num_bands;
    int32_t band_index;
    /* MCRT_INTEGRATOR_PT (0, default) or MCRT_INTEGRATOR_BDPT (RTBDPTPass::update,
     * APP/.../RTBDPTPass.cpp:67-128).  BDPT with num_bands > 1 renders the band's camera and
     * light subpaths; its light-tracing strategies splat into any pixel, so the frame stops after
     * the visibility pass: the caller sums the ranks' splats (mcrt_bdpt_splats_copy + a
     * reduce-scatter) and completes it with mcrt_bdpt_gather. */
    int32_t integrator;
    /* 1: textures at camera-ray hits are read mip-mapped over the pixel footprint (ray
     * differentials, computeSurfaceInteractionWithDifferentials + readTexture2Df_lod +
     * computeMipmapLOD: KRN/geometry.cl:92-175, KRN/textures.cl:148-202).  The reference carries
     * this path switched off (KRN/textures.cl:204-209); 0 (default) = its bilinear level-0
     * reads.  PT only; needs the textures' mip chains (mcrt_texture_desc.numMipLevels). */
    int32_t texture_lod;
} mcrt_frame_params;

typedef struct mcrt_ctx_s*         mcrt_ctx;
typedef struct mcrt_scene_s*       mcrt_scene;
typedef struct mcrt_framebuffer_s* mcrt_framebuffer;

/* ------------------------------------------------------------------------ */
/* Context (replaces PlatformManager/KernelManager/RTBufferManager,
 * APP/raytracing/system/{Kernel,Platform}Manager.cpp, and RadeonRays::CreateFromOpenClContext,
 * RR/src/api/radeon_rays.cpp:288-318).  One context per GPU.               */
/* ------------------------------------------------------------------------ */
MCRT_API mcrt_status mcrt_ctx_create(int device, mcrt_ctx* out);
MCRT_API mcrt_status mcrt_ctx_destroy(mcrt_ctx ctx);
MCRT_API const char* mcrt_last_error(mcrt_ctx ctx);   /* ctx may be NULL: last global error */
MCRT_API mcrt_status mcrt_ctx_synchronize(mcrt_ctx ctx);
/* stream: a hipStream_t (as void*) all work of this context is enqueued on; NULL = the context's own stream. */
MCRT_API mcrt_status mcrt_ctx_set_stream(mcrt_ctx ctx, void* stream);
/* The context stream (hipStream_t) that accumulation and the frame-buffer copies are enqueued on:
 * a caller orders its own work (e.g. an RCCL collective) after them with it. */
MCRT_API mcrt_status mcrt_ctx_get_stream(mcrt_ctx ctx, void** stream);
/* Per-kernel HIP-event timing (replaces QueryManager GPU timers, source/engine/util/QueryManager.h:141-164).
 * enable = 2 also counts the shadow rays answered by their occluder hint (mcrt_framebuffer_hint_counts);
 * those counters are device atomics that slow the shadow launches by a few per cent, so timing runs use 1. */
MCRT_API mcrt_status mcrt_ctx_set_profiling(mcrt_ctx ctx, int enable);
/* Synchronizes, then fills up to max entries: kernel name, summed HIP-event time (ms),
 * launch count and items processed (pixels / rays / paths); *count = kernels with stats. */
MCRT_API mcrt_status mcrt_ctx_kernel_stats(mcrt_ctx ctx, int max, const char** names,
                                           double* total_ms, int64_t* launches,
                                           int64_t* items, int* count);
MCRT_API mcrt_status mcrt_ctx_reset_stats(mcrt_ctx ctx);
/* Attainable HBM bandwidth: a float4 stream-copy kernel over `bytes` (>= 1 GiB recommended,
 * well above the 256 MB Infinity Cache), best of `iters` launches; *gbps = (read + write)
 * bytes / time.  The roofline's "attainable" figure next to the 8 TB/s spec peak. */
MCRT_API mcrt_status mcrt_ctx_stream_copy(mcrt_ctx ctx, uint64_t bytes, int iters, double* gbps);
/* Dependent-gather ceiling of the traversal's access pattern: every lane of 32 waves per CU
 * follows a chain of 64-B records over an array of `records` records (uniformly random links
 * read from the record just fetched, four 16-B loads per step), `steps` steps, best of `iters`
 * launches; *gsteps = dependent record fetches per second / 1e9.  The roofline's reference for
 * the node-visit rate of the latency-bound traversal kernels (records ~ the tree's node count:
 * served from HBM; ~2 M: Infinity Cache; ~32 K: L2). */
MCRT_API mcrt_status mcrt_ctx_gather_chase(mcrt_ctx ctx, uint64_t records, int steps, int iters, double* gsteps);
/* The same probe over the compact records' layout (the per-ray walks, mcrt_traverse.h qwalk):
 * records of 32 B (an internal node: 2 x 16-B loads) or 48 B (a leaf: 3 loads in the same round
 * trip, its type carried in the link) packed back to back, a share leaf_frac of them leaves. */
MCRT_API mcrt_status mcrt_ctx_gather_chase_compact(mcrt_ctx ctx, uint64_t records, double leaf_frac, int steps,
                                                   int iters, double* gsteps);

/* ------------------------------------------------------------------------ */
/* Scene (replaces RTScene upload + RadeonRays CreateMesh/AttachShape/SetId/
 * SetTransform/Commit: APP/raytracing/scene/RTScene.cpp:28-56,199-267,564-809;
 * RR/include/radeon_rays.h:214-237).                                        */
/* ------------------------------------------------------------------------ */
MCRT_API mcrt_status mcrt_scene_create(mcrt_ctx ctx, const mcrt_scene_desc* desc, mcrt_scene* out);
MCRT_API mcrt_status mcrt_scene_destroy(mcrt_scene scene);
/* Dynamic updates (RTScene::update, APP/raytracing/scene/RTScene.cpp:317-391). Shapes
 * whose transforms change require mcrt_accel_build again. */
MCRT_API mcrt_status mcrt_scene_update_lights(mcrt_scene scene, const mcrt_light* lights, uint32_t n);
MCRT_API mcrt_status mcrt_scene_update_materials(mcrt_scene scene, const mcrt_material* m, uint32_t n);
MCRT_API mcrt_status mcrt_scene_update_shapes(mcrt_scene scene, const mcrt_shape* s, uint32_t n);
/* BVH build over all shapes in world space (IntersectionApi::Commit ->
 * IntersectorLDS::Process -> Bvh2::Build, RR/src/accelerator/bvh2.h:206-315).
 * Hit shapeid = index into the shapes array (RTScene assigns SetId(nextShapeId++)
 * in shape order, RTScene.cpp:592,668). opts may be NULL (defaults). */
MCRT_API mcrt_status mcrt_accel_build(mcrt_scene scene, const mcrt_accel_opts* opts);
/* Build statistics: node count, bytes on device, host build milliseconds. */
MCRT_API mcrt_status mcrt_accel_info(mcrt_scene scene, uint64_t* num_nodes, uint64_t* device_bytes,
                                     double* build_ms, uint32_t* num_triangles);
/* Which structure mcrt_accel_build made: two_level 0 (flat Bvh2) / 1 (instanced), distinct
 * meshes and instances of the two-level one, deepest traversal path. */
MCRT_API mcrt_status mcrt_accel_layout(mcrt_scene scene, int32_t* two_level, uint32_t* num_meshes,
                                       uint32_t* num_instances, int32_t* depth);
/* Copy of the device records (64 B each, the mcrt_accel_build_host_records layout) into out
 * (up to max_records; out may be NULL to query *num_records).  In a flat structure a triangle
 * leaf's int word 13 holds its parent record's index on the device (the occluder hints' box test)
 * where the host build leaves -1. */
MCRT_API mcrt_status mcrt_accel_read_records(mcrt_scene scene, float* out, uint64_t max_records,
                                             uint64_t* num_records);
/* ------------------------------------------------------------------------ */
/* Scene ingestion for C/C++ hosts (mcrt_objload.cpp): OBJ + MTL + PNG into the
 * SCENE_PARAMS arrays, replacing the reference's assimp import + RTScene mesh,
 * material and texture conversion (source/engine/resource/AssetImporter.cpp:40,
 * APP/raytracing/scene/RTScene.cpp:564-766, 826-880).  Left-handed (z negated,
 * winding flipped), fan triangulation, face normals where vn is missing,
 * uber materials from Kd/Ks/Ns + map_Kd/map_bump/map_d/map_Ks, RGBA8 textures.  */
/* ------------------------------------------------------------------------ */
typedef struct mcrt_obj_scene_s* mcrt_obj_scene;
#define MCRT_OBJ_MIPS            1   /* store each texture's glGenerateMipmap chain (uploadTextures) */
#define MCRT_OBJ_EMISSIVE_LIGHTS 2   /* materials with Ke > 0 become triangle-mesh area lights */
MCRT_API mcrt_status mcrt_obj_load(const char* path, uint32_t flags, mcrt_obj_scene* out);
/* Extra lights (the demo's sun: PathTracingApp.cpp:395-401).  Directional lights are placed on
 * the scene's bounding sphere like RTScene::setLight (RTScene.cpp:482-494). */
MCRT_API mcrt_status mcrt_obj_add_directional_light(mcrt_obj_scene s, const float dir[3], const float intensity[3]);
MCRT_API mcrt_status mcrt_obj_add_point_light(mcrt_obj_scene s, const float pos[3], const float intensity[3]);
/* The arrays as a mcrt_scene_desc for mcrt_scene_create (pointers owned by s, valid until the
 * next add_* call or mcrt_obj_free; sobol_matrices left NULL for the caller to set). */
MCRT_API mcrt_status mcrt_obj_scene_desc(mcrt_obj_scene s, mcrt_scene_desc* desc);
MCRT_API const char* mcrt_obj_warnings(mcrt_obj_scene s);   /* missing MTL / skipped textures */
MCRT_API void mcrt_obj_free(mcrt_obj_scene s);

/* Which builder made the flat structure: 0 host (or two-level), 1 device LBVH, 2 device SAH
 * (mcrt_accel_opts.device_build 0 and 2), 4 the host 3-axis SAH perf tree (device_build 4). */
MCRT_API mcrt_status mcrt_accel_builder(mcrt_scene scene, int32_t* builder);
/* Host-only build of the structure mcrt_accel_build would upload (no device needed): 64-B
 * records (mcrt_bvh.cpp / mcrt_bvh2l.cpp layouts) into out_records (up to max_records; may be
 * NULL to query *num_records); info[4] = {two_level, top-level records, depth, meshes}.
 * For tools and tests (e.g. pinning the trees against the reference builders). */
MCRT_API mcrt_status mcrt_accel_build_host_records(const mcrt_scene_desc* desc, const mcrt_accel_opts* opts,
                                                   float* out_records, uint64_t max_records,
                                                   uint64_t* num_records, int32_t* info);

/* ------------------------------------------------------------------------ */
/* Ray queries on DEVICE buffers (IntersectionApi::QueryIntersection /
 * QueryOcclusion, RR/include/radeon_rays.h:267-277 -> IntersectorLDS::Intersect/
 * Occluded, RR/src/intersector/intersector_lds.cpp:266-326).
 * Semantics of intersect_main/occluded_main (RR/src/kernels/CL/intersect_bvh2_lds.cl):
 *  - rays with extra[1] == 0 leave their output untouched;
 *  - a leaf is skipped when ray mask (extra[0]) == shape id (RR_RAY_MASK);
 *  - closest: miss -> shapeid = primid = -1 (uvwt untouched), hit -> uvwt = (u,v,0,t);
 *  - any: 1 = occluded, -1 = not occluded.                                 */
/* ------------------------------------------------------------------------ */
MCRT_API mcrt_status mcrt_trace_closest(mcrt_scene scene, const mcrt_ray* d_rays, int32_t n,
                                        mcrt_intersection* d_hits);
MCRT_API mcrt_status mcrt_trace_any(mcrt_scene scene, const mcrt_ray* d_rays, int32_t n,
                                    int32_t* d_hits);
/* The variants with the ray count in device memory (QueryIntersection / QueryOcclusion with
 * `Buffer const* numrays, int maxrays`, RR/include/radeon_rays.h:272-277; the count a previous
 * kernel wrote, read by the query kernel itself, so no host round trip): min(*d_numrays, maxrays)
 * rays are traced, the grid covers maxrays.  Asynchronous on the context stream, as RR's queries:
 * the query waits for wait_event (NULL: none) and, when done_event is not NULL, *done_event
 * receives a new event recorded after it (RR's `Event** event`; mcrt_event_wait = Event::Wait,
 * mcrt_event_destroy = IntersectionApi::DeleteEvent). */
typedef struct mcrt_event_s* mcrt_event;
MCRT_API mcrt_status mcrt_trace_closest_count(mcrt_scene scene, const mcrt_ray* d_rays, const int32_t* d_numrays,
                                              int32_t maxrays, mcrt_intersection* d_hits, mcrt_event wait_event,
                                              mcrt_event* done_event);
MCRT_API mcrt_status mcrt_trace_any_count(mcrt_scene scene, const mcrt_ray* d_rays, const int32_t* d_numrays,
                                          int32_t maxrays, int32_t* d_hits, mcrt_event wait_event,
                                          mcrt_event* done_event);
MCRT_API mcrt_status mcrt_event_wait(mcrt_event event);
MCRT_API mcrt_status mcrt_event_destroy(mcrt_event event);

/* ------------------------------------------------------------------------ */
/* Frame buffer + integrator (RTPrimaryRaysPass, RTPathTracingPass,
 * RTReconstructionPass: APP/raytracing/renderPasses/RT*Pass.cpp; kernels
 * KRN/PathTracing.cl, KRN/reconstruction.cl).                              */
/* ------------------------------------------------------------------------ */
MCRT_API mcrt_status mcrt_framebuffer_create(mcrt_ctx ctx, uint32_t width, uint32_t height,
                                             mcrt_framebuffer* out);
MCRT_API mcrt_status mcrt_framebuffer_destroy(mcrt_framebuffer fb);
/* Frames in flight (PT): mcrt_render_frame for frame i uses buffer slot i mod n on its own HIP
 * stream and returns at once; mcrt_accumulate runs on the context stream in call order, after
 * that frame's render, so n frames overlap on the GPU and the image is unchanged bit for bit
 * (the reference's pass sequence per frame, RTPathTracingPass::update then
 * RTReconstructionPass::updateReconstruction, is kept; only its clFinish after every launch is
 * gone).  0 = auto = 2: each launch's divergent tail of long rays is filled by the next
 * frame's launches (small band shares are better widened by mcrt_render_frames).  Reads of the frame
 * buffer synchronise every slot.  No reference counterpart (its passes are synchronous). */
#define MCRT_MAX_FRAMES_IN_FLIGHT 4
MCRT_API mcrt_status mcrt_framebuffer_set_frames_in_flight(mcrt_framebuffer fb, int32_t n);
/* Renders one 1-spp frame: PrimaryRays + maxDepth x (shade, shadow, extend).
 * Result: per-pixel frame radiance ("RadianceBufferCL"). */
MCRT_API mcrt_status mcrt_render_frame(mcrt_scene scene, mcrt_framebuffer fb, const mcrt_camera* camera,
                                       const mcrt_frame_params* params);
/* ReconstructionPass (KRN/reconstruction.cl:6-60): clamp [0,1000] (NaN->0),
 * frame_index 0 overwrites, else accumulates sum(w*L), sum(w); image = ratio.
 * After mcrt_render_frames it accumulates every frame of that batch in frame order
 * (frame_index = the batch's first frame), all with this filter. */
MCRT_API mcrt_status mcrt_accumulate(mcrt_framebuffer fb, const mcrt_filter* filter, int32_t frame_index);
/* Batched frames (PT and BDPT): renders the `count` (PT 1..256, BDPT 1..32: its per-frame arrays
 * are whole-frame sized) consecutive 1-spp frames
 * params->frame_index + k, k < count, with cameras[k] (per-frame TAA jitter), in ONE pass --
 * every launch (camera rays, shading, shadow + extension rays) covers all count frames' paths,
 * so a small per-rank band share (tile split over N GPUs) still fills the 256 CUs and the
 * divergent tail of each launch is paid once per batch (1/8 of the bands x 160 frames = the
 * paths of one GPU's 20-frame call).  Per frame the arithmetic, the RNG
 * streams (keyed by pixel, frame_index + k, bounce) and the radiance are exactly those of
 * mcrt_render_frame; mcrt_accumulate_frames (or mcrt_accumulate) then sums them in frame order,
 * so the image equals count x (mcrt_render_frame + mcrt_accumulate) bit for bit.  Radiance read
 * back (mcrt_framebuffer_read 0) is the batch's first frame.  The reference renders one frame
 * per RTPathTracingPass::update; this is the same sequence, launched wider.
 * BDPT (RTBDPTPass::update per frame): every launch covers the batch's (tile, frame) paths; the
 * s = 1 strategies walk the batch's frames in order, so the sampled-light-vertex slot each frame
 * reads is the one the previous frame wrote (BDPT.cl:585-586), as in count single calls; vertices
 * and own strategies are those of count single calls bit for bit, splat sums up to atomic order.
 * With a band split, mcrt_bdpt_splat_layout's chunk then holds the batch's frames.
 * Memory (PT): each frame slot (2 in flight) holds about 0.8 KB per path of the call (ray queues,
 * hit records, the per-ray traversal stack spill and, for calls of >= 16 M paths, the stopped
 * walks' state) plus 32 B per pixel and frame: 1080p x 20 frames ~ 34 GB per slot.  A call that does not fit fails with the hipMalloc error (nothing is
 * rendered; smaller calls still work), e.g. 256 whole 1080p frames; 256 band-frames of a 1/8
 * band share fit. */
MCRT_API mcrt_status mcrt_render_frames(mcrt_scene scene, mcrt_framebuffer fb, const mcrt_camera* cameras,
                                        int32_t count, const mcrt_frame_params* params);
/* filters: `count` filters (one per frame of the last mcrt_render_frames; the per-frame filter
 * props of RTReconstructionPass) or 1 shared by all; frame_index = the batch's first frame. */
MCRT_API mcrt_status mcrt_accumulate_frames(mcrt_framebuffer fb, const mcrt_filter* filters, int32_t count,
                                            int32_t frame_index);
/* Device pointers of the frame buffer's arrays (float4 x W*H, float x W*H).  The radiance
 * pointer is the plane of the LAST rendered frame: frames rotate through the frame slots
 * (mcrt_framebuffer_set_frames_in_flight), so it is valid only until the next render call on this
 * frame buffer, and work on another stream must first synchronise with the frame (e.g.
 * mcrt_ctx_synchronize).  The accumulator and image pointers are fixed for the frame buffer's life. */
MCRT_API mcrt_status mcrt_framebuffer_device_ptrs(mcrt_framebuffer fb, void** radiance, void** weighted_sum,
                                                  void** weight_sum, void** image);
/* Post-process of the accumulated image, the passes after RTReconstructionPass in the
 * reference pipeline (PathTracingApp.cpp:240-254): RTDenoisePass (BilateralDenoise,
 * KRN/Denoise.cl:6-47, RTDenoisePass.cpp) then RTToneMappingPass (ReinhardToneMapping,
 * KRN/ToneMapping.cl:42-63, RTToneMappingPass.cpp; the pass passes GI.minLuminance as Lwhite).
 * Result: the display image (mcrt_framebuffer_read which = 3), = the image when both are off. */
typedef struct {
    int32_t use_denoise;        /* GI.useDenoise (default 0) */
    int32_t denoise_radius;     /* GI.denoiseKernelRadius (default 1) */
    float   sigma_spatial;      /* GI.bilateralDenoiseSigmaSpatial (default 1.0) */
    float   sigma_range;        /* GI.bilateralDenoiseSigmaRange (default 0.1) */
    int32_t use_tonemapping;    /* GI.useTonemapping (default 0) */
    float   min_luminance;      /* GI.minLuminance (default 2.0), Reinhard's Lwhite */
} mcrt_postprocess_params;
MCRT_API mcrt_status mcrt_postprocess(mcrt_framebuffer fb, const mcrt_postprocess_params* params);
/* Per-pixel outputs at the camera-ray hits (camera rays traced by this call; no shading):
 *  MCRT_AOV_ALBEDO:      float4 per pixel = (uber diffuse Kd incl. texture, opacity.x), zero on
 *                        a miss; mip-mapped when params->texture_lod (an albedo guide for denoisers)
 *  MCRT_AOV_TEXTURE_LOD: 3 float4 per pixel = (duvdx, duvdy), (diffuse-texture LOD, shape index
 *                        bits, uv), the diffuse texture read at that LOD (zeros where untextured).
 * host_out: W*H*{1|3}*4 floats.  Band fields of params select the rows as in mcrt_render_frame. */
#define MCRT_AOV_ALBEDO      0
#define MCRT_AOV_TEXTURE_LOD 1
MCRT_API mcrt_status mcrt_render_aov(mcrt_scene scene, mcrt_framebuffer fb, const mcrt_camera* camera,
                                     const mcrt_frame_params* params, int aov, float* host_out);
/* Copies device -> host (RGBA32F, W*H*4 floats).  which: 0 radiance, 1 weighted sum, 2 image,
 * 3 display image (mcrt_postprocess). */
MCRT_API mcrt_status mcrt_framebuffer_read(mcrt_framebuffer fb, int which, float* host_rgba);
/* Radiance of frame k (0 <= k < count) of the last mcrt_render_frames call (k = 0: the same as
 * mcrt_framebuffer_read 0): the reference's RadianceBufferCL of that frame
 * (RTPathTracingPass.cpp:106), RGBA32F, W*H*4 floats. */
MCRT_API mcrt_status mcrt_framebuffer_read_frame(mcrt_framebuffer fb, int32_t k, float* host_rgba);
/* Device-to-device copy of one frame-buffer array into caller memory (e.g. a torch/RCCL
 * buffer for the multi-GPU reduce): which 0 radiance (float4), 1 weighted sum (float4),
 * 2 image (float4), 3 weight sum (float).  Enqueued on the context stream, ordered after the
 * last render; the radiance copy keeps that frame's slot from taking a new frame until read. */
MCRT_API mcrt_status mcrt_framebuffer_copy_device(mcrt_framebuffer fb, int which, void* d_dst);
/* Inverse for multi-GPU: overwrite the weighted sums (float4) and weights (float) from device
 * memory (after a reduce) and recompute the image = sum / weight on the device. */
MCRT_API mcrt_status mcrt_framebuffer_set_accumulation(mcrt_framebuffer fb, const void* d_wsum, const void* d_wts);
/* Tile split (mcrt_frame_params.num_bands > 1), end of job, without full-frame copies: pack this
 * rank's own rows of the accumulators (its bands of the last render, local 8-row block tb at rows
 * 8 tb .. 8 tb + 7) into d_dst, one row = W x float4 weighted sum then W x float weight (5 W
 * floats), straight from the frame buffer.  Rows past the rank's last row are left untouched.
 * Enqueued on the context stream after the last accumulate.  Replaces the all-reduce of the two
 * accumulation buffers the reference would need (RTPathTracingPass.cpp:99-117 accumulates on one
 * device) with the gather of mcrt.dist.gather_bands_fb. */
MCRT_API mcrt_status mcrt_framebuffer_bands_pack(mcrt_framebuffer fb, void* d_dst);
/* On the gathering rank: d_recv = num_bands chunks of max_rows packed rows (chunk r = rank r's
 * mcrt_framebuffer_bands_pack output); every other rank's rows are written into this frame
 * buffer's accumulators in place and the image = sum / weight is recomputed (the same division
 * as mcrt_framebuffer_set_accumulation).  Enqueued on the context stream. */
MCRT_API mcrt_status mcrt_framebuffer_bands_unpack(mcrt_framebuffer fb, const void* d_recv, int32_t max_rows);
/* Band geometry of the last render, for a C++ host sizing the gather of the packed rows:
 * max_rows = the largest rank's row count (whole 8-row blocks; one packed chunk = max_rows x 5 W
 * floats, the max_rows argument of mcrt_framebuffer_bands_unpack), and the num_bands / band_index
 * the frame was rendered with.  Any output pointer may be NULL. */
MCRT_API mcrt_status mcrt_framebuffer_band_layout(mcrt_framebuffer fb, int32_t* max_rows, int32_t* num_bands,
                                                  int32_t* band_index);
/* Per-frame path statistics of the last render (paths, closest rays, any rays, ...). */
MCRT_API mcrt_status mcrt_framebuffer_stats(mcrt_framebuffer fb, int64_t* closest_rays, int64_t* any_rays,
                                            int64_t* shaded_paths);
/* Queue sizes of the last PT render, per bounce b < max: shadow[b] = shadow rays queued by
 * bounce b's shading, extension[b] = extension rays queued for bounce b+1. */
MCRT_API mcrt_status mcrt_framebuffer_queue_counts(mcrt_framebuffer fb, int32_t* shadow, int32_t* extension, int max);
/* Shadow rays of the last PT render answered by their occluder hint, per bounce b < max (the rest
 * walked the tree; the reference walks every one, intersect_bvh2_lds.cl:229-363, with the same
 * answers).  Counted while mcrt_ctx_set_profiling(ctx, 2) is on; zero otherwise, when the hints are
 * off (MCRT_SHADOW_HINTS=0) or the structure is two-level. */
MCRT_API mcrt_status mcrt_framebuffer_hint_counts(mcrt_framebuffer fb, int32_t* hits, int max);
/* Extension rays of the last PT render whose closest-hit walk over the compact records ended on a
 * near tie and was repeated on the exact 64-B records (so the reference's visit order resolves it),
 * per bounce b < max (rays traced for bounce b + 1).  Counted while mcrt_ctx_set_profiling(ctx, 2)
 * is on; zero otherwise and with MCRT_QUANT_NODES=0. */
MCRT_API mcrt_status mcrt_framebuffer_retrace_counts(mcrt_framebuffer fb, int32_t* retraces, int max);
/* Diagnostics: with MCRT_WAVE_CLOCK=1 in the environment, the last PT call's launches record each
 * workgroup's (start, end) on the constant 100-MHz clock (s_memrealtime, low 32 bits); which = 0
 * camera launch, 1 bounce-0 shadow + extension launch (extension workgroups), 2 last-bounce shadow
 * launch.  Copies min(max_blocks, *blocks) pairs; (0, 0) = a workgroup that had no work.  While
 * MCRT_WAVE_CLOCK is set every render keeps ONE frame in flight (the buffers are per frame buffer). */
MCRT_API mcrt_status mcrt_framebuffer_wave_clock(mcrt_framebuffer fb, int which, uint32_t* host_out, int64_t max_blocks,
                                                 int64_t* blocks);
/* Host copy of a ray queue of the last render (the state the reference keeps in its
 * per-pixel trace_shadowRays / trace_rays / throughput buffers):
 *   which 0: shadow queue of the last bounce    -- origin.xyz|tmax, dir.xyz|pixel(int bits), throughput*L
 *   which 1: last extension queue (bounce D-2)  -- origin.xyz|pixel(int bits), dir.xyz|bsdf flags, throughput
 * Writes min(count, max_records) records as three float4 arrays back to back
 * (dst = [a0..a(n-1) | b0.. | c0..], 48 * max_records bytes) and the full count.
 * The ORDER of the records is not deterministic: the shading kernels append them per workgroup
 * through LDS atomics (grouped by octant x dominant axis), so two runs hold the same set of
 * records in different orders.  Every record carries its pixel, and the radiance does not depend
 * on the order; compare queues as sets (e.g. sorted by pixel). */
MCRT_API mcrt_status mcrt_framebuffer_read_queue(mcrt_framebuffer fb, int which, void* host_dst,
                                                 int64_t max_records, int32_t* count);
/* Host copy of the BDPT state of the last BDPT frame (the reference keeps it in RTBDPTPass's
 * m_cameraVertices / m_lightVertices / vertex-count buffers, RTBDPTPass.cpp:456-470):
 *   which 0: camera vertices, (D+2) depths x 8 planes of float4 x W*H (layout: mcrt_bdpt.hip)
 *         1: light vertices, (D+1) depths x 8 planes     2/3: camera / light vertex counts (int32 x W*H)
 *         4: own-strategy contributions ((C-D) planes)   5: persistent s=1 sampled light vertices (D planes)
 *         6: light-tracing (t=1) splat sums of the frame (float4 x W*H)
 * Copies min(bytes, size) bytes; *needed = the array's size (host_dst may be NULL to query it). */
/* Band-split BDPT (num_bands > 1): the frame's light-tracing splats land in any pixel, so the ranks
 * exchange them once per frame (the reference's ConnectVertices atomics + CopyBuffer,
 * BDPT.cl:671-913).  The splats are laid out RANK-MAJOR: `chunks` (= num_bands) chunks of
 * `chunk_pixels` pixels of MCRT_SPLAT_CHANNELS (3) floats -- r, g, b, as the reference's splat
 * buffer (BDPT.cl:654-669, 888-899) -- chunk r holding the rows of rank r's bands in its own tile order (zero
 * past its last row), so ONE reduce-scatter hands each rank exactly its rows' sums:
 *   mcrt_bdpt_splat_layout   the chunk geometry of the last frame's band split;
 *   mcrt_bdpt_splats_copy    this rank's splats, rank-major, into d_dst (chunks x chunk_pixels
 *                            x 3 floats of device memory), ENQUEUED on the frame's stream
 *                            (mcrt_framebuffer_stream): order the collective after it there (no
 *                            host synchronisation, so frames in flight keep overlapping);
 *   mcrt_bdpt_gather         completes the rank's bands with d_own_chunk = chunk band_index of the
 *                            ranks' summed buffers (chunk_pixels x 3 floats; NULL: the rank's own splats
 *                            in its natural layout -- a 1-rank check).  It reads d_own_chunk on the
 *                            frame's stream; a later mcrt_bdpt_splats_copy waits for it.
 * Rendering or accumulating in between fails with MCRT_ERROR_NOT_READY.  With no frame pending (a
 * light-less scene, a whole-image frame) the copy writes zeros and the gather does nothing. */
#define MCRT_SPLAT_CHANNELS 3
MCRT_API mcrt_status mcrt_bdpt_splat_layout(mcrt_framebuffer fb, uint64_t* chunk_pixels, int32_t* chunks);
/* The HIP stream (hipStream_t) the last frame of fb was enqueued on (its frame slot's). */
MCRT_API mcrt_status mcrt_framebuffer_stream(mcrt_framebuffer fb, void** stream);
MCRT_API mcrt_status mcrt_bdpt_splats_copy(mcrt_framebuffer fb, void* d_dst);
MCRT_API mcrt_status mcrt_bdpt_gather(mcrt_framebuffer fb, const void* d_own_chunk);
/* Sparse splat exchange (the band split's alternative to the dense rank-major buffer above): only a
 * few per cent of a rank's paths splat into another rank's rows (San-Miguel proxy: ~2.6 %), so the
 * ranks exchange those splats as records -- 4 floats: the target path index (k * W*H + pixel, int
 * bits), r, g, b -- with one all-to-all instead of reducing whole frames:
 *   mcrt_framebuffer_set_splat_exchange  MCRT_SPLAT_EXCHANGE_SPARSE before rendering (DENSE: default);
 *                            k_bdpt_vis then adds the rank's own-row splats in place and lists the rest;
 *   mcrt_bdpt_splats_sparse  counts[r] = records for rank r (counts[band_index] = 0), SYNCHRONOUS up to
 *                            the frame's visibility pass (the sizes are host data for the all-to-all);
 *                            when d_dst holds capacity >= sum(counts) records of device memory it also
 *                            groups the records by rank into it, enqueued on the frame's stream (else
 *                            counts only: grow the buffer and call again);
 *   mcrt_bdpt_gather_sparse  adds the `records` received records (targets in this rank's rows) and
 *                            completes the rank's bands, on the frame's stream.
 * The frame equals the dense exchange's (and one GPU's) up to the order of the splat sums. */
#define MCRT_SPLAT_EXCHANGE_DENSE 0
#define MCRT_SPLAT_EXCHANGE_SPARSE 1
MCRT_API mcrt_status mcrt_framebuffer_set_splat_exchange(mcrt_framebuffer fb, int32_t mode);
MCRT_API mcrt_status mcrt_bdpt_splats_sparse(mcrt_framebuffer fb, void* d_dst, int64_t capacity, int64_t* counts,
                                             int32_t num_counts);
MCRT_API mcrt_status mcrt_bdpt_gather_sparse(mcrt_framebuffer fb, const void* d_recv, int64_t records);
MCRT_API mcrt_status mcrt_framebuffer_read_bdpt(mcrt_framebuffer fb, int which, void* host_dst, uint64_t bytes,
                                                uint64_t* needed);

/* ------------------------------------------------------------------------ */
/* Host helpers                                                              */
/* ------------------------------------------------------------------------ */
/* The reference host's RTPinholeCamera (kernel_data.h:246-264), bit for bit: CameraComponent
 * (source/engine/camera/CameraComponent.cpp:61-134: glm::perspective -- left-handed, the vendored
 * glm forces GLM_FORCE_LEFT_HANDED -- and the view matrix from the transform's rotation columns
 * right / up / look), RTUtil::screenToRay for the four image corners at the near plane
 * (APP/raytracing/util/RTUtil.cpp:9-41, RTPrimaryRaysPass.cpp:81-104) with pixel_offset = the
 * TAA jitter in pixels (GI.filterSettings.curPixelOffset), worldToClip = viewProj (row major) and
 * the z = 1 image-plane area of RTBDPTPass.cpp:158-166.  fov_y is the value the reference hands to
 * glm::perspective, i.e. RADIANS (note: PathTracingApp.cpp:387 passes 45.0f, so the reference
 * app's vertical field of view is 45 rad mod pi ~ 58.3 degrees).  float32 in glm's operation
 * order (mcrt_camera.cpp), pinned against the reference's own glm (tests/test_camera_cpu.py). */
MCRT_API mcrt_status mcrt_make_pinhole_camera_axes(const float pos[3], const float right[3], const float up[3],
                                                   const float look[3], float fov_y, float near_z, float far_z,
                                                   uint32_t width, uint32_t height, const float pixel_offset[2],
                                                   mcrt_camera* out);
/* Convenience form: a look-at camera (Camera::lookAt, source/engine/camera/Camera.cpp:58-63, with
 * forward = target - position) and the field of view in DEGREES (glm::radians); otherwise
 * mcrt_make_pinhole_camera_axes. */
MCRT_API mcrt_status mcrt_make_pinhole_camera(const float pos[3], const float forward[3], const float up[3],
                                              float fov_y_deg, float near_z, float far_z,
                                              uint32_t width, uint32_t height,
                                              const float pixel_offset[2], mcrt_camera* out);
/* TAA jitter of frame `frame` (PathTracingApp.cpp:208-215): pixel offset =
 * (lerp(-rx, rx, sobol(frame, 0)), lerp(-ry, ry, sobol(frame, 1))), Sampler::sobolSample with
 * scramble 0 over the 1024 x 52 g_SobolMatrices32 (the scene's sobol_matrices); radius = the
 * reconstruction filter radius (GI.filterSettings.radius). */
MCRT_API mcrt_status mcrt_taa_pixel_offset(const uint32_t* sobol_matrices, uint32_t frame, float radius_x,
                                           float radius_y, float out[2]);
/* Library version / build string. */
MCRT_API const char* mcrt_version(void);

#ifdef __cplusplus
}
#endif

#ifdef __cplusplus
static_assert(sizeof(mcrt_shape) == 160, "RTShape is 160 B");
static_assert(sizeof(mcrt_material) == 128, "RTMaterial is 128 B");
static_assert(sizeof(mcrt_light) == 80, "RTLight is 80 B");
static_assert(sizeof(mcrt_camera) == 176, "RTPinholeCamera is 176 B");
static_assert(sizeof(mcrt_texture_desc) == 16, "TextureDesc2D is 16 B");
static_assert(sizeof(mcrt_ray) == 48, "RR ray is 48 B");
static_assert(sizeof(mcrt_intersection) == 32, "RR Intersection is 32 B");
static_assert(sizeof(mcrt_filter) == 56, "RTFilterProperties (device) is 56 B");
static_assert(offsetof(mcrt_material, uber_roughness) == 80, "roughness @80");
static_assert(offsetof(mcrt_material, uber_normalMapId) == 96, "normalMapId @96");
static_assert(offsetof(mcrt_camera, width) == 160, "width @160");
static_assert(offsetof(mcrt_filter, radius) == 8, "radius @8 (device)");
static_assert(offsetof(mcrt_filter, mitchellB) == 16, "B @16 (device)");
static_assert(offsetof(mcrt_filter, pixelOffset) == 40, "pixelOffset @40 (device)");
#else
_Static_assert(sizeof(mcrt_shape) == 160, "RTShape is 160 B");
_Static_assert(sizeof(mcrt_material) == 128, "RTMaterial is 128 B");
_Static_assert(sizeof(mcrt_light) == 80, "RTLight is 80 B");
_Static_assert(sizeof(mcrt_camera) == 176, "RTPinholeCamera is 176 B");
_Static_assert(sizeof(mcrt_ray) == 48, "RR ray is 48 B");
_Static_assert(sizeof(mcrt_intersection) == 32, "RR Intersection is 32 B");
_Static_assert(sizeof(mcrt_filter) == 56, "RTFilterProperties (device) is 56 B");
#endif

#endif /* MCRT_CAPI_H */

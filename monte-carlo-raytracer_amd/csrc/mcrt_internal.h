// mcrt_internal.h -- structures shared by the host runtime (mcrt_capi.cpp) and the
// HIP kernels (mcrt_kernels.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstddef>
#include <string>

#include "../../include/mcrt_capi.h"

// Device view of the scene (the 15 SCENE_PARAMS arrays + our BVH).
struct SceneArgs {
    const mcrt_shape* shapes;
    const uint32_t* indices;
    const float4* positions;
    const float2* uvs;
    const float4* normals;
    const mcrt_texture_desc* textures;
    const uint8_t* texData;
    const uint32_t* sobol;
    const mcrt_light* lights;
    const mcrt_material* materials;
    const float4* nodes;  // unified BVH (mcrt_bvh.cpp): leaf k = (v0, shape), (e1, prim), (e2, -), marker
    // Surface records (built at scene upload, mcrt_build_surface_records): one 128-B record per
    // triangle of each distinct (startIdx, startVertex) mesh with the object-space p0..p2,
    // uv0..uv2 and n0..n2 computeSurfaceInteraction reads (geometry.cl:180-191), so a hit costs
    // one cache line instead of an index line + 9 scattered vertex lines.  Shape k's triangle p
    // is record surfBase[k] + p.
    const float4* surf;
    const uint32_t* surfBase;
    int numLights;
};

struct FrameArgs {
    uint32_t W, H;
    int frame, maxDepth, sampler;
    int russianRoulette, rrStartDepth;
    int bandRows, numBands, bandIndex;
    int tilesX, numTiles;   // 8x8 tiles of this rank's bands
    int textureLod;         // mip-mapped texture reads at camera-ray hits (PT)
    int batch;              // frames per launch (mcrt_render_frames): path id = k * W*H + pixel, frame f.frame + k
    int tileMajor;          // launch order of (tile, frame k): 1 = a tile's frames adjacent, 0 = frame-major
    int primaryPack;        // camera launch: 1 = a wave holds a few pixels x all batch frames
    int shadePack;          // first shading launch: the same packing (its ray queues inherit the order)
    // Longest-first tile order of the camera and first-shading launches (NULL: tile order): slot j
    // of the launch takes tile tileOrder[j]; tileCost (NULL: not recorded) accumulates each tile's
    // camera-wave time for the next call's order (mcrt_kernels.hip k_tile_order)
    const uint32_t* tileOrder;
    uint32_t* tileCost;
};
// Frames per mcrt_render_frames call.  PT: a rank's share of a multi-GPU step (1/N of each frame's
// bands) x N frames per step keeps its launches as large as one GPU's (N = 8: 20 steps = 160
// band-frames in one call).  BDPT's per-frame arrays are whole-frame sized (~3.2 KB per pixel), so
// its calls stay at 32 frames.
#define MCRT_MAX_BATCH_FRAMES 256
#define MCRT_MAX_BDPT_BATCH_FRAMES 32

struct QueueArgs {
    int* shadowCount;
    float4 *sO, *sD, *sL;
    int* extCountOut;
    float4 *eOout, *eDout, *eTout;
};

// float4 planes per BDPT vertex: 8 for the vertex, 5 for its uber-material properties
#define BDPT_VERTEX_PLANES 13
// BDPT per-frame state (mcrt_bdpt.hip header comment has the layout)
struct BdptArgs {
    float4* camV;        // (D+2) x 8 planes x N
    float4* lightV;      // (D+1) x 8 planes x N
    int* camCount;       // N
    int* lightCount;     // N
    float4* sampLight;   // D planes x N, persistent across frames
    float4* slots;       // ownSlots planes x N
    float4* splat;       // N
    int ownSlots;        // strategies with t >= 2 = maxConnections - D
    int depth0Const;     // 1: the frame-invariant planes of the depth-0 vertices are already in place
                         // at this plane stride (k_bdpt_start writes only the per-frame ones)
    uint32_t* lightKey;  // per start-queue slot: the light ray's origin / direction cell (NULL: no sort)
    uint32_t* lightSlot; //   and its slot (the radix sort's values)
    uint32_t* extKey;    // per slot of a bounce queue that will be traced: the ray's direction octant and
    uint32_t* extSlot;   //   origin cell (NULL: no sort), and its slot
    float keyLo[3], keyScale[3];   // origin cell = (o - keyLo) * keyScale, 32 x 8 x 32 cells
    // Band split, sparse splat exchange (NULL list: the dense rank-major exchange): light-tracing
    // splats landing in another rank's rows are appended here as (target path index bits, r, g, b);
    // the rank's own land in `splat`.  Owner of pixel row y: ((y / 8) / bpb) % bands.
    float4* splatList;
    int* splatListCount;
    int splatListCap;
    int splatW, splatN0, splatBpb, splatBands, splatBand;
    // the light-tracing strategies (t = 1) evaluated by the vertex launch that creates their light
    // vertex (lightInVertex), appending to the connection queue: the batch's cameras and that queue
    const mcrt_camera* cams;
    int* connCount;
    float4 *connO, *connD, *connL;
    int lightInVertex;
};
struct BdptQueue {
    int* count;
    float4 *o, *d, *t;
};

// entries of a wave packet's stack (one VGPR lane each: node word + 64-bit lane mask); a level
// pushes at most 2, so trees of depth <= MCRT_PK_STACK / 2 take the packets
#define MCRT_PK_STACK 64
struct TraceCtx {
    const float4* nodes;   // 4 float4 per node (mcrt_bvh.cpp): internal = child boxes + indices, leaf = triangle
                           // two-level (mcrt_bvh2l.cpp): + instance records (world->object rows, bottom root)
    int twoLevel;          // selects the kernels' two-level instantiation (launch-time, not per lane)
    int packet;            // coherent launches (camera rays, bounce-0 shadow rays) walk the tree as wave
                           // packets (mcrt_traverse.h traversePacket); flat trees of depth <= MCRT_PK_STACK / 2
    uint32_t* spill;
    int spillCap;           // spill entries per ray (a multiple of STACK_LDS)
    int* overflow;
    // Occluder hints of the any-hit launches over plain records (mcrt_traverse.h hintOccludes):
    // a table of leaf indices that shadow rays test before walking the tree.  NULL = off.
    uint32_t* hint;
    int hintMode;           // MCRT_HINT_PIXEL: slot = path id % hintPixels; MCRT_HINT_CELL: hash of the
                            // ray's origin cell (MCRT_HINT_GRID^3 over the scene bounds) and octant
    uint32_t hintPixels;
    uint32_t* hintCell;     // the origin-cell table (also given to pixel-mode launches)
    uint32_t hintMask;      // cell table entries - 1 (a power of two)
    float hintLo[3], hintInvExt[3];   // cell = (o - hintLo) * hintInvExt * MCRT_HINT_GRID
    uint32_t numNodes;      // records in `nodes` (hints are range-checked against it)
    int* hintHits;          // rays answered by their hint are counted here (NULL: not counted)
    // Compact records of the same tree (mcrt_kernels.hip k_qnodes_convert; the per-ray walks of the
    // LAY_QUANT instantiations, mcrt_traverse.h traverseQOct): 32-B internal records with 8-bit
    // outward-rounded child boxes, 48-B leaves; a record reference is (offset / 16) << 1 | leaf.
    // NULL: not built (two-level, non-DFS trees, MCRT_QUANT_NODES=0).
    const float4* qnodes;
    uint32_t qroot;
    int* retraces;          // closest-hit walks repeated on the exact records (near ties; NULL: not counted)
    uint32_t* waveClock;    // diagnostics (MCRT_WAVE_CLOCK=1): per workgroup (start, end) of the 100-MHz clock
    // Stop rule of the extension rays' compact walks in k_shadow_extend (walkCap 0: none).  A wave
    // stops once it has taken walkCap steps and at most walkLanes of its lanes are still walking;
    // the unfinished walks are appended to `suspend` (MCRT_SUSPEND_F4 float4 each, *suspendCount of
    // them) and k_walk_resume finishes them in dense waves.
    int walkCap, walkLanes;
    float4* suspend;
    int* suspendCount;
};
#define MCRT_SUSPEND_F4 6

#define MCRT_HINT_PIXEL 1
#define MCRT_HINT_CELL 2
#define MCRT_HINT_CELL_BITS 25
#ifndef MCRT_HINT_GRID
#define MCRT_HINT_GRID 768
#endif

namespace mcrt {
// n rays, or with countDev (device memory) min(*countDev, n) of them
void launch_trace_rays(bool any, const TraceCtx& c, const mcrt_ray* rays, int n, const int* countDev,
                       mcrt_intersection* hits, int* occl, hipStream_t st);
void launch_surface_records(const uint32_t* meshStartIdx, const uint32_t* meshStartVertex, const uint32_t* meshBase,
                            int numMeshes, uint32_t numRecords, const uint32_t* indices, const float4* positions,
                            const float2* uvs, const float4* normals, float4* surf, hipStream_t st);
void launch_primary(const TraceCtx& c, const FrameArgs& f, const mcrt_camera* cam, float4* hits, hipStream_t st);
// closest hit over two queues in one launch: queue 0 over cc's records, queue 1 over c's
// the light-start queue of a BDPT call sorted by cell (keys, slots from k_bdpt_start) -> perm
size_t bdpt_light_sort_temp_bytes(int n);
hipError_t bdpt_light_sort(uint32_t* keys, uint32_t* keys2, uint32_t* slots, uint32_t* perm, int n, void* tmp,
                           size_t tmpBytes, hipStream_t st, int bits = 13);
void launch_extend_pair(const TraceCtx& cc, const TraceCtx& c, const int* count0, const float4* qO0, const float4* qD0,
                        float4* hit0, const int* count1, const float4* qO1, const float4* qD1, float4* hit1,
                        int maxCount0, int maxCount1, hipStream_t st, const uint32_t* perm1 = nullptr);
void launch_extend(const TraceCtx& c, const int* count, const float4* qO, const float4* qD, float4* hits, int maxCount,
                   hipStream_t st, const uint32_t* perm = nullptr);
void launch_shadow(const TraceCtx& c, const int* count, const float4* sO, const float4* sD, const float4* sL,
                   float4* radiance, int maxCount, hipStream_t st);
void launch_shadow_extend(const TraceCtx& c, const int* extCount, const float4* qO, const float4* qD, float4* hits,
                          const int* shadowCount, const float4* sO, const float4* sD, const float4* sL,
                          float4* radiance, int maxExt, int maxShadow, hipStream_t st);
// the walks k_shadow_extend suspended (c.walkCap > 0): at most maxExt of them
void launch_walk_resume(const TraceCtx& c, const float4* qO, const float4* qD, float4* hits, int maxExt,
                        hipStream_t st);
void launch_shade0(const SceneArgs& s, const FrameArgs& f, const mcrt_camera* cam, const float4* hits,
                   float4* radiance, const QueueArgs& q, hipStream_t st);
void launch_shadeN(const SceneArgs& s, const FrameArgs& f, int bounce, const int* countIn, const float4* qO,
                   const float4* qD, const float4* qT, const float4* hits, float4* radiance, const QueueArgs& q,
                   int maxCount, hipStream_t st);
void launch_aov(const SceneArgs& s, const FrameArgs& f, const mcrt_camera* cam, const float4* hits, int which,
                float4* out, hipStream_t st);
// filters: the reconstruction filter of each batch frame in device memory (KRN/kernel_data.h:63-80), k_accumulate
// evaluates its weight like ReconstructionPass (reconstruction.cl:21-42); filterStride 0 = one filter for all frames
void launch_accumulate(const FrameArgs& f, int frame, const mcrt_filter* filters, int filterStride, const float4* radiance, float4* wsum, float* wts,
                       float4* image, hipStream_t st);
void launch_resolve(uint32_t W, uint32_t H, const float4* wsum, const float* wts, float4* image, hipStream_t st);
void launch_band_pack(const FrameArgs& f, const float4* wsum, const float* wts, float* out, hipStream_t st);
void launch_band_unpack(const FrameArgs& f, int maxRows, const float* recv, float4* wsum, float* wts, float4* image,
                        hipStream_t st);
void launch_denoise(int W, int H, int r, float ss, float sr, const float4* in, float4* out, hipStream_t st);
void launch_tonemap(int n, float Lwhite, const float4* in, float4* out, hipStream_t st);
void launch_stream_copy(const float4* src, float4* dst, size_t n4, int numCUs, hipStream_t st);
// parent index of each triangle leaf into its record's word 13 (flat trees, finish_accel)
void launch_leaf_parents(float4* nodes, uint32_t n, hipStream_t st);
// order[0..n) = tiles by descending cost[tile] (bucketed; one workgroup)
void launch_tile_order(const uint32_t* cost, int n, uint32_t* order, hipStream_t st);
// compact records of a flat DFS tree (after launch_leaf_parents): *qOut (16-B units, caller frees),
// *units its size; hipErrorNotSupported when the tree is not in DFS order (left child = i + 1)
hipError_t build_qnodes(const float4* nodes, uint32_t n, float4** qOut, size_t* units, hipStream_t st);
void launch_chase_init(void* rec, uint32_t n, hipStream_t st);
void launch_chase(const void* rec, uint32_t n, int steps, int waves, uint32_t* sink, hipStream_t st);
// the chase over packed 32-B / 48-B records (mcrt_ctx_gather_chase_compact): best of iters launches
hipError_t chase_compact(uint32_t n, double leafFrac, int steps, int waves, int iters, hipStream_t st, float* bestMs);
void launch_bdpt_start(const SceneArgs& s, const FrameArgs& f, const BdptArgs& b, const mcrt_camera* cam,
                       const BdptQueue& camQ, const BdptQueue& lightQ, hipStream_t st);
void launch_bdpt_vertex(const SceneArgs& s, const FrameArgs& f, const BdptArgs& b, int depth, const BdptQueue& qIn,
                        const float4* hits, const BdptQueue& qOut, int maxCount, hipStream_t st);
void launch_bdpt_connect(const SceneArgs& s, const FrameArgs& f, const BdptArgs& b, const mcrt_camera* cam,
                         const BdptQueue& q, hipStream_t st);
// k_bdpt_vis is a grid-stride launch of at most this many one-wave workgroups (spill columns per wave)
constexpr int BDPT_VIS_MAX_WAVES = 65536;
void launch_bdpt_vis(const TraceCtx& c, const BdptArgs& b, const BdptQueue& q, int maxCount, hipStream_t st);
void launch_bdpt_gather(const FrameArgs& f, const BdptArgs& b, float4* radiance, const float* chunk,
                        size_t chunkPixels, hipStream_t st);
void launch_bdpt_splat_pack(const FrameArgs& f, size_t chunkPixels, const float4* splat, float* out, hipStream_t st);
void launch_bdpt_clear_splat(int n, float4* splat, hipStream_t st);
// sparse splat exchange: per-owner counts of the list (hist[bands], zeroed by the caller), the list
// grouped by owner into dst at off[owner] (cursor[bands] zeroed), received records added to splat
void launch_splat_hist(const BdptArgs& b, int* hist, hipStream_t st);
struct SplatOffsets { int off[64]; };
void launch_splat_group(const BdptArgs& b, SplatOffsets off, int* cursor, float4* dst, hipStream_t st);
void launch_splat_unpack(const float4* recv, int n, float4* splat, hipStream_t st);
}  // namespace mcrt

// Device BVH builder (mcrt_gpubuild.hip): linear BVH in the mcrt_bvh.cpp record format
#include <vector>
namespace mcrt {
hipError_t gpu_build_bvh(const mcrt_shape* dShapes, const std::vector<uint32_t>& shapeFirst, const uint32_t* dIndices,
                         const float4* dPositions, size_t n, hipStream_t st, float4** nodesOut, int* depthOut);
hipError_t launch_build_prims(int n, const mcrt_shape* dShapes, const uint32_t* dShapeFirst, int numShapes,
                              const uint32_t* dIndices, const float4* dPositions, float* tri, int* shapeOf, int* primOf,
                              float4* amin, float4* amax, float4* cen, int* cbounds, hipStream_t st);
// Device SAH build node-identical to the host / RadeonRays Bvh2 build (mcrt_sahbuild.hip); on
// failure *why names the reason (the caller falls back to the host build)
hipError_t gpu_build_sah(const mcrt_shape* dShapes, const std::vector<uint32_t>& shapeFirst, const uint32_t* dIndices,
                         const float4* dPositions, size_t n, float cost, int bins, bool sah, hipStream_t st,
                         float4** nodesOut, int* depthOut, const char** why);
// The running host's _mm_rcp_ps over the mantissa bits it reads (exponent 127), and whether the
// device rule mcrt_sah.h rcp_ps / sa4 reproduces _mm_rcp_ps / _mm_dp_ps here (mcrt_bvh.cpp)
struct HostRcp {
    std::vector<uint32_t> t;
    int bits = 0;
    bool ok = false;
};
const HostRcp& host_rcp_table();
}
// the thread's mcrt_last_error(NULL) text (mcrt_capi.cpp), for entry points without a context
namespace mcrt {
void set_last_error(const std::string& msg);
}
// Host BVH builder (mcrt_bvh.cpp)
namespace mcrt {
struct BvhOut {
    // GPU layout
    std::size_t numNodes = 0;
    std::size_t numTris = 0;
    float* nodes = nullptr;   // 16 floats per node
    float* tris = nullptr;    // unused (leaves live in `nodes`)
    int depth = 0;
};
// world-space triangles (9 floats each), shape id / prim id per triangle
bool build_bvh(const float* tri, const int32_t* shapeOf, const int32_t* primOf, std::size_t n, float cost, int bins,
               bool sah, int threads, BvhOut& out, bool axes3 = false);
void free_bvh(BvhOut& out);
}  // namespace mcrt
// Host two-level (instanced) build (mcrt_bvh2l.cpp)
namespace mcrt {
struct Bvh2lOut {
    std::vector<float> records;   // 16 floats per record
    std::size_t numNodes = 0, topNodes = 0;
    int numMeshes = 0, numInstances = 0;
    int depth = 0;                // deepest top + bottom path (+ the return marker)
    float topBox[6] = {};         // world bounds (lo xyz, hi xyz)
};
// true when two shapes share (startIdx, startVertex, numTriangles): RTScene::attachMesh then
// creates RadeonRays instances and RR switches to its two-level intersector
bool shapes_are_instanced(const mcrt_shape* shapes, std::size_t n);
bool build_bvh2l(const mcrt_shape* shapes, std::size_t nshapes, const uint32_t* indices, const mcrt_float4* positions,
                 const mcrt_mat4* worldToLocal, float cost, int bins, bool sah, int threads, Bvh2lOut& out);
}  // namespace mcrt

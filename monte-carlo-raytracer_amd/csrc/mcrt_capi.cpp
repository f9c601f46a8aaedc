// mcrt_capi.cpp -- host runtime behind include/mcrt_capi.h.
//
// Replaces the reference's OpenCL host plumbing (PlatformManager / KernelManager /
// RTBufferManager, RTScene uploads, RadeonRays IntersectionApi, and the per-pass
// launch + clFinish sequence of RTPrimaryRaysPass / RTPathTracingPass /
// RTReconstructionPass) with: one HIP stream per context, all per-frame work enqueued
// without host synchronisation (queue sizes stay on the device), one memset per frame.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <tuple>
#include <vector>
#include <map>
#include <tuple>
#include <vector>

#include "mcrt_internal.h"

namespace {

thread_local std::string g_lastError;
}  // namespace
namespace mcrt {
void set_last_error(const std::string& msg) { g_lastError = msg; }
}  // namespace mcrt
namespace {

#define MCRT_MAX_BOUNCES 32

enum KernelId {
    K_PRIMARY, K_SHADE0, K_SHADEN, K_SHADOW, K_EXTEND, K_ACCUM, K_TRACE_CLOSEST, K_TRACE_ANY,
    K_BDPT_START, K_BDPT_VERTEX, K_BDPT_CONNECT, K_BDPT_VIS, K_BDPT_GATHER, K_SHADOW_EXTEND, K_COUNT
};
const char* kKernelNames[K_COUNT] = {"k_primary",    "k_shade0",      "k_shadeN",       "k_shadow",   "k_extend",
                                     "k_accumulate", "k_trace_closest", "k_trace_any",  "k_bdpt_start",
                                     "k_bdpt_vertex", "k_bdpt_connect", "k_bdpt_vis",   "k_bdpt_gather",
                                     "k_shadow_extend"};

}  // namespace

struct mcrt_ctx_s {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    int numCUs = 256;
    bool profiling = false;
    bool countHints = false;   // mcrt_ctx_set_profiling(2): occluder-hint counters (one atomic per wave)
    int* dFlags = nullptr;          // device flags: [0] traversal-stack overflow (mcrt_traverse.h), set by any launch
    std::string error;
    struct Pending {
        int kernel;
        hipEvent_t a, b;
        const int* countDev;   // device counter holding the item count (or nullptr)
        const int* countDev2;  // a second counter added to it (fused launches), or nullptr
        int64_t items;
    };
    std::vector<Pending> pending;
    double totalMs[K_COUNT] = {};
    int64_t launches[K_COUNT] = {};
    int64_t items[K_COUNT] = {};
};

struct mcrt_scene_s {
    mcrt_ctx ctx = nullptr;
    // host copies needed for the BVH build and dynamic updates
    std::vector<mcrt_shape> shapes;
    std::vector<uint32_t> indices;
    std::vector<mcrt_float4> positions;
    // device arrays
    void* dShapes = nullptr;
    void* dIndices = nullptr;
    void* dPositions = nullptr;
    void* dUvs = nullptr;
    void* dNormals = nullptr;
    void* dTextures = nullptr;
    void* dTexData = nullptr;
    void* dSobol = nullptr;
    void* dLights = nullptr;
    void* dMaterials = nullptr;
    void* dSurf = nullptr;       // surface records (SceneArgs::surf), 128 B per distinct mesh triangle
    void* dSurfBase = nullptr;   // per shape: its first surface record
    void* dSurfMeshes = nullptr; // build scratch: startIdx | startVertex | base per distinct mesh
    uint32_t numLights = 0, numMaterials = 0, numTextures = 0;
    bool hasSobol = false;
    // BVH
    void* dNodes = nullptr;
    void* dTris = nullptr;
    bool packets = false;      // coherent launches as wave packets (finish_accel)
    uint64_t numNodes = 0;
    uint32_t numTris = 0;
    double buildMs = 0.0;
    int builder = 0;   // which builder made the flat structure: 0 host, 1 device LBVH, 2 device SAH
    int bvhDepth = 0;
    bool twoLevel = false;          // instanced scene: two-level records (mcrt_bvh2l.cpp)
    int numMeshes = 0, numInstances = 0;
    // traversal scratch
    uint32_t* dSpill = nullptr;
    int spillCap = 0;
    size_t spillRays = 0;           // rays the spill buffer covers (spillCap words each)
    int* dScratch = nullptr;   // work counters for API queries
    float bbLo[3] = {0, 0, 0}, bbHi[3] = {0, 0, 0};   // world bounds (root record of the BVH)
    // occluder hints of the shadow rays after bounce 0, by origin cell (TraceCtx::hint, flat trees):
    // allocated on the first shadow launch that uses hints (ensure_hint_cell), 2^hintBits words
    uint32_t* dHintCell = nullptr;
    int hintBits = 0;
    // compact records of the flat tree (TraceCtx::qnodes; mcrt::build_qnodes), NULL when not built
    float4* dQNodes = nullptr;
    size_t qUnits = 0;
    uint32_t qRoot = 0;
    bool hintAllocFailed = false;   // no memory for the table: hints stay off for this scene
};

// One frame in flight (PT): the per-frame buffers of mcrt_render_frame, its own stream and
// spill columns.  Frame i renders in slot i mod S on that slot's stream while mcrt_accumulate
// runs on the context stream in frame order (it waits for the slot's `done` event and records
// `free` after reading the slot's radiance), so S frames overlap on the GPU -- each frame's
// arithmetic and the per-pixel accumulation order are unchanged, so the image is the same bit
// for bit.  Small per-rank frames (tile split over many GPUs) do not fill 256 CUs alone.
struct FrameSlot {
    float4* radiance = nullptr;
    float4* hitsP = nullptr;     // primary hits (mcrt_kernels.hip hitSlot)
    float4* hitsE = nullptr;     // extension hits by queue slot
    float4* eO[2] = {};
    float4* eD[2] = {};
    float4* eT[2] = {};
    float4 *sO = nullptr, *sD = nullptr, *sL = nullptr;
    int* counters = nullptr;     // [0..31] shadow counts, [32..63] ext counts, [64..] work counters, camera @128
    uint32_t* spill = nullptr;   // per-ray traversal spill columns of this slot's launches
    size_t spillWords = 0;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;   // recorded after the slot's last render
    hipEvent_t free = nullptr;   // recorded on the context stream after the slot's buffers were last read
    int lastMaxDepth = 0;
    int64_t lastPixels = 0;
    int lastBatch = 1;           // frames of the slot's last render (mcrt_render_frames)
    int frames = 1;              // radiance / primary-hit planes of W*H allocated (batch capacity)
    size_t queueCap = 0;         // entries of each ray-queue buffer
    // longest-first tile order (FrameArgs::tileOrder): the camera-wave cost of each tile recorded by
    // this slot's last call, and the order made from it; stream-ordered on the slot's stream
    uint32_t* tileCost = nullptr;
    uint32_t* tileOrder = nullptr;
    int costTiles = 0;           // tiles of the recorded costs (0: none)
    int tileCap = 0;
    // suspended extension walks (TraceCtx::walkCap): MCRT_SUSPEND_F4 float4 per queue entry, and
    // one count per bounce (zeroed per call)
    float4* suspend = nullptr;
    size_t suspendCap = 0;
    int* suspendCnt = nullptr;
};
#define SLOT_FILTER_OFFSET (512 + 176 * MCRT_MAX_BATCH_FRAMES)   // the batch's filters (mcrt_accumulate_frames)
#define SLOT_COUNTER_BYTES (SLOT_FILTER_OFFSET + (int)sizeof(mcrt_filter) * MCRT_MAX_BATCH_FRAMES + 1536)

// Per-frame BDPT arrays (RTBDPTPass::createBuffers, RTBDPTPass.cpp:442-479), one set per frame
// slot so BDPT frames overlap like PT frames; layouts in mcrt_bdpt.hip.
struct BdptSet {
    float4 *camV = nullptr, *lightV = nullptr, *slots = nullptr, *splat = nullptr;
    int *camCount = nullptr, *lightCount = nullptr, *bdptCounters = nullptr;
    float4 *bqO[2] = {}, *bqD[2] = {}, *bqT[2] = {}, *bHits = nullptr;
    float4 *cO = nullptr, *cD = nullptr, *cL = nullptr;
    uint32_t* spill = nullptr;   // traversal spill columns of this set's launches
    // the light-start queue's sort (mcrt::bdpt_light_sort): keys, sorted keys, slots, permutation
    uint32_t *lkey = nullptr, *lkey2 = nullptr, *lslot = nullptr, *lperm = nullptr;
    // the traced bounce queues' sort (same routine; k_bdpt_vertex's keys over 2 N slots)
    uint32_t *ekey = nullptr, *ekey2 = nullptr, *eslot = nullptr, *eperm = nullptr;
    void* sortTmp = nullptr;
    size_t sortTmpBytes = 0;
    int frames = 0;              // batch frames the per-frame arrays hold (plane stride N x frames)
    size_t spillWords = 0;
    // plane stride and band (rows, count, index) whose depth-0 frame-invariant planes k_bdpt_start
    // wrote for every path of the band
    size_t constStride = 0;
    int constBand[3] = {0, 0, -1};
    // band split, sparse splat exchange: the splats landing in other ranks' rows (BdptArgs::splatList)
    // and 128 ints of grouping scratch (per-owner counts, cursors)
    float4* splatList = nullptr;
    size_t splatListCap = 0;
    int* splatAux = nullptr;
    // suspended closest-hit walks (TraceCtx::walkCap): MCRT_SUSPEND_F4 float4 per queue entry, one
    // count per traced queue (zeroed per call)
    float4* suspend = nullptr;
    size_t suspendCap = 0;
    int* suspendCnt = nullptr;
};   // [0..127] ints: counters; cameras (176 B each, <= MCRT_MAX_BATCH_FRAMES) from byte 512, then filters

struct mcrt_framebuffer_s {
    mcrt_ctx ctx = nullptr;
    uint32_t W = 0, H = 0;
    size_t N = 0;
    std::vector<FrameSlot> slot;   // slot[0] always allocated; others on first use
    int cur = 0, next = 0;         // slot of the last rendered frame / of the next one
    int framesInFlight = 0;        // 0 = auto (mcrt_framebuffer_set_frames_in_flight)
    // views of slot[cur] (the last rendered frame)
    float4* radiance = nullptr;
    float4* wsum = nullptr;
    float* wts = nullptr;
    float4* image = nullptr;
    float4* denoised = nullptr;  // RTDenoisePass output (persistent: the reference keeps its image)
    float4* display = nullptr;   // post-processed image (mcrt_postprocess)
    uint32_t* hintPix = nullptr; // occluder hint of each pixel's bounce-0 shadow ray (TraceCtx::hint)
    float4* hitsP = nullptr;     // primary hits (mcrt_kernels.hip hitSlot)
    float4* hitsE = nullptr;     // extension hits by queue slot
    float4* eO[2] = {};
    float4* eD[2] = {};
    float4* eT[2] = {};
    float4 *sO = nullptr, *sD = nullptr, *sL = nullptr;
    int* counters = nullptr;
    int lastMaxDepth = 0;
    int64_t lastPixels = 0;
    FrameArgs bands{};      // band layout of the last mcrt_render_frame (used by mcrt_accumulate)
    bool haveBands = false;
    // BDPT state (allocated on the first BDPT frame for a max depth; mcrt_bdpt.hip has the layout):
    // per-frame arrays per frame slot; the sampled-light-vertex planes carry state from frame to
    // frame (BDPT.cl:585), so they are shared and the connect launches stay in frame order
    int bdptDepth = 0;
    BdptSet bset[MCRT_MAX_FRAMES_IN_FLIGHT];
    hipEvent_t bdptConnect = nullptr;   // recorded after the last enqueued frame's connect launch
    // diagnostics (MCRT_WAVE_CLOCK=1): per-workgroup (start, end) clocks of the last PT call's camera,
    // shadow+extension and last shadow launches (mcrt_framebuffer_wave_clock)
    uint32_t* waveClk[3] = {};
    size_t waveClkBlocks[3] = {};
    // views of the set of the last BDPT frame (read-back API)
    float4 *camV = nullptr, *lightV = nullptr, *sampLight = nullptr, *slots = nullptr, *splat = nullptr;
    int *camCount = nullptr, *lightCount = nullptr, *bdptCounters = nullptr;
    float4 *bqO[2] = {}, *bqD[2] = {}, *bqT[2] = {}, *bHits = nullptr;
    float4 *cO = nullptr, *cD = nullptr, *cL = nullptr;   // connection queue
    int lastIntegrator = MCRT_INTEGRATOR_PT;
    int bdptBatch = 1;           // frames of the last BDPT call (plane stride N x bdptBatch)
    bool bdptOneSet = false;     // a second BDPT set did not fit in HBM: BDPT frames use slot 0 only
    bool bdptPendingGather = false;   // band-split BDPT frame waiting for the ranks' summed splats
    int splatExchange = MCRT_SPLAT_EXCHANGE_DENSE;   // mcrt_framebuffer_set_splat_exchange
    int bdptSet = 0;             // the BDPT set of the last BDPT call
};

// BDPT queue counters (64 ints per frame set): [d] the subpath-ray queue of depth d (d <= 33;
// at depth 0 the light rays only), then these
enum { BDPT_CNT_CONN = 40, BDPT_CNT_CAM0 = 41, BDPT_CNT_SPLATS = 42 };
static int bdpt_max_connections(int D) { const int t = D + 2; return t * (t + 1) / 2 - 2; }   // RTBDPTPass.cpp:404-408

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
static mcrt_status fail(mcrt_ctx ctx, mcrt_status code, const std::string& msg) {
    g_lastError = msg;
    if (ctx) ctx->error = msg;
    return code;
}
#define HIPCHK(ctx, expr)                                                                                   \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess)                                                                               \
            return fail(ctx, e_ == hipErrorOutOfMemory ? MCRT_ERROR_OUT_OF_MEMORY : MCRT_ERROR_DEVICE,      \
                        std::string(#expr) + ": " + hipGetErrorString(e_));                                 \
    } while (0)

template <class T>
static hipError_t upload(void** dst, const T* src, size_t count, hipStream_t st) {
    *dst = nullptr;
    if (!src || count == 0) return hipSuccess;
    hipError_t e = hipMalloc(dst, sizeof(T) * count);
    if (e != hipSuccess) return e;
    return hipMemcpyAsync(*dst, src, sizeof(T) * count, hipMemcpyHostToDevice, st);
}

struct Timed {
    mcrt_ctx c;
    int k;
    hipEvent_t a = nullptr, b = nullptr;
    const int* countDev;
    int64_t items;
    hipStream_t st;
    const int* countDev2;
    Timed(mcrt_ctx ctx, int kernel, const int* countDev_, int64_t items_, hipStream_t stream = nullptr,
          const int* countDev2_ = nullptr)
        : c(ctx), k(kernel), countDev(countDev_), items(items_), st(stream ? stream : ctx->stream),
          countDev2(countDev2_) {
        if (c->profiling) {
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a, st);
        }
    }
    ~Timed() {
        if (c->profiling) {
            hipEventRecord(b, st);
            c->pending.push_back({k, a, b, countDev, countDev2, items});
        }
    }
};

static void drain_pending(mcrt_ctx ctx) {
    if (ctx->pending.empty()) return;
    for (auto& p : ctx->pending) {
        hipEventSynchronize(p.b);   // events may sit on frame-slot streams
        float ms = 0.0f;
        hipEventElapsedTime(&ms, p.a, p.b);
        ctx->totalMs[p.kernel] += ms;
        ctx->launches[p.kernel] += 1;
        int64_t it = p.items;
        if (p.countDev) {
            int v = 0, v2 = 0;
            hipMemcpy(&v, p.countDev, sizeof(int), hipMemcpyDeviceToHost);
            if (p.countDev2) hipMemcpy(&v2, p.countDev2, sizeof(int), hipMemcpyDeviceToHost);
            it = (int64_t)v + v2;
        }
        ctx->items[p.kernel] += it;
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    ctx->pending.clear();
}

// RR transform_point (RR/include/math/mathutils.h:111-118) for the BVH's world-space triangles
static inline void xformPoint(const mcrt_mat4& m, const mcrt_float4& p, float* o) {
    const mcrt_float4* r[3] = {&m.m0, &m.m1, &m.m2};
    for (int i = 0; i < 3; ++i) {
        float acc = 0.0f;
        acc += r[i]->x * p.x;
        acc += r[i]->y * p.y;
        acc += r[i]->z * p.z;
        acc += r[i]->w * 0.0f;
        o[i] = acc + r[i]->w;
    }
}

// Per-ray spill columns for `rays` rays (rounded up to whole waves); grown on demand.
static bool ensure_spill(mcrt_scene s, size_t rays) {
    rays = (rays + 63) / 64 * 64;
    if (rays <= s->spillRays && s->dSpill) return true;
    hipStreamSynchronize(s->ctx->stream);   // the old buffer may still be in use
    if (s->dSpill) hipFree(s->dSpill);
    s->dSpill = nullptr;
    s->spillRays = 0;
    if (hipMalloc(&s->dSpill, rays * (size_t)s->spillCap * sizeof(uint32_t)) != hipSuccess) return false;
    s->spillRays = rays;
    return true;
}

static TraceCtx trace_ctx(mcrt_scene s) {
    TraceCtx c = {};
    c.nodes = (const float4*)s->dNodes;
    c.packet = 0;
    c.spill = s->dSpill;
    c.spillCap = s->spillCap;
    c.overflow = s->ctx->dFlags;
    c.twoLevel = s->twoLevel ? 1 : 0;
    c.numNodes = (uint32_t)s->numNodes;
    c.qnodes = s->dQNodes;
    c.qroot = s->qRoot;
    return c;
}

// Occluder hints for a shadow launch (mcrt_traverse.h hintOccludes; flat trees only -- the leaf test
// of a two-level record would need the instance transform): bounce-0 rays by pixel (table `pix`,
// n pixels), later ones by origin cell.  The answers are the walk's with or without them;
// MCRT_SHADOW_HINTS=0 turns them off (A/B, tests).
static bool hints_enabled() {
    const char* e = std::getenv("MCRT_SHADOW_HINTS");
    return !(e && std::atoi(e) == 0);
}
// test hook: MCRT_TEST_HINT_FILL=seed fills a new hint table with pseudo-random words below
// `range` instead of "no hint", so a test can check that arbitrary hints change no answer
static hipError_t fill_hints(uint32_t* d, size_t n, uint32_t range, hipStream_t st) {
    const char* e = std::getenv("MCRT_TEST_HINT_FILL");
    if (!e) return hipMemsetAsync(d, 0xff, 4 * n, st);
    std::vector<uint32_t> h(n);
    uint32_t x = 2463534242u + (uint32_t)std::atoi(e);
    for (auto& v : h) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        v = x % range;
    }
    hipError_t r = hipMemcpyAsync(d, h.data(), 4 * n, hipMemcpyHostToDevice, st);
    if (r == hipSuccess) r = hipStreamSynchronize(st);
    return r;
}
// Entries of the origin-cell table: 2^25 words (128 MB) for trees of more than 2^22 nodes (the
// headline scene: 20 M nodes), fewer for smaller trees (2 words per node, at least 2^18).  Any size
// is safe -- a slot is a hint, never an answer.
static int hint_bits_for(uint32_t numNodes) {
    int b = 18;
    while (b < MCRT_HINT_CELL_BITS && (1u << b) < 2u * numNodes) ++b;
    return b;
}
// The table is allocated (and emptied) on the first launch that uses it, on the context stream,
// which is finished before the launch's own stream reads it; if it does not fit, hints stay off.
static bool ensure_hint_cell(mcrt_scene s) {
    if (s->dHintCell) return true;
    if (s->hintAllocFailed) return false;
    mcrt_ctx ctx = s->ctx;
    const int bits = hint_bits_for((uint32_t)s->numNodes);
    hipError_t e = hipMalloc(&s->dHintCell, sizeof(uint32_t) << bits);
    if (e == hipSuccess) e = fill_hints(s->dHintCell, (size_t)1 << bits, (uint32_t)s->numNodes + 64, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    if (e != hipSuccess) {
        hipGetLastError();
        if (s->dHintCell) hipFree(s->dHintCell);
        s->dHintCell = nullptr;
        s->hintAllocFailed = true;
        return false;
    }
    s->hintBits = bits;
    return true;
}
static void with_hints(TraceCtx& c, mcrt_scene s, uint32_t* pix, uint32_t n) {
    if (s->twoLevel || !hints_enabled() || !ensure_hint_cell(s)) return;
    c.hintCell = s->dHintCell;
    c.hintMask = (1u << s->hintBits) - 1;
    for (int a = 0; a < 3; ++a) {
        const float ext = s->bbHi[a] - s->bbLo[a];
        c.hintLo[a] = s->bbLo[a];
        c.hintInvExt[a] = ext > 0.0f ? 1.0f / ext : 0.0f;
    }
    c.hint = pix ? pix : s->dHintCell;
    c.hintMode = pix ? MCRT_HINT_PIXEL : MCRT_HINT_CELL;
    c.hintPixels = n;
}

// Stop rule of the extension rays' compact walks (TraceCtx::walkCap / walkLanes): a wave stops
// once it has taken MCRT_WALK_CAP steps (0 = never) and MCRT_WALK_LANES of its lanes or fewer are
// still walking (64: a fixed step limit).  Default 60 / 8: k_shadow_extend 0.643 -> 0.603 ms per
// frame on the headline (a fixed 130-step limit 0.609; profiles/r05/ab/README.txt item 20)
static int walk_cap() {
    const char* e = std::getenv("MCRT_WALK_CAP");
    return e ? std::max(0, std::atoi(e)) : 60;
}
// PT: the stop rule for the extension launches of bounces <= MCRT_WALK_MAXB (default 0: the first,
// full-size one).  At depth 5 the later, smaller launches -- whose any-hit shadow blocks otherwise
// overlap the long walks' tail -- lost what the first gained: k_shadow_extend 2.951 ms per frame
// without the rule, 2.943 with it on every launch, 2.915 on the first only (item 20)
// ... and only for calls of at least MCRT_WALK_MIN_PATHS paths (default 16 M): a rank's share of a
// strong-scaled frame (N = 8: 5 M paths per call) finishes the resumed walks in a launch too small
// to hide their tail (emulated N = 8 rank 0.175 -> 0.179 ms per frame with the rule; BDPT 0.649 ->
// 0.659).  The tests set it to 0 to run the rule on small frames.
static int64_t walk_min_paths() {
    const char* e = std::getenv("MCRT_WALK_MIN_PATHS");
    return e ? std::atoll(e) : 16000000;
}
static int walk_max_bounce() {
    const char* e = std::getenv("MCRT_WALK_MAXB");
    return e ? std::atoi(e) : 0;
}
// BDPT: the light-tracing strategies (t = 1) evaluated by the vertex launches that create their
// light vertices instead of by a connection launch that re-reads them (MCRT_BDPT_LIGHT_IN_VERTEX)
static int bdpt_light_in_vertex() {
    const char* e = std::getenv("MCRT_BDPT_LIGHT_IN_VERTEX");
    return e ? (std::atoi(e) != 0) : 1;
}
static int walk_lanes() {
    const char* e = std::getenv("MCRT_WALK_LANES");
    return e ? std::min(64, std::max(0, std::atoi(e))) : 8;
}

// the coherent launches' view (camera rays, bounce-0 shadow rays): wave packets when the tree allows
static TraceCtx packet_ctx(mcrt_scene s) {
    TraceCtx c = trace_ctx(s);
    c.packet = s->packets ? 1 : 0;
    return c;
}

static SceneArgs scene_args(mcrt_scene s) {
    SceneArgs a;
    a.shapes = (const mcrt_shape*)s->dShapes;
    a.indices = (const uint32_t*)s->dIndices;
    a.positions = (const float4*)s->dPositions;
    a.uvs = (const float2*)s->dUvs;
    a.normals = (const float4*)s->dNormals;
    a.textures = (const mcrt_texture_desc*)s->dTextures;
    a.texData = (const uint8_t*)s->dTexData;
    a.sobol = (const uint32_t*)s->dSobol;
    a.lights = (const mcrt_light*)s->dLights;
    a.materials = (const mcrt_material*)s->dMaterials;
    a.nodes = (const float4*)s->dNodes;
    a.surf = (const float4*)s->dSurf;
    a.surfBase = (const uint32_t*)s->dSurfBase;
    a.numLights = (int)s->numLights;
    return a;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
extern "C" {

MCRT_API const char* mcrt_version(void) { return "mcrt-mi355x 0.1 (gfx950, HIP)"; }

MCRT_API const char* mcrt_last_error(mcrt_ctx ctx) { return ctx ? ctx->error.c_str() : g_lastError.c_str(); }

MCRT_API mcrt_status mcrt_ctx_create(int device, mcrt_ctx* out) {
    if (!out) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "out is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(nullptr, MCRT_ERROR_NO_DEVICE, "no HIP device");
    if (device < 0 || device >= n) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "device index out of range");
    auto* c = new mcrt_ctx_s();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess) { delete c; return fail(nullptr, MCRT_ERROR_DEVICE, "hipSetDevice failed"); }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess) c->numCUs = prop.multiProcessorCount;
    if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return fail(nullptr, MCRT_ERROR_DEVICE, "hipStreamCreate failed");
    }
    c->stream = c->own;
    if (hipMalloc(&c->dFlags, 64 * sizeof(int)) != hipSuccess || hipMemset(c->dFlags, 0, 64 * sizeof(int)) != hipSuccess) {
        hipStreamDestroy(c->own);
        delete c;
        return fail(nullptr, MCRT_ERROR_OUT_OF_MEMORY, "device flags");
    }
    *out = c;
    return MCRT_OK;
}

// Device-side error flags raised by kernels since the last check (call after a synchronisation):
// a traversal whose stack needed more entries than its spill column holds drops entries
// (mcrt_traverse.h), so its hits may be wrong -- reported, never silent.
static mcrt_status check_device_flags(mcrt_ctx ctx) {
    int f = 0;
    HIPCHK(ctx, hipMemcpy(&f, ctx->dFlags, sizeof(int), hipMemcpyDeviceToHost));
    if (f != 0) {
        HIPCHK(ctx, hipMemset(ctx->dFlags, 0, sizeof(int)));
        return fail(ctx, MCRT_ERROR_DEVICE,
                    "traversal stack overflow: a ray needed more stack entries than its spill column holds "
                    "(results of the affected launches are unreliable)");
    }
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_destroy(mcrt_ctx ctx) {
    if (!ctx) return MCRT_OK;
    hipSetDevice(ctx->device);
    drain_pending(ctx);
    hipStreamSynchronize(ctx->stream);
    hipStreamDestroy(ctx->own);
    if (ctx->dFlags) hipFree(ctx->dFlags);
    delete ctx;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_synchronize(mcrt_ctx ctx) {
    if (!ctx) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "ctx is NULL");
    hipSetDevice(ctx->device);
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHK(ctx, hipDeviceSynchronize());   // frame-slot streams of the context's frame buffers
    return check_device_flags(ctx);
}

MCRT_API mcrt_status mcrt_ctx_set_stream(mcrt_ctx ctx, void* stream) {
    if (!ctx) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "ctx is NULL");
    ctx->stream = stream ? (hipStream_t)stream : ctx->own;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_get_stream(mcrt_ctx ctx, void** stream) {
    if (!ctx || !stream) return fail(ctx, MCRT_ERROR_INVALID_ARG, "NULL argument");
    *stream = (void*)ctx->stream;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_set_profiling(mcrt_ctx ctx, int enable) {
    if (!ctx) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "ctx is NULL");
    ctx->profiling = enable != 0;
    ctx->countHints = enable >= 2;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_kernel_stats(mcrt_ctx ctx, int max, const char** names, double* total_ms,
                                           int64_t* launches, int64_t* items, int* count) {
    if (!ctx) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "ctx is NULL");
    hipSetDevice(ctx->device);
    drain_pending(ctx);
    int k = 0;
    for (int i = 0; i < K_COUNT && k < max; ++i) {
        if (ctx->launches[i] == 0) continue;
        if (names) names[k] = kKernelNames[i];
        if (total_ms) total_ms[k] = ctx->totalMs[i];
        if (launches) launches[k] = ctx->launches[i];
        if (items) items[k] = ctx->items[i];
        ++k;
    }
    if (count) *count = k;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_stream_copy(mcrt_ctx ctx, uint64_t bytes, int iters, double* gbps) {
    if (!ctx || !gbps || bytes < 4096 || iters < 1) return fail(ctx, MCRT_ERROR_INVALID_ARG, "bad stream-copy args");
    hipSetDevice(ctx->device);
    const size_t n4 = (size_t)(bytes / 2 / 16);   // half the bytes read, half written
    float4 *a = nullptr, *b = nullptr;
    HIPCHK(ctx, hipMalloc(&a, n4 * 16));
    if (hipMalloc(&b, n4 * 16) != hipSuccess) { hipFree(a); return fail(ctx, MCRT_ERROR_OUT_OF_MEMORY, "stream copy"); }
    hipMemsetAsync(a, 0, n4 * 16, ctx->stream);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int i = 0; i < iters + 1; ++i) {
        hipEventRecord(e0, ctx->stream);
        mcrt::launch_stream_copy(a, b, n4, ctx->numCUs, ctx->stream);
        hipEventRecord(e1, ctx->stream);
        hipEventSynchronize(e1);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        if (i > 0 && ms < best) best = ms;   // launch 0 warms up
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipFree(a);
    hipFree(b);
    HIPCHK(ctx, hipGetLastError());
    *gbps = (double)(2 * n4 * 16) / (best * 1e-3) / 1e9;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_gather_chase(mcrt_ctx ctx, uint64_t records, int steps, int iters, double* gsteps) {
    if (!ctx || !gsteps || records < 64 || records > 0xffffffffull || steps < 1 || iters < 1)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "bad gather-chase args");
    hipSetDevice(ctx->device);
    void* rec = nullptr;
    uint32_t* sink = nullptr;
    HIPCHK(ctx, hipMalloc(&rec, 64 * records));
    if (hipMalloc(&sink, 4) != hipSuccess) { hipFree(rec); return fail(ctx, MCRT_ERROR_OUT_OF_MEMORY, "gather chase"); }
    mcrt::launch_chase_init(rec, (uint32_t)records, ctx->stream);
    const int waves = ctx->numCUs * 32;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    for (int i = 0; i < iters + 1; ++i) {
        hipEventRecord(e0, ctx->stream);
        mcrt::launch_chase(rec, (uint32_t)records, i == 0 ? std::max(1, steps / 4) : steps, waves, sink, ctx->stream);
        hipEventRecord(e1, ctx->stream);
        hipEventSynchronize(e1);
        float ms = 0.0f;
        hipEventElapsedTime(&ms, e0, e1);
        if (i > 0 && ms < best) best = ms;   // launch 0 warms caches and translations
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipFree(rec);
    hipFree(sink);
    HIPCHK(ctx, hipGetLastError());
    *gsteps = (double)waves * 64.0 * steps / (best * 1e-3) / 1e9;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_gather_chase_compact(mcrt_ctx ctx, uint64_t records, double leaf_frac, int steps,
                                                   int iters, double* gsteps) {
    if (!ctx || !gsteps || records < 64 || records > 0x3fffffffull || steps < 1 || iters < 1 || !(leaf_frac >= 0.0) ||
        leaf_frac > 1.0)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "bad gather-chase args");
    hipSetDevice(ctx->device);
    const int waves = ctx->numCUs * 32;
    float best = 0.0f;
    HIPCHK(ctx, mcrt::chase_compact((uint32_t)records, leaf_frac, steps, waves, iters, ctx->stream, &best));
    *gsteps = (double)waves * 64.0 * steps / (best * 1e-3) / 1e9;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_ctx_reset_stats(mcrt_ctx ctx) {
    if (!ctx) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "ctx is NULL");
    drain_pending(ctx);
    for (int i = 0; i < K_COUNT; ++i) { ctx->totalMs[i] = 0.0; ctx->launches[i] = 0; ctx->items[i] = 0; }
    return MCRT_OK;
}

// ---------------------------------------------------------------------------
// scene
// ---------------------------------------------------------------------------
static void scene_free_device(mcrt_scene s) {
    void** ptrs[] = {&s->dShapes, &s->dIndices, &s->dPositions, &s->dUvs, &s->dNormals, &s->dTextures,
                     &s->dTexData, &s->dSobol, &s->dLights, &s->dMaterials, &s->dNodes, &s->dTris,
                     &s->dSurf, &s->dSurfBase, &s->dSurfMeshes};
    for (void** p : ptrs) {
        if (*p) hipFree(*p);
        *p = nullptr;
    }
    if (s->dSpill) hipFree(s->dSpill);
    if (s->dScratch) hipFree(s->dScratch);
    if (s->dHintCell) hipFree(s->dHintCell);
    s->dHintCell = nullptr;
    if (s->dQNodes) hipFree(s->dQNodes);
    s->dQNodes = nullptr;
    s->qUnits = 0;
    s->dSpill = nullptr;
    s->spillRays = 0;
    s->dScratch = nullptr;
}

// Surface records (SceneArgs::surf): shapes with the same (startIdx, startVertex, numTriangles)
// -- RTScene's instances of one mesh -- share one record range; the records are gathered on the
// device from the uploaded index/vertex arrays.  Rebuilt when shapes change.
static hipError_t build_surface_records(mcrt_scene s) {
    hipStream_t st = s->ctx->stream;
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, uint32_t> meshOf;
    std::vector<uint32_t> mStart, mVert, mBase, shapeBase(s->shapes.size());
    uint32_t total = 0;
    for (size_t i = 0; i < s->shapes.size(); ++i) {
        const mcrt_shape& sh = s->shapes[i];
        auto key = std::make_tuple((uint32_t)sh.startIdx, (uint32_t)sh.startVertex, (uint32_t)sh.numTriangles);
        auto it = meshOf.find(key);
        if (it == meshOf.end()) {
            it = meshOf.emplace(key, total).first;
            if (sh.numTriangles > 0) {
                mStart.push_back(sh.startIdx);
                mVert.push_back(sh.startVertex);
                mBase.push_back(total);
            }
            total += sh.numTriangles;
        }
        shapeBase[i] = it->second;
    }
    hipError_t e = hipStreamSynchronize(st);   // the old records may still be read
    void** old[] = {&s->dSurf, &s->dSurfBase, &s->dSurfMeshes};
    for (void** p : old) {
        if (*p) hipFree(*p);
        *p = nullptr;
    }
    const int nm = (int)mBase.size();
    std::vector<uint32_t> meshes(3 * (size_t)std::max(nm, 1));
    std::copy(mStart.begin(), mStart.end(), meshes.begin());
    std::copy(mVert.begin(), mVert.end(), meshes.begin() + nm);
    std::copy(mBase.begin(), mBase.end(), meshes.begin() + 2 * nm);
    if (e == hipSuccess) e = hipMalloc(&s->dSurf, (size_t)std::max(total, 1u) * 128);
    if (e == hipSuccess) e = upload(&s->dSurfBase, shapeBase.data(), shapeBase.size(), st);
    if (e == hipSuccess) e = upload(&s->dSurfMeshes, meshes.data(), meshes.size(), st);
    if (e == hipSuccess && nm > 0) {
        const uint32_t* m = (const uint32_t*)s->dSurfMeshes;
        mcrt::launch_surface_records(m, m + nm, m + 2 * nm, nm, total, (const uint32_t*)s->dIndices,
                                     (const float4*)s->dPositions, (const float2*)s->dUvs, (const float4*)s->dNormals,
                                     (float4*)s->dSurf, st);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    return e;
}

MCRT_API mcrt_status mcrt_scene_create(mcrt_ctx ctx, const mcrt_scene_desc* d, mcrt_scene* out) {
    if (!ctx || !d || !out) return fail(ctx, MCRT_ERROR_INVALID_ARG, "NULL argument");
    if (d->num_shapes == 0 || !d->shapes) return fail(ctx, MCRT_ERROR_INVALID_ARG, "scene has no shapes");
    if (!d->indices || !d->positions || !d->uvs || !d->normals)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "indices/positions/uvs/normals are required");
    for (uint32_t i = 0; i < d->num_shapes; ++i) {
        const mcrt_shape& s = d->shapes[i];
        if ((uint64_t)s.startIdx + 3ull * s.numTriangles > d->num_indices)
            return fail(ctx, MCRT_ERROR_INVALID_ARG, "shape " + std::to_string(i) + " indexes past the index array");
        if (s.materialId >= (int)d->num_materials)
            return fail(ctx, MCRT_ERROR_INVALID_ARG, "shape " + std::to_string(i) + " has an invalid material id");
        if (s.lightID >= (int)d->num_lights) return fail(ctx, MCRT_ERROR_INVALID_ARG, "invalid light id");
    }
    for (uint32_t i = 0; i < d->num_shapes; ++i) {
        const mcrt_shape& s = d->shapes[i];
        for (uint32_t k = 0; k < 3u * s.numTriangles; ++k)
            if ((uint64_t)s.startVertex + d->indices[s.startIdx + k] >= d->num_vertices)
                return fail(ctx, MCRT_ERROR_INVALID_ARG, "vertex index out of range in shape " + std::to_string(i));
    }
    for (uint32_t i = 0; i < d->num_lights; ++i) {
        const mcrt_light& L = d->lights[i];
        if (L.type == MCRT_TRIANGLE_MESH_AREA_LIGHT && (L.shapeId < 0 || L.shapeId >= (int)d->num_shapes ||
                                                        d->shapes[L.shapeId].numTriangles == 0))
            return fail(ctx, MCRT_ERROR_INVALID_ARG, "mesh light " + std::to_string(i) + " has an invalid shape");
    }
    for (uint32_t i = 0; i < d->num_textures; ++i) {
        const mcrt_texture_desc& t = d->textures[i];
        if (t.width == 0 || t.height == 0 || (uint64_t)t.memOffset + 4ull * t.width * t.height > d->tex_data_bytes)
            return fail(ctx, MCRT_ERROR_INVALID_ARG, "texture " + std::to_string(i) + " is out of the texel buffer");
    }
    hipSetDevice(ctx->device);
    auto* s = new mcrt_scene_s();
    s->ctx = ctx;
    s->shapes.assign(d->shapes, d->shapes + d->num_shapes);
    s->indices.assign(d->indices, d->indices + d->num_indices);
    s->positions.assign(d->positions, d->positions + d->num_vertices);
    hipStream_t st = ctx->stream;
    hipError_t e = hipSuccess;
#define UP(dst, src, cnt) if (e == hipSuccess) e = upload(&s->dst, src, cnt, st)
    UP(dShapes, d->shapes, d->num_shapes);
    UP(dIndices, d->indices, d->num_indices);
    UP(dPositions, d->positions, d->num_vertices);
    UP(dUvs, d->uvs, d->num_vertices);
    UP(dNormals, d->normals, d->num_vertices);
    UP(dTextures, d->textures, d->num_textures);
    UP(dTexData, d->tex_data, d->tex_data_bytes);
    UP(dSobol, d->sobol_matrices, d->num_sobol_words);
    UP(dLights, d->lights, d->num_lights);
    UP(dMaterials, d->materials, d->num_materials);
#undef UP
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = build_surface_records(s);
    if (e != hipSuccess) {
        scene_free_device(s);
        delete s;
        return fail(ctx, e == hipErrorOutOfMemory ? MCRT_ERROR_OUT_OF_MEMORY : MCRT_ERROR_DEVICE,
                    std::string("scene upload: ") + hipGetErrorString(e));
    }
    s->numLights = d->num_lights;
    s->numMaterials = d->num_materials;
    s->numTextures = d->num_textures;
    s->hasSobol = d->sobol_matrices != nullptr && d->num_sobol_words >= 1024u * 52u;
    *out = s;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_scene_destroy(mcrt_scene s) {
    if (!s) return MCRT_OK;
    hipSetDevice(s->ctx->device);
    hipStreamSynchronize(s->ctx->stream);
    scene_free_device(s);
    delete s;
    return MCRT_OK;
}

static mcrt_status replace_array(mcrt_scene s, void** dst, const void* src, size_t bytes) {
    mcrt_ctx ctx = s->ctx;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (*dst) HIPCHK(ctx, hipFree(*dst));
    *dst = nullptr;
    if (bytes) {
        HIPCHK(ctx, hipMalloc(dst, bytes));
        HIPCHK(ctx, hipMemcpy(*dst, src, bytes, hipMemcpyHostToDevice));
    }
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_scene_update_lights(mcrt_scene s, const mcrt_light* lights, uint32_t n) {
    if (!s || (n && !lights)) return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "invalid lights");
    mcrt_status st = replace_array(s, &s->dLights, lights, sizeof(mcrt_light) * n);
    if (st == MCRT_OK) s->numLights = n;
    return st;
}

MCRT_API mcrt_status mcrt_scene_update_materials(mcrt_scene s, const mcrt_material* m, uint32_t n) {
    if (!s || (n && !m)) return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "invalid materials");
    mcrt_status st = replace_array(s, &s->dMaterials, m, sizeof(mcrt_material) * n);
    if (st == MCRT_OK) s->numMaterials = n;
    return st;
}

MCRT_API mcrt_status mcrt_scene_update_shapes(mcrt_scene s, const mcrt_shape* sh, uint32_t n) {
    if (!s || !sh || n != s->shapes.size())
        return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "shape count must not change");
    for (uint32_t i = 0; i < n; ++i)
        if (sh[i].startIdx != s->shapes[i].startIdx || sh[i].numTriangles != s->shapes[i].numTriangles)
            return fail(s->ctx, MCRT_ERROR_INVALID_ARG, "shape topology must not change");
    s->shapes.assign(sh, sh + n);
    mcrt_status st = replace_array(s, &s->dShapes, sh, sizeof(mcrt_shape) * n);
    if (st != MCRT_OK) return st;
    HIPCHK(s->ctx, build_surface_records(s));   // startVertex may have moved
    return MCRT_OK;
}

static mcrt_status finish_accel(mcrt_scene s, std::chrono::steady_clock::time_point t0, const float* box6);

MCRT_API mcrt_status mcrt_accel_build(mcrt_scene s, const mcrt_accel_opts* opts) {
    if (!s) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "scene is NULL");
    mcrt_ctx ctx = s->ctx;
    const float cost = opts ? opts->traversal_cost : 10.0f;
    const int bins = opts ? opts->num_bins : 64;
    const bool sah = opts ? opts->use_sah != 0 : true;
    if (bins < 2 || bins > 4096) return fail(ctx, MCRT_ERROR_INVALID_ARG, "num_bins out of range");
    auto t0 = std::chrono::steady_clock::now();
    size_t n = 0;
    for (auto& sh : s->shapes) n += sh.numTriangles;
    if (n == 0) return fail(ctx, MCRT_ERROR_INVALID_ARG, "scene has no triangles (RR: Commit on empty scene throws)");
    if (n > (size_t)0x7fffffff) return fail(ctx, MCRT_ERROR_INVALID_ARG, "too many triangles");
    // IntersectorTwoLevel when forced or when a mesh is shared, unless flat is forced
    // (CalcIntersectionDevice::Preprocess, RR/src/device/calc_intersection_device.cpp:68-105)
    const bool use2 = (opts && opts->force_2level) ||
                      (!(opts && opts->force_flat) && mcrt::shapes_are_instanced(s->shapes.data(), s->shapes.size()));
    if (use2) {
        int threads = (int)std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
        mcrt::Bvh2lOut b2;
        if (!mcrt::build_bvh2l(s->shapes.data(), s->shapes.size(), s->indices.data(), s->positions.data(),
                               opts ? opts->world_to_local : nullptr, cost, bins, sah, threads, b2))
            return fail(ctx, MCRT_ERROR_INVALID_ARG, "two-level BVH build failed");
        hipSetDevice(ctx->device);
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        if (s->dNodes) hipFree(s->dNodes);
        if (s->dTris) hipFree(s->dTris);
        s->dNodes = s->dTris = nullptr;
        hipError_t e = hipMalloc(&s->dNodes, 64 * b2.numNodes);
        if (e == hipSuccess) e = hipMemcpy(s->dNodes, b2.records.data(), 64 * b2.numNodes, hipMemcpyHostToDevice);
        if (e != hipSuccess) return fail(ctx, MCRT_ERROR_OUT_OF_MEMORY, std::string("BVH upload: ") + hipGetErrorString(e));
        s->numNodes = b2.numNodes;
        s->numTris = (uint32_t)n;
        s->bvhDepth = b2.depth;
        s->twoLevel = true;
        s->numMeshes = b2.numMeshes;
        s->numInstances = b2.numInstances;
        return finish_accel(s, t0, b2.topBox);
    }
    s->twoLevel = false;
    s->numMeshes = s->numInstances = 0;
    const int buildMode = opts ? opts->device_build : 0;
    if (buildMode == 0 || buildMode == 2) {   // on-device SAH, node-identical to the host build
        hipSetDevice(ctx->device);
        std::vector<uint32_t> first(s->shapes.size());
        uint32_t acc = 0;
        for (size_t si = 0; si < s->shapes.size(); ++si) { first[si] = acc; acc += s->shapes[si].numTriangles; }
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        float4* nodes = nullptr;
        int depth = 0;
        const char* why = nullptr;
        const hipError_t e = mcrt::gpu_build_sah((const mcrt_shape*)s->dShapes, first, (const uint32_t*)s->dIndices,
                                                 (const float4*)s->dPositions, n, cost, bins, sah, ctx->stream, &nodes,
                                                 &depth, &why);
        if (e == hipSuccess) {
            if (s->dNodes) hipFree(s->dNodes);
            if (s->dTris) hipFree(s->dTris);
            s->dTris = nullptr;
            s->dNodes = nodes;
            s->numNodes = 2 * n - 1;
            s->numTris = (uint32_t)n;
            s->bvhDepth = depth;
            s->builder = 2;
            return finish_accel(s, t0, nullptr);
        }
        // configurations the device path does not reproduce (> 64 bins, a host whose rcpps the
        // table cannot model, pathological level counts) take the host build: same tree; so does a
        // device without room for the build's scratch (~230 B per triangle beyond the records)
        if (e != hipErrorNotSupported && e != hipErrorInvalidValue && e != hipErrorOutOfMemory)
            return fail(ctx, MCRT_ERROR_DEVICE, std::string("device SAH build: ") + (why ? why : hipGetErrorString(e)));
        (void)hipGetLastError();
        if (e == hipErrorOutOfMemory)
            std::fprintf(stderr, "mcrt: device SAH build out of memory, building the same tree on the host\n");
    }
    s->builder = 0;
    if (buildMode == 1) {   // on-device linear BVH (mcrt_gpubuild.hip)
        hipSetDevice(ctx->device);
        std::vector<uint32_t> first(s->shapes.size());
        uint32_t acc = 0;
        for (size_t si = 0; si < s->shapes.size(); ++si) { first[si] = acc; acc += s->shapes[si].numTriangles; }
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        float4* nodes = nullptr;
        int depth = 0;
        HIPCHK(ctx, mcrt::gpu_build_bvh((const mcrt_shape*)s->dShapes, first, (const uint32_t*)s->dIndices,
                                        (const float4*)s->dPositions, n, ctx->stream, &nodes, &depth));
        if (s->dNodes) hipFree(s->dNodes);
        if (s->dTris) hipFree(s->dTris);
        s->dTris = nullptr;
        s->dNodes = nodes;
        s->numNodes = 2 * n - 1;
        s->numTris = (uint32_t)n;
        s->bvhDepth = depth;
        s->builder = 1;
        return finish_accel(s, t0, nullptr);
    }
    std::vector<float> tri(9 * n);
    std::vector<int32_t> shapeOf(n), primOf(n);
    size_t k = 0;
    for (size_t si = 0; si < s->shapes.size(); ++si) {
        const mcrt_shape& sh = s->shapes[si];
        for (uint32_t f = 0; f < sh.numTriangles; ++f, ++k) {
            for (int c = 0; c < 3; ++c)
                xformPoint(sh.toWorldTransform, s->positions[sh.startVertex + s->indices[sh.startIdx + 3 * f + c]],
                           &tri[9 * k + 3 * c]);
            shapeOf[k] = (int32_t)si;
            primOf[k] = (int32_t)f;
        }
    }
    int threads = (int)std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
    mcrt::BvhOut bvh;
    if (!mcrt::build_bvh(tri.data(), shapeOf.data(), primOf.data(), n, cost, bins, sah, threads, bvh, buildMode == 4))
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "BVH build failed");
    if (buildMode == 4) s->builder = 4;   // the perf tree (3-axis SAH), not the reference's
    hipSetDevice(ctx->device);
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    if (s->dNodes) hipFree(s->dNodes);
    if (s->dTris) hipFree(s->dTris);
    s->dNodes = s->dTris = nullptr;
    hipError_t e = hipMalloc(&s->dNodes, 64 * bvh.numNodes);
    if (e == hipSuccess) e = hipMemcpy(s->dNodes, bvh.nodes, 64 * bvh.numNodes, hipMemcpyHostToDevice);
    s->numNodes = bvh.numNodes;
    s->numTris = (uint32_t)bvh.numTris;
    s->bvhDepth = bvh.depth;
    mcrt::free_bvh(bvh);
    if (e != hipSuccess) return fail(ctx, MCRT_ERROR_OUT_OF_MEMORY, std::string("BVH upload: ") + hipGetErrorString(e));
    return finish_accel(s, t0, nullptr);
}

// traversal scratch: overflow flag; per-ray spill columns deep enough for the tree
// (allocated by ensure_spill for the largest launch)
static mcrt_status finish_accel(mcrt_scene s, std::chrono::steady_clock::time_point t0, const float* box6) {
    mcrt_ctx ctx = s->ctx;
    // wave packets for the coherent launches (mcrt_traverse.h traversePacket): flat trees whose
    // depth fits the packet stack (at most 2 entries per internal level: 2 x depth, the leaves'
    // level).  MCRT_CAMERA_PACKETS=0 walks them per ray (A/B and tests: the results are the same bit
    // for bit).
    const char* pe = std::getenv("MCRT_CAMERA_PACKETS");
    s->packets = !s->twoLevel && 2 * s->bvhDepth <= MCRT_PK_STACK && s->numNodes < (1u << 26) &&   // 32-bit offsets
                 !(pe && std::atoi(pe) == 0);
    if (!s->dScratch) HIPCHK(ctx, hipMalloc(&s->dScratch, 256 * sizeof(int)));
    HIPCHK(ctx, hipMemset(s->dScratch, 0, 256 * sizeof(int)));
    if (!s->twoLevel) {
        // parent links of the leaves (occluder hints).  The origin-cell hint table is allocated on
        // its first use (ensure_hint_cell, sized for the tree); a rebuild drops the old one
        mcrt::launch_leaf_parents((float4*)s->dNodes, (uint32_t)s->numNodes, ctx->stream);
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        if (s->dHintCell) hipFree(s->dHintCell);
        s->dHintCell = nullptr;
        s->hintAllocFailed = false;
    }
    // compact records for the per-ray walks (mcrt_traverse.h traverseQOct): depth-first flat trees;
    // MCRT_QUANT_NODES=0 keeps the 64-B records everywhere (A/B, tests).  A tree the converter
    // cannot take (LBVH numbering) or a device without room for it (~0.8 GB at 10 M triangles)
    // keeps the 64-B walk: the same answers.
    if (s->dQNodes) hipFree(s->dQNodes);
    s->dQNodes = nullptr;
    s->qUnits = 0;
    const char* qe = std::getenv("MCRT_QUANT_NODES");
    if (!s->twoLevel && !(qe && std::atoi(qe) == 0)) {
        float4* q = nullptr;
        size_t units = 0;
        const hipError_t e = mcrt::build_qnodes((const float4*)s->dNodes, (uint32_t)s->numNodes, &q, &units, ctx->stream);
        if (e == hipSuccess) {
            s->dQNodes = q;
            s->qUnits = units;
        } else if (e != hipErrorNotSupported && e != hipErrorOutOfMemory) {
            return fail(ctx, MCRT_ERROR_DEVICE, std::string("compact records: ") + hipGetErrorString(e));
        } else {
            (void)hipGetLastError();
        }
    }
    int needCap = ((s->bvhDepth + 2 + 15) / 16) * 16;   // whole spill blocks of STACK_LDS entries
    // test hook: MCRT_TEST_SPILL_CAP=k caps the spill columns at k entries (0 = LDS stack only) so a
    // test can drive a traversal past its capacity and check that the overflow is reported
    if (const char* tc = std::getenv("MCRT_TEST_SPILL_CAP")) needCap = std::max(0, std::atoi(tc) / 16 * 16);
    if (needCap != s->spillCap) {
        if (s->dSpill) hipFree(s->dSpill);
        s->dSpill = nullptr;
        s->spillRays = 0;
        s->spillCap = needCap;
    }
    if (box6) {
        for (int a = 0; a < 3; ++a) { s->bbLo[a] = box6[a]; s->bbHi[a] = box6[3 + a]; }
        s->buildMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        return MCRT_OK;
    }
    // world bounds = the root record's two child boxes (or its triangle)
    float r[16];
    HIPCHK(ctx, hipMemcpy(r, s->dNodes, 64, hipMemcpyDeviceToHost));
    int32_t mark;
    std::memcpy(&mark, &r[12], 4);
    s->qRoot = mark >= 0 ? 0u : 1u;   // compact reference of the root: offset 0, leaf bit
    if (mark >= 0) {
        const float lo[3] = {std::min(r[0], r[4]), std::min(r[2], r[6]), std::min(r[8], r[10])};
        const float hi[3] = {std::max(r[1], r[5]), std::max(r[3], r[7]), std::max(r[9], r[11])};
        for (int a = 0; a < 3; ++a) { s->bbLo[a] = lo[a]; s->bbHi[a] = hi[a]; }
    } else {
        for (int a = 0; a < 3; ++a) {
            const float v0 = r[a], v1 = r[a] + r[4 + a], v2 = r[a] + r[8 + a];
            s->bbLo[a] = std::min(v0, std::min(v1, v2));
            s->bbHi[a] = std::max(v0, std::max(v1, v2));
        }
    }
    s->buildMs = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_accel_info(mcrt_scene s, uint64_t* num_nodes, uint64_t* device_bytes, double* build_ms,
                                     uint32_t* num_triangles) {
    if (!s) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "scene is NULL");
    if (num_nodes) *num_nodes = s->numNodes;
    if (device_bytes) *device_bytes = 64ull * s->numNodes + 16ull * s->qUnits;
    if (build_ms) *build_ms = s->buildMs;
    if (num_triangles) *num_triangles = s->numTris;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_accel_layout(mcrt_scene s, int32_t* two_level, uint32_t* num_meshes,
                                       uint32_t* num_instances, int32_t* depth) {
    if (!s) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "scene is NULL");
    if (!s->dNodes) return fail(s->ctx, MCRT_ERROR_NOT_READY, "mcrt_accel_build has not been called");
    if (two_level) *two_level = s->twoLevel ? 1 : 0;
    if (num_meshes) *num_meshes = (uint32_t)s->numMeshes;
    if (num_instances) *num_instances = (uint32_t)s->numInstances;
    if (depth) *depth = s->bvhDepth;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_accel_read_records(mcrt_scene s, float* out, uint64_t max_records, uint64_t* num_records) {
    if (!s || !num_records) return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    if (!s->dNodes) return fail(s->ctx, MCRT_ERROR_INVALID_ARG, "scene has no acceleration structure");
    *num_records = s->numNodes;
    if (!out) return MCRT_OK;
    mcrt_ctx ctx = s->ctx;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    HIPCHK(ctx, hipMemcpy(out, s->dNodes, 64 * std::min<uint64_t>(max_records, s->numNodes), hipMemcpyDeviceToHost));
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_accel_builder(mcrt_scene s, int32_t* builder) {
    if (!s || !builder) return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    *builder = s->twoLevel ? 0 : s->builder;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_accel_build_host_records(const mcrt_scene_desc* d, const mcrt_accel_opts* opts,
                                                   float* out_records, uint64_t max_records, uint64_t* num_records,
                                                   int32_t* info) {
    if (!d || !d->shapes || !d->indices || !d->positions || !num_records)
        return fail(nullptr, MCRT_ERROR_INVALID_ARG, "invalid arguments");
    const float cost = opts ? opts->traversal_cost : 10.0f;
    const int bins = opts ? opts->num_bins : 64;
    const bool sah = opts ? opts->use_sah != 0 : true;
    if (bins < 2 || bins > 4096) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "num_bins out of range");
    for (uint32_t i = 0; i < d->num_shapes; ++i) {
        const mcrt_shape& sh = d->shapes[i];
        if ((uint64_t)sh.startIdx + 3ull * sh.numTriangles > d->num_indices)
            return fail(nullptr, MCRT_ERROR_INVALID_ARG, "shape indices out of range");
        for (uint64_t k = 0; k < 3ull * sh.numTriangles; ++k)
            if ((uint64_t)sh.startVertex + d->indices[sh.startIdx + k] >= d->num_vertices)
                return fail(nullptr, MCRT_ERROR_INVALID_ARG, "vertex index out of range");
    }
    const int threads = (int)std::max(1u, std::min(64u, std::thread::hardware_concurrency()));
    const bool use2 = (opts && opts->force_2level) ||
                      (!(opts && opts->force_flat) && mcrt::shapes_are_instanced(d->shapes, d->num_shapes));
    int32_t inf[4] = {use2 ? 1 : 0, 0, 0, 0};
    if (use2) {
        mcrt::Bvh2lOut b2;
        if (!mcrt::build_bvh2l(d->shapes, d->num_shapes, d->indices, d->positions, opts ? opts->world_to_local : nullptr,
                               cost, bins, sah, threads, b2))
            return fail(nullptr, MCRT_ERROR_INVALID_ARG, "two-level BVH build failed");
        *num_records = b2.numNodes;
        if (out_records) std::memcpy(out_records, b2.records.data(), 64 * std::min<uint64_t>(max_records, b2.numNodes));
        inf[1] = (int32_t)b2.topNodes;
        inf[2] = b2.depth;
        inf[3] = b2.numMeshes;
    } else {
        size_t n = 0;
        for (uint32_t i = 0; i < d->num_shapes; ++i) n += d->shapes[i].numTriangles;
        if (n == 0) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "scene has no triangles");
        std::vector<float> tri(9 * n);
        std::vector<int32_t> shapeOf(n), primOf(n);
        size_t k = 0;
        for (uint32_t si = 0; si < d->num_shapes; ++si) {
            const mcrt_shape& sh = d->shapes[si];
            for (uint32_t f = 0; f < sh.numTriangles; ++f, ++k) {
                for (int c = 0; c < 3; ++c)
                    xformPoint(sh.toWorldTransform, d->positions[sh.startVertex + d->indices[sh.startIdx + 3 * f + c]],
                               &tri[9 * k + 3 * c]);
                shapeOf[k] = (int32_t)si;
                primOf[k] = (int32_t)f;
            }
        }
        mcrt::BvhOut bvh;
        if (!mcrt::build_bvh(tri.data(), shapeOf.data(), primOf.data(), n, cost, bins, sah, threads, bvh,
                             opts && opts->device_build == 4))
            return fail(nullptr, MCRT_ERROR_INVALID_ARG, "BVH build failed");
        *num_records = bvh.numNodes;
        if (out_records) std::memcpy(out_records, bvh.nodes, 64 * std::min<uint64_t>(max_records, bvh.numNodes));
        inf[1] = (int32_t)bvh.numNodes;
        inf[2] = bvh.depth;
        mcrt::free_bvh(bvh);
    }
    if (info) std::memcpy(info, inf, sizeof(inf));
    return MCRT_OK;
}

// ---------------------------------------------------------------------------
// RadeonRays-style queries
// ---------------------------------------------------------------------------
struct mcrt_event_s {
    hipEvent_t e = nullptr;
    int device = 0;
};

// n: the host count, or with countDev the grid's capacity (maxrays) and the device count
static mcrt_status trace_common(mcrt_scene s, const mcrt_ray* rays, int32_t n, const int32_t* countDev,
                                mcrt_intersection* hits, int32_t* occl, bool any, mcrt_event wait = nullptr,
                                mcrt_event* done = nullptr) {
    if (done) *done = nullptr;
    if (!s) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "scene is NULL");
    mcrt_ctx ctx = s->ctx;
    if (!s->dNodes) return fail(ctx, MCRT_ERROR_NOT_READY, "mcrt_accel_build has not been called");
    if (n < 0 || (n > 0 && !rays) || (n > 0 && !any && !hits) || (n > 0 && any && !occl))
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "invalid ray query arguments");
    hipSetDevice(ctx->device);
    if (wait) HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, wait->e, 0));
    if (n > 0) {
        if (!ensure_spill(s, (size_t)n)) return fail(ctx, MCRT_ERROR_OUT_OF_MEMORY, "traversal spill buffer");
        Timed t(ctx, any ? K_TRACE_ANY : K_TRACE_CLOSEST, countDev, countDev ? 0 : n);
        mcrt::launch_trace_rays(any, trace_ctx(s), rays, n, countDev, hits, occl, ctx->stream);
    }
    HIPCHK(ctx, hipGetLastError());
    if (done) {
        auto* ev = new mcrt_event_s();
        ev->device = ctx->device;
        hipError_t e = hipEventCreateWithFlags(&ev->e, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventRecord(ev->e, ctx->stream);
        if (e != hipSuccess) {
            if (ev->e) hipEventDestroy(ev->e);
            delete ev;
            return fail(ctx, MCRT_ERROR_DEVICE, std::string("query event: ") + hipGetErrorString(e));
        }
        *done = ev;
    }
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_trace_closest(mcrt_scene s, const mcrt_ray* d_rays, int32_t n, mcrt_intersection* d_hits) {
    return trace_common(s, d_rays, n, nullptr, d_hits, nullptr, false);
}

MCRT_API mcrt_status mcrt_trace_any(mcrt_scene s, const mcrt_ray* d_rays, int32_t n, int32_t* d_hits) {
    return trace_common(s, d_rays, n, nullptr, nullptr, d_hits, true);
}

MCRT_API mcrt_status mcrt_trace_closest_count(mcrt_scene s, const mcrt_ray* d_rays, const int32_t* d_numrays,
                                              int32_t maxrays, mcrt_intersection* d_hits, mcrt_event wait_event,
                                              mcrt_event* done_event) {
    if (!d_numrays) return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "d_numrays is NULL");
    return trace_common(s, d_rays, maxrays, d_numrays, d_hits, nullptr, false, wait_event, done_event);
}

MCRT_API mcrt_status mcrt_trace_any_count(mcrt_scene s, const mcrt_ray* d_rays, const int32_t* d_numrays,
                                          int32_t maxrays, int32_t* d_hits, mcrt_event wait_event,
                                          mcrt_event* done_event) {
    if (!d_numrays) return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "d_numrays is NULL");
    return trace_common(s, d_rays, maxrays, d_numrays, nullptr, d_hits, true, wait_event, done_event);
}

MCRT_API mcrt_status mcrt_event_wait(mcrt_event ev) {
    if (!ev) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "event is NULL");
    hipSetDevice(ev->device);
    const hipError_t e = hipEventSynchronize(ev->e);
    if (e != hipSuccess) return fail(nullptr, MCRT_ERROR_DEVICE, std::string("event wait: ") + hipGetErrorString(e));
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_event_destroy(mcrt_event ev) {
    if (!ev) return MCRT_OK;
    hipSetDevice(ev->device);
    hipEventDestroy(ev->e);
    delete ev;
    return MCRT_OK;
}

// ---------------------------------------------------------------------------
// frame buffer + integrator
// ---------------------------------------------------------------------------
static void bset_free(BdptSet& b) {
    void* ptrs[] = {b.camV,   b.lightV, b.slots,  b.splat,  b.camCount, b.lightCount, b.bdptCounters,
                    b.bqO[0], b.bqO[1], b.bqD[0], b.bqD[1], b.bqT[0], b.bqT[1], b.bHits, b.cO, b.cD, b.cL, b.spill,
                    b.lkey, b.lkey2, b.lslot, b.lperm, b.ekey, b.ekey2, b.eslot, b.eperm, b.sortTmp,
                    b.splatList, b.splatAux, b.suspend, b.suspendCnt};
    for (void* p : ptrs)
        if (p) hipFree(p);
    b = BdptSet();
}

static void fb_free_bdpt(mcrt_framebuffer fb) {
    for (auto& b : fb->bset) bset_free(b);
    if (fb->sampLight) hipFree(fb->sampLight);
    if (fb->bdptConnect) hipEventDestroy(fb->bdptConnect);
    fb->bdptConnect = nullptr;
    fb->camV = fb->lightV = fb->sampLight = fb->slots = fb->splat = fb->bHits = fb->cO = fb->cD = fb->cL = nullptr;
    fb->camCount = fb->lightCount = fb->bdptCounters = nullptr;
    for (int i = 0; i < 2; ++i) fb->bqO[i] = fb->bqD[i] = fb->bqT[i] = nullptr;
    fb->bdptDepth = 0;
}

static void slot_free(FrameSlot& k) {
    if (k.stream) hipStreamSynchronize(k.stream);
    void* ptrs[] = {k.radiance, k.hitsP, k.hitsE, k.eO[0], k.eO[1], k.eD[0], k.eD[1], k.eT[0], k.eT[1],
                    k.sO,       k.sD,    k.sL,    k.counters, k.spill, k.tileCost, k.tileOrder,
                    k.suspend,  k.suspendCnt};
    for (void* p : ptrs)
        if (p) hipFree(p);
    if (k.done) hipEventDestroy(k.done);
    if (k.free) hipEventDestroy(k.free);
    if (k.stream) hipStreamDestroy(k.stream);
    k = FrameSlot();
}

static void fb_free(mcrt_framebuffer fb) {
    for (auto& k : fb->slot) slot_free(k);
    for (auto& w : fb->waveClk) {
        if (w) hipFree(w);
        w = nullptr;
    }
    void* ptrs[] = {fb->wsum, fb->wts, fb->image, fb->denoised, fb->display, fb->hintPix};
    for (void* p : ptrs)
        if (p) hipFree(p);
    fb_free_bdpt(fb);
}

// Per-frame planes (radiance, primary hits) for `frames` frames of N pixels; ray queues of Q entries.
// N: pixels; T: the frame's 8x8 tiles x 64 (the packed hit slots, mcrt_kernels.hip hitSlot)
static hipError_t slot_alloc(FrameSlot& k, size_t N, size_t T, int frames = 1, size_t Q = 0) {
    hipError_t e = hipSuccess;
    if (Q < N) Q = N;
    auto A = [&](auto** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc((void**)p, bytes);
    };
    A(&k.radiance, 16 * N * frames);
    A(&k.hitsP, 16 * std::max(N, T) * frames);
    A(&k.hitsE, 16 * Q);
    for (int i = 0; i < 2; ++i) { A(&k.eO[i], 16 * Q); A(&k.eD[i], 16 * Q); A(&k.eT[i], 16 * Q); }
    A(&k.sO, 16 * Q);
    A(&k.sD, 16 * Q);
    A(&k.sL, 16 * Q);
    A(&k.counters, SLOT_COUNTER_BYTES);
    k.frames = frames;
    k.queueCap = Q;
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&k.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&k.done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&k.free, hipEventDisableTiming);
    // zero-fills on the slot's own stream, ahead of its first launch; `done` covers them for
    // readers on other streams (ctx_wait_slots) before the slot's first frame records it
    if (e == hipSuccess) e = hipMemsetAsync(k.radiance, 0, 16 * N * frames, k.stream);
    if (e == hipSuccess) e = hipMemsetAsync(k.counters, 0, SLOT_COUNTER_BYTES, k.stream);
    if (e == hipSuccess) e = hipEventRecord(k.done, k.stream);
    if (e != hipSuccess) slot_free(k);
    return e;
}

// The fb's radiance/queue/counter fields view slot k (the last rendered frame).
static void fb_bind(mcrt_framebuffer fb, int k) {
    FrameSlot& s = fb->slot[k];
    fb->cur = k;
    fb->radiance = s.radiance;
    fb->hitsP = s.hitsP;
    fb->hitsE = s.hitsE;
    for (int i = 0; i < 2; ++i) { fb->eO[i] = s.eO[i]; fb->eD[i] = s.eD[i]; fb->eT[i] = s.eT[i]; }
    fb->sO = s.sO;
    fb->sD = s.sD;
    fb->sL = s.sL;
    fb->counters = s.counters;
    fb->lastMaxDepth = s.lastMaxDepth;
    fb->lastPixels = s.lastPixels;
}

// Host reads and context-stream work that touch the slots: all slot streams first.
static hipError_t fb_sync(mcrt_framebuffer fb) {
    hipError_t e = hipSuccess;
    for (auto& k : fb->slot)
        if (k.stream && e == hipSuccess) e = hipStreamSynchronize(k.stream);
    if (e == hipSuccess) e = hipStreamSynchronize(fb->ctx->stream);
    return e;
}

// Makes the context stream wait for every slot's last render (work on the context stream
// that reads or rewrites slot buffers: BDPT, AOVs, device copies).
static void ctx_wait_slots(mcrt_framebuffer fb) {
    for (auto& k : fb->slot)
        if (k.stream) hipStreamWaitEvent(fb->ctx->stream, k.done, 0);
}

// NQ = the pixels of the whole 8x8 tiles covering the image (>= N): the start queues hold one slot
// per lane of the tile walk.  Ray queues and hits hold 2 x NQ (the depth-1 camera and light halves).
static hipError_t bset_alloc(BdptSet& b, size_t N, size_t NQ, int D, int frames, hipStream_t st) {
    const size_t C = (size_t)bdpt_max_connections(D);
    N *= frames;    // every per-frame array holds the batch's frames
    NQ *= frames;
    hipError_t e = hipSuccess;
    auto A = [&](auto** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc((void**)p, bytes);
    };
    A(&b.camV, 16 * N * BDPT_VERTEX_PLANES * (D + 2));
    A(&b.lightV, 16 * N * BDPT_VERTEX_PLANES * (D + 1));
    A(&b.slots, 16 * N * (C - D));
    A(&b.splat, 16 * N);
    A(&b.camCount, 4 * N);
    A(&b.lightCount, 4 * N);
    A(&b.bdptCounters, 64 * sizeof(int));
    for (int i = 0; i < 2; ++i) { A(&b.bqO[i], 32 * NQ); A(&b.bqD[i], 32 * NQ); A(&b.bqT[i], 32 * NQ); }
    A(&b.bHits, 32 * NQ);
    A(&b.cO, 16 * N * C);
    A(&b.cD, 16 * N * C);
    A(&b.cL, 16 * N * C);
    A(&b.lkey, 4 * NQ);
    A(&b.lkey2, 4 * NQ);
    A(&b.lslot, 4 * NQ);
    A(&b.lperm, 4 * NQ);
    A(&b.ekey, 8 * N);
    A(&b.ekey2, 8 * N);
    A(&b.eslot, 8 * N);
    A(&b.eperm, 8 * N);
    b.sortTmpBytes = mcrt::bdpt_light_sort_temp_bytes((int)std::max(NQ, 2 * N));
    A(&b.sortTmp, b.sortTmpBytes);
    // zero-fills on the stream of the set's frames (st, its slot's), ahead of the first launch
    // that writes the set: a 3 GB vertex-plane memset on another stream could still be running
    // under k_bdpt_start and zero its vertices
    if (e == hipSuccess) e = hipMemsetAsync(b.splat, 0, 16 * N, st);
    if (e == hipSuccess) e = hipMemsetAsync(b.camV, 0, 16 * N * BDPT_VERTEX_PLANES * (D + 2), st);
    if (e == hipSuccess) e = hipMemsetAsync(b.lightV, 0, 16 * N * BDPT_VERTEX_PLANES * (D + 1), st);
    if (e != hipSuccess) bset_free(b);
    else b.frames = frames;
    return e;
}

// The fb's BDPT views show set k (the last BDPT frame).
static void fb_bind_bdpt(mcrt_framebuffer fb, int k) {
    const BdptSet& b = fb->bset[k];
    fb->bdptSet = k;
    fb->camV = b.camV; fb->lightV = b.lightV; fb->slots = b.slots; fb->splat = b.splat;
    fb->camCount = b.camCount; fb->lightCount = b.lightCount; fb->bdptCounters = b.bdptCounters;
    for (int i = 0; i < 2; ++i) { fb->bqO[i] = b.bqO[i]; fb->bqD[i] = b.bqD[i]; fb->bqT[i] = b.bqT[i]; }
    fb->bHits = b.bHits; fb->cO = b.cO; fb->cD = b.cD; fb->cL = b.cL;
}

// RTBDPTPass::createBuffers (RTBDPTPass.cpp:442-479), sized for max depth D: set k of the
// per-frame arrays, plus the persistent sampled-light-vertex planes, which start zeroed (the
// reference's buffer starts with whatever the allocation holds; its clref runner zero-fills it too).
// (also the packed camera-hit slots per frame: every 8x8 tile of the frame x 64)
static size_t bdpt_queue_cap(mcrt_framebuffer fb) {
    return (size_t)((fb->W + 7) / 8) * ((fb->H + 7) / 8) * 64;
}
static hipError_t fb_ensure_bdpt(mcrt_framebuffer fb, int D, int k, int frames, hipStream_t st) {
    const size_t N = fb->N;
    if (fb->bdptDepth != D) {
        for (auto& sl : fb->slot)
            if (sl.stream) hipStreamSynchronize(sl.stream);
        hipStreamSynchronize(fb->ctx->stream);
        fb_free_bdpt(fb);
        hipError_t e = hipMalloc(&fb->sampLight, 16 * N * D);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&fb->bdptConnect, hipEventDisableTiming);
        // zeroed on this frame's stream; every connect launch (the planes' only reader and writer)
        // waits for bdptConnect, recorded here first
        if (e == hipSuccess) e = hipMemsetAsync(fb->sampLight, 0, 16 * N * D, st);
        if (e == hipSuccess) e = hipEventRecord(fb->bdptConnect, st);
        if (e != hipSuccess) { fb_free_bdpt(fb); return e; }
        fb->bdptDepth = D;
    }
    BdptSet& bs = fb->bset[k];
    if (bs.camV && bs.frames < frames) {   // a larger batch: the set's last frames must be done
        for (auto& sl : fb->slot)
            if (sl.stream) hipStreamSynchronize(sl.stream);
        hipStreamSynchronize(fb->ctx->stream);
        bset_free(bs);
        bs = BdptSet{};
    }
    if (!bs.camV) return bset_alloc(bs, N, bdpt_queue_cap(fb), D, frames, st);
    return hipSuccess;
}

MCRT_API mcrt_status mcrt_framebuffer_create(mcrt_ctx ctx, uint32_t width, uint32_t height, mcrt_framebuffer* out) {
    if (!ctx || !out || width == 0 || height == 0 || (uint64_t)width * height > (1ull << 30))
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "invalid frame buffer size");
    hipSetDevice(ctx->device);
    auto* fb = new mcrt_framebuffer_s();
    fb->ctx = ctx;
    fb->W = width;
    fb->H = height;
    fb->N = (size_t)width * height;
    const size_t N = fb->N;
    hipError_t e = hipSuccess;
    auto A = [&](auto** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc((void**)p, bytes);
    };
    A(&fb->wsum, 16 * N);
    A(&fb->wts, 4 * N);
    A(&fb->image, 16 * N);
    A(&fb->denoised, 16 * N);
    A(&fb->display, 16 * N);
    A(&fb->hintPix, 4 * N);
    fb->slot.resize(MCRT_MAX_FRAMES_IN_FLIGHT);
    if (e == hipSuccess) e = slot_alloc(fb->slot[0], N, N);   // one frame: hits by pixel
    if (e == hipSuccess) fb_bind(fb, 0);
    // zero-fills on slot 0's (private) stream, finished before the frame buffer is handed out:
    // only this buffer's work is waited for, not the device (other contexts, a captured caller stream)
    if (e == hipSuccess) e = hipMemsetAsync(fb->wsum, 0, 16 * N, fb->slot[0].stream);
    if (e == hipSuccess) e = hipMemsetAsync(fb->wts, 0, 4 * N, fb->slot[0].stream);
    if (e == hipSuccess) e = hipMemsetAsync(fb->image, 0, 16 * N, fb->slot[0].stream);
    if (e == hipSuccess) e = hipMemsetAsync(fb->denoised, 0, 16 * N, fb->slot[0].stream);
    if (e == hipSuccess) e = hipMemsetAsync(fb->display, 0, 16 * N, fb->slot[0].stream);
    if (e == hipSuccess) e = fill_hints(fb->hintPix, N, 1u << 22, fb->slot[0].stream);   // no hints
    if (e == hipSuccess) e = hipStreamSynchronize(fb->slot[0].stream);
    if (e != hipSuccess) {
        fb_free(fb);
        delete fb;
        return fail(ctx, e == hipErrorOutOfMemory ? MCRT_ERROR_OUT_OF_MEMORY : MCRT_ERROR_DEVICE,
                    std::string("frame buffer: ") + hipGetErrorString(e));
    }
    *out = fb;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_set_frames_in_flight(mcrt_framebuffer fb, int32_t n) {
    if (!fb || n < 0 || n > MCRT_MAX_FRAMES_IN_FLIGHT)
        return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "frames in flight must be 0 (auto) .. 4");
    fb->framesInFlight = n;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_destroy(mcrt_framebuffer fb) {
    if (!fb) return MCRT_OK;
    hipSetDevice(fb->ctx->device);
    fb_sync(fb);
    fb_free(fb);
    delete fb;
    return MCRT_OK;
}

static bool frame_args(mcrt_framebuffer fb, const mcrt_frame_params* p, FrameArgs& f, std::string& err) {
    f.W = fb->W;
    f.H = fb->H;
    f.frame = p->frame_index;
    f.maxDepth = p->max_depth;
    f.sampler = p->sampler;
    f.russianRoulette = p->russian_roulette;
    f.rrStartDepth = p->rr_start_depth;
    f.textureLod = p->texture_lod ? 1 : 0;
    // batched frames: workgroups of the camera / first-bounce launches walk (tile, frame) with the
    // frames of a tile adjacent, so one XCD traces a tile's batch of jittered frames back to back,
    // and a camera / first-shading wave holds 64 consecutive (pixel, frame) paths of one tile
    // (profiles/r02/ab/README.txt items 11, 14, 15); the order changes no result
    f.tileMajor = 1;
    f.primaryPack = 1;
    f.shadePack = 1;
    f.batch = 1;
    f.tileOrder = nullptr;   // set per call by render_frames (longest-first)
    f.tileCost = nullptr;
    f.numBands = p->num_bands <= 0 ? 1 : p->num_bands;
    f.bandIndex = p->band_index;
    f.bandRows = f.numBands == 1 ? 8 : p->band_rows;
    if (f.bandRows <= 0 || (f.bandRows & 7) != 0) { err = "band_rows must be a positive multiple of 8"; return false; }
    if (f.bandIndex < 0 || f.bandIndex >= f.numBands) { err = "band_index out of range"; return false; }
    f.tilesX = (int)((fb->W + 7) / 8);
    // row-blocks (8 rows) of this band set inside the image
    const int blocksTotal = (int)((fb->H + 7) / 8);
    const int bpb = f.bandRows / 8;
    int myBlocks = 0;
    for (int gb = 0; gb < blocksTotal; ++gb)
        if ((gb / bpb) % f.numBands == f.bandIndex) ++myBlocks;
    // tile ids are dealt in the kernel as tb -> gb; count the band-local blocks that map inside
    f.numTiles = myBlocks * f.tilesX;
    return true;
}

// Frames in flight for a render: the frame buffer's setting; auto = 2.  Each launch of a frame ends in a divergent tail of long rays that the next
// frame's launches fill (San-Miguel proxy 1080p: 2.33 -> 1.91 ms/frame with 2 slots, 2.06 with 4;
// tools/scale_emulate.py).  Small per-rank band shares are widened by batching frames
// (mcrt_render_frames) rather than by more slots: 4 slots of 1/8-image frames reach 0.49 ms per
// frame at N = 8, 2 slots of 16-frame batches 0.25.
// MCRT_WAVE_CLOCK=1: record per-workgroup clocks of launch `which` (grid of `blocks`) on stream st
static uint32_t* wave_clock_buf(mcrt_framebuffer fb, int which, size_t blocks, hipStream_t st) {
    static const bool on = [] { const char* e = std::getenv("MCRT_WAVE_CLOCK"); return e && std::atoi(e) != 0; }();
    if (!on) return nullptr;
    if (fb->waveClkBlocks[which] < blocks) {
        hipStreamSynchronize(st);
        if (fb->waveClk[which]) hipFree(fb->waveClk[which]);
        fb->waveClk[which] = nullptr;
        fb->waveClkBlocks[which] = 0;
        if (hipMalloc(&fb->waveClk[which], 8 * blocks) != hipSuccess) { hipGetLastError(); return nullptr; }
        fb->waveClkBlocks[which] = blocks;
    }
    hipMemsetAsync(fb->waveClk[which], 0, 8 * fb->waveClkBlocks[which], st);
    return fb->waveClk[which];
}

#define MCRT_LPT_SHADE_MAX_PATHS 16000000
// MCRT_LONGEST_FIRST=0: camera / first-shading tiles in plain tile order (A/B)
static bool longest_first() {
    static const bool on = [] { const char* e = std::getenv("MCRT_LONGEST_FIRST"); return !(e && std::atoi(e) == 0); }();
    return on;
}

static int frames_in_flight(mcrt_framebuffer fb, const FrameArgs& f) {
    // MCRT_WAVE_CLOCK=1: one frame in flight -- the clock buffers are per frame buffer, so two slots'
    // launches in flight would write the same per-workgroup entries
    static const bool clocks = [] { const char* e = std::getenv("MCRT_WAVE_CLOCK"); return e && std::atoi(e) != 0; }();
    if (clocks) return 1;
    int n = fb->framesInFlight;
    if (n <= 0) n = 2;
    return std::max(1, std::min(n, MCRT_MAX_FRAMES_IN_FLIGHT));
}

// RTBDPTPass::update (RTBDPTPass.cpp:67-128): start vertices, D+1 rounds of (trace, vertex),
// connections + MIS, visibility, gather.  Rays of both subpaths share one compacted queue.
static mcrt_status render_bdpt(mcrt_scene s, mcrt_framebuffer fb, const mcrt_camera* cam, const mcrt_frame_params* p,
                               const FrameArgs& f, int k, hipStream_t st) {
    // frame slot k on stream st: per-frame arrays of set k; the connect launch (the only reader
    // and writer of the shared sampled-light-vertex planes) waits for the previous frame's connect
    mcrt_ctx ctx = s->ctx;
    const int D = p->max_depth;
    const int B = f.batch;   // frames of this call (mcrt_render_frames): path = k * W*H + pixel
    HIPCHK(ctx, fb_ensure_bdpt(fb, D, k, B, st));
    fb_bind_bdpt(fb, k);
    fb->lastMaxDepth = D;
    fb->lastPixels = 0;
    fb->bands = f;
    fb->haveBands = true;
    fb->lastIntegrator = MCRT_INTEGRATOR_BDPT;
    fb->bdptBatch = B;
    mcrt_camera* dCam = reinterpret_cast<mcrt_camera*>(fb->counters + 128);
    HIPCHK(ctx, hipMemcpyAsync(dCam, cam, sizeof(mcrt_camera) * B, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemsetAsync(fb->bdptCounters, 0, 64 * sizeof(int), st));
    if (s->numLights == 0) {   // RTBDPTPass.cpp:69: no lights -> pass skipped
        HIPCHK(ctx, hipMemsetAsync(fb->radiance, 0, 16 * fb->N * (size_t)B, st));
        return MCRT_OK;
    }
    const size_t N = fb->N * (size_t)B, C = (size_t)bdpt_max_connections(D);   // N: paths of the batch
    BdptSet& bs = fb->bset[k];
    const size_t NQ = bdpt_queue_cap(fb) * (size_t)B;
    // spill columns: one per ray of the widest closest-hit launch (2 NQ) and one per wave of the
    // grid-stride visibility launch (mcrt::BDPT_VIS_MAX_WAVES)
    const size_t spillWords = (std::max(2 * NQ, (size_t)mcrt::BDPT_VIS_MAX_WAVES * 64) + 63) / 64 * 64 * (size_t)s->spillCap;
    if (bs.spillWords < spillWords) {
        HIPCHK(ctx, hipStreamSynchronize(st));
        if (bs.spill) hipFree(bs.spill);
        bs.spill = nullptr;
        bs.spillWords = 0;
        HIPCHK(ctx, hipMalloc(&bs.spill, spillWords * sizeof(uint32_t)));
        bs.spillWords = spillWords;
    }
    TraceCtx tcs = trace_ctx(s);
    tcs.spill = bs.spill;
    const SceneArgs sa = scene_args(s);
    // the closest-hit launches' stop rule (TraceCtx::walkCap): a traced queue holds at most
    // max(bandQ, nSort) = nSort rays (below)
    const int wcap = tcs.qnodes && !tcs.twoLevel && (int64_t)f.numTiles * 64 * B >= walk_min_paths() ? walk_cap() : 0;
    TraceCtx tce = tcs;
    if (wcap > 0) {
        const size_t need = (size_t)std::min((size_t)2 * N, (size_t)2 * (size_t)f.numTiles * 64 * B);
        if (bs.suspendCap < need) {
            HIPCHK(ctx, hipStreamSynchronize(st));
            if (bs.suspend) hipFree(bs.suspend);
            bs.suspend = nullptr;
            bs.suspendCap = 0;
            HIPCHK(ctx, hipMalloc(&bs.suspend, sizeof(float4) * MCRT_SUSPEND_F4 * need));
            bs.suspendCap = need;
        }
        if (!bs.suspendCnt) HIPCHK(ctx, hipMalloc(&bs.suspendCnt, 64 * sizeof(int)));
        HIPCHK(ctx, hipMemsetAsync(bs.suspendCnt, 0, 64 * sizeof(int), st));
        tce.walkCap = wcap;
        tce.walkLanes = walk_lanes();
        tce.suspend = bs.suspend;
    }
    BdptArgs b{};
    b.camV = fb->camV;
    b.lightV = fb->lightV;
    b.camCount = fb->camCount;
    b.lightCount = fb->lightCount;
    b.sampLight = fb->sampLight;
    b.slots = fb->slots;
    b.splat = fb->splat;
    b.ownSlots = (int)C - D;
    // (planes at another stride hold other data; another band's paths were never written)
    // the light-start rays are traced in cell order (keys from k_bdpt_start, rocPRIM sort below):
    // k_extend 3.07 -> 2.82 ms per frame at 1080p (profiles/r04/ab/README.txt)
    b.lightKey = bs.lkey;
    b.lightSlot = bs.lslot;
    // the bounce queues that are traced (depths 1..D) in octant / origin-cell order: keys written by
    // k_bdpt_vertex, sorted below, walked through the permutation by k_extend
    b.extKey = nullptr;
    b.extSlot = nullptr;
    for (int a = 0; a < 3; ++a) {
        const float ext = s->bbHi[a] - s->bbLo[a];
        b.keyLo[a] = s->bbLo[a];
        b.keyScale[a] = ext > 0.0f ? (a == 1 ? 8.0f : 32.0f) / ext : 0.0f;
    }
    b.cams = dCam;
    b.connCount = fb->bdptCounters + BDPT_CNT_CONN;
    b.connO = fb->cO;
    b.connD = fb->cD;
    b.connL = fb->cL;
    b.lightInVertex = bdpt_light_in_vertex();
    BdptArgs bk = b;   // the vertex launches whose output queue is traced
    bk.extKey = bs.ekey;
    bk.extSlot = bs.eslot;
    // a bounce queue holds at most the band's camera + light rays (2 per path of this rank's tiles),
    // appended compactly from slot 0: sort (and clear) only that range, not the whole frame's -- a
    // rank of a band split would otherwise sort 8 x its own rays at N = 8
    const int bandQ = f.numTiles * 64 * B;   // this rank's paths: a start queue holds at most one ray each
    const int nSort = (int)std::min((size_t)2 * N, (size_t)2 * (size_t)bandQ);
    // the queue traced at round D + 1 holds camera rays only (the light subpaths end at depth D): at
    // most one per path, so it is sorted (and its keys cleared) over bandQ slots, not 2 x bandQ
    auto sortRange = [&](int tracedAt) { return tracedAt == D + 1 ? std::min(nSort, bandQ) : nSort; };
    auto clearKeys = [&](int n) {   // unwritten slots sort last (stable sort: after the written ones)
        return hipMemsetAsync(bs.ekey, 0xFF, 4 * (size_t)n, st);
    };
    b.depth0Const = bs.constStride == N && bs.constBand[0] == f.bandRows && bs.constBand[1] == f.numBands &&
                    bs.constBand[2] == f.bandIndex ? 1 : 0;
    bs.constStride = N;
    bs.constBand[0] = f.bandRows;
    bs.constBand[1] = f.numBands;
    bs.constBand[2] = f.bandIndex;
    int* cnt = fb->bdptCounters;   // [d] ray queue of depth d (d <= D + 1 <= 33), BDPT_CNT_* below
    auto queue = [&](int d) {
        BdptQueue q;
        q.count = cnt + d;
        q.o = fb->bqO[d & 1];
        q.d = fb->bqD[d & 1];
        q.t = fb->bqT[d & 1];
        return q;
    };
    const bool bandSplit = f.numBands > 1;
    const bool sparse = bandSplit && fb->splatExchange == MCRT_SPLAT_EXCHANGE_SPARSE;
    if (sparse) {
        // the splats landing in other ranks' rows go to a list (at most D per path: t = 1, s = 2..D+1);
        // the rank's own rows are zeroed by k_bdpt_start, the other rows of its plane stay unused
        const size_t cap = (size_t)D * (size_t)bandQ;
        if (bs.splatListCap < cap || !bs.splatAux) {
            HIPCHK(ctx, hipStreamSynchronize(st));
            if (bs.splatList) hipFree(bs.splatList);
            bs.splatList = nullptr;
            bs.splatListCap = 0;
            HIPCHK(ctx, hipMalloc(&bs.splatList, 16 * cap));
            bs.splatListCap = cap;
            if (!bs.splatAux) HIPCHK(ctx, hipMalloc(&bs.splatAux, 128 * sizeof(int)));
        }
        b.splatList = bs.splatList;
        b.splatListCount = cnt + BDPT_CNT_SPLATS;
        b.splatListCap = (int)std::min(cap, (size_t)INT32_MAX);
        b.splatW = (int)f.W;
        b.splatN0 = (int)(f.W * f.H);
        b.splatBpb = f.bandRows / 8;
        b.splatBands = f.numBands;
        b.splatBand = f.bandIndex;
    } else if (bandSplit) {   // splats of this rank's light paths land in any pixel: clear the whole buffer
        mcrt::launch_bdpt_clear_splat((int)N, fb->splat, st);
    }
    // depth 0: camera rays (coherent, 8x8 tiles in order) in the first half of queue 0's buffers
    // with their own count, light rays in the second half with count [0]; ONE launch traces both,
    // the camera rays as wave packets like PT's camera rays (packet_ctx); both
    // halves then feed the depth-1 vertex launches, which append to queue 1
    BdptQueue camQ = queue(0), lightQ = queue(0);
    camQ.count = cnt + BDPT_CNT_CAM0;
    lightQ.o += NQ;
    lightQ.d += NQ;
    lightQ.t += NQ;
    {
        Timed t(ctx, K_BDPT_START, nullptr, (int64_t)f.numTiles * 64 * B, st);
        mcrt::launch_bdpt_start(sa, f, b, dCam, camQ, lightQ, st);
    }
    {
        TraceCtx tcc = packet_ctx(s);
        tcc.spill = bs.spill;
        Timed t(ctx, K_EXTEND, camQ.count, 0, st);
        // exactly the slots k_bdpt_start wrote (the light queue's count, f.numTiles x 64 x B <= NQ)
        HIPCHK(ctx, mcrt::bdpt_light_sort(bs.lkey, bs.lkey2, bs.lslot, bs.lperm, f.numTiles * 64 * B, bs.sortTmp,
                                          bs.sortTmpBytes, st));
        TraceCtx tl = tce;
        tl.suspendCount = wcap > 0 ? bs.suspendCnt : nullptr;
        mcrt::launch_extend_pair(tcc, tl, camQ.count, camQ.o, camQ.d, fb->bHits, lightQ.count, lightQ.o, lightQ.d,
                                 fb->bHits + NQ, bandQ, bandQ, st, bs.lperm);   // grids sized to the band
        if (wcap > 0) mcrt::launch_walk_resume(tl, lightQ.o, lightQ.d, fb->bHits + NQ, bandQ, st);
    }
    HIPCHK(ctx, clearKeys(sortRange(2)));   // queue 1 is traced (D >= 1), at round 2
    {
        Timed t(ctx, K_BDPT_VERTEX, camQ.count, 0, st);
        mcrt::launch_bdpt_vertex(sa, f, bk, 1, camQ, fb->bHits, queue(1), bandQ, st);
    }
    {
        Timed t(ctx, K_BDPT_VERTEX, lightQ.count, 0, st);
        mcrt::launch_bdpt_vertex(sa, f, bk, 1, lightQ, fb->bHits + NQ, queue(1), bandQ, st);
    }
    for (int d = 2; d <= D + 1; ++d) {
        const BdptQueue qIn = queue(d - 1), qOut = queue(d);
        {
            Timed t(ctx, K_EXTEND, qIn.count, 0, st);
            const int nQ = sortRange(d);
            HIPCHK(ctx, mcrt::bdpt_light_sort(bs.ekey, bs.ekey2, bs.eslot, bs.eperm, nQ, bs.sortTmp,
                                              bs.sortTmpBytes, st, 16));
            TraceCtx te = tce;
            te.suspendCount = wcap > 0 ? bs.suspendCnt + d : nullptr;
            mcrt::launch_extend(te, qIn.count, qIn.o, qIn.d, fb->bHits, nQ, st, bs.eperm);
            if (wcap > 0) mcrt::launch_walk_resume(te, qIn.o, qIn.d, fb->bHits, nQ, st);
        }
        const bool traced = d <= D;   // queue d is traced by the next round
        if (traced) HIPCHK(ctx, clearKeys(sortRange(d + 1)));
        Timed t(ctx, K_BDPT_VERTEX, qIn.count, 0, st);
        mcrt::launch_bdpt_vertex(sa, f, traced ? bk : b, d, qIn, fb->bHits, qOut, nSort, st);
    }
    BdptQueue cq;
    cq.count = cnt + BDPT_CNT_CONN;
    cq.o = fb->cO;
    cq.d = fb->cD;
    cq.t = fb->cL;
    HIPCHK(ctx, hipStreamWaitEvent(st, fb->bdptConnect, 0));   // sampled-light planes in frame order
    {
        Timed t(ctx, K_BDPT_CONNECT, nullptr, (int64_t)f.numTiles * 64 * B, st);
        mcrt::launch_bdpt_connect(sa, f, b, dCam, cq, st);
    }
    HIPCHK(ctx, hipEventRecord(fb->bdptConnect, st));
    {
        Timed t(ctx, K_BDPT_VIS, cq.count, 0, st);
        TraceCtx tvis = tcs;
        with_hints(tvis, s, nullptr, 0);   // occluder hints by origin cell
        mcrt::launch_bdpt_vis(tvis, b, cq, (int)(C * N), st);
    }
    if (bandSplit) {   // completed by mcrt_bdpt_gather once the ranks' splats are summed
        fb->bdptPendingGather = true;
    } else {
        Timed t(ctx, K_BDPT_GATHER, nullptr, (int64_t)f.numTiles * 64 * B, st);
        mcrt::launch_bdpt_gather(f, b, fb->radiance, nullptr, 0, st);
    }
    HIPCHK(ctx, hipGetLastError());
    fb->lastPixels = (int64_t)f.numTiles * 64 * B;
    return MCRT_OK;
}

static mcrt_status render_frames(mcrt_scene s, mcrt_framebuffer fb, const mcrt_camera* cam, int count,
                                 const mcrt_frame_params* p) {
    if (!s || !fb || !cam || !p) return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    mcrt_ctx ctx = s->ctx;
    if (fb->ctx != ctx) return fail(ctx, MCRT_ERROR_INVALID_ARG, "frame buffer belongs to another context");
    if (!s->dNodes) return fail(ctx, MCRT_ERROR_NOT_READY, "mcrt_accel_build has not been called");
    if (count < 1 || count > MCRT_MAX_BATCH_FRAMES)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "frame count must be 1 .. MCRT_MAX_BATCH_FRAMES (256)");
    if (p->integrator == MCRT_INTEGRATOR_BDPT && count > MCRT_MAX_BDPT_BATCH_FRAMES)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "BDPT frame count must be 1 .. MCRT_MAX_BDPT_BATCH_FRAMES (32)");
    for (int k = 0; k < count; ++k)
        if (cam[k].width != fb->W || cam[k].height != fb->H)
            return fail(ctx, MCRT_ERROR_INVALID_ARG, "camera size differs from the frame buffer");
    if (p->integrator == MCRT_INTEGRATOR_BDPT) {   // slot codes (own strategy x paths) and ray tags are int32
        const uint64_t NB = (uint64_t)fb->N * count, C = (uint64_t)bdpt_max_connections(p->max_depth);
        if ((C - (uint64_t)p->max_depth) * NB >= (1ull << 31) || 2 * NB >= (1ull << 31))
            return fail(ctx, MCRT_ERROR_INVALID_ARG, "BDPT: strategies x frames x pixels must stay below 2^31");
    }
    if ((uint64_t)fb->N * count >= (1ull << 31))
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "frame count x pixels must stay below 2^31 (path ids are int32)");
    if (p->max_depth < 1 || p->max_depth > MCRT_MAX_BOUNCES) return fail(ctx, MCRT_ERROR_INVALID_ARG, "max_depth out of range");
    if (p->sampler != MCRT_SAMPLER_RANDOM && p->sampler != MCRT_SAMPLER_SOBOL)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "unknown sampler");
    if (p->sampler == MCRT_SAMPLER_SOBOL && !s->hasSobol)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "Sobol sampler requires the 1024x52 Sobol matrices in the scene");
    if (p->integrator != MCRT_INTEGRATOR_PT && p->integrator != MCRT_INTEGRATOR_BDPT)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "unknown integrator");
    if (fb->bdptPendingGather)
        return fail(ctx, MCRT_ERROR_NOT_READY, "band-split BDPT frame not completed (mcrt_bdpt_gather)");
    FrameArgs f;
    std::string err;
    if (!frame_args(fb, p, f, err)) return fail(ctx, MCRT_ERROR_INVALID_ARG, err);
    hipSetDevice(ctx->device);
    f.batch = count;
    // frame slot: its buffers are free once the accumulation of its previous frame has read them
    const bool bdpt = p->integrator == MCRT_INTEGRATOR_BDPT;
    const int S = bdpt && fb->bdptOneSet ? 1 : frames_in_flight(fb, f);
    int ks = fb->next % S;
    if (bdpt && ks != 0 && fb->bdptDepth == p->max_depth && !fb->bset[ks].camV) {
        // each BDPT set holds ~C x N x 48 B of connection rays (2.5 GB at 1080p, D = 2): when a
        // second one does not fit, fall back to one frame in flight instead of failing the frame
        // (zero-filled on slot ks's stream when it exists, else on slot 0's and finished here: set ks
        // is then first written on slot ks's stream)
        hipStream_t zs = fb->slot[ks].stream ? fb->slot[ks].stream : fb->slot[0].stream;
        hipError_t e = bset_alloc(fb->bset[ks], fb->N, bdpt_queue_cap(fb), p->max_depth, count, zs);
        if (e == hipSuccess && zs != fb->slot[ks].stream) e = hipStreamSynchronize(zs);
        if (e == hipErrorOutOfMemory) {
            hipGetLastError();
            fb->bdptOneSet = true;
            ks = 0;
        } else if (e != hipSuccess) {
            return fail(ctx, MCRT_ERROR_DEVICE, std::string("BDPT buffers: ") + hipGetErrorString(e));
        }
    }
    FrameSlot& slot = fb->slot[ks];
    if (bdpt) {   // BDPT frames overlap the same way (set ks)
        if (!slot.stream) {
            HIPCHK(ctx, slot_alloc(slot, fb->N, bdpt_queue_cap(fb), count));
        } else if (slot.frames < count) {   // radiance planes for a larger batch
            HIPCHK(ctx, hipEventSynchronize(slot.free));
            HIPCHK(ctx, hipStreamSynchronize(slot.stream));
            slot_free(slot);
            HIPCHK(ctx, slot_alloc(slot, fb->N, bdpt_queue_cap(fb), count));
        }
        HIPCHK(ctx, hipStreamWaitEvent(slot.stream, slot.free, 0));
        fb_bind(fb, ks);
        fb->next = (ks + 1) % (fb->bdptOneSet ? 1 : S);
        slot.lastBatch = count;
        const mcrt_status r = render_bdpt(s, fb, cam, p, f, ks, slot.stream);
        slot.lastMaxDepth = fb->lastMaxDepth;
        slot.lastPixels = fb->lastPixels;
        hipEventRecord(slot.done, slot.stream);
        return r;
    }
    // the queues hold at most the batch's paths of the band: size the ray grids to them
    const int bandPaths = f.numTiles * 64 * count;
    const size_t qNeed = std::max(fb->N, (size_t)bandPaths);
    if (!slot.stream) {
        HIPCHK(ctx, slot_alloc(slot, fb->N, bdpt_queue_cap(fb), count, qNeed));
    } else if (slot.frames < count || slot.queueCap < qNeed) {   // grow for a larger batch
        HIPCHK(ctx, hipEventSynchronize(slot.free));
        slot_free(slot);
        HIPCHK(ctx, slot_alloc(slot, fb->N, bdpt_queue_cap(fb), count, qNeed));
    }
    const int cap = s->spillCap;
    const size_t spillRays = (std::max((size_t)bandPaths, 2 * qNeed + 64) + 63) / 64 * 64;
    if (!slot.spill || slot.spillWords < spillRays * cap) {
        HIPCHK(ctx, hipStreamSynchronize(slot.stream));
        if (slot.spill) hipFree(slot.spill);
        slot.spill = nullptr;
        slot.spillWords = 0;
        HIPCHK(ctx, hipMalloc(&slot.spill, spillRays * cap * sizeof(uint32_t)));
        slot.spillWords = spillRays * cap;
    }
    hipStream_t st = slot.stream;
    HIPCHK(ctx, hipStreamWaitEvent(st, slot.free, 0));
    fb_bind(fb, ks);
    fb->next = (ks + 1) % S;
    fb->lastMaxDepth = slot.lastMaxDepth = p->max_depth;
    fb->lastPixels = slot.lastPixels = 0;
    slot.lastBatch = count;
    fb->bands = f;
    fb->haveBands = true;
    mcrt_camera* dCam = reinterpret_cast<mcrt_camera*>(fb->counters + 128);   // 176 B per frame after the counters
    HIPCHK(ctx, hipMemcpyAsync(dCam, cam, sizeof(mcrt_camera) * count, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, hipMemsetAsync(fb->counters, 0, 128 * sizeof(int), st));
    int* shadowCnt = fb->counters;          // [b]
    int* extCnt = fb->counters + 32;        // [b]
    const SceneArgs sa = scene_args(s);
    fb->lastIntegrator = MCRT_INTEGRATOR_PT;
    if (s->numLights == 0) {   // RTPathTracingPass.cpp:42: no lights -> pass skipped; radiance = 0 here
        // every frame plane of the batch: accumulate reads `count` of them
        HIPCHK(ctx, hipMemsetAsync(fb->radiance, 0, 16 * fb->N * (size_t)count, st));
        HIPCHK(ctx, hipEventRecord(slot.done, st));
        return MCRT_OK;
    }
    TraceCtx tcs = trace_ctx(s);
    tcs.spill = slot.spill;
    const int qCap = bandPaths;
    const int wcap = tcs.qnodes && !tcs.twoLevel && p->max_depth > 1 && bandPaths >= walk_min_paths() ? walk_cap() : 0;
    if (wcap > 0) {
        if (slot.suspendCap < (size_t)qCap) {
            HIPCHK(ctx, hipStreamSynchronize(st));
            if (slot.suspend) hipFree(slot.suspend);
            slot.suspend = nullptr;
            slot.suspendCap = 0;
            HIPCHK(ctx, hipMalloc(&slot.suspend, sizeof(float4) * MCRT_SUSPEND_F4 * (size_t)qCap));
            slot.suspendCap = qCap;
        }
        if (!slot.suspendCnt) HIPCHK(ctx, hipMalloc(&slot.suspendCnt, 32 * sizeof(int)));
        HIPCHK(ctx, hipMemsetAsync(slot.suspendCnt, 0, 32 * sizeof(int), st));
    }
    if (longest_first()) {
        // the camera / first-shading tiles in descending cost of this slot's previous call (same
        // tiles), and this call's costs recorded for the next one -- all on the slot's stream
        if (slot.tileCap < f.numTiles) {
            HIPCHK(ctx, hipStreamSynchronize(st));
            if (slot.tileCost) hipFree(slot.tileCost);
            if (slot.tileOrder) hipFree(slot.tileOrder);
            slot.tileCost = slot.tileOrder = nullptr;
            slot.tileCap = slot.costTiles = 0;
            HIPCHK(ctx, hipMalloc(&slot.tileCost, 4 * (size_t)f.numTiles));
            HIPCHK(ctx, hipMalloc(&slot.tileOrder, 4 * (size_t)f.numTiles));
            slot.tileCap = f.numTiles;
        }
        if (slot.costTiles == f.numTiles) {
            mcrt::launch_tile_order(slot.tileCost, f.numTiles, slot.tileOrder, st);
            f.tileOrder = slot.tileOrder;
        }
        HIPCHK(ctx, hipMemsetAsync(slot.tileCost, 0, 4 * (size_t)f.numTiles, st));
        f.tileCost = slot.tileCost;
        slot.costTiles = f.numTiles;
    }
    {
        Timed t(ctx, K_PRIMARY, nullptr, (int64_t)bandPaths, st);
        TraceCtx tcp = packet_ctx(s);   // coherent camera rays: wave packets
        tcp.spill = slot.spill;
        tcp.waveClock = wave_clock_buf(fb, 0, (size_t)f.numTiles * count, st);
        mcrt::launch_primary(tcp, f, dCam, fb->hitsP, st);
    }
    for (int b = 0; b < p->max_depth; ++b) {
        QueueArgs q;
        q.shadowCount = shadowCnt + b;
        q.sO = fb->sO; q.sD = fb->sD; q.sL = fb->sL;
        q.extCountOut = extCnt + b;
        q.eOout = fb->eO[b & 1]; q.eDout = fb->eD[b & 1]; q.eTout = fb->eT[b & 1];
        if (b == 0) {
            Timed t(ctx, K_SHADE0, nullptr, (int64_t)bandPaths, st);
            // the longest-first order also for the first shading (its extension queue then starts with
            // the expensive tiles' rays) only for small launches: at a rank's share of N >= 4 GPUs it
            // trims the extension launch's tail, on a whole 1080p image it costs the shading's
            // spatial locality (+2.8 % k_shade0, +1.2 % k_shadow_extend; profiles/r05/ab/longest_first)
            FrameArgs fs = f;
            if ((int64_t)bandPaths > MCRT_LPT_SHADE_MAX_PATHS) fs.tileOrder = nullptr;
            mcrt::launch_shade0(sa, fs, dCam, fb->hitsP, fb->radiance, q, st);
        } else {
            Timed t(ctx, K_SHADEN, extCnt + b - 1, 0, st);
            mcrt::launch_shadeN(sa, f, b, extCnt + b - 1, fb->eO[(b - 1) & 1], fb->eD[(b - 1) & 1],
                                fb->eT[(b - 1) & 1], fb->hitsE, fb->radiance, q, qCap, st);
        }
        if (b + 1 < p->max_depth) {
            // shadow rays of bounce b + extension rays for bounce b+1 (both from this shading pass) in
            // one launch: separate k_extend + k_shadow launches cost 0.18 ms more per frame (r01)
            Timed t(ctx, K_SHADOW_EXTEND, extCnt + b, 0, st, shadowCnt + b);   // items: extension + shadow rays
            // bounce-0 shadow rays are coherent (a packed wave's paths share a pixel): wave packets
            TraceCtx tse = b == 0 ? packet_ctx(s) : tcs;
            tse.spill = slot.spill;
            with_hints(tse, s, b == 0 ? fb->hintPix : nullptr, (uint32_t)fb->N);
            if (tse.hint && ctx->countHints) tse.hintHits = fb->counters + 64 + b;
            if (tse.qnodes && ctx->countHints) tse.retraces = fb->counters + 96 + b;
            if (b == 0) tse.waveClock = wave_clock_buf(fb, 1, 2 * (((size_t)qCap + 63) / 64), st);
            if (wcap > 0 && b <= walk_max_bounce()) {
                tse.walkCap = wcap;
                tse.walkLanes = walk_lanes();
                tse.suspend = slot.suspend;
                tse.suspendCount = slot.suspendCnt + b;
            }
            mcrt::launch_shadow_extend(tse, extCnt + b, fb->eO[b & 1], fb->eD[b & 1], fb->hitsE, shadowCnt + b,
                                       fb->sO, fb->sD, fb->sL, fb->radiance, qCap, qCap, st);
            if (tse.walkCap > 0) mcrt::launch_walk_resume(tse, fb->eO[b & 1], fb->eD[b & 1], fb->hitsE, qCap, st);
        } else {
            Timed t(ctx, K_SHADOW, shadowCnt + b, 0, st);
            TraceCtx tsh = tcs;
            with_hints(tsh, s, b == 0 ? fb->hintPix : nullptr, (uint32_t)fb->N);
            if (tsh.hint && ctx->countHints) tsh.hintHits = fb->counters + 64 + b;
            tsh.waveClock = wave_clock_buf(fb, 2, ((size_t)qCap + 63) / 64, st);
            mcrt::launch_shadow(tsh, shadowCnt + b, fb->sO, fb->sD, fb->sL, fb->radiance, qCap, st);
        }
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(slot.done, st));
    fb->lastPixels = slot.lastPixels = (int64_t)bandPaths;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_render_frame(mcrt_scene s, mcrt_framebuffer fb, const mcrt_camera* cam,
                                       const mcrt_frame_params* p) {
    return render_frames(s, fb, cam, 1, p);
}

MCRT_API mcrt_status mcrt_render_frames(mcrt_scene s, mcrt_framebuffer fb, const mcrt_camera* cameras, int32_t count,
                                        const mcrt_frame_params* p) {
    return render_frames(s, fb, cameras, count, p);
}

MCRT_API mcrt_status mcrt_render_aov(mcrt_scene s, mcrt_framebuffer fb, const mcrt_camera* cam,
                                     const mcrt_frame_params* p, int aov, float* host_out) {
    if (!s || !fb || !cam || !p || !host_out) return fail(s ? s->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    mcrt_ctx ctx = s->ctx;
    if (!s->dNodes) return fail(ctx, MCRT_ERROR_NOT_READY, "mcrt_accel_build has not been called");
    if (aov != MCRT_AOV_ALBEDO && aov != MCRT_AOV_TEXTURE_LOD) return fail(ctx, MCRT_ERROR_INVALID_ARG, "unknown aov");
    if (cam->width != fb->W || cam->height != fb->H)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "camera size differs from the frame buffer");
    FrameArgs f;
    std::string err;
    if (!frame_args(fb, p, f, err)) return fail(ctx, MCRT_ERROR_INVALID_ARG, err);
    hipSetDevice(ctx->device);
    hipStream_t st = ctx->stream;
    ctx_wait_slots(fb);   // the AOV pass reuses the bound slot's camera and primary-hit buffers
    mcrt_camera* dCam = reinterpret_cast<mcrt_camera*>(fb->counters + 128);
    HIPCHK(ctx, hipMemcpyAsync(dCam, cam, sizeof(mcrt_camera), hipMemcpyHostToDevice, st));
    if (!ensure_spill(s, std::max((size_t)f.numTiles * 64, 2 * fb->N + 64)))
        return fail(ctx, MCRT_ERROR_OUT_OF_MEMORY, "traversal spill buffer");
    const TraceCtx tcs = packet_ctx(s);
    mcrt::launch_primary(tcs, f, dCam, fb->hitsP, st);
    const size_t stride = aov == MCRT_AOV_TEXTURE_LOD ? 3 : 1;
    float4* dOut = nullptr;
    HIPCHK(ctx, hipMallocAsync((void**)&dOut, 16 * stride * fb->N, st));
    HIPCHK(ctx, hipMemsetAsync(dOut, 0, 16 * stride * fb->N, st));
    mcrt::launch_aov(scene_args(s), f, dCam, fb->hitsP, aov, dOut, st);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(host_out, dOut, 16 * stride * fb->N, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    hipFreeAsync(dOut, st);
    hipStreamSynchronize(st);
    if (e != hipSuccess) return fail(ctx, MCRT_ERROR_DEVICE, std::string("aov: ") + hipGetErrorString(e));
    return MCRT_OK;
}

static mcrt_status accumulate(mcrt_framebuffer fb, const mcrt_filter* filters, int nfilters, int32_t frame_index) {
    if (!fb || !filters) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    mcrt_ctx ctx = fb->ctx;
    if (fb->bdptPendingGather)
        return fail(ctx, MCRT_ERROR_NOT_READY, "band-split BDPT frame not completed (mcrt_bdpt_gather)");
    if (!fb->haveBands) {   // no frame rendered yet: whole image
        mcrt_frame_params p{};
        std::memset(&p, 0, sizeof(p));
        p.num_bands = 1;
        std::string err;
        frame_args(fb, &p, fb->bands, err);
        fb->haveBands = true;
    }
    hipSetDevice(ctx->device);
    FrameSlot& slot = fb->slot[fb->cur];
    const int batch = slot.lastBatch;
    if (nfilters != 1 && nfilters != batch)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "one filter, or one per frame of the last mcrt_render_frames");
    FrameArgs f = fb->bands;
    f.batch = batch;
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, slot.done, 0));   // the frame's render (its slot stream)
    // weights are evaluated on the device (k_accumulate, filters.cl); the filters go to the slot's
    // counter block, which its next render (after slot.free below) does not touch before this launch
    mcrt_filter* dFilt = reinterpret_cast<mcrt_filter*>(reinterpret_cast<char*>(slot.counters) + SLOT_FILTER_OFFSET);
    HIPCHK(ctx, hipMemcpyAsync(dFilt, filters, sizeof(mcrt_filter) * nfilters, hipMemcpyHostToDevice, ctx->stream));
    {
        Timed t(ctx, K_ACCUM, nullptr, (int64_t)f.numTiles * 64 * batch);
        mcrt::launch_accumulate(f, frame_index, dFilt, nfilters == 1 ? 0 : 1, fb->radiance, fb->wsum, fb->wts, fb->image,
                                ctx->stream);
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(slot.free, ctx->stream));   // the slot may take its next frame
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_accumulate(mcrt_framebuffer fb, const mcrt_filter* filter, int32_t frame_index) {
    return accumulate(fb, filter, 1, frame_index);
}

MCRT_API mcrt_status mcrt_accumulate_frames(mcrt_framebuffer fb, const mcrt_filter* filters, int32_t count,
                                            int32_t frame_index) {
    return accumulate(fb, filters, count, frame_index);
}

MCRT_API mcrt_status mcrt_framebuffer_device_ptrs(mcrt_framebuffer fb, void** radiance, void** weighted_sum,
                                                  void** weight_sum, void** image) {
    if (!fb) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "fb is NULL");
    if (radiance) *radiance = fb->radiance;
    if (weighted_sum) *weighted_sum = fb->wsum;
    if (weight_sum) *weight_sum = fb->wts;
    if (image) *image = fb->image;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_postprocess(mcrt_framebuffer fb, const mcrt_postprocess_params* p) {
    if (!fb || !p) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    const int W = (int)fb->W, H = (int)fb->H;
    const float4* src = fb->image;
    if (p->use_denoise) {
        // RTDenoisePass (RTDenoisePass.cpp:21-60): the kernel writes nothing for a non-positive
        // radius or sigma (Denoise.cl:18-19), so the pass then shows its image's old content.
        if (p->denoise_radius > 16) return fail(ctx, MCRT_ERROR_INVALID_ARG, "denoise_radius > 16 (the GUI allows <= 10)");
        if (p->denoise_radius > 0 && p->sigma_spatial > 0.0f && p->sigma_range > 0.0f)
            mcrt::launch_denoise(W, H, p->denoise_radius, p->sigma_spatial, p->sigma_range, fb->image, fb->denoised,
                                 ctx->stream);
        src = fb->denoised;
    }
    if (p->use_tonemapping)   // RTToneMappingPass::applyReinhardToneMapping (RTToneMappingPass.cpp:38-72)
        mcrt::launch_tonemap(W * H, p->min_luminance, src, fb->display, ctx->stream);
    else
        HIPCHK(ctx, hipMemcpyAsync(fb->display, src, 16 * fb->N, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipGetLastError());
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_read(mcrt_framebuffer fb, int which, float* host_rgba) {
    if (!fb || !host_rgba || which < 0 || which > 3) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    const void* src = which == 0 ? (const void*)fb->radiance : which == 1 ? (const void*)fb->wsum
                      : which == 2 ? (const void*)fb->image : (const void*)fb->display;
    HIPCHK(ctx, fb_sync(fb));
    HIPCHK(ctx, hipMemcpy(host_rgba, src, 16 * fb->N, hipMemcpyDeviceToHost));
    return check_device_flags(ctx);
}

MCRT_API mcrt_status mcrt_framebuffer_read_frame(mcrt_framebuffer fb, int32_t k, float* host_rgba) {
    if (!fb || !host_rgba) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    mcrt_ctx ctx = fb->ctx;
    const int batch = fb->slot[fb->cur].lastBatch;
    if (k < 0 || k >= std::max(batch, 1))
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "frame index outside the last mcrt_render_frames batch");
    hipSetDevice(ctx->device);
    HIPCHK(ctx, fb_sync(fb));
    HIPCHK(ctx, hipMemcpy(host_rgba, fb->radiance + (size_t)k * fb->N, 16 * fb->N, hipMemcpyDeviceToHost));
    return check_device_flags(ctx);
}

MCRT_API mcrt_status mcrt_framebuffer_copy_device(mcrt_framebuffer fb, int which, void* d_dst) {
    if (!fb || !d_dst || which < 0 || which > 3) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    const void* src = which == 0 ? (const void*)fb->radiance : which == 1 ? (const void*)fb->wsum
                      : which == 2 ? (const void*)fb->image : (const void*)fb->wts;
    if (which == 0) ctx_wait_slots(fb);
    HIPCHK(ctx, hipMemcpyAsync(d_dst, src, (which == 3 ? 4 : 16) * fb->N, hipMemcpyDeviceToDevice, ctx->stream));
    // the slot may take its next frame only after this copy has read its radiance
    if (which == 0) HIPCHK(ctx, hipEventRecord(fb->slot[fb->cur].free, ctx->stream));
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_set_accumulation(mcrt_framebuffer fb, const void* d_wsum, const void* d_wts) {
    if (!fb || !d_wsum || !d_wts) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, hipMemcpyAsync(fb->wsum, d_wsum, 16 * fb->N, hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(fb->wts, d_wts, 4 * fb->N, hipMemcpyDeviceToDevice, ctx->stream));
    mcrt::launch_resolve(fb->W, fb->H, fb->wsum, fb->wts, fb->image, ctx->stream);
    HIPCHK(ctx, hipGetLastError());
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_bands_pack(mcrt_framebuffer fb, void* d_dst) {
    if (!fb || !d_dst) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    if (!fb->haveBands) return fail(fb->ctx, MCRT_ERROR_NOT_READY, "no frame rendered");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    mcrt::launch_band_pack(fb->bands, fb->wsum, fb->wts, static_cast<float*>(d_dst), ctx->stream);
    HIPCHK(ctx, hipGetLastError());
    return MCRT_OK;
}

// The largest rank's row count of a band split (whole 8-row blocks): the rows of one packed chunk.
static int band_max_rows(const FrameArgs& f) {
    const int blocks = (int)((f.H + 7) / 8), bpb = f.bandRows / 8;
    const int perCycle = bpb * f.numBands;
    return 8 * ((blocks / perCycle) * bpb + std::min(blocks % perCycle, bpb));
}

MCRT_API mcrt_status mcrt_framebuffer_band_layout(mcrt_framebuffer fb, int32_t* max_rows, int32_t* num_bands,
                                                  int32_t* band_index) {
    if (!fb) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "fb is NULL");
    if (!fb->haveBands) return fail(fb->ctx, MCRT_ERROR_NOT_READY, "no frame rendered");
    if (max_rows) *max_rows = band_max_rows(fb->bands);
    if (num_bands) *num_bands = fb->bands.numBands;
    if (band_index) *band_index = fb->bands.bandIndex;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_bands_unpack(mcrt_framebuffer fb, const void* d_recv, int32_t max_rows) {
    if (!fb || !d_recv) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    if (!fb->haveBands) return fail(fb->ctx, MCRT_ERROR_NOT_READY, "no frame rendered");
    const FrameArgs& f = fb->bands;
    // every chunk of d_recv must hold the largest rank's rows
    if (max_rows < band_max_rows(f))
        return fail(fb->ctx, MCRT_ERROR_INVALID_ARG, "max_rows below the largest rank's row count");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    mcrt::launch_band_unpack(f, max_rows, static_cast<const float*>(d_recv), fb->wsum, fb->wts, fb->image,
                             ctx->stream);
    HIPCHK(ctx, hipGetLastError());
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_stats(mcrt_framebuffer fb, int64_t* closest_rays, int64_t* any_rays,
                                            int64_t* shaded_paths) {
    if (!fb) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "fb is NULL");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, fb_sync(fb));
    int c[64];
    if (fb->lastIntegrator == MCRT_INTEGRATOR_BDPT) {   // closest: all subpath rays; any: connection rays
        HIPCHK(ctx, hipMemcpy(c, fb->bdptCounters, sizeof(c), hipMemcpyDeviceToHost));
        int64_t cl = 0;
        for (int d = 0; d <= fb->lastMaxDepth; ++d) cl += c[d];
        cl += c[BDPT_CNT_CAM0];
        if (closest_rays) *closest_rays = cl;
        if (any_rays) *any_rays = c[BDPT_CNT_CONN];
        if (shaded_paths) *shaded_paths = cl;
        return MCRT_OK;
    }
    HIPCHK(ctx, hipMemcpy(c, fb->counters, sizeof(c), hipMemcpyDeviceToHost));
    int64_t cl = fb->lastPixels, an = 0, sh = fb->lastPixels;
    for (int b = 0; b < fb->lastMaxDepth; ++b) {
        an += c[b];
        if (b + 1 < fb->lastMaxDepth) { cl += c[32 + b]; sh += c[32 + b]; }
    }
    if (closest_rays) *closest_rays = cl;
    if (any_rays) *any_rays = an;
    if (shaded_paths) *shaded_paths = sh;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_queue_counts(mcrt_framebuffer fb, int32_t* shadow, int32_t* extension, int max) {
    if (!fb || max < 0) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, fb_sync(fb));
    int c[64];
    HIPCHK(ctx, hipMemcpy(c, fb->counters, sizeof(c), hipMemcpyDeviceToHost));
    for (int b = 0; b < max && b < 32; ++b) {
        const bool live = b < fb->lastMaxDepth && fb->lastIntegrator == MCRT_INTEGRATOR_PT;
        if (shadow) shadow[b] = live ? c[b] : 0;
        if (extension) extension[b] = live && b + 1 < fb->lastMaxDepth ? c[32 + b] : 0;
    }
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_hint_counts(mcrt_framebuffer fb, int32_t* hits, int max) {
    if (!fb || max < 0) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, fb_sync(fb));
    int c[128];
    HIPCHK(ctx, hipMemcpy(c, fb->counters, sizeof(c), hipMemcpyDeviceToHost));
    for (int b = 0; b < max && b < 32; ++b) {
        const bool live = b < fb->lastMaxDepth && fb->lastIntegrator == MCRT_INTEGRATOR_PT;
        if (hits) hits[b] = live ? c[64 + b] : 0;
    }
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_retrace_counts(mcrt_framebuffer fb, int32_t* retraces, int max) {
    if (!fb || max < 0) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    mcrt_ctx ctx = fb->ctx;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, fb_sync(fb));
    int c[128];
    HIPCHK(ctx, hipMemcpy(c, fb->counters, sizeof(c), hipMemcpyDeviceToHost));
    for (int b = 0; b < max && b < 32; ++b) {
        const bool live = b + 1 < fb->lastMaxDepth && fb->lastIntegrator == MCRT_INTEGRATOR_PT;
        if (retraces) retraces[b] = live ? c[96 + b] : 0;
    }
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_wave_clock(mcrt_framebuffer fb, int which, uint32_t* host_out, int64_t max_blocks,
                                                 int64_t* blocks) {
    if (!fb || which < 0 || which > 2 || !blocks) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "bad args");
    mcrt_ctx ctx = fb->ctx;
    *blocks = (int64_t)fb->waveClkBlocks[which];
    if (!host_out || !fb->waveClk[which]) return MCRT_OK;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, fb_sync(fb));
    const size_t n = std::min((size_t)std::max<int64_t>(max_blocks, 0), fb->waveClkBlocks[which]);
    HIPCHK(ctx, hipMemcpy(host_out, fb->waveClk[which], 8 * n, hipMemcpyDeviceToHost));
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_read_queue(mcrt_framebuffer fb, int which, void* host_dst,
                                                 int64_t max_records, int32_t* count) {
    if (!fb) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "fb is NULL");
    mcrt_ctx ctx = fb->ctx;
    if (which != 0 && which != 1) return fail(ctx, MCRT_ERROR_INVALID_ARG, "which must be 0 (shadow) or 1 (extension)");
    if (max_records < 0 || (max_records > 0 && !host_dst)) return fail(ctx, MCRT_ERROR_INVALID_ARG, "bad destination");
    if (fb->lastMaxDepth <= 0) return fail(ctx, MCRT_ERROR_INVALID_ARG, "nothing rendered yet");
    hipSetDevice(ctx->device);
    HIPCHK(ctx, fb_sync(fb));
    int c[64];
    HIPCHK(ctx, hipMemcpy(c, fb->counters, sizeof(c), hipMemcpyDeviceToHost));
    const int b = which == 0 ? fb->lastMaxDepth - 1 : fb->lastMaxDepth - 2;   // last shadow / last extension queue
    const int n = b < 0 ? 0 : (which == 0 ? c[b] : c[32 + b]);
    if (count) *count = n;
    const int64_t m = std::min<int64_t>(n, max_records);
    if (m == 0) return MCRT_OK;
    const float4* src[3];
    if (which == 0) { src[0] = fb->sO; src[1] = fb->sD; src[2] = fb->sL; }
    else { src[0] = fb->eO[b & 1]; src[1] = fb->eD[b & 1]; src[2] = fb->eT[b & 1]; }   // b >= 0 here
    for (int k = 0; k < 3; ++k)
        HIPCHK(ctx, hipMemcpy(static_cast<char*>(host_dst) + (size_t)k * 16 * max_records, src[k], 16 * (size_t)m,
                              hipMemcpyDeviceToHost));
    return MCRT_OK;
}

// Rank-major splat layout of a band split of H rows into num_bands interleaved sets of band_rows
// rows: chunks = num_bands, each of (the largest rank's 8-row block count) x 8 rows x W pixels.
static size_t splat_chunk_pixels(const FrameArgs& f) {
    const int blocksTotal = (int)((f.H + 7) / 8), bpb = f.bandRows / 8;
    int maxBlocks = 0;
    for (int r = 0; r < f.numBands; ++r) {
        int nb = 0;
        for (int gb = 0; gb < blocksTotal; ++gb) nb += ((gb / bpb) % f.numBands == r) ? 1 : 0;
        maxBlocks = std::max(maxBlocks, nb);
    }
    return (size_t)maxBlocks * 8 * f.W;
}

MCRT_API mcrt_status mcrt_bdpt_splat_layout(mcrt_framebuffer fb, uint64_t* chunk_pixels, int32_t* chunks) {
    if (!fb || !chunk_pixels || !chunks) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    if (!fb->haveBands) return fail(fb->ctx, MCRT_ERROR_NOT_READY, "no frame rendered yet");
    *chunk_pixels = splat_chunk_pixels(fb->bands) * (size_t)std::max(fb->bands.batch, 1);   // batch frames per chunk
    *chunks = fb->bands.numBands;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_set_splat_exchange(mcrt_framebuffer fb, int32_t mode) {
    if (!fb || (mode != MCRT_SPLAT_EXCHANGE_DENSE && mode != MCRT_SPLAT_EXCHANGE_SPARSE))
        return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "unknown splat exchange mode");
    if (fb->bdptPendingGather) return fail(fb->ctx, MCRT_ERROR_NOT_READY, "band-split BDPT frame not completed");
    fb->splatExchange = mode;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_bdpt_splats_sparse(mcrt_framebuffer fb, void* d_dst, int64_t capacity, int64_t* counts,
                                             int32_t num_counts) {
    if (!fb || !counts) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    mcrt_ctx ctx = fb->ctx;
    const int bands = fb->bands.numBands;
    if (num_counts < bands) return fail(ctx, MCRT_ERROR_INVALID_ARG, "counts must hold num_bands entries");
    for (int r = 0; r < num_counts; ++r) counts[r] = 0;
    if (!fb->bdptPendingGather) return MCRT_OK;   // nothing pending (light-less scene): no splats
    if (fb->splatExchange != MCRT_SPLAT_EXCHANGE_SPARSE)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "frame rendered with the dense splat exchange (mcrt_bdpt_splats_copy)");
    if (bands > 64) return fail(ctx, MCRT_ERROR_INVALID_ARG, "sparse splat exchange: at most 64 bands");
    hipSetDevice(ctx->device);
    BdptSet& bs = fb->bset[fb->bdptSet];
    hipStream_t st = fb->slot[fb->cur].stream;
    BdptArgs b{};
    b.splatList = bs.splatList;
    b.splatListCount = fb->bdptCounters + BDPT_CNT_SPLATS;
    b.splatListCap = (int)std::min(bs.splatListCap, (size_t)INT32_MAX);
    b.splatW = (int)fb->bands.W;
    b.splatN0 = (int)(fb->bands.W * fb->bands.H);
    b.splatBpb = fb->bands.bandRows / 8;
    b.splatBands = bands;
    b.splatBand = fb->bands.bandIndex;
    int h[64];
    HIPCHK(ctx, hipMemsetAsync(bs.splatAux, 0, 128 * sizeof(int), st));
    mcrt::launch_splat_hist(b, bs.splatAux, st);
    HIPCHK(ctx, hipMemcpyAsync(h, bs.splatAux, sizeof(int) * bands, hipMemcpyDeviceToHost, st));
    HIPCHK(ctx, hipStreamSynchronize(st));   // the sizes go to the host (an all-to-all's split sizes)
    mcrt::SplatOffsets off{};
    int64_t total = 0;
    for (int r = 0; r < bands; ++r) {
        off.off[r] = (int)total;
        counts[r] = h[r];
        total += h[r];
    }
    if (!d_dst || capacity < total) return MCRT_OK;   // sizes only (the caller grows its buffer and calls again)
    // the caller's send buffer may still be read by an earlier call's all-to-all on another frame
    // slot's stream (two frames in flight), and that call's unpack must read its receive buffer
    // before this call's all-to-all (ordered after this grouping on this stream) overwrites it: wait
    // for every other slot's completed frame, as mcrt_bdpt_splats_copy does
    for (auto& k : fb->slot)
        if (k.stream && k.stream != st) HIPCHK(ctx, hipStreamWaitEvent(st, k.done, 0));
    mcrt::launch_splat_group(b, off, bs.splatAux + 64, (float4*)d_dst, st);
    HIPCHK(ctx, hipGetLastError());
    return MCRT_OK;   // grouping enqueued on the frame's stream
}

MCRT_API mcrt_status mcrt_bdpt_gather_sparse(mcrt_framebuffer fb, const void* d_recv, int64_t records) {
    if (!fb || (records > 0 && !d_recv)) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    mcrt_ctx ctx = fb->ctx;
    if (!fb->bdptPendingGather) return MCRT_OK;
    if (fb->splatExchange != MCRT_SPLAT_EXCHANGE_SPARSE)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "frame rendered with the dense splat exchange (mcrt_bdpt_gather)");
    if (records < 0 || records > INT32_MAX) return fail(ctx, MCRT_ERROR_INVALID_ARG, "bad record count");
    hipSetDevice(ctx->device);
    FrameSlot& slot = fb->slot[fb->cur];
    hipStream_t st = slot.stream;
    mcrt::launch_splat_unpack((const float4*)d_recv, (int)records, fb->splat, st);
    BdptArgs b{};
    b.slots = fb->slots;
    b.splat = fb->splat;
    b.ownSlots = bdpt_max_connections(fb->bdptDepth) - fb->bdptDepth;
    {
        Timed t(ctx, K_BDPT_GATHER, nullptr, (int64_t)fb->bands.numTiles * 64 * fb->bands.batch, st);
        mcrt::launch_bdpt_gather(fb->bands, b, fb->radiance, nullptr, 0, st);   // the rank's own plane
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(slot.done, st));
    fb->bdptPendingGather = false;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_bdpt_splats_copy(mcrt_framebuffer fb, void* d_dst) {
    if (!fb || !d_dst) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    mcrt_ctx ctx = fb->ctx;
    if (fb->bdptPendingGather && fb->splatExchange == MCRT_SPLAT_EXCHANGE_SPARSE)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "frame rendered with the sparse splat exchange (mcrt_bdpt_splats_sparse)");
    if (!fb->haveBands) return fail(ctx, MCRT_ERROR_NOT_READY, "no frame rendered yet");
    hipSetDevice(ctx->device);
    const size_t chunk = splat_chunk_pixels(fb->bands);   // per frame; a rank's chunk holds batch of them
    const size_t total = chunk * (size_t)std::max(fb->bands.batch, 1) * (size_t)fb->bands.numBands;
    FrameSlot& slot = fb->slot[fb->cur];
    hipStream_t st = slot.stream ? slot.stream : ctx->stream;
    // the caller's buffer may still be read by an earlier frame's gather on another slot's stream
    for (auto& k : fb->slot)
        if (k.stream && k.stream != st) HIPCHK(ctx, hipStreamWaitEvent(st, k.done, 0));
    HIPCHK(ctx, hipMemsetAsync(d_dst, 0, sizeof(float) * MCRT_SPLAT_CHANNELS * total, st));
    if (fb->bdptPendingGather)   // (else, e.g. a scene without lights: the frame is complete, no splats)
        mcrt::launch_bdpt_splat_pack(fb->bands, chunk, fb->splat, (float*)d_dst, st);
    HIPCHK(ctx, hipGetLastError());
    return MCRT_OK;   // enqueued on the frame's stream (mcrt_framebuffer_stream): no host sync
}

MCRT_API mcrt_status mcrt_framebuffer_stream(mcrt_framebuffer fb, void** stream) {
    if (!fb || !stream) return fail(fb ? fb->ctx : nullptr, MCRT_ERROR_INVALID_ARG, "NULL argument");
    const FrameSlot& slot = fb->slot[fb->cur];
    *stream = (void*)(slot.stream ? slot.stream : fb->ctx->stream);
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_bdpt_gather(mcrt_framebuffer fb, const void* d_own_chunk) {
    if (!fb) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "fb is NULL");
    mcrt_ctx ctx = fb->ctx;
    if (!fb->bdptPendingGather) return MCRT_OK;   // nothing deferred (whole-image or light-less frame)
    if (fb->splatExchange == MCRT_SPLAT_EXCHANGE_SPARSE)
        return fail(ctx, MCRT_ERROR_INVALID_ARG, "frame rendered with the sparse splat exchange (mcrt_bdpt_gather_sparse)");
    hipSetDevice(ctx->device);
    FrameSlot& slot = fb->slot[fb->cur];
    hipStream_t st = slot.stream;
    BdptArgs b{};
    b.slots = fb->slots;
    b.splat = fb->splat;
    b.ownSlots = bdpt_max_connections(fb->bdptDepth) - fb->bdptDepth;
    {
        Timed t(ctx, K_BDPT_GATHER, nullptr, (int64_t)fb->bands.numTiles * 64 * fb->bands.batch, st);
        mcrt::launch_bdpt_gather(fb->bands, b, fb->radiance, (const float*)d_own_chunk,
                                 splat_chunk_pixels(fb->bands), st);
    }
    HIPCHK(ctx, hipGetLastError());
    HIPCHK(ctx, hipEventRecord(slot.done, st));
    fb->bdptPendingGather = false;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_framebuffer_read_bdpt(mcrt_framebuffer fb, int which, void* host_dst, uint64_t bytes,
                                                uint64_t* needed) {
    if (!fb) return fail(nullptr, MCRT_ERROR_INVALID_ARG, "fb is NULL");
    mcrt_ctx ctx = fb->ctx;
    if (fb->bdptDepth <= 0) return fail(ctx, MCRT_ERROR_INVALID_ARG, "no BDPT frame rendered yet");
    // the planes of the last BDPT call's batch (plane stride N x batch)
    const size_t N = fb->N * (size_t)fb->bdptBatch, D = (size_t)fb->bdptDepth;
    const size_t C = (size_t)bdpt_max_connections(fb->bdptDepth);
    const void* src = nullptr;
    size_t sz = 0;
    switch (which) {
    case 0: src = fb->camV; sz = 16 * N * BDPT_VERTEX_PLANES * (D + 2); break;
    case 1: src = fb->lightV; sz = 16 * N * BDPT_VERTEX_PLANES * (D + 1); break;
    case 2: src = fb->camCount; sz = 4 * N; break;
    case 3: src = fb->lightCount; sz = 4 * N; break;
    case 4: src = fb->slots; sz = 16 * N * (C - D); break;
    case 5: src = fb->sampLight; sz = 16 * fb->N * D; break;   // per pixel, carried across frames
    case 6: src = fb->splat; sz = 16 * N; break;
    default: return fail(ctx, MCRT_ERROR_INVALID_ARG, "which must be 0..6");
    }
    if (needed) *needed = sz;
    if (!host_dst || bytes == 0) return MCRT_OK;
    hipSetDevice(ctx->device);
    HIPCHK(ctx, fb_sync(fb));
    HIPCHK(ctx, hipMemcpy(host_dst, src, std::min<size_t>(sz, bytes), hipMemcpyDeviceToHost));
    return MCRT_OK;
}

// host camera helpers: mcrt_camera.cpp

}  // extern "C"

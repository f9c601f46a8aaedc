// TEST INFRASTRUCTURE ONLY -- runs the REFERENCE's own OpenCL kernels on the GPU box.
//
// The code objects in oracle/_ref/clref_*.hsaco are the reference's assets/kernels/PathTracing.cl,
// reconstruction.cl and RadeonRays' intersect_bvh2_lds.cl, compiled here for gfx950 by ROCm clang
// against ROCm's OpenCL device libraries (oracle/refbuild/Makefile).  This host driver (ours)
// loads them through the ROCm OpenCL runtime (clCreateProgramWithBinary) and replays the
// reference's host launch sequence:
//   RTPrimaryRaysPass::update   (RTPrimaryRaysPass.cpp:32-67): GeneratePerspectiveRays, intersect_main
//   RTPathTracingPass::update   (RTPathTracingPass.cpp:40-114): per bounce PathTracing, occluded_main,
//                                ShadowPass, intersect_main
//   RTReconstructionPass        (RTReconstructionPass.cpp:71-123): ReconstructionPass
// with 8x8 work-groups for application kernels and 64-wide groups for RadeonRays
// (IntersectorLDS::Intersect, intersector_lds.cpp:266-295).  The BVH node array is the
// reference builder's (oracle/_ref/librrref.so = RadeonRays bvh2.cpp).
#define CL_TARGET_OPENCL_VERSION 120
#include <CL/cl.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "../../include/mcrt_capi.h"

namespace {
std::string g_err;

bool ok(cl_int e, const char* what) {
    if (e != CL_SUCCESS) {
        g_err = std::string(what) + " failed: " + std::to_string(e);
        return false;
    }
    return true;
}

std::vector<unsigned char> readFile(const std::string& p) {
    std::ifstream f(p, std::ios::binary);
    return std::vector<unsigned char>((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
}

struct Runtime {
    cl_platform_id plat = nullptr;
    cl_device_id dev = nullptr;
    cl_context ctx = nullptr;
    cl_command_queue q = nullptr;
    cl_program pt = nullptr, rr = nullptr, recon = nullptr, bdpt = nullptr;
    cl_kernel kGen = nullptr, kPT = nullptr, kShadow = nullptr, kIsect = nullptr, kOccl = nullptr, kRecon = nullptr;
    cl_kernel kBStart = nullptr, kBSec = nullptr, kBPrep = nullptr, kBConn = nullptr, kBCopy = nullptr;
    // RadeonRays IntersectorTwoLevel (intersect_bvh2level_skiplinks.cl), loaded on first use
    cl_program rr2l = nullptr;
    cl_kernel kIsect2 = nullptr, kOccl2 = nullptr;
    std::string deviceName, dir;
} R;

cl_program loadProgram(const std::string& path) {
    auto bin = readFile(path);
    if (bin.empty()) { g_err = "cannot read " + path; return nullptr; }
    size_t len = bin.size();
    const unsigned char* p = bin.data();
    cl_int st = 0, e = 0;
    cl_program prog = clCreateProgramWithBinary(R.ctx, 1, &R.dev, &len, &p, &st, &e);
    if (!ok(e, "clCreateProgramWithBinary") || !ok(st, "binary status")) return nullptr;
    e = clBuildProgram(prog, 1, &R.dev, "", nullptr, nullptr);
    if (e != CL_SUCCESS) {
        size_t n = 0;
        clGetProgramBuildInfo(prog, R.dev, CL_PROGRAM_BUILD_LOG, 0, nullptr, &n);
        std::string log(n, '\0');
        clGetProgramBuildInfo(prog, R.dev, CL_PROGRAM_BUILD_LOG, n, &log[0], nullptr);
        g_err = "clBuildProgram(" + path + "): " + std::to_string(e) + " " + log;
        return nullptr;
    }
    return prog;
}

cl_mem buf(size_t bytes, const void* host) {
    cl_int e = 0;
    if (bytes == 0) bytes = 16;
    cl_mem m = clCreateBuffer(R.ctx, CL_MEM_READ_WRITE | (host ? CL_MEM_COPY_HOST_PTR : 0), bytes, (void*)host, &e);
    if (!ok(e, "clCreateBuffer")) return nullptr;
    if (!host) {
        std::vector<unsigned char> z(bytes, 0);
        clEnqueueWriteBuffer(R.q, m, CL_TRUE, 0, bytes, z.data(), 0, nullptr, nullptr);
    }
    return m;
}

struct Scene {
    cl_mem shapes, indices, positions, uvs, normals, tangents, binormals, colors, textures, texData, sobol, lights,
        materials, camera, nodes;
    int numLights;
    // per-resolution buffers
    int W = 0, H = 0;
    cl_mem rays = nullptr, rayDiff = nullptr, isect = nullptr, shadowRays = nullptr, occl = nullptr, thr = nullptr,
           temp = nullptr, radiance = nullptr, stack = nullptr, count = nullptr, wsum = nullptr, wts = nullptr,
           filter = nullptr, image = nullptr;
    // RTBDPTPass::createBuffers (RTBDPTPass.cpp:442-479)
    int bW = 0, bH = 0, bD = 0;
    cl_mem bFinal = nullptr, bRadiance = nullptr, camV = nullptr, lightV = nullptr, camRays = nullptr, camIsect = nullptr,
           camThr = nullptr, camPdf = nullptr, camCnt = nullptr, lightRays = nullptr, lightIsect = nullptr,
           lightThr = nullptr, lightPdf = nullptr, lightCnt = nullptr, connRays = nullptr, connVis = nullptr,
           sampCamV = nullptr, sampLightV = nullptr, bTemp = nullptr, bStack = nullptr, bCount = nullptr,
           bConnCount = nullptr;
    // two-level mode: IntersectorTwoLevel's buffers (intersector_2level.cpp:300-470)
    bool twoLevel = false;
    cl_mem n2 = nullptr, v2 = nullptr, f2 = nullptr, s2 = nullptr;
    int root2 = -1;
};

template <class T>
cl_int arg(cl_kernel k, int i, const T& v) { return clSetKernelArg(k, i, sizeof(T), &v); }

bool launch2D(cl_kernel k, int W, int H) {
    size_t gs[2] = {(size_t)(W + 7) / 8 * 8, (size_t)(H + 7) / 8 * 8}, ls[2] = {8, 8};
    return ok(clEnqueueNDRangeKernel(R.q, k, 2, nullptr, gs, ls, 0, nullptr, nullptr), "launch2D") &&
           ok(clFinish(R.q), "clFinish");
}
// IntersectorTwoLevel::Intersect / Occluded argument order (intersector_2level.cpp:640-690)
bool launchRR2(cl_kernel k, Scene* s, cl_mem rays, cl_mem out, cl_mem count, int n) {
    k = (k == R.kIsect) ? R.kIsect2 : R.kOccl2;
    cl_int e = 0;
    e |= arg(k, 0, s->n2);
    e |= arg(k, 1, s->v2);
    e |= arg(k, 2, s->f2);
    e |= arg(k, 3, s->s2);
    e |= arg(k, 4, s->root2);
    e |= arg(k, 5, rays);
    e |= arg(k, 6, count);
    e |= arg(k, 7, out);
    if (!ok(e, "set RR2L args")) return false;
    size_t gs = (size_t)(n + 63) / 64 * 64, ls = 64;
    return ok(clEnqueueNDRangeKernel(R.q, k, 1, nullptr, &gs, &ls, 0, nullptr, nullptr), "launchRR2") &&
           ok(clFinish(R.q), "clFinish");
}
bool launchRR(cl_kernel k, Scene* s, cl_mem rays, cl_mem out, int n) {
    if (s->twoLevel) return launchRR2(k, s, rays, out, s->count, n);
    cl_int e = 0;
    e |= arg(k, 0, s->nodes);
    e |= arg(k, 1, rays);
    e |= arg(k, 2, s->count);
    e |= arg(k, 3, s->stack);
    e |= arg(k, 4, out);
    if (!ok(e, "set RR args")) return false;
    size_t gs = (size_t)(n + 63) / 64 * 64, ls = 64;
    return ok(clEnqueueNDRangeKernel(R.q, k, 1, nullptr, &gs, &ls, 0, nullptr, nullptr), "launchRR") &&
           ok(clFinish(R.q), "clFinish");
}
bool ensureBuffers(Scene* s, int W, int H) {
    if (s->W == W && s->H == H) return true;
    cl_mem* old[] = {&s->rays, &s->rayDiff, &s->isect, &s->shadowRays, &s->occl, &s->thr, &s->temp, &s->radiance,
                     &s->stack, &s->count, &s->wsum, &s->wts, &s->filter};
    for (auto* m : old)
        if (*m) clReleaseMemObject(*m), *m = nullptr;
    if (s->image) clReleaseMemObject(s->image), s->image = nullptr;
    size_t N = (size_t)W * H;
    s->rays = buf(48 * N, nullptr);
    s->rayDiff = buf(64 * N, nullptr);
    s->isect = buf(32 * N, nullptr);
    s->shadowRays = buf(48 * N, nullptr);
    s->occl = buf(4 * N, nullptr);
    s->thr = buf(32 * N, nullptr);
    s->temp = buf(16 * N, nullptr);
    s->radiance = buf(16 * N, nullptr);
    s->stack = buf(4 * N * 64, nullptr);
    int n = (int)N;
    s->count = buf(4, &n);
    s->wsum = buf(16 * N, nullptr);
    s->wts = buf(4 * N, nullptr);
    s->filter = buf(sizeof(mcrt_filter), nullptr);
    cl_image_format fmt = {CL_RGBA, CL_FLOAT};
    cl_int e = 0;
    // CDNA devices report no image support: ReconstructionPass then cannot run (its
    // output is a write_only image2d_t); the frame pipeline does not need it.
    s->image = clCreateImage2D(R.ctx, CL_MEM_READ_WRITE, &fmt, W, H, 0, nullptr, &e);
    if (e != CL_SUCCESS) s->image = nullptr;
    s->W = W;
    s->H = H;
    return s->rays && s->stack;
}
}  // namespace

extern "C" {

__attribute__((visibility("default"))) const char* clref_error() { return g_err.c_str(); }

__attribute__((visibility("default"))) const char* clref_device() { return R.deviceName.c_str(); }

// variant: "fast" = the reference's build options (-cl-mad-enable -cl-fast-relaxed-math), "ieee" = none
__attribute__((visibility("default"))) int clref_init(const char* dir, const char* variant) {
    cl_uint np = 0;
    if (!ok(clGetPlatformIDs(0, nullptr, &np), "clGetPlatformIDs") || np == 0) { g_err = "no OpenCL platform"; return -1; }
    std::vector<cl_platform_id> ps(np);
    clGetPlatformIDs(np, ps.data(), nullptr);
    for (auto p : ps) {
        cl_uint nd = 0;
        if (clGetDeviceIDs(p, CL_DEVICE_TYPE_GPU, 0, nullptr, &nd) == CL_SUCCESS && nd > 0) {
            R.plat = p;
            clGetDeviceIDs(p, CL_DEVICE_TYPE_GPU, 1, &R.dev, nullptr);
            break;
        }
    }
    if (!R.dev) { g_err = "no OpenCL GPU device"; return -2; }
    char name[256] = {0};
    clGetDeviceInfo(R.dev, CL_DEVICE_NAME, sizeof(name), name, nullptr);
    R.deviceName = name;
    cl_int e = 0;
    R.ctx = clCreateContext(nullptr, 1, &R.dev, nullptr, nullptr, &e);
    if (!ok(e, "clCreateContext")) return -3;
    R.q = clCreateCommandQueue(R.ctx, R.dev, 0, &e);
    if (!ok(e, "clCreateCommandQueue")) return -4;
    std::string d(dir);
    R.dir = d;
    R.pt = loadProgram(d + "/clref_pt_" + variant + ".hsaco");
    R.rr = loadProgram(d + "/clref_rr.hsaco");
    R.recon = loadProgram(d + "/clref_recon.hsaco");
    if (!R.pt || !R.rr || !R.recon) return -5;
    R.kGen = clCreateKernel(R.pt, "GeneratePerspectiveRays", &e);
    if (!ok(e, "kernel GeneratePerspectiveRays")) return -6;
    R.kPT = clCreateKernel(R.pt, "PathTracing", &e);
    if (!ok(e, "kernel PathTracing")) return -6;
    R.kShadow = clCreateKernel(R.pt, "ShadowPass", &e);
    if (!ok(e, "kernel ShadowPass")) return -6;
    R.kIsect = clCreateKernel(R.rr, "intersect_main", &e);
    if (!ok(e, "kernel intersect_main")) return -6;
    R.kOccl = clCreateKernel(R.rr, "occluded_main", &e);
    if (!ok(e, "kernel occluded_main")) return -6;
    R.kRecon = clCreateKernel(R.recon, "ReconstructionPass", &e);
    if (!ok(e, "kernel ReconstructionPass")) return -6;
    R.bdpt = loadProgram(d + "/clref_bdpt_" + variant + ".hsaco");
    if (!R.bdpt) return -5;
    const char* bk[5] = {"GenerateStartVertices", "GenerateSecondaryVertices", "PrepareConnections", "ConnectVertices",
                         "CopyBuffer"};
    cl_kernel* bp[5] = {&R.kBStart, &R.kBSec, &R.kBPrep, &R.kBConn, &R.kBCopy};
    for (int i = 0; i < 5; ++i) {
        *bp[i] = clCreateKernel(R.bdpt, bk[i], &e);
        if (!ok(e, bk[i])) return -6;
    }
    return 0;
}

// nodes: RadeonRays Bvh2 node array (64 B each) from the reference builder
__attribute__((visibility("default"))) void* clref_scene_create(const mcrt_scene_desc* d, const void* nodes,
                                                                int64_t num_nodes) {
    auto* s = new Scene();
    s->shapes = buf(sizeof(mcrt_shape) * d->num_shapes, d->shapes);
    s->indices = buf(4ull * d->num_indices, d->indices);
    s->positions = buf(16ull * d->num_vertices, d->positions);
    s->uvs = buf(8ull * d->num_vertices, d->uvs);
    s->normals = buf(16ull * d->num_vertices, d->normals);
    s->tangents = buf(16ull * d->num_vertices, d->tangents);
    s->binormals = buf(16ull * d->num_vertices, d->binormals);
    s->colors = d->colors ? buf(16ull * d->num_vertices, d->colors) : buf(16, nullptr);
    s->textures = d->num_textures ? buf(16ull * d->num_textures, d->textures) : buf(16, nullptr);
    s->texData = d->tex_data_bytes ? buf(d->tex_data_bytes, d->tex_data) : buf(16, nullptr);
    s->sobol = d->sobol_matrices ? buf(4ull * d->num_sobol_words, d->sobol_matrices) : buf(16, nullptr);
    s->lights = d->num_lights ? buf(sizeof(mcrt_light) * d->num_lights, d->lights) : buf(16, nullptr);
    s->materials = d->num_materials ? buf(sizeof(mcrt_material) * d->num_materials, d->materials) : buf(16, nullptr);
    s->camera = buf(sizeof(mcrt_camera), nullptr);
    s->nodes = buf(64ull * num_nodes, nodes);
    s->numLights = (int)d->num_lights;
    if (!s->shapes || !s->nodes) { delete s; return nullptr; }
    return s;
}

// Switch the scene's ray queries to RadeonRays' two-level intersector over the reference's own
// two-level buffers (oracle/_ref/librrref.so rr2l_build): nodes 32 B, vertices 16 B, faces 20 B,
// shapes 112 B.
__attribute__((visibility("default"))) int clref_scene_set_two_level(void* sp, const void* nodes, int64_t nn,
                                                                     const void* verts, int64_t nv, const void* faces,
                                                                     int64_t nf, const void* shapes, int64_t ns,
                                                                     int root) {
    Scene* s = (Scene*)sp;
    if (!R.rr2l) {
        R.rr2l = loadProgram(R.dir + "/clref_rr2l.hsaco");
        if (!R.rr2l) return -1;
        cl_int e = 0;
        R.kIsect2 = clCreateKernel(R.rr2l, "intersect_main", &e);
        if (!ok(e, "kernel intersect_main (2l)")) return -2;
        R.kOccl2 = clCreateKernel(R.rr2l, "occluded_main", &e);
        if (!ok(e, "kernel occluded_main (2l)")) return -2;
    }
    cl_mem* old[] = {&s->n2, &s->v2, &s->f2, &s->s2};
    for (auto* m : old)
        if (*m) clReleaseMemObject(*m), *m = nullptr;
    s->n2 = buf(32ull * nn, nodes);
    s->v2 = buf(16ull * nv, verts);
    s->f2 = buf(20ull * nf, faces);
    s->s2 = buf(112ull * ns, shapes);
    s->root2 = root;
    s->twoLevel = s->n2 && s->v2 && s->f2 && s->s2;
    return s->twoLevel ? 0 : -3;
}

static bool setSceneArgs(cl_kernel k, Scene* s, int& a) {   // RTScene::setSceneArgs, RTScene.cpp:178-197
    cl_int e = 0;
    e |= arg(k, a++, s->shapes);
    e |= arg(k, a++, s->indices);
    e |= arg(k, a++, s->positions);
    e |= arg(k, a++, s->uvs);
    e |= arg(k, a++, s->normals);
    e |= arg(k, a++, s->tangents);
    e |= arg(k, a++, s->binormals);
    e |= arg(k, a++, s->colors);
    e |= arg(k, a++, s->textures);
    e |= arg(k, a++, s->texData);
    e |= arg(k, a++, s->sobol);
    e |= arg(k, a++, s->lights);
    e |= arg(k, a++, s->numLights);
    e |= arg(k, a++, s->materials);
    e |= arg(k, a++, s->camera);
    return ok(e, "scene args");
}

// One frame (RTPrimaryRaysPass + RTPathTracingPass); radiance_out: W*H float4 ("RadianceBufferCL").
__attribute__((visibility("default"))) int clref_render(void* sp, const mcrt_camera* cam, int frame, int maxDepth,
                                                        float* radiance_out, double* ms_out) {
    Scene* s = (Scene*)sp;
    const int W = (int)cam->width, H = (int)cam->height;
    if (!ensureBuffers(s, W, H)) return -1;
    if (!ok(clEnqueueWriteBuffer(R.q, s->camera, CL_TRUE, 0, sizeof(mcrt_camera), cam, 0, nullptr, nullptr), "camera"))
        return -1;
    cl_int e = 0;
    e |= arg(R.kGen, 0, s->rays);
    e |= arg(R.kGen, 1, s->rayDiff);
    e |= arg(R.kGen, 2, s->camera);
    if (!ok(e, "gen args") || !launch2D(R.kGen, W, H)) return -2;
    if (!launchRR(R.kIsect, s, s->rays, s->isect, W * H)) return -3;
    for (int b = 0; b < maxDepth; ++b) {
        int a = 0;
        if (!setSceneArgs(R.kPT, s, a)) return -4;
        e = 0;
        e |= arg(R.kPT, a++, W);
        e |= arg(R.kPT, a++, H);
        e |= arg(R.kPT, a++, s->shadowRays);
        e |= arg(R.kPT, a++, s->rays);
        e |= arg(R.kPT, a++, s->isect);
        e |= arg(R.kPT, a++, frame);
        e |= arg(R.kPT, a++, maxDepth);
        e |= arg(R.kPT, a++, b);
        e |= arg(R.kPT, a++, s->temp);
        e |= arg(R.kPT, a++, s->thr);
        if (!ok(e, "PT args") || !launch2D(R.kPT, W, H)) return -5;
        if (!launchRR(R.kOccl, s, s->shadowRays, s->occl, W * H)) return -6;
        e = 0;
        e |= arg(R.kShadow, 0, s->shadowRays);
        e |= arg(R.kShadow, 1, s->occl);
        e |= arg(R.kShadow, 2, W);
        e |= arg(R.kShadow, 3, H);
        e |= arg(R.kShadow, 4, b);
        e |= arg(R.kShadow, 5, s->thr);
        e |= arg(R.kShadow, 6, s->temp);
        e |= arg(R.kShadow, 7, s->radiance);
        if (!ok(e, "shadow args") || !launch2D(R.kShadow, W, H)) return -7;
        if (b + 1 < maxDepth && !launchRR(R.kIsect, s, s->rays, s->isect, W * H)) return -8;
    }
    clFinish(R.q);
    (void)ms_out;
    if (radiance_out &&
        !ok(clEnqueueReadBuffer(R.q, s->radiance, CL_TRUE, 0, 16ull * W * H, radiance_out, 0, nullptr, nullptr), "read"))
        return -9;
    return 0;
}

// ReconstructionPass (reconstruction.cl:6-60); image_out: W*H float4
__attribute__((visibility("default"))) int clref_accumulate(void* sp, int frame, const mcrt_filter* f, float* image_out) {
    Scene* s = (Scene*)sp;
    if (!s->image) { g_err = "device has no OpenCL image support (ReconstructionPass writes an image2d_t)"; return -10; }
    if (!ok(clEnqueueWriteBuffer(R.q, s->filter, CL_TRUE, 0, sizeof(mcrt_filter), f, 0, nullptr, nullptr), "filter"))
        return -1;
    cl_int e = 0;
    e |= arg(R.kRecon, 0, s->W);
    e |= arg(R.kRecon, 1, s->H);
    e |= arg(R.kRecon, 2, frame);
    e |= arg(R.kRecon, 3, s->filter);
    e |= arg(R.kRecon, 4, s->radiance);
    e |= arg(R.kRecon, 5, s->wsum);
    e |= arg(R.kRecon, 6, s->wts);
    e |= arg(R.kRecon, 7, s->image);
    if (!ok(e, "recon args") || !launch2D(R.kRecon, s->W, s->H)) return -2;
    size_t origin[3] = {0, 0, 0}, region[3] = {(size_t)s->W, (size_t)s->H, 1};
    if (image_out &&
        !ok(clEnqueueReadImage(R.q, s->image, CL_TRUE, origin, region, 0, 0, image_out, 0, nullptr, nullptr), "read image"))
        return -3;
    return 0;
}

// RadeonRays QueryIntersection / QueryOcclusion on host rays (48 B) -> host hits (32 B / int)
__attribute__((visibility("default"))) int clref_trace(void* sp, const void* rays, int n, void* out, int any) {
    Scene* s = (Scene*)sp;
    cl_mem r = buf(48ull * n, rays);
    cl_mem o = buf((any ? 4ull : 32ull) * n, out);   // pre-filled: inactive rays stay untouched
    cl_mem st = buf(4ull * n * 64, nullptr);
    cl_mem cnt = buf(4, &n);
    cl_mem saveStack = s->stack, saveCount = s->count;
    s->stack = st;
    s->count = cnt;
    bool good = launchRR(any ? R.kOccl : R.kIsect, s, r, o, n);
    s->stack = saveStack;
    s->count = saveCount;
    if (good) good = ok(clEnqueueReadBuffer(R.q, o, CL_TRUE, 0, (any ? 4ull : 32ull) * n, out, 0, nullptr, nullptr), "read");
    clReleaseMemObject(r);
    clReleaseMemObject(o);
    clReleaseMemObject(st);
    clReleaseMemObject(cnt);
    return good ? 0 : -1;
}

// Debug read-back of the last frame's intermediate buffers (stage-level parity diagnostics):
// which 0 rays (48 B), 1 isect (32 B), 2 shadow rays (48 B), 3 temp radiance (16 B),
// 4 throughput records (32 B), 5 occlusion (4 B), 6 radiance (16 B); per pixel.
__attribute__((visibility("default"))) int clref_read(void* sp, int which, void* out) {
    Scene* s = (Scene*)sp;
    const size_t n = (size_t)s->W * s->H;
    cl_mem m[8] = {s->rays, s->isect, s->shadowRays, s->temp, s->thr, s->occl, s->radiance, s->rayDiff};
    size_t sz[8] = {48, 32, 48, 16, 32, 4, 16, 64};
    if (which < 0 || which > 7 || !m[which]) { g_err = "clref_read: bad buffer"; return -1; }
    return ok(clEnqueueReadBuffer(R.q, m[which], CL_TRUE, 0, sz[which] * n, out, 0, nullptr, nullptr), "read") ? 0 : -2;
}

// Stage probe (clprobe.cl, test infrastructure): per-pixel intermediates of the reference's
// PathTracing functions for given intersections / incoming directions; out: 20 float4 / pixel.
__attribute__((visibility("default"))) int clref_probe(void* sp, const char* hsaco, const void* isects,
                                                       const float* dirs, int W, int H, int frame, float* out) {
    Scene* s = (Scene*)sp;
    static cl_program prog = nullptr;
    static cl_kernel k = nullptr;
    cl_int e = 0;
    if (!k) {
        prog = loadProgram(hsaco);
        if (!prog) return -1;
        k = clCreateKernel(prog, "ProbeShade", &e);
        if (!ok(e, "kernel ProbeShade")) return -2;
    }
    const size_t n = (size_t)W * H;
    cl_mem bi = buf(32 * n, isects), bd = buf(16 * n, dirs), bs = buf(48 * n, nullptr);
    std::vector<float> zero(80 * n, 0.0f);
    cl_mem bo = buf(80 * 4 * n, zero.data());
    int a = 0;
    if (!setSceneArgs(k, s, a)) return -3;
    e = 0;
    e |= arg(k, a++, W);
    e |= arg(k, a++, H);
    e |= arg(k, a++, frame);
    e |= arg(k, a++, bi);
    e |= arg(k, a++, bd);
    e |= arg(k, a++, bs);
    e |= arg(k, a++, bo);
    if (!ok(e, "probe args")) return -4;
    size_t gs = (n + 63) / 64 * 64, ls = 64;
    bool good = ok(clEnqueueNDRangeKernel(R.q, k, 1, nullptr, &gs, &ls, 0, nullptr, nullptr), "probe launch") &&
                ok(clEnqueueReadBuffer(R.q, bo, CL_TRUE, 0, 80 * 4 * n, out, 0, nullptr, nullptr), "probe read");
    clReleaseMemObject(bi);
    clReleaseMemObject(bd);
    clReleaseMemObject(bs);
    clReleaseMemObject(bo);
    return good ? 0 : -5;
}

// Texture-LOD probe (clprobe_lod.cl, test infrastructure): the reference's unused LOD functions
// over given primary intersections (32 B) and ray differentials (64 B); out: 3 float4 / pixel.
__attribute__((visibility("default"))) int clref_probe_lod(void* sp, const char* hsaco, const void* isects,
                                                           const void* diffs, int W, int H, float* out) {
    Scene* s = (Scene*)sp;
    static cl_program prog = nullptr;
    static cl_kernel k = nullptr;
    cl_int e = 0;
    if (!k) {
        prog = loadProgram(hsaco);
        if (!prog) return -1;
        k = clCreateKernel(prog, "ProbeLOD", &e);
        if (!ok(e, "kernel ProbeLOD")) return -2;
    }
    const size_t n = (size_t)W * H;
    cl_mem bi = buf(32 * n, isects), bd = buf(64 * n, diffs);
    std::vector<float> zero(12 * n, 0.0f);
    cl_mem bo = buf(12 * 4 * n, zero.data());
    int a = 0;
    if (!setSceneArgs(k, s, a)) return -3;
    e = 0;
    e |= arg(k, a++, W);
    e |= arg(k, a++, H);
    e |= arg(k, a++, bi);
    e |= arg(k, a++, bd);
    e |= arg(k, a++, bo);
    if (!ok(e, "probe lod args")) return -4;
    size_t gs = (n + 63) / 64 * 64, ls = 64;
    bool good = ok(clEnqueueNDRangeKernel(R.q, k, 1, nullptr, &gs, &ls, 0, nullptr, nullptr), "probe lod launch") &&
                ok(clEnqueueReadBuffer(R.q, bo, CL_TRUE, 0, 12 * 4 * n, out, 0, nullptr, nullptr), "probe lod read");
    clReleaseMemObject(bi);
    clReleaseMemObject(bd);
    clReleaseMemObject(bo);
    return good ? 0 : -5;
}

// Filter probe (clprobe_filters.cl, test infrastructure): the reference's filter weight for each of
// n 56-B RTFilterProperties records.
__attribute__((visibility("default"))) int clref_probe_filters(const char* hsaco, const void* props, int n,
                                                               float* out) {
    static cl_program prog = nullptr;
    static cl_kernel k = nullptr;
    cl_int e = 0;
    if (!k) {
        prog = loadProgram(hsaco);
        if (!prog) return -1;
        k = clCreateKernel(prog, "ProbeFilters", &e);
        if (!ok(e, "kernel ProbeFilters")) return -2;
    }
    cl_mem bp = buf(56 * (size_t)n, props);
    std::vector<float> zero((size_t)n, 0.0f);
    cl_mem bo = buf(4 * (size_t)n, zero.data());
    e = 0;
    e |= arg(k, 0, bp);
    e |= arg(k, 1, n);
    e |= arg(k, 2, bo);
    if (!ok(e, "probe filter args")) return -4;
    size_t gs = ((size_t)n + 63) / 64 * 64, ls = 64;
    bool good = ok(clEnqueueNDRangeKernel(R.q, k, 1, nullptr, &gs, &ls, 0, nullptr, nullptr), "probe filter launch") &&
                ok(clEnqueueReadBuffer(R.q, bo, CL_TRUE, 0, 4 * (size_t)n, out, 0, nullptr, nullptr), "probe filter read");
    clReleaseMemObject(bp);
    clReleaseMemObject(bo);
    return good ? 0 : -5;
}

// Tone-mapping probe (clprobe_tonemap.cl, test infrastructure): the reference's Reinhard operator
// (computeLuminanceFromRGB + toneMapControlled) on n float4 pixels.
__attribute__((visibility("default"))) int clref_probe_tonemap(const char* hsaco, const float* in, int n, float Lwhite,
                                                               float* out) {
    static cl_program prog = nullptr;
    static cl_kernel k = nullptr;
    cl_int e = 0;
    if (!k) {
        prog = loadProgram(hsaco);
        if (!prog) return -1;
        k = clCreateKernel(prog, "ProbeToneMap", &e);
        if (!ok(e, "kernel ProbeToneMap")) return -2;
    }
    cl_mem bi = buf(16 * (size_t)n, in);
    cl_mem bo = buf(16 * (size_t)n, nullptr);
    e = 0;
    e |= arg(k, 0, bi);
    e |= arg(k, 1, n);
    e |= arg(k, 2, Lwhite);
    e |= arg(k, 3, bo);
    if (!ok(e, "probe tonemap args")) return -4;
    size_t gs = ((size_t)n + 63) / 64 * 64, ls = 64;
    bool good = ok(clEnqueueNDRangeKernel(R.q, k, 1, nullptr, &gs, &ls, 0, nullptr, nullptr), "probe tonemap launch") &&
                ok(clEnqueueReadBuffer(R.q, bo, CL_TRUE, 0, 16 * (size_t)n, out, 0, nullptr, nullptr), "probe tonemap read");
    clReleaseMemObject(bi);
    clReleaseMemObject(bo);
    return good ? 0 : -5;
}

// ---------------------------------------------------------------------------
// BDPT (RTBDPTPass::update, RTBDPTPass.cpp:67-128; kernels BDPT.cl:240-932)
// ---------------------------------------------------------------------------
static const size_t kVertexBytes = 240;   // sizeof(RTBDPTVertex), kernel_data.h:220-244
static int maxConnections(int D) { const int t = D + 2; return t * (t + 1) / 2 - 2; }   // RTBDPTPass.cpp:404-408

static bool ensureBdptBuffers(Scene* s, int W, int H, int D) {
    if (s->bW == W && s->bH == H && s->bD == D) return true;
    cl_mem* old[] = {&s->bFinal, &s->bRadiance, &s->camV, &s->lightV, &s->camRays, &s->camIsect, &s->camThr,
                     &s->camPdf, &s->camCnt, &s->lightRays, &s->lightIsect, &s->lightThr, &s->lightPdf, &s->lightCnt,
                     &s->connRays, &s->connVis, &s->sampCamV, &s->sampLightV, &s->bTemp, &s->bStack, &s->bCount,
                     &s->bConnCount};
    for (auto* m : old)
        if (*m) clReleaseMemObject(*m), *m = nullptr;
    const size_t N = (size_t)W * H, C = (size_t)maxConnections(D);
    // All buffers start zero-filled (buf()); the reference allocates them uninitialised.
    s->bRadiance = buf(16 * N, nullptr);
    s->bFinal = buf(12 * N, nullptr);
    s->camV = buf(kVertexBytes * N * (D + 2), nullptr);
    s->lightV = buf(kVertexBytes * N * (D + 1), nullptr);
    s->camRays = buf(48 * N, nullptr);
    s->camIsect = buf(32 * N, nullptr);
    s->camThr = buf(16 * N, nullptr);
    s->camPdf = buf(4 * N, nullptr);
    s->camCnt = buf(4 * N, nullptr);
    s->lightRays = buf(48 * N, nullptr);
    s->lightIsect = buf(32 * N, nullptr);
    s->lightThr = buf(16 * N, nullptr);
    s->lightPdf = buf(4 * N, nullptr);
    s->lightCnt = buf(4 * N, nullptr);
    s->connRays = buf(48 * N * C, nullptr);
    s->connVis = buf(4 * N * C, nullptr);
    s->sampCamV = buf(kVertexBytes * N * D, nullptr);
    s->sampLightV = buf(kVertexBytes * N * D, nullptr);
    s->bTemp = buf(16 * N * C, nullptr);
    s->bStack = buf(4 * N * C * 64, nullptr);
    int n = (int)N, nc = (int)(N * C);
    s->bCount = buf(4, &n);
    s->bConnCount = buf(4, &nc);
    s->bW = W;
    s->bH = H;
    s->bD = D;
    return s->bStack && s->connRays && s->camV;
}

static bool launchRRn(cl_kernel k, Scene* s, cl_mem rays, cl_mem out, cl_mem count, int n) {
    if (s->twoLevel) return launchRR2(k, s, rays, out, count, n);
    cl_int e = 0;
    e |= arg(k, 0, s->nodes);
    e |= arg(k, 1, rays);
    e |= arg(k, 2, count);
    e |= arg(k, 3, s->bStack);
    e |= arg(k, 4, out);
    if (!ok(e, "set RR args")) return false;
    size_t gs = (size_t)(n + 63) / 64 * 64, ls = 64;
    return ok(clEnqueueNDRangeKernel(R.q, k, 1, nullptr, &gs, &ls, 0, nullptr, nullptr), "launchRR") &&
           ok(clFinish(R.q), "clFinish");
}

// One BDPT frame; radiance_out: W*H float4 (the pass's "RadianceBufferCL" after CopyBuffer).
__attribute__((visibility("default"))) int clref_bdpt_render(void* sp, const mcrt_camera* cam, int frame, int maxDepth,
                                                             float* radiance_out) {
    Scene* s = (Scene*)sp;
    const int W = (int)cam->width, H = (int)cam->height, N = W * H;
    if (!ensureBdptBuffers(s, W, H, maxDepth)) return -1;
    if (!ok(clEnqueueWriteBuffer(R.q, s->camera, CL_TRUE, 0, sizeof(mcrt_camera), cam, 0, nullptr, nullptr), "camera"))
        return -1;
    cl_int e = 0;
    int a = 0;
    // generateStartVertices (RTBDPTPass.cpp:130-221)
    if (!setSceneArgs(R.kBStart, s, a)) return -2;
    e |= arg(R.kBStart, a++, W);
    e |= arg(R.kBStart, a++, H);
    e |= arg(R.kBStart, a++, frame);
    e |= arg(R.kBStart, a++, maxDepth);
    e |= arg(R.kBStart, a++, s->camV);
    e |= arg(R.kBStart, a++, s->camRays);
    e |= arg(R.kBStart, a++, s->camThr);
    e |= arg(R.kBStart, a++, s->camPdf);
    e |= arg(R.kBStart, a++, s->camCnt);
    e |= arg(R.kBStart, a++, s->lightV);
    e |= arg(R.kBStart, a++, s->lightRays);
    e |= arg(R.kBStart, a++, s->lightThr);
    e |= arg(R.kBStart, a++, s->lightPdf);
    e |= arg(R.kBStart, a++, s->lightCnt);
    e |= arg(R.kBStart, a++, s->bFinal);
    if (!ok(e, "start args") || !launch2D(R.kBStart, W, H)) return -2;
    if (!launchRRn(R.kIsect, s, s->camRays, s->camIsect, s->bCount, N)) return -3;
    if (!launchRRn(R.kIsect, s, s->lightRays, s->lightIsect, s->bCount, N)) return -3;
    // generateSecondaryVertices (RTBDPTPass.cpp:223-307)
    a = 0;
    if (!setSceneArgs(R.kBSec, s, a)) return -4;
    e = 0;
    e |= arg(R.kBSec, a++, W);
    e |= arg(R.kBSec, a++, H);
    e |= arg(R.kBSec, a++, frame);
    e |= arg(R.kBSec, a++, maxDepth);
    const int pathArg = a;
    if (!ok(e, "secondary args")) return -4;
    for (int depth = 1; depth <= maxDepth + 1; ++depth) {
        for (int isCam = 1; isCam >= 0; --isCam) {
            if (!isCam && depth > maxDepth) continue;
            a = pathArg;
            e = 0;
            e |= arg(R.kBSec, a++, isCam);
            e |= arg(R.kBSec, a++, isCam ? s->camV : s->lightV);
            e |= arg(R.kBSec, a++, isCam ? s->camRays : s->lightRays);
            e |= arg(R.kBSec, a++, isCam ? s->camIsect : s->lightIsect);
            e |= arg(R.kBSec, a++, isCam ? s->camThr : s->lightThr);
            e |= arg(R.kBSec, a++, isCam ? s->camPdf : s->lightPdf);
            e |= arg(R.kBSec, a++, isCam ? s->camCnt : s->lightCnt);
            e |= arg(R.kBSec, a++, depth);
            if (!ok(e, "secondary path args") || !launch2D(R.kBSec, W, H)) return -5;
        }
        if (!launchRRn(R.kIsect, s, s->camRays, s->camIsect, s->bCount, N)) return -6;
        if (depth <= maxDepth && !launchRRn(R.kIsect, s, s->lightRays, s->lightIsect, s->bCount, N)) return -6;
    }
    // prepareVertexConnections (RTBDPTPass.cpp:309-359)
    a = 0;
    if (!setSceneArgs(R.kBPrep, s, a)) return -7;
    e = 0;
    e |= arg(R.kBPrep, a++, W);
    e |= arg(R.kBPrep, a++, H);
    e |= arg(R.kBPrep, a++, frame);
    e |= arg(R.kBPrep, a++, maxDepth);
    e |= arg(R.kBPrep, a++, s->camV);
    e |= arg(R.kBPrep, a++, s->lightV);
    e |= arg(R.kBPrep, a++, s->sampCamV);
    e |= arg(R.kBPrep, a++, s->sampLightV);
    e |= arg(R.kBPrep, a++, s->connRays);
    e |= arg(R.kBPrep, a++, s->camCnt);
    e |= arg(R.kBPrep, a++, s->lightCnt);
    e |= arg(R.kBPrep, a++, s->bTemp);
    if (!ok(e, "prepare args") || !launch2D(R.kBPrep, W, H)) return -7;
    const int NC = N * maxConnections(maxDepth);
    if (!launchRRn(R.kOccl, s, s->connRays, s->connVis, s->bConnCount, NC)) return -8;
    // makeConnections (RTBDPTPass.cpp:361-402)
    a = 0;
    if (!setSceneArgs(R.kBConn, s, a)) return -9;
    e = 0;
    e |= arg(R.kBConn, a++, W);
    e |= arg(R.kBConn, a++, H);
    e |= arg(R.kBConn, a++, frame);
    e |= arg(R.kBConn, a++, maxDepth);
    e |= arg(R.kBConn, a++, s->camV);
    e |= arg(R.kBConn, a++, s->lightV);
    e |= arg(R.kBConn, a++, s->sampCamV);
    e |= arg(R.kBConn, a++, s->sampLightV);
    e |= arg(R.kBConn, a++, s->connRays);
    e |= arg(R.kBConn, a++, s->connVis);
    e |= arg(R.kBConn, a++, s->camCnt);
    e |= arg(R.kBConn, a++, s->lightCnt);
    e |= arg(R.kBConn, a++, s->bTemp);
    e |= arg(R.kBConn, a++, s->bFinal);
    if (!ok(e, "connect args") || !launch2D(R.kBConn, W, H)) return -9;
    // copyRadianceBuffer (RTBDPTPass.cpp:410-440)
    e = 0;
    e |= arg(R.kBCopy, 0, W);
    e |= arg(R.kBCopy, 1, H);
    e |= arg(R.kBCopy, 2, s->bFinal);
    e |= arg(R.kBCopy, 3, s->bRadiance);
    if (!ok(e, "copy args") || !launch2D(R.kBCopy, W, H)) return -10;
    if (radiance_out &&
        !ok(clEnqueueReadBuffer(R.q, s->bRadiance, CL_TRUE, 0, 16ull * N, radiance_out, 0, nullptr, nullptr), "read"))
        return -11;
    return 0;
}

// Debug read-back of the last BDPT frame: which 0 camera vertices (240 B x (D+2) per pixel),
// 1 light vertices (240 B x (D+1)), 2 camera vertex counts (int), 3 light vertex counts (int),
// 4 connection rays (48 B x C per pixel), 5 connection visibilities (int x C), 6 temp radiance
// (float4 x C), 7 sampled light vertices (240 B x D), 8 sampled camera vertices (240 B x D).
__attribute__((visibility("default"))) int64_t clref_bdpt_read(void* sp, int which, void* out) {
    Scene* s = (Scene*)sp;
    const size_t N = (size_t)s->bW * s->bH, C = (size_t)maxConnections(s->bD), D = (size_t)s->bD;
    cl_mem m[9] = {s->camV, s->lightV, s->camCnt, s->lightCnt, s->connRays, s->connVis, s->bTemp, s->sampLightV,
                   s->sampCamV};
    size_t sz[9] = {kVertexBytes * N * (D + 2), kVertexBytes * N * (D + 1), 4 * N, 4 * N, 48 * N * C, 4 * N * C,
                    16 * N * C, kVertexBytes * N * D, kVertexBytes * N * D};
    if (which < 0 || which > 8 || !m[which]) { g_err = "clref_bdpt_read: bad buffer"; return -1; }
    if (!out) return (int64_t)sz[which];
    return ok(clEnqueueReadBuffer(R.q, m[which], CL_TRUE, 0, sz[which], out, 0, nullptr, nullptr), "read")
               ? (int64_t)sz[which] : -2;
}

}  // extern "C"

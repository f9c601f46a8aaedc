// The multi-GPU end of job from a C++ host: the reference host's passes (which have no Python;
// RTReconstructionPass.cpp:71-123 is where the single reduce sits, RTBDPTPass.cpp:410-440 where
// BDPT's splats are resolved) driving the C ABI and RCCL directly, as INTEGRATION.md "Multi-GPU"
// prescribes:
//
//   PT:   every band renders its rows (mcrt_frame_params band_rows/num_bands/band_index) and
//         accumulates -> mcrt_framebuffer_bands_pack on the context stream -> ONE gather as
//         ncclGroupStart / ncclSend / ncclRecv / ncclGroupEnd on that stream ->
//         mcrt_framebuffer_bands_unpack on the gathering rank (image = the 1-GPU image bit for bit);
//   BDPT: per frame mcrt_bdpt_splats_copy (rank-major, on the frame's stream) -> ONE
//         ncclReduceScatter -> mcrt_bdpt_gather -> accumulate; the same band gather at the end.
//
// One process per GPU (device = rank % visible devices), `world` ranks, communicator from a unique
// id that rank 0 writes to ID_FILE.  Each process renders `bands / world` consecutive band indices
// (rank-major: rank r owns bands r*per .. r*per+per-1), each in its own frame buffer: per = 1 is the
// deployment shape; per > 1 lets a single GPU with a 1-rank communicator run the whole exchange
// through RCCL (self sends / receives; the reduce-scatter sums the process's bands first, as a
// host with several bands per GPU would).  Rank 0 also renders the whole image on one frame
// buffer (no split) for the comparison.
//
// usage: capi_rccl SCENE_DIR OUT_DIR frames max_depth bands [world rank ID_FILE]
//   OUT_DIR (rank 0): pt_plain.bin, pt_split.bin, bdpt_plain.bin, bdpt_split.bin (RGBA32F images);
//   one JSON line on stdout.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <unistd.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "consumer_util.h"
#include "mcrt_capi.h"

namespace {

using consumer::check;
using consumer::hipCheck;
using consumer::save;

inline void ncclCheck(ncclResult_t r) {
    if (r != ncclSuccess) throw std::runtime_error(std::string("RCCL: ") + ncclGetErrorString(r));
}

// The local pre-sum of a process's rank-major splat buffers (only with several bands per process).
__global__ void k_add(float* __restrict__ a, const float* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] += b[i];
}

ncclUniqueId shareId(int rank, const std::string& path) {
    ncclUniqueId id;
    if (rank == 0) {
        ncclCheck(ncclGetUniqueId(&id));
        const std::string tmp = path + ".tmp";
        consumer::save(tmp, reinterpret_cast<const char*>(&id), sizeof(id));
        if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("cannot publish the RCCL id");
        return id;
    }
    for (int i = 0; i < 6000; ++i) {   // up to 60 s for rank 0
        auto v = consumer::load<char>(path);
        if (v.size() == sizeof(id)) {
            std::memcpy(&id, v.data(), sizeof(id));
            return id;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(10));
    }
    throw std::runtime_error("timed out waiting for rank 0's RCCL id");
}

mcrt_frame_params params(int frame, int maxDepth, int integrator, int bands, int band) {
    mcrt_frame_params p = {};
    p.frame_index = frame;
    p.max_depth = maxDepth;
    p.sampler = MCRT_SAMPLER_RANDOM;
    p.integrator = integrator;
    p.band_rows = 8;
    p.num_bands = bands;
    p.band_index = band;
    return p;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 6) {
        std::fprintf(stderr, "usage: %s SCENE_DIR OUT_DIR frames max_depth bands [world rank ID_FILE]\n", argv[0]);
        return 2;
    }
    const std::string in = argv[1], out = argv[2];
    const int frames = std::atoi(argv[3]), maxDepth = std::atoi(argv[4]), bands = std::atoi(argv[5]);
    const int world = argc > 6 ? std::atoi(argv[6]) : 1, rank = argc > 7 ? std::atoi(argv[7]) : 0;
    const std::string idFile = argc > 8 ? argv[8] : out + "/rccl.id";
    if (world < 1 || rank < 0 || rank >= world || bands < world || bands % world != 0 || frames < 1) {
        std::fprintf(stderr, "capi_rccl: need 0 <= rank < world, bands a multiple of world, frames >= 1\n");
        return 2;
    }
    const int per = bands / world;
    mcrt_ctx ctx = nullptr;
    ncclComm_t comm = nullptr;
    try {
        int ndev = 0;
        hipCheck(hipGetDeviceCount(&ndev));
        const int dev = rank % ndev;
        hipCheck(hipSetDevice(dev));
        const ncclUniqueId id = shareId(rank, idFile);
        ncclCheck(ncclCommInitRank(&comm, world, id, rank));
        check(mcrt_ctx_create(dev, &ctx), nullptr);
        void* stv = nullptr;
        check(mcrt_ctx_get_stream(ctx, &stv), ctx);
        hipStream_t st = static_cast<hipStream_t>(stv);   // accumulate, pack, unpack and the collectives

        // ---- RTScene::commit ------------------------------------------------------------------
        const consumer::SceneFiles files(in);
        if (files.camera.size() != 1 || files.shapes.empty()) throw std::runtime_error("bad scene directory");
        const mcrt_scene_desc d = files.desc();
        mcrt_scene scene = nullptr;
        check(mcrt_scene_create(ctx, &d, &scene), ctx);
        mcrt_accel_opts o = {10.0f, 64, 1};
        check(mcrt_accel_build(scene, &o), ctx);
        const mcrt_camera cam = files.camera[0];
        const size_t N = (size_t)cam.width * cam.height;
        mcrt_filter filt = {};
        filt.filterType = MCRT_BOX_FILTER;
        filt.radius.x = filt.radius.y = 2.0f;

        std::vector<float> img(4 * N);
        int ptIdentical = -1;
        double bdptMaxRel = -1.0;
        for (int integrator : {MCRT_INTEGRATOR_PT, MCRT_INTEGRATOR_BDPT}) {
            const char* tag = integrator == MCRT_INTEGRATOR_PT ? "pt" : "bdpt";
            // ---- rank 0: the whole image on one frame buffer (the comparison) ----------------
            std::vector<float> plain(4 * N);
            if (rank == 0) {
                mcrt_framebuffer fb = nullptr;
                check(mcrt_framebuffer_create(ctx, cam.width, cam.height, &fb), ctx);
                for (int f = 0; f < frames; ++f) {
                    const mcrt_frame_params p = params(f, maxDepth, integrator, 1, 0);
                    check(mcrt_render_frame(scene, fb, &cam, &p), ctx);
                    check(mcrt_accumulate(fb, &filt, f), ctx);
                }
                check(mcrt_framebuffer_read(fb, 2, plain.data()), ctx);
                save(out + "/" + tag + "_plain.bin", plain.data(), 4 * N);
                check(mcrt_framebuffer_destroy(fb), ctx);
            }
            // ---- this process's bands ----------------------------------------------------------
            std::vector<mcrt_framebuffer> fbs(per, nullptr);
            for (auto& fb : fbs) check(mcrt_framebuffer_create(ctx, cam.width, cam.height, &fb), ctx);
            float* dFull = nullptr;   // BDPT: per band, the rank-major splats (bands chunks)
            float* dOwn = nullptr;    // BDPT: this rank's chunks of the sum (per chunks)
            size_t cp4 = 0;           // floats of one chunk
            std::vector<hipEvent_t> ev(per + 1, nullptr);
            for (auto& e : ev) hipCheck(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            for (int f = 0; f < frames; ++f) {
                for (int j = 0; j < per; ++j) {
                    const mcrt_frame_params p = params(f, maxDepth, integrator, bands, rank * per + j);
                    check(mcrt_render_frame(scene, fbs[j], &cam, &p), ctx);
                }
                if (integrator == MCRT_INTEGRATOR_BDPT) {
                    uint64_t chunkPixels = 0;
                    int32_t chunks = 0;
                    check(mcrt_bdpt_splat_layout(fbs[0], &chunkPixels, &chunks), ctx);
                    if (chunks != bands) throw std::runtime_error("splat layout: chunks != bands");
                    if (!dFull) {
                        cp4 = MCRT_SPLAT_CHANNELS * (size_t)chunkPixels;
                        hipCheck(hipMalloc(&dFull, sizeof(float) * cp4 * bands * per));
                        hipCheck(hipMalloc(&dOwn, sizeof(float) * cp4 * per));
                    }
                    // each band's splats, rank-major, on its frame's stream; the collective's stream
                    // waits for them (events, no host synchronisation)
                    for (int j = 0; j < per; ++j) {
                        void* fst = nullptr;
                        check(mcrt_framebuffer_stream(fbs[j], &fst), ctx);
                        // the previous frame's reduce-scatter has read dFull (ev[per]; a no-op before
                        // the first); its gathers have read dOwn (splats_copy waits for those itself)
                        hipCheck(hipStreamWaitEvent(static_cast<hipStream_t>(fst), ev[per], 0));
                        check(mcrt_bdpt_splats_copy(fbs[j], dFull + (size_t)j * cp4 * bands), ctx);
                        hipCheck(hipEventRecord(ev[j], static_cast<hipStream_t>(fst)));
                        hipCheck(hipStreamWaitEvent(st, ev[j], 0));
                    }
                    for (int j = 1; j < per; ++j)
                        k_add<<<1024, 256, 0, st>>>(dFull, dFull + (size_t)j * cp4 * bands, cp4 * bands);
                    hipCheck(hipGetLastError());
                    // ONE reduce-scatter: rank r receives the sums of chunks r*per .. r*per+per-1
                    ncclCheck(ncclReduceScatter(dFull, dOwn, cp4 * per, ncclFloat, ncclSum, comm, st));
                    hipCheck(hipEventRecord(ev[per], st));
                    for (int j = 0; j < per; ++j) {
                        void* fst = nullptr;
                        check(mcrt_framebuffer_stream(fbs[j], &fst), ctx);
                        hipCheck(hipStreamWaitEvent(static_cast<hipStream_t>(fst), ev[per], 0));
                        check(mcrt_bdpt_gather(fbs[j], dOwn + (size_t)j * cp4), ctx);
                    }
                }
                for (int j = 0; j < per; ++j) check(mcrt_accumulate(fbs[j], &filt, f), ctx);
            }
            // ---- end of job: ONE gather of the bands' packed rows to rank 0 -------------------
            int32_t maxRows = 0, nb = 0, bi = 0;
            check(mcrt_framebuffer_band_layout(fbs[0], &maxRows, &nb, &bi), ctx);
            if (nb != bands || bi != rank * per) throw std::runtime_error("band layout mismatch");
            const size_t n = (size_t)maxRows * 5 * cam.width;   // floats of one band's packed rows
            float* dSend = nullptr;
            float* dRecv = nullptr;
            hipCheck(hipMalloc(&dSend, sizeof(float) * n * per));
            if (rank == 0) hipCheck(hipMalloc(&dRecv, sizeof(float) * n * bands));
            for (int j = 0; j < per; ++j) check(mcrt_framebuffer_bands_pack(fbs[j], dSend + (size_t)j * n), ctx);
            ncclCheck(ncclGroupStart());
            for (int j = 0; j < per; ++j) ncclCheck(ncclSend(dSend + (size_t)j * n, n, ncclFloat, 0, comm, st));
            if (rank == 0)
                for (int b = 0; b < bands; ++b)   // band b comes from rank b / per, in its band order
                    ncclCheck(ncclRecv(dRecv + (size_t)b * n, n, ncclFloat, b / per, comm, st));
            ncclCheck(ncclGroupEnd());
            if (rank == 0) {
                check(mcrt_framebuffer_bands_unpack(fbs[0], dRecv, maxRows), ctx);   // fbs[0] = band 0
                check(mcrt_framebuffer_read(fbs[0], 2, img.data()), ctx);
                save(out + "/" + tag + "_split.bin", img.data(), 4 * N);
                if (integrator == MCRT_INTEGRATOR_PT) {
                    ptIdentical = std::memcmp(img.data(), plain.data(), sizeof(float) * 4 * N) == 0 ? 1 : 0;
                } else {
                    bdptMaxRel = 0.0;
                    for (size_t i = 0; i < 4 * N; ++i)
                        bdptMaxRel = std::max(bdptMaxRel, std::fabs((double)img[i] - plain[i]) /
                                                              std::max(1.0, std::fabs((double)plain[i])));
                }
            }
            check(mcrt_ctx_synchronize(ctx), ctx);
            (void)hipFree(dSend);
            if (dRecv) (void)hipFree(dRecv);
            if (dFull) (void)hipFree(dFull);
            if (dOwn) (void)hipFree(dOwn);
            for (auto& e : ev) (void)hipEventDestroy(e);
            for (auto& fb : fbs) check(mcrt_framebuffer_destroy(fb), ctx);
        }
        if (rank == 0) {
            int ver = 0;
            ncclCheck(ncclGetVersion(&ver));
            std::printf("{\"pixels\": %zu, \"world\": %d, \"bands\": %d, \"pt_identical\": %d, "
                        "\"bdpt_max_rel\": %.3e, \"rccl_version\": %d}\n",
                        N, world, bands, ptIdentical, bdptMaxRel, ver);
        }
        check(mcrt_scene_destroy(scene), ctx);
        check(mcrt_ctx_destroy(ctx), nullptr);
        ncclCheck(ncclCommDestroy(comm));
    } catch (const std::exception& e) {
        std::fprintf(stderr, "capi_rccl (rank %d): %s\n", rank, e.what());
        if (ctx) mcrt_ctx_destroy(ctx);
        if (comm) ncclCommAbort(comm);
        return 1;
    }
    return 0;
}

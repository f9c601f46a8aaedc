// A compiled C++ consumer of include/mcrt_capi.h that replays INTEGRATION.md's reference-side
// code: RTScene::commit (RTScene.cpp:199-244) -> mcrt_scene_create + mcrt_accel_build;
// RTPrimaryRaysPass (RTPrimaryRaysPass.cpp:32-67) -> 48-B rays in hipMalloc'd memory traced with
// mcrt_trace_closest / mcrt_trace_any where g_isectApi->QueryIntersection / QueryOcclusion are
// called; RTPathTracingPass::update (RTPathTracingPass.cpp:40-114) -> mcrt_render_frame;
// RTReconstructionPass::updateReconstruction (RTReconstructionPass.cpp:71-123) -> mcrt_accumulate
// + mcrt_framebuffer_read; errors surface through check() as std::runtime_error, which the passes
// already catch (RTPathTracingPass.cpp:89-104).
//
// usage: capi_consumer SCENE_DIR OUT_DIR frames max_depth
//   SCENE_DIR: raw little-endian arrays written by tests/test_gpu_capi_consumer.py
//   OUT_DIR:   rays.bin, hits.bin, occl.bin, radiance.bin (last frame), image.bin; one JSON line on stdout
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "consumer_util.h"
#include "mcrt_capi.h"

namespace {

using consumer::check;
using consumer::hipCheck;
using consumer::load;
using consumer::save;

// GeneratePerspectiveRays (PathTracing.cl:13-35) on the host: d = normalize(mix(mix(r00, r10, u),
// mix(r01, r11, u), v)), u = x / W, v = y / H; tmax 1000; active, mask -1
void perspectiveRays(const mcrt_camera& cam, std::vector<mcrt_ray>& rays) {
    const uint32_t W = cam.width, H = cam.height;
    rays.assign((size_t)W * H, mcrt_ray{});
    auto mix = [](float a, float b, float t) { return a + (b - a) * t; };
    for (uint32_t y = 0; y < H; ++y)
        for (uint32_t x = 0; x < W; ++x) {
            const float u = (float)x / (float)W, v = (float)y / (float)H;
            float d[3];
            const float* r00 = &cam.r00.x; const float* r10 = &cam.r10.x;
            const float* r01 = &cam.r01.x; const float* r11 = &cam.r11.x;
            for (int k = 0; k < 3; ++k) d[k] = mix(mix(r00[k], r10[k], u), mix(r01[k], r11[k], u), v);
            const float l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            mcrt_ray& r = rays[(size_t)y * W + x];
            r.o = cam.pos;
            r.o.w = 1000.0f;
            r.d.x = d[0] / l; r.d.y = d[1] / l; r.d.z = d[2] / l; r.d.w = 0.0f;
            r.extra[0] = -1;
            r.extra[1] = (x + y) % 7 == 3 ? 0 : 1;   // a few inactive rays: their records stay untouched
        }
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s SCENE_DIR OUT_DIR frames max_depth [OBJ_FILE]\n", argv[0]);
        return 2;
    }
    const std::string in = argv[1], out = argv[2];
    const int frames = std::atoi(argv[3]), maxDepth = std::atoi(argv[4]);
    mcrt_ctx ctx = nullptr;
    int caught = 0;
    try {
        check(mcrt_ctx_create(0, &ctx), nullptr);
        // ---- AssetImporter + RTScene (optional): an OBJ file through mcrt_obj_load ------------
        mcrt_obj_scene objScene = nullptr;
        if (argc > 5) {
            check(mcrt_obj_load(argv[5], MCRT_OBJ_MIPS | MCRT_OBJ_EMISSIVE_LIGHTS, &objScene), ctx);
            auto sun = load<float>(in + "/sun.bin");   // direction xyz, intensity rgb
            if (sun.size() == 6) check(mcrt_obj_add_directional_light(objScene, &sun[0], &sun[3]), ctx);
        }
        // ---- RTScene::commit ------------------------------------------------------------------
        const consumer::SceneFiles files(in);
        const auto& camv = files.camera;
        if (camv.size() != 1 || (files.shapes.empty() && !objScene)) throw std::runtime_error("bad scene directory");
        mcrt_scene_desc d = files.desc();
        if (objScene) {
            check(mcrt_obj_scene_desc(objScene, &d), ctx);
            d.sobol_matrices = files.sobol.empty() ? nullptr : files.sobol.data();
            d.num_sobol_words = (uint32_t)files.sobol.size();
        }
        mcrt_scene scene = nullptr;
        check(mcrt_scene_create(ctx, &d, &scene), ctx);
        if (objScene) mcrt_obj_free(objScene);   // the scene holds device copies
        mcrt_accel_opts o = {10.0f, 64, 1};       // RTScene::commit: SAH, 64 bins, cost 10 (rest zero)
        check(mcrt_accel_build(scene, &o), ctx);
        const mcrt_camera cam = camv[0];
        const size_t N = (size_t)cam.width * cam.height;

        // ---- RTPrimaryRaysPass with the RadeonRays queries swapped ---------------------------
        std::vector<mcrt_ray> rays;
        perspectiveRays(cam, rays);
        mcrt_ray* dRays = nullptr;
        mcrt_intersection* dHits = nullptr;
        int32_t* dOccl = nullptr;
        hipCheck(hipMalloc(&dRays, sizeof(mcrt_ray) * N));
        hipCheck(hipMalloc(&dHits, sizeof(mcrt_intersection) * N));
        hipCheck(hipMalloc(&dOccl, sizeof(int32_t) * N));
        hipCheck(hipMemcpy(dRays, rays.data(), sizeof(mcrt_ray) * N, hipMemcpyHostToDevice));
        hipCheck(hipMemset(dHits, 0xff, sizeof(mcrt_intersection) * N));   // sentinel: -1 bytes
        hipCheck(hipMemset(dOccl, 0x7f, sizeof(int32_t) * N));
        check(mcrt_trace_closest(scene, dRays, (int32_t)N, dHits), ctx);    // g_isectApi->QueryIntersection
        check(mcrt_trace_any(scene, dRays, (int32_t)N, dOccl), ctx);        // g_isectApi->QueryOcclusion
        check(mcrt_ctx_synchronize(ctx), ctx);
        std::vector<mcrt_intersection> hits(N);
        std::vector<int32_t> occl(N);
        hipCheck(hipMemcpy(hits.data(), dHits, sizeof(mcrt_intersection) * N, hipMemcpyDeviceToHost));
        hipCheck(hipMemcpy(occl.data(), dOccl, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
        size_t nhit = 0;
        for (auto& h : hits) nhit += h.shapeid >= 0;

        // ---- the device-count queries (QueryIntersection / QueryOcclusion with numrays in remote
        // memory and events, radeon_rays.h:272-277): k = N/2 + 37 rays of a grid for N; the second
        // query waits for the first's event; records past k stay untouched -------------------------
        int countMatch = 1;
        {
            const int32_t k = (int32_t)(N / 2 + 37);
            int32_t* dCount = nullptr;
            hipCheck(hipMalloc(&dCount, sizeof(int32_t)));
            hipCheck(hipMemcpy(dCount, &k, sizeof(int32_t), hipMemcpyHostToDevice));
            hipCheck(hipMemset(dHits, 0xff, sizeof(mcrt_intersection) * N));
            hipCheck(hipMemset(dOccl, 0x7f, sizeof(int32_t) * N));
            mcrt_event e1 = nullptr, e2 = nullptr;
            check(mcrt_trace_closest_count(scene, dRays, dCount, (int32_t)N, dHits, nullptr, &e1), ctx);
            check(mcrt_trace_any_count(scene, dRays, dCount, (int32_t)N, dOccl, e1, &e2), ctx);
            check(mcrt_event_wait(e2), ctx);
            std::vector<mcrt_intersection> h2(N);
            std::vector<int32_t> o2(N);
            hipCheck(hipMemcpy(h2.data(), dHits, sizeof(mcrt_intersection) * N, hipMemcpyDeviceToHost));
            hipCheck(hipMemcpy(o2.data(), dOccl, sizeof(int32_t) * N, hipMemcpyDeviceToHost));
            for (size_t i = 0; i < N; ++i) {
                mcrt_intersection sentinel;
                std::memset(&sentinel, 0xff, sizeof(sentinel));
                const bool in = (int32_t)i < k;
                if (std::memcmp(&h2[i], in ? &hits[i] : &sentinel, sizeof(mcrt_intersection)) != 0) countMatch = 0;
                if (o2[i] != (in ? occl[i] : 0x7f7f7f7f)) countMatch = 0;
            }
            check(mcrt_event_destroy(e1), ctx);
            check(mcrt_event_destroy(e2), ctx);
            (void)hipFree(dCount);
        }

        // ---- RTPathTracingPass::update + RTReconstructionPass::updateReconstruction ----------
        mcrt_framebuffer fb = nullptr;
        check(mcrt_framebuffer_create(ctx, cam.width, cam.height, &fb), ctx);
        std::vector<float> radiance(4 * N), image(4 * N);
        for (int frame = 0; frame < frames; ++frame) {
            mcrt_frame_params p = {};
            p.frame_index = frame;
            p.max_depth = maxDepth;
            p.sampler = MCRT_SAMPLER_RANDOM;       // RT_SAMPLER in samplers.cl
            p.band_rows = 8; p.num_bands = 1; p.band_index = 0;
            check(mcrt_render_frame(scene, fb, &cam, &p), ctx);
            mcrt_filter f = {};                    // explicit 56-B device layout
            f.filterType = MCRT_BOX_FILTER;
            f.radius.x = 2.0f; f.radius.y = 2.0f;
            check(mcrt_accumulate(fb, &f, frame), ctx);
        }
        check(mcrt_framebuffer_read(fb, 0, radiance.data()), ctx);
        check(mcrt_framebuffer_read(fb, 2, image.data()), ctx);   // upload to the GL texture as before

        // ---- the error path the passes rely on -------------------------------------------------
        try {
            mcrt_frame_params bad = {};
            bad.max_depth = 0;                       // invalid
            check(mcrt_render_frame(scene, fb, &cam, &bad), ctx);
        } catch (const std::runtime_error& e) {
            caught = std::strlen(e.what()) > 0 ? 1 : 0;
        }

        save(out + "/rays.bin", rays.data(), N);
        save(out + "/hits.bin", hits.data(), N);
        save(out + "/occl.bin", occl.data(), N);
        save(out + "/radiance.bin", radiance.data(), 4 * N);
        save(out + "/image.bin", image.data(), 4 * N);
        double mean = 0.0;
        for (size_t i = 0; i < N; ++i) mean += image[4 * i] + image[4 * i + 1] + image[4 * i + 2];
        std::printf("{\"pixels\": %zu, \"closest_hits\": %zu, \"image_mean\": %.6f, \"error_caught\": %d, "
                    "\"count_queries_match\": %d, \"version\": \"%s\"}\n", N, nhit, mean / (3.0 * N), caught,
                    countMatch, mcrt_version());
        check(mcrt_framebuffer_destroy(fb), ctx);
        check(mcrt_scene_destroy(scene), ctx);
        (void)hipFree(dRays);
        (void)hipFree(dHits);
        (void)hipFree(dOccl);
        check(mcrt_ctx_destroy(ctx), nullptr);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "capi_consumer: %s\n", e.what());
        if (ctx) mcrt_ctx_destroy(ctx);
        return 1;
    }
    return 0;
}

// Diagnostics only: the product's shading device functions evaluated for given
// intersections, emitting the same 20 float4 per pixel as oracle/refbuild/clprobe.cl does
// for the reference, so the two can be compared stage by stage (tools/probe/probe.py).
#include "../../monte-carlo-raytracer_amd/csrc/mcrt_kernels.hip"

#define PROBE_STRIDE 20

__global__ void k_probe(SceneArgs s, FrameArgs f, const mcrt_intersection* isects, const float4* dirs, float4* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int)(f.W * f.H)) return;
    const mcrt_intersection isect = isects[i];
    float4* o = out + (size_t)i * PROBE_STRIDE;
    if (isect.shapeid == -1 || isect.primid == -1 || s.numLights <= 0) return;
    auto st = [&](int k, f3 v, float w) { o[k] = make_float4(v.x, v.y, v.z, w); };
    Frame si = computeSurfaceInteraction(s, isect.shapeid, isect.primid, f2{isect.uvwt.x, isect.uvwt.y});
    const f3 wo = -ld3(dirs[i]);
    const bool isBackfacing = cl_dot(si.gn, wo) < 0.0f;
    const float traceErrorOffset = isBackfacing ? -RT_TRACE_OFFSET_F : RT_TRACE_OFFSET_F;
    st(0, si.p, traceErrorOffset);
    st(1, si.gn, 0.f);
    st(2, si.sn, 0.f);
    st(3, si.sdpdu, 0.f);
    st(4, si.sdpdv, 0.f);
    o[5] = make_float4(si.uv.x, si.uv.y, 0.f, 0.f);
    const mcrt_shape& shape = s.shapes[isect.shapeid];
    const int materialId = shape.materialId;
    mcrt_material mat;
    if (materialId != -1) {
        mat = s.materials[materialId];
        if (mat.uber_normalMapId != -1) applyNormalMapping(s, mat.uber_normalMapId, si);
    }
    st(6, si.sn, 0.f);
    st(7, si.sdpdu, 0.f);
    st(8, si.sdpdv, 0.f);
    Sampler sampler = makeSampler(f.sampler, (uint32_t)i, f.frame, 0, f.W, f.H, s.sobol);
    uint32_t lightIdx = (uint32_t)floorf(getSample1D(sampler) * s.numLights);
    lightIdx %= (uint32_t)s.numLights;
    const f2 u = getSample2D(sampler);
    const mcrt_light light = s.lights[lightIdx];
    const LightSample ls = sampleLightLi(s, light, si, traceErrorOffset, u);
    st(9, ls.Li, ls.pdf);
    st(10, ls.wi, (float)lightIdx);
    const float lightPdf = ls.pdf * light.choicePdf;
    f3 L = splat3(0.0f);
    if (materialId != -1) {
        const Uber um = uberProps(s, mat, si.uv);
        st(16, um.Kd, um.eta);
        st(17, um.Ks, um.roughness.x);
        st(18, um.opacity, um.roughness.y);
        o[19] = make_float4(um.Kt.x, um.Kt.y, um.Kt.z, um.Kt.w);
        f3 bsdf = evaluateUberBSDF(um, si, wo, ls.wi);
        st(11, bsdf, 0.f);
        bsdf *= absDot(ls.wi, si.sn);
        st(12, bsdf, lightPdf);
        if (!isNearZero(lightPdf)) L = ls.Li * bsdf / lightPdf;
        const f2 bsdfSample = getSample2D(sampler);
        f3 wn;
        float pdf = 0.0f;
        int sampledType;
        const f3 fs = sampleUberBSDF(um, si, bsdfSample, wo, &wn, &pdf, &sampledType);
        st(14, fs, pdf);
        st(15, wn, (float)sampledType);
    }
    st(13, L, 0.f);
}

extern "C" int probe_shade(const mcrt_scene_desc* d, const void* isects, const float* dirs, int W, int H, int frame,
                           int sampler, float* out) {
    auto up = [](const void* p, size_t bytes) -> void* {
        void* q = nullptr;
        if (!p || bytes == 0) { hipMalloc(&q, 16); return q; }
        hipMalloc(&q, bytes);
        hipMemcpy(q, p, bytes, hipMemcpyHostToDevice);
        return q;
    };
    SceneArgs s{};
    s.shapes = (const mcrt_shape*)up(d->shapes, sizeof(mcrt_shape) * d->num_shapes);
    s.indices = (const uint32_t*)up(d->indices, 4ull * d->num_indices);
    s.positions = (const float4*)up(d->positions, 16ull * d->num_vertices);
    s.uvs = (const float2*)up(d->uvs, 8ull * d->num_vertices);
    s.normals = (const float4*)up(d->normals, 16ull * d->num_vertices);
    s.textures = (const mcrt_texture_desc*)up(d->textures, 16ull * d->num_textures);
    s.texData = (const uint8_t*)up(d->tex_data, d->tex_data_bytes);
    s.sobol = (const uint32_t*)up(d->sobol_matrices, 4ull * d->num_sobol_words);
    s.lights = (const mcrt_light*)up(d->lights, sizeof(mcrt_light) * d->num_lights);
    s.materials = (const mcrt_material*)up(d->materials, sizeof(mcrt_material) * d->num_materials);
    s.numLights = (int)d->num_lights;
    FrameArgs f{};
    f.W = W;
    f.H = H;
    f.frame = frame;
    f.maxDepth = 2;
    f.sampler = sampler;
    const size_t n = (size_t)W * H;
    void* bi = up(isects, 32 * n);
    void* bd = up(dirs, 16 * n);
    void* bo = nullptr;
    hipMalloc(&bo, 320 * n);
    hipMemset(bo, 0, 320 * n);
    hipLaunchKernelGGL(k_probe, dim3((n + 63) / 64), dim3(64), 0, 0, s, f, (const mcrt_intersection*)bi,
                       (const float4*)bd, (float4*)bo);
    const hipError_t e = hipMemcpy(out, bo, 320 * n, hipMemcpyDeviceToHost);
    for (const void* p : {(const void*)s.shapes, (const void*)s.indices, (const void*)s.positions, (const void*)s.uvs,
                          (const void*)s.normals, (const void*)s.textures, (const void*)s.texData,
                          (const void*)s.sobol, (const void*)s.lights, (const void*)s.materials, (const void*)bi,
                          (const void*)bd, (const void*)bo})
        hipFree(const_cast<void*>(p));
    return e == hipSuccess ? 0 : -1;
}

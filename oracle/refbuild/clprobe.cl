// TEST INFRASTRUCTURE ONLY (oracle/refbuild): stage probe over the reference's own OpenCL
// functions, compiled from the reference sources where they lie (-I assets/kernels).
// For each pixel's RTIntersection + incoming direction it records the intermediates of the
// PathTracing kernel (PathTracing.cl:52-184) at bounce 0, so that tools/probe can compare
// the product's device functions with the reference's stage by stage.
#include "PathTracing.cl"

#define PROBE_STRIDE 20

__kernel void ProbeShade(SCENE_PARAMS, int image_width, int image_height, int integrator_frameNum,
                         __global const RTIntersection* isects, __global const float4* dirs,
                         __global RTRay* shadowRays, __global float4* out)
{
    int i = get_global_id(0);
    if (i >= image_width * image_height) return;
    MAKE_SCENE(scene);
    RTIntersection isect = isects[i];
    __global float4* o = out + i * PROBE_STRIDE;
    if (isect.shapeid == -1 || isect.primid == -1 || scene.numLights <= 0) return;
    RTInteraction si = computeSurfaceInteraction(&scene, &isect);
    si.wo = -dirs[i].xyz;
    const bool isBackfacing = dot(si.gn, si.wo) < 0.0f;
    si.traceErrorOffset = isBackfacing ? -RT_TRACE_OFFSET : RT_TRACE_OFFSET;
    o[0] = (float4)(si.p, si.traceErrorOffset);
    o[1] = (float4)(si.gn, 0.0f);
    o[2] = (float4)(si.sn, 0.0f);
    o[3] = (float4)(si.sdpdu, 0.0f);
    o[4] = (float4)(si.sdpdv, 0.0f);
    o[5] = (float4)(si.uv, 0.0f, 0.0f);
    int materialId = scene_shapes[isect.shapeid].materialId;
    applyNormalMapping(&scene, materialId, &si);
    o[6] = (float4)(si.sn, 0.0f);
    o[7] = (float4)(si.sdpdu, 0.0f);
    o[8] = (float4)(si.sdpdv, 0.0f);
    MAKE_SAMPLER(sampler, i, 0);
    float lightPdf = 0.0f;
    uint lightIdx = ((uint)floor(getSample1D(&sampler) * scene.numLights));
    lightIdx %= scene.numLights;
    float3 wi = (float3)(0.0f);
    float2 u = getSample2D(&sampler);
    float3 unusedN, unusedP;
    float3 Li = sampleLightLi(lightIdx, &scene, &si, u, &unusedP, &unusedN, &wi, &lightPdf, shadowRays + i);
    o[9] = (float4)(Li, lightPdf);
    o[10] = (float4)(wi, (float)lightIdx);
    lightPdf *= scene.lights[lightIdx].choicePdf;
    float3 L = (float3)(0.0f);
    if (materialId != RT_INVALID_ID)
    {
        RTUberMaterialProperties um;
        getUberMaterialProperties(&scene, materialId, &si, &um);
        o[16] = (float4)(um.Kd, um.eta);
        o[17] = (float4)(um.Ks, um.roughness.x);
        o[18] = (float4)(um.opacity, um.roughness.y);
        o[19] = um.Kt;
        float3 bsdf = evaluateMaterial(&scene, materialId, si.wo, wi, &si, TRANSPORT_MODE_RADIANCE);
        o[11] = (float4)(bsdf, 0.0f);
        bsdf *= absDot(wi, si.sn);
        o[12] = (float4)(bsdf, lightPdf);
        if (!isNearZero(lightPdf))
            L = Li * bsdf / lightPdf;
        float2 bsdfSample = getSample2D(&sampler);
        float pdf = 0.0f;
        BxDFType sampledType;
        int unused;
        float3 wn;
        float3 f = sampleMaterial(&scene, materialId, &si, bsdfSample, TRANSPORT_MODE_RADIANCE, BSDF_ALL, si.wo, &wn, &pdf, &unused, &sampledType);
        o[14] = (float4)(f, pdf);
        o[15] = (float4)(wn, (float)sampledType);
    }
    o[13] = (float4)(L, 0.0f);
}

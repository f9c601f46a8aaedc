// mcrt_device.h -- device-side math of the MI355X path-tracing core.
//
// Numerics policy (DESIGN.md "Numerics"): the reference's GPU build is OpenCL C compiled by
// ROCm clang with OpenCL-default floating point: contraction only inside one expression
// (FP_CONTRACT ON), 2.5-ulp division, 3-ulp sqrt, and the ROCm device-library builtins
// (dot = fma chain, cross = fma with a negated product, mix = fma, normalize = x * rsqrt with
// range scaling, clamp = med3).  This file reproduces exactly those operation sequences with
// clang ext_vector types (so expressions contract as in OpenCL) and is compiled with
// -ffp-contract=on -fno-hip-fp32-correctly-rounded-divide-sqrt; the HIP path therefore
// computes the same fp32 results as the reference kernels on the same hardware for
// identical inputs (and uses the cheaper division / sqrt sequences).
// Paths: KRN = assets/kernels, RR = third_party/RadeonRays/RadeonRays.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mcrt_capi.h"

#define MCRT_DEV __device__ __forceinline__

typedef float f3 __attribute__((ext_vector_type(3)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

MCRT_DEV f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
MCRT_DEV f3 splat3(float x) { return f3{x, x, x}; }
MCRT_DEV f3 ld3(const mcrt_float4& p) { return f3{p.x, p.y, p.z}; }
MCRT_DEV f3 ld3(const float4& p) { return f3{p.x, p.y, p.z}; }

// ---- OpenCL builtins as implemented by the ROCm device libraries (opencl.bc / ocml.bc) ----
MCRT_DEV float cl_dot(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
MCRT_DEV f3 cl_cross(f3 a, f3 b) {
    return f3{fmaf(a.y, b.z, b.y * -a.z), fmaf(a.z, b.x, b.z * -a.x), fmaf(a.x, b.y, b.x * -a.y)};
}
MCRT_DEV f3 cl_mix(f3 a, f3 b, float t) {
    const f3 d = b - a;
    return f3{fmaf(d.x, t, a.x), fmaf(d.y, t, a.y), fmaf(d.z, t, a.z)};
}
MCRT_DEV float cl_mixf(float a, float b, float t) { return fmaf(b - a, t, a); }
// fp32 division and sqrt exactly as the AMDGPU backend lowers the reference's OpenCL `/`
// (2.5 ulp: frexp / v_rcp / ldexp) and `sqrt` (3 ulp: v_sqrt with range scaling) with fp32
// denormals enabled.  Spelled out with target builtins because compiler transforms (LICM,
// branch merging) may drop the accuracy metadata of a plain `/` and silently switch to the
// correctly rounded sequence -- in the product and in the reference alike, at different sites.
MCRT_DEV float cl_div(float a, float b) {
    const float r = __builtin_amdgcn_rcpf(__builtin_amdgcn_frexp_mantf(b));
    return __builtin_ldexpf(__builtin_amdgcn_frexp_mantf(a) * r,
                            __builtin_amdgcn_frexp_expf(a) - __builtin_amdgcn_frexp_expf(b));
}
MCRT_DEV f2 cl_div(f2 a, float b) { return f2{cl_div(a.x, b), cl_div(a.y, b)}; }
MCRT_DEV f3 cl_div(f3 a, float b) { return f3{cl_div(a.x, b), cl_div(a.y, b), cl_div(a.z, b)}; }
MCRT_DEV f4 cl_div(f4 a, float b) { return f4{cl_div(a.x, b), cl_div(a.y, b), cl_div(a.z, b), cl_div(a.w, b)}; }
MCRT_DEV float cl_sqrt(float x) {
    const bool tiny = x < 0x1.0p-126f;
    return __builtin_ldexpf(__builtin_amdgcn_sqrtf(__builtin_ldexpf(x, tiny ? 32 : 0)), tiny ? -16 : 0);
}
// Correctly rounded division (f32 operands, f64 quotient: exact rounding).  Only where the
// reference's own compiled kernel ends up with a precise fdiv (see evaluateUberBSDF).
MCRT_DEV float cr_div(float a, float b) { return (float)((double)a / (double)b); }
MCRT_DEV f3 cl_normalize(f3 p) {
    if (p.x == 0.0f && p.y == 0.0f && p.z == 0.0f) return p;
    float l2 = cl_dot(p, p);
    if (l2 < 0x1.0p-126f) {
        p = p * 0x1.0p+86f;
        l2 = cl_dot(p, p);
    } else if (l2 == __builtin_inff()) {
        p = p * 0x1.0p-66f;
        l2 = cl_dot(p, p);
        if (l2 == __builtin_inff()) {
            p = f3{__builtin_copysignf(__builtin_isinf(p.x) ? 1.0f : 0.0f, p.x),
                   __builtin_copysignf(__builtin_isinf(p.y) ? 1.0f : 0.0f, p.y),
                   __builtin_copysignf(__builtin_isinf(p.z) ? 1.0f : 0.0f, p.z)};
            l2 = cl_dot(p, p);
        }
    }
    return p * rsqrtf(l2);
}
MCRT_DEV float cl_length(f3 p) {
    const float l2 = cl_dot(p, p);
    if (l2 < 0x1.0p-126f) return cl_sqrt(cl_dot(p * 0x1.0p+86f, p * 0x1.0p+86f)) * 0x1.0p-86f;
    if (l2 == __builtin_inff()) return cl_sqrt(cl_dot(p * 0x1.0p-66f, p * 0x1.0p-66f)) * 0x1.0p+66f;
    return cl_sqrt(l2);
}
MCRT_DEV float cl_distance(f3 a, f3 b) { return cl_length(a - b); }
MCRT_DEV float cl_clamp(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
MCRT_DEV float cl_sign(float x) {
    return __builtin_copysignf((__builtin_isnan(x) || x == 0.0f) ? 0.0f : 1.0f, x);
}

// ---- KRN/math.cl, KRN/matrix.cl ----
#define PI_F 3.14159265359f
#define PI_INV_F 0.31830988618f
#define PI2_F 6.28318530718f
#define PI_DIV_4_F 0.78539816339f
#define PI_DIV_2_F 1.57079632679f
#define RT_TRACE_OFFSET_F 0.00001f
#define RT_MAX_TRACE_F 1000.0f

MCRT_DEV f3 computeOrthogonalVector(f3 n) {   // math.cl:53-66
    if (fabsf(n.z) > 0.0f) {
        float d = cl_sqrt(n.z * n.z + n.x * n.x);
        return f3{cl_div(-n.z, d), 0.0f, cl_div(n.x, d)};
    }
    float d = cl_sqrt(n.y * n.y + n.x * n.x);
    return f3{cl_div(n.y, d), cl_div(-n.x, d), 0.0f};
}
MCRT_DEV float absDot(f3 a, f3 b) { return fabsf(cl_dot(a, b)); }
MCRT_DEV bool isNearZero(float v) { return fabsf(v) < 1e-8f; }
MCRT_DEV bool isNotNearZero(float v) { return fabsf(v) > 1e-8f; }
MCRT_DEV float distanceSquared(f3 p0, f3 p1) { return cl_dot(p0 - p1, p0 - p1); }
MCRT_DEV f3 lerpDirection(f3 d0, f3 d1, f3 d2, f3 d3, float t0, float t1) {   // math.cl:88-91
    return cl_normalize(cl_mix(cl_mix(d0, d1, t0), cl_mix(d3, d2, t0), t1));
}
MCRT_DEV f3 transformVector3(const mcrt_mat4& m, f3 v) {   // matrix.cl:44-51
    f3 r;
    r.x = cl_dot(ld3(m.m0), v);
    r.y = cl_dot(ld3(m.m1), v);
    r.z = cl_dot(ld3(m.m2), v);
    return r;
}
MCRT_DEV f3 transformPoint3(const mcrt_mat4& m, f3 v) {   // matrix.cl:53-60
    f3 r;
    r.x = cl_dot(ld3(m.m0), v) + m.m0.w;
    r.y = cl_dot(ld3(m.m1), v) + m.m1.w;
    r.z = cl_dot(ld3(m.m2), v) + m.m2.w;
    return r;
}

// ---- RNG + samplers: KRN/rng.cl:48-107, KRN/samplers.cl:64-122 ----
MCRT_DEV uint32_t wangHash(uint32_t s) {
    s = (s ^ 61u) ^ (s >> 16);
    s *= 9u;
    s = s ^ (s >> 4);
    s *= 0x27d4eb2du;
    s = s ^ (s >> 15);
    return s;
}
MCRT_DEV uint32_t xorshift(uint32_t& s) {
    s += 2463534242u;
    s ^= (s << 13);
    s ^= (s >> 17);
    s ^= (s << 5);
    return s;
}
struct Sampler {
    uint32_t idx, dim, scramble;
    const uint32_t* mats;   // nullptr => random sampler
};
MCRT_DEV Sampler makeSampler(int kind, uint32_t pix, int frame, int bounce, uint32_t W, uint32_t H, const uint32_t* mats) {
    Sampler s;
    s.dim = 0;
    if (kind == MCRT_SAMPLER_SOBOL) {   // samplers.cl:75-80
        s.idx = pix + (uint32_t)frame * W * H;
        uint32_t seed = wangHash((uint32_t)(frame + 1) * (uint32_t)(bounce + 1));
        s.scramble = xorshift(seed);
        s.mats = mats;
    } else {                             // samplers.cl:83-84
        s.idx = wangHash(pix + (uint32_t)(frame + 1) * W * H * (uint32_t)(bounce + 1));
        s.scramble = 0;
        s.mats = nullptr;
    }
    return s;
}
MCRT_DEV float getSample1D(Sampler& s) {
    if (s.mats) {
        uint32_t v = s.scramble;
        uint32_t idx = s.idx;
        const uint32_t* C = s.mats + s.dim * 52u;
        for (int i = 0; idx != 0; idx >>= 1, ++i)
            if (idx & 1u) v ^= C[i];
        s.dim++;
        return (float)v * 0x1p-32f;
    }
    return (float)xorshift(s.idx) * 0x1p-32f;   // (float)x / 0xffffffff == x * 2^-32 exactly
}
MCRT_DEV f2 getSample2D(Sampler& s) {
    f2 u;
    u.x = getSample1D(s);
    u.y = getSample1D(s);
    return u;
}

MCRT_DEV f2 concentricSampleDisc(f2 u) {   // samplers.cl:169-191
    f2 uOffset = 2.0f * u - f2{1.0f, 1.0f};
    if (u.x < 1e-8f && u.y < 1e-8f) return f2{0.0f, 0.0f};
    float theta, r;
    if (fabsf(uOffset.x) > fabsf(uOffset.y)) {
        r = uOffset.x;
        theta = PI_DIV_4_F * cl_div(uOffset.y, uOffset.x);
    } else {
        r = uOffset.y;
        theta = PI_DIV_2_F - PI_DIV_4_F * cl_div(uOffset.x, uOffset.y);
    }
    return r * f2{cosf(theta), sinf(theta)};
}
MCRT_DEV f3 cosineSampleHemisphere(f2 u) {   // samplers.cl:193-198
    f2 d = concentricSampleDisc(u);
    float y = cl_sqrt(fmaxf(0.0f, 1.0f - d.x * d.x - d.y * d.y));
    return f3{d.x, y, d.y};
}

// ---- Uber BSDF: KRN/bxdfs.cl (shading frame: normal = y, tangent = x, binormal = z) ----
enum : int {
    BSDF_REFLECTION = 1, BSDF_TRANSMISSION = 2, BSDF_DIFFUSE = 4, BSDF_GLOSSY = 8, BSDF_SPECULAR = 16,
    BSDF_SPEC_REFL = 17, BSDF_SPEC_TRANS = 18, BSDF_LAMBERT = 5, BSDF_MF_REFL = 9, BSDF_MF_TRANS = 10,
};
MCRT_DEV float evalCosTheta(f3 w) { return w.y; }
MCRT_DEV float evalCosSqTheta(f3 w) { return w.y * w.y; }
MCRT_DEV float evalAbsCosTheta(f3 w) { return fabsf(w.y); }
MCRT_DEV float evalSinSqTheta(f3 w) { return fmaxf(0.0f, 1.0f - evalCosSqTheta(w)); }
MCRT_DEV float evalSinTheta(f3 w) { return cl_sqrt(evalSinSqTheta(w)); }
MCRT_DEV float evalTanTheta(f3 w) { return cl_div(evalSinTheta(w), evalCosTheta(w)); }
MCRT_DEV float evalTanSqTheta(f3 w) { return cl_div(evalSinSqTheta(w), evalCosSqTheta(w)); }
MCRT_DEV float evalCosPhi(f3 w) {
    float st = evalSinTheta(w);
    return st == 0 ? 1.0f : cl_clamp(cl_div(w.x, st), -1.0f, 1.0f);
}
MCRT_DEV float evalSinPhi(f3 w) {   // bxdfs.cl:35-39: the `evalSinTheta == 0` test is always false
    float st = evalSinTheta(w);
    return cl_clamp(cl_div(w.z, st), -1.0f, 1.0f);
}
MCRT_DEV float evalCosSqPhi(f3 w) { return evalCosPhi(w) * evalCosPhi(w); }
MCRT_DEV float evalSinSqPhi(f3 w) { return evalSinPhi(w) * evalSinPhi(w); }
MCRT_DEV bool isSameHemisphere(f3 a, f3 b) { return a.y * b.y > 0.0f; }
MCRT_DEV bool isBlack(f3 c) { return c.x < 0.000001f && c.y < 0.000001f && c.z < 0.000001f; }
MCRT_DEV bool isNotBlack(f3 c) { return c.x > 0.000001f || c.y > 0.000001f || c.z > 0.000001f; }

MCRT_DEV float evaluateFresnelDielectric(float cosThetaI, float etaI, float etaT) {   // bxdfs.cl:159-190
    cosThetaI = cl_clamp(cosThetaI, -1.0f, 1.0f);
    if (cosThetaI <= 0.0f) {
        float h = etaI;
        etaI = etaT;
        etaT = h;
        cosThetaI = fabsf(cosThetaI);
    }
    float sinThetaI = cl_sqrt(fmaxf(0.0f, 1.0f - cosThetaI * cosThetaI));
    float sinThetaT = cl_div(etaI, etaT) * sinThetaI;
    if (sinThetaT >= 1.0f) return 1.0f;
    float cosThetaT = cl_sqrt(fmaxf(0.0f, 1.0f - sinThetaT * sinThetaT));
    float rparl = cl_div(((etaT * cosThetaI) - (etaI * cosThetaT)), ((etaT * cosThetaI) + (etaI * cosThetaT)));
    float rperp = cl_div(((etaI * cosThetaI) - (etaT * cosThetaT)), ((etaI * cosThetaI) + (etaT * cosThetaT)));
    return (rparl * rparl + rperp * rperp) * 0.5f;
}
MCRT_DEV f3 reflect(f3 wo, f3 n) { return -wo + 2.0f * cl_dot(n, wo) * n; }   // bxdfs.cl:228-231
MCRT_DEV bool refract(f3 wi, f3 n, float eta, f3* wt) {   // bxdfs.cl:233-245
    float cosThetaI = cl_dot(n, wi);
    float sin2ThetaI = fmaxf(0.0f, 1.0f - cosThetaI * cosThetaI);
    float sin2ThetaT = eta * eta * sin2ThetaI;
    if (sin2ThetaT >= 1.0f) return false;
    float cosThetaT = cl_sqrt(1.0f - sin2ThetaT);
    *wt = -eta * wi + (eta * cosThetaI - cosThetaT) * n;
    return true;
}
// bxdfs.cl:330-347.  Kept as calls: in the reference these terms enter `f +=` through a
// function call, so they must not contract into the accumulation.
MCRT_DEV f3 evaluateLambertianReflection(f3 R) { return R * PI_INV_F; }
MCRT_DEV float evaluateLambertianReflectionPdf(f3 wo, f3 wi) {
    return isSameHemisphere(wo, wi) ? evalAbsCosTheta(wi) * PI_INV_F : 0.0f;
}
MCRT_DEV f3 sampleSpecularReflection_Dielectric(f3 R, float etaI, float etaT, f3 wo, f3* wi, float* pdf) {
    *wi = f3{-wo.x, wo.y, -wo.z};   // bxdfs.cl:259-268
    *pdf = 1.0f;
    float F = evaluateFresnelDielectric(evalCosTheta(*wi), etaI, etaT);
    return cl_div(F * R, evalAbsCosTheta(*wi));
}
// TransportMode (bxdfs.cl:143-147): the path tracer is radiance transport; BDPT light
// subpaths are importance transport.
enum { TRANSPORT_MODE_RADIANCE = 0, TRANSPORT_MODE_IMPORTANCE = 1 };

MCRT_DEV f3 sampleSpecularTransmission(f3 T, float etaA, float etaB, f3 wo, f3* wi, float* pdf,
                                       int mode = TRANSPORT_MODE_RADIANCE) {   // :288-307
    bool isEntering = evalCosTheta(wo) > 0.0f;
    float etaI = isEntering ? etaA : etaB;
    float etaT = isEntering ? etaB : etaA;
    f3 n = f3{0.0f, 1.0f, 0.0f} * cl_sign(wo.y);
    if (!refract(wo, n, cl_div(etaI, etaT), wi)) return f3{0.0f, 0.0f, 0.0f};
    *pdf = 1.0f;
    f3 ft = T * (1.0f - evaluateFresnelDielectric(evalCosTheta(*wi), etaA, etaB));
    if (mode == TRANSPORT_MODE_RADIANCE) ft *= cl_div((etaI * etaI), (etaT * etaT));
    return cl_div(ft, evalAbsCosTheta(*wi));
}
MCRT_DEV float roughnessToAlpha(float roughness) {   // bxdfs.cl:385-390
    roughness = fmaxf(roughness, 1e-3f);
    float x = logf(roughness);
    return 1.62142f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
}
MCRT_DEV float computeTrowbridgeReitzDistribution(f3 wh, f2 alpha) {   // :406-415
    float tan2Theta = evalTanSqTheta(wh);
    if (__builtin_isinf(tan2Theta)) return 0.0f;
    const float cos4Theta = evalCosSqTheta(wh) * evalCosSqTheta(wh);
    float e = (cl_div(evalCosSqPhi(wh), (alpha.x * alpha.x)) + cl_div(evalSinSqPhi(wh), (alpha.y * alpha.y))) * tan2Theta;
    return cl_div(1.0f, (PI_F * alpha.x * alpha.y * cos4Theta * (1.0f + e) * (1.0f + e)));
}
MCRT_DEV float computeTrowbridgeReitzDistributionLambda(f3 w, f2 alpha) {   // :435-445
    float absTanTheta = fabsf(evalTanTheta(w));
    if (__builtin_isinf(absTanTheta)) return 0.0f;
    float alphaW = cl_sqrt(evalCosSqPhi(w) * alpha.x * alpha.x + evalSinSqPhi(w) * alpha.y * alpha.y);
    float alpha2Tan2Theta = (alphaW * absTanTheta) * (alphaW * absTanTheta);
    return (-1.0f + cl_sqrt(1.f + alpha2Tan2Theta)) * 0.5f;   // x / 2.0f folds to x * 0.5f
}
MCRT_DEV float computeTrowbridgeReitzDistributionG(f3 wo, f3 wi, f2 alpha) {   // :461-474
    return cl_div(1.0f, (1.0f + computeTrowbridgeReitzDistributionLambda(wo, alpha) + computeTrowbridgeReitzDistributionLambda(wi, alpha)));
}
MCRT_DEV f3 evaluateMicrofacetReflection(f3 R, f2 alpha, float etaI, float etaT, f3 wo, f3 wi) {   // :481-500
    float cosThetaO = evalAbsCosTheta(wo);
    float cosThetaI = evalAbsCosTheta(wi);
    f3 wh = wi + wo;
    if (cosThetaI == 0.0f || cosThetaO == 0.0f) return f3{0.0f, 0.0f, 0.0f};
    if (wh.x == 0.0f && wh.y == 0.0f && wh.z == 0.0f) return f3{0.0f, 0.0f, 0.0f};
    wh = cl_normalize(wh);
    float F = evaluateFresnelDielectric(cl_dot(wi, wh), etaI, etaT);
    return cl_div(R * computeTrowbridgeReitzDistribution(wh, alpha) * computeTrowbridgeReitzDistributionG(wo, wi, alpha) * F,
                  (4.0f * cosThetaI * cosThetaO));
}
// The reciprocals of eta in the microfacet-transmission functions are correctly rounded:
// the reference's compiler hoists `etaI / etaT` (etaI = 1) out of the eta selects, which drops
// its 2.5-ulp accuracy metadata, in the NEE evaluation and in the sampling path alike
// (the sampled, evaluated and pdf etas are one CSE'd value there).
MCRT_DEV f3 evaluateMicrofacetTransmission(f3 T, f2 alpha, float etaI, float etaT, f3 wo, f3 wi,
                                          int mode = TRANSPORT_MODE_RADIANCE) {   // :563-588
    if (isSameHemisphere(wo, wi)) return f3{0.0f, 0.0f, 0.0f};
    float cosThetaO = evalCosTheta(wo);
    float cosThetaI = evalCosTheta(wi);
    if (cosThetaI == 0.0f || cosThetaO == 0.0f) return f3{0.0f, 0.0f, 0.0f};
    float eta = evalCosTheta(wo) > 0.0f ? cr_div(etaT, etaI) : cr_div(etaI, etaT);
    f3 wh = cl_normalize(wo + wi * eta);
    if (wh.z < 0) wh = -wh;   // bxdfs.cl:577 (z, not y: SURVEY App. A Q4)
    float F = evaluateFresnelDielectric(cl_dot(wo, wh), etaI, etaT);
    float sqrtDenom = cl_dot(wo, wh) + eta * cl_dot(wi, wh);
    float factor = (mode == TRANSPORT_MODE_RADIANCE) ? cr_div(1.0f, eta) : 1.0f;
    return (f3{1.0f, 1.0f, 1.0f} - F) * T *
           fabsf(cl_div(computeTrowbridgeReitzDistribution(wh, alpha) * computeTrowbridgeReitzDistributionG(wo, wi, alpha) *
                            eta * eta * absDot(wi, wh) * absDot(wo, wh) * factor * factor,
                        (cosThetaI * cosThetaO * sqrtDenom * sqrtDenom)));
}
MCRT_DEV f3 sampleTrowbridgeReitzDistribution_wh(f2 u, f3 wo, f2 alpha) {   // :647-675
    // cosTheta = 1 / sqrt(.) is correctly rounded: the reference's compiler merges the two
    // branches' divisions after the if/else and drops their accuracy metadata.
    float cosTheta = 0.0f;
    float phi = (2.0f * PI_F) * u.y;
    if (alpha.x == alpha.y) {
        float tanTheta2 = cl_div(alpha.x * alpha.x * u.x, (1.0f - u.x));
        cosTheta = cr_div(1.0f, cl_sqrt(1.0f + tanTheta2));
    } else {
        phi = atanf(cl_div(alpha.y, alpha.x) * tanf(2.0f * PI_F * u.y + 0.5f * PI_F));
        if (u.y > .5f) phi += PI_F;
        float sinPhi = sinf(phi);
        float cosPhi = cosf(phi);
        const float alphax2 = alpha.x * alpha.x, alphay2 = alpha.y * alpha.y;
        const float alpha2 = cl_div(1.0f, (cl_div(cosPhi * cosPhi, alphax2) + cl_div(sinPhi * sinPhi, alphay2)));
        float tanTheta2 = cl_div(alpha2 * u.x, (1.0f - u.x));
        cosTheta = cr_div(1.0f, cl_sqrt(1.0f + tanTheta2));
    }
    float sinTheta = cl_sqrt(fmaxf(0.0f, 1.0f - cosTheta * cosTheta));
    f3 wh = f3{sinTheta * cosf(phi), cosTheta, sinTheta * sinf(phi)};   // math.cl:18-23
    if (!isSameHemisphere(wo, wh)) wh = -wh;
    return wh;
}
MCRT_DEV float evalTrowbridgeReitzPdf_wh(f3 wo, f3 wh, f2 alpha) {
    return computeTrowbridgeReitzDistribution(wh, alpha) * evalAbsCosTheta(wh);
}
MCRT_DEV float evalMicrofacetReflectionPdf(f3 wo, f3 wi, f3 wh, f2 alpha) {   // :695-701
    if (!isSameHemisphere(wo, wi)) return 0.0f;
    return cl_div(evalTrowbridgeReitzPdf_wh(wo, wh, alpha), (4.0f * cl_dot(wo, wh)));
}
MCRT_DEV float evalMicrofacetTransmissionPdf(f3 wo, f3 wi, f2 alpha, float etaA, float etaB) {   // :717-729
    if (isSameHemisphere(wo, wi)) return 0.0f;
    float eta = evalCosTheta(wo) > 0.0f ? cr_div(etaB, etaA) : cr_div(etaA, etaB);
    f3 wh = cl_normalize(wo + wi * eta);
    float sqrtDenom = cl_dot(wo, wh) + eta * cl_dot(wi, wh);
    float dwh_dwi = fabsf(cl_div((eta * eta * cl_dot(wi, wh)), (sqrtDenom * sqrtDenom)));
    return evalTrowbridgeReitzPdf_wh(wo, wh, alpha) * dwh_dwi;
}
MCRT_DEV f3 sampleMicrofacetReflection(f2 u, f3 R, f2 alpha, float etaI, float etaT, f3 wo, f3* wi, float* pdf) {
    f3 wh = sampleTrowbridgeReitzDistribution_wh(u, wo, alpha);   // :731-749
    *wi = reflect(wo, wh);
    if (!isSameHemisphere(wo, *wi)) return f3{0.0f, 0.0f, 0.0f};
    *pdf = evalMicrofacetReflectionPdf(wo, *wi, wh, alpha);
    return evaluateMicrofacetReflection(R, alpha, etaI, etaT, wo, *wi);
}
MCRT_DEV f3 sampleMicrofacetTransmission(f2 u, f3 T, f2 alpha, float etaA, float etaB, f3 wo, f3* wi, float* pdf,
                                         int mode = TRANSPORT_MODE_RADIANCE) {
    f3 wh = sampleTrowbridgeReitzDistribution_wh(u, wo, alpha);   // :751-762
    float eta = evalCosTheta(wo) > 0.0f ? cr_div(etaA, etaB) : cr_div(etaB, etaA);
    if (!refract(wo, wh, eta, wi)) return f3{0.0f, 0.0f, 0.0f};
    *pdf = evalMicrofacetTransmissionPdf(wo, *wi, alpha, etaA, etaB);
    return evaluateMicrofacetTransmission(T, alpha, etaA, etaB, wo, *wi, mode);
}

struct Frame {   // the RTInteraction fields the shading uses
    f3 p, gn, sn, sdpdu, sdpdv;
    f2 uv;
};
MCRT_DEV f3 dirToShadingSpace(f3 w, const Frame& si) {   // bxdfs.cl:81-107
    return f3{cl_dot(si.sdpdu, w), cl_dot(si.sn, w), cl_dot(si.sdpdv, w)};
}
MCRT_DEV f3 dirFromShadingToWorld(f3 w, const Frame& si) {   // bxdfs.cl:94-112
    const f3 t = si.sdpdu, n = si.sn, bn = si.sdpdv;
    return f3{t.x * w.x + n.x * w.y + bn.x * w.z, t.y * w.x + n.y * w.y + bn.y * w.z, t.z * w.x + n.z * w.y + bn.z * w.z};
}
MCRT_DEV bool isReflection(f3 woWorld, f3 wiWorld, const Frame& si) {
    return cl_dot(si.gn, woWorld) * cl_dot(si.gn, wiWorld) > 0.0f;
}

struct Uber {   // RTUberMaterialProperties (materials.cl:67-74)
    f3 Kd, Ks, Kr, opacity;
    f4 Kt;
    f2 roughness;
    float eta;
};

// bxdfs.cl:804-827
MCRT_DEV f3 evaluateUberBSDF(const Uber& m, const Frame& si, f3 woWorld, f3 wiWorld, int mode = TRANSPORT_MODE_RADIANCE) {
    if (!isReflection(woWorld, wiWorld, si)) {
        bool isPerfectSpecularTransmission = m.Kt.w < 0.5f;
        if (isPerfectSpecularTransmission) return f3{0.0f, 0.0f, 0.0f};
        f3 wo = dirToShadingSpace(woWorld, si);
        f3 wi = dirToShadingSpace(wiWorld, si);
        f3 kt = m.Kt.xyz * m.opacity;
        return evaluateMicrofacetTransmission(kt, m.roughness, 1.0f, m.eta, wo, wi, mode);
    }
    f3 wo = dirToShadingSpace(woWorld, si);
    f3 wi = dirToShadingSpace(wiWorld, si);
    f3 kd = m.Kd * m.opacity;
    f3 ks = m.Ks * m.opacity;
    return evaluateMicrofacetReflection(ks, m.roughness, 1.0f, m.eta, wo, wi) + evaluateLambertianReflection(kd);
}

// bxdfs.cl:892-1053, type = BSDF_ALL; `wi` zero-initialised.
// numNonDeltaTypes (optional) counts the matching non-specular lobes (BDPT connectibility).
MCRT_DEV f3 sampleUberBSDF(const Uber& m, const Frame& si, f2 u, f3 woWorld, f3* wiWorld, float* pdf, int* sampledType,
                           int mode = TRANSPORT_MODE_RADIANCE, int* numNonDeltaTypes = nullptr) {
    f3 t = f3{1.0f, 1.0f, 1.0f} - m.opacity;
    int numBxDFs = 0;
    f3 kd = m.Kd * m.opacity;
    f3 ks = m.Ks * m.opacity;
    f3 kt = m.Kt.xyz * m.opacity;
    f3 kr = m.Kr * m.opacity;
    f3 wo = dirToShadingSpace(woWorld, si);
    f3 wi = f3{0.0f, 0.0f, 0.0f};
    bool isPerfectSpecularTransmission = m.Kt.w < 0.5f;
    *sampledType = 0;
    const bool hasT = isNotBlack(t), hasKd = isNotBlack(kd), hasKs = isNotBlack(ks), hasKr = isNotBlack(kr),
               hasKt = isNotBlack(kt);
    numBxDFs = (int)hasT + (int)hasKd + (int)hasKs + (int)hasKr + (int)hasKt;
    if (numNonDeltaTypes) *numNonDeltaTypes = (int)hasKd + (int)hasKs + (int)(hasKt && !isPerfectSpecularTransmission);
    if (numBxDFs == 0) return f3{0.0f, 0.0f, 0.0f};
    int chosenBxDFIdx = min((int)floorf(u.x * numBxDFs), numBxDFs - 1);
    u.x = u.x * numBxDFs - chosenBxDFIdx;
    f3 f = f3{0.0f, 0.0f, 0.0f};
    *pdf = 0.0f;
    bool isSamplingSpecular = false;
    if (hasT) {
        if (chosenBxDFIdx-- == 0) {
            f += sampleSpecularTransmission(t, 1.0f, 1.0f, wo, &wi, pdf, mode);
            *sampledType |= BSDF_SPEC_TRANS;
            isSamplingSpecular = true;
        }
    }
    if (isPerfectSpecularTransmission && hasKt) {
        if (chosenBxDFIdx-- == 0) {
            f += sampleSpecularTransmission(kt, 1.0f, m.eta, wo, &wi, pdf, mode);
            *sampledType |= BSDF_SPEC_TRANS;
            isSamplingSpecular = true;
        }
    }
    if (hasKr) {
        if (chosenBxDFIdx-- == 0) {
            f += sampleSpecularReflection_Dielectric(kr, 1.0f, m.eta, wo, &wi, pdf);
            *sampledType |= BSDF_SPEC_REFL;
            isSamplingSpecular = true;
        }
    }
    if (hasKt) {   // bxdfs.cl:1004, independent of Kt.w
        if (chosenBxDFIdx-- == 0) {
            f += sampleMicrofacetTransmission(u, kt, m.roughness, 1.0f, m.eta, wo, &wi, pdf, mode);
            *sampledType |= BSDF_MF_TRANS;
        }
    }
    bool isLambertianEvaluationRequested = false;
    if (hasKd) {
        if (chosenBxDFIdx-- == 0) {
            wi = cosineSampleHemisphere(u);   // sampleCosineHemisphere, bxdfs.cl:317-328
            if (wo.y < 0.0f) wi.y *= -1.0f;
            *pdf = evalAbsCosTheta(wi) * PI_INV_F;
            f += evaluateLambertianReflection(kd);
            *sampledType |= BSDF_LAMBERT;
        } else if (!isSamplingSpecular && isSameHemisphere(wi, wo)) {
            isLambertianEvaluationRequested = true;
        }
    }
    if (hasKs) {
        if (chosenBxDFIdx-- == 0) {
            f += sampleMicrofacetReflection(u, ks, m.roughness, 1.0f, m.eta, wo, &wi, pdf);
            *sampledType |= BSDF_MF_REFL;
        } else if (!isSamplingSpecular && isSameHemisphere(wi, wo)) {
            f += evaluateMicrofacetReflection(ks, m.roughness, 1.0f, m.eta, wo, wi);
            *pdf += evalMicrofacetReflectionPdf(wo, wi, cl_normalize(wo + wi), m.roughness);
        }
    }
    if (isLambertianEvaluationRequested) {
        f += evaluateLambertianReflection(kd);
        *pdf += evaluateLambertianReflectionPdf(wo, wi);
    }
    *pdf = cl_div(*pdf, (float)numBxDFs);
    *wiWorld = dirFromShadingToWorld(wi, si);
    return f;
}

// bxdfs.cl:829-880 (evaluateUberBSDF_Pdf), type = BSDF_ALL
MCRT_DEV float evaluateUberBSDF_Pdf(const Uber& m, const Frame& si, f3 woWorld, f3 wiWorld) {
    f3 wo = dirToShadingSpace(woWorld, si);
    f3 wi = dirToShadingSpace(wiWorld, si);
    if (isNearZero(wo.y)) return 0.0f;
    f3 t = f3{1.0f, 1.0f, 1.0f} - m.opacity;
    int numBxDFs = 0;
    f3 kd = m.Kd * m.opacity;
    f3 ks = m.Ks * m.opacity;
    f3 kt = m.Kt.xyz * m.opacity;
    f3 kr = m.Kr * m.opacity;
    float pdf = 0.0f;
    if (isNotBlack(t)) ++numBxDFs;
    if (isNotBlack(kr)) ++numBxDFs;
    if (isNotBlack(kt)) {
        if (m.Kt.w < 0.5f) {
            ++numBxDFs;
        } else {
            pdf += evalMicrofacetTransmissionPdf(wo, wi, m.roughness, 1.0f, m.eta);
            ++numBxDFs;
        }
    }
    if (isNotBlack(kd)) {
        pdf += evaluateLambertianReflectionPdf(wo, wi);
        ++numBxDFs;
    }
    if (isNotBlack(ks)) {
        pdf += evalMicrofacetReflectionPdf(wo, wi, cl_normalize(wo + wi), m.roughness);
        ++numBxDFs;
    }
    if (numBxDFs > 1) pdf = cl_div(pdf, (float)numBxDFs);
    return pdf;
}

/*
 * mcrt_oracle.c -- TEST INFRASTRUCTURE ONLY (see mcrt_oracle.h).
 *
 * Plain-C restatement of the reference hot path.  Every function cites the
 * reference file:line it follows.  Paths:
 *   KRN = assets/kernels
 *   RR  = third_party/RadeonRays/RadeonRays
 *   RRT = third_party/RadeonRays/UnitTest
 *
 * Arithmetic policy: IEEE fp32, no FMA contraction (-ffp-contract=off), left-
 * to-right evaluation exactly as written in the reference; OpenCL `mad` in the
 * RR box test is restated as fmaf (what the reference's GPU build emits).
 * Deliberate decisions on reference UB:
 *   Q1 bxdfs.cl:38  evalSinPhi always clamps (function-address compare is false)
 *   Q3 bxdfs.cl:908 `wi` zero-initialised before the lobe chain
 *   Q13 lights.cl:64 point light at distance 0: pdf and wi zero-initialised
 */
#include "mcrt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <stdatomic.h>
#include <immintrin.h>

/* ======================================================================= */
/* Vector helpers (OpenCL builtin semantics)                               */
/* ======================================================================= */
typedef struct { float x, y, z; } v3;
typedef struct { float x, y; } v2;

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 vadd(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 vsub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 vmul(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 vdiv(v3 a, v3 b) { return V3(a.x / b.x, a.y / b.y, a.z / b.z); }
static inline v3 vs(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }      /* a * s  */
static inline v3 sv(float s, v3 a) { return V3(s * a.x, s * a.y, s * a.z); }      /* s * a  */
static inline v3 vdivs(v3 a, float s) { return V3(a.x / s, a.y / s, a.z / s); }
static inline v3 vneg(v3 a) { return V3(-a.x, -a.y, -a.z); }
static inline float vdot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 vcross(v3 a, v3 b) {
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* OpenCL normalize / length with the ROCm device-library range scaling. */
static inline v3 vnormalize(v3 p) {
    float l2 = vdot(p, p);
    if (l2 < FLT_MIN) { p = vs(p, 0x1.0p+86f); l2 = vdot(p, p); }
    else if (isinf(l2)) { p = vs(p, 0x1.0p-65f); l2 = vdot(p, p); }
    if (l2 == 0.0f) return p;
    return vs(p, 1.0f / sqrtf(l2));
}
static inline float vlength(v3 p) { return sqrtf(vdot(p, p)); }
static inline v3 vmix(v3 a, v3 b, float t) { return vadd(a, vs(vsub(b, a), t)); }   /* mix = a + (b-a)*t */
static inline float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
static inline float signf(float x) {
    if (x > 0.0f) return 1.0f;
    if (x < 0.0f) return -1.0f;
    if (x == 0.0f) return x;   /* +-0 */
    return 0.0f;               /* NaN */
}
static inline v3 load3(const mcrt_float3* p) { return V3(p->x, p->y, p->z); }
static inline v3 load3a(const float* p) { return V3(p[0], p[1], p[2]); }

#define PI 3.14159265359f         /* KRN/math.cl:8 */
#define PI_INV 0.31830988618f
#define PI2_INV 0.15915494309f
#define PI4_INV 0.07957747154f
#define PI2 6.28318530718f
#define PI_DIV_4 0.78539816339f
#define PI_DIV_2 1.57079632679f
#define RT_TRACE_OFFSET 0.00001f  /* KRN/kernel_data.h:10 */
#define RT_MAX_TRACE_DISTANCE 1000.0f

/* KRN/math.cl:53-66 */
static v3 computeOrthogonalVector(v3 n) {
    if (fabsf(n.z) > 0.0f) {
        float d = sqrtf(n.z * n.z + n.x * n.x);
        return V3(-n.z / d, 0.0f, n.x / d);
    } else {
        float d = sqrtf(n.y * n.y + n.x * n.x);
        return V3(n.y / d, -n.x / d, 0.0f);
    }
}
static inline float absDot(v3 a, v3 b) { return fabsf(vdot(a, b)); }       /* math.cl:68-71 */
static inline int isNearZero(float v) { return fabsf(v) < 1e-8f; }          /* math.cl:73-76 */
static inline int isNotNearZero(float v) { return fabsf(v) > 1e-8f; }       /* math.cl:78-81 */
static inline float distanceSquared(v3 a, v3 b) { return vdot(vsub(a, b), vsub(a, b)); }
/* math.cl:88-91 */
static inline v3 lerpDirection(v3 d0, v3 d1, v3 d2, v3 d3, float t0, float t1) {
    return vnormalize(vmix(vmix(d0, d1, t0), vmix(d3, d2, t0), t1));
}
/* KRN/matrix.cl:44-60 */
static inline v3 transformVector3(const mcrt_mat4* m, v3 v) {
    return V3(vdot(load3(&m->m0), v), vdot(load3(&m->m1), v), vdot(load3(&m->m2), v));
}
static inline v3 transformPoint3(const mcrt_mat4* m, v3 v) {
    return V3(vdot(load3(&m->m0), v) + m->m0.w, vdot(load3(&m->m1), v) + m->m1.w,
              vdot(load3(&m->m2), v) + m->m2.w);
}

/* ======================================================================= */
/* RNG + samplers: KRN/rng.cl, KRN/samplers.cl                             */
/* ======================================================================= */
/* rng.cl:58-66 */
uint32_t orc_wang_hash(uint32_t seed) {
    seed = (seed ^ 61u) ^ (seed >> 16);
    seed *= 9u;
    seed = seed ^ (seed >> 4);
    seed *= 0x27d4eb2du;
    seed = seed ^ (seed >> 15);
    return seed;
}
/* rng.cl:48-56 */
uint32_t orc_xorshift(uint32_t* s) {
    *s += 2463534242u;
    *s ^= (*s << 13);
    *s ^= (*s >> 17);
    *s ^= (*s << 5);
    return *s;
}
/* rng.cl:104-107: (float)x / 0xffffffff; the constant converts to 2^32 (Q10). */
float orc_rand_float(uint32_t* s) { return ((float)orc_xorshift(s)) / 4294967296.0f; }

/* samplers.cl:64-72 */
float orc_sobol_sample(uint32_t idx, uint32_t dim, uint32_t scramble, const uint32_t* m) {
    uint32_t v = scramble;
    for (uint32_t i = dim * 52u; idx != 0; idx >>= 1, ++i)
        if (idx & 1u) v ^= m[i];
    return (float)v * 0x1p-32f;
}

typedef struct {
    int kind;            /* 0 sobol, 1 random (samplers.cl:16-18) */
    uint32_t idx;        /* random: xorshift state; sobol: sample index */
    uint32_t dimension;
    uint32_t scramble;
    const uint32_t* mats;
} Sampler;

/* MAKE_SAMPLER, samplers.cl:74-85 (uint32 wrap for the int products, Q5/Q6). */
static void makeSampler(Sampler* s, int kind, uint32_t bufferIdx, int frame, int bounce, int W, int H,
                        const uint32_t* mats) {
    s->kind = kind;
    s->mats = mats;
    s->dimension = 0;
    if (kind == MCRT_SAMPLER_SOBOL) {
        s->idx = bufferIdx + (uint32_t)frame * (uint32_t)W * (uint32_t)H;
        uint32_t seed = orc_wang_hash((uint32_t)(frame + 1) * (uint32_t)(bounce + 1));
        s->scramble = orc_xorshift(&seed);
    } else {
        s->idx = orc_wang_hash(bufferIdx + (uint32_t)(frame + 1) * (uint32_t)W * (uint32_t)H * (uint32_t)(bounce + 1));
        s->scramble = 0;
    }
}
/* samplers.cl:99-122 */
static float getSample1D(Sampler* s) {
    if (s->kind == MCRT_SAMPLER_SOBOL) {
        float u = orc_sobol_sample(s->idx, s->dimension, s->scramble, s->mats);
        s->dimension++;
        return u;
    }
    return orc_rand_float(&s->idx);
}
static v2 getSample2D(Sampler* s) {
    v2 u;
    u.x = getSample1D(s);   /* (float2)(a, b): x is evaluated first */
    u.y = getSample1D(s);
    return u;
}

void orc_sampler_draws(int kind, uint32_t pix, int frame, int bounce, int W, int H,
                       const uint32_t* sobol, float out[5]) {
    Sampler s;
    makeSampler(&s, kind, pix, frame, bounce, W, H, sobol);
    out[0] = getSample1D(&s);
    v2 a = getSample2D(&s);
    v2 b = getSample2D(&s);
    out[1] = a.x; out[2] = a.y; out[3] = b.x; out[4] = b.y;
}

/* samplers.cl:169-191 */
static v2 concentricSampleDisc(v2 u) {
    v2 uo = {2.0f * u.x - 1.0f, 2.0f * u.y - 1.0f};
    if (u.x < 1e-8f && u.y < 1e-8f) { v2 z = {0.0f, 0.0f}; return z; }
    float theta, r;
    if (fabsf(uo.x) > fabsf(uo.y)) { r = uo.x; theta = PI_DIV_4 * (uo.y / uo.x); }
    else { r = uo.y; theta = PI_DIV_2 - PI_DIV_4 * (uo.x / uo.y); }
    v2 res = {r * cosf(theta), r * sinf(theta)};
    return res;
}
/* samplers.cl:193-198 */
static v3 cosineSampleHemisphere(v2 u) {
    v2 d = concentricSampleDisc(u);
    float y = sqrtf(fmaxf(0.0f, 1.0f - d.x * d.x - d.y * d.y));
    return V3(d.x, y, d.y);
}
/* samplers.cl:227-231 */
static v2 uniformSampleTriangle(v2 u) {
    float su0 = sqrtf(u.x);
    v2 r = {1.0f - su0, u.y * su0};
    return r;
}

typedef struct { v3 p, gn; } ShapeSample;
/* samplers.cl:259-269 */
static ShapeSample sampleDisk(v3 p, v3 n, float radius, v2 u, float* pdf) {
    v2 p2d = concentricSampleDisc(u);
    ShapeSample it;
    it.gn = n;
    v3 t = computeOrthogonalVector(n);
    v3 b = vnormalize(vcross(n, t));
    it.p = vadd(vadd(p, vs(vs(t, p2d.x), radius)), vs(vs(b, p2d.y), radius));
    *pdf = 1.0f / (PI * radius * radius);
    return it;
}
/* samplers.cl:275-285 */
static ShapeSample sampleTriangle(v3 p0, v3 p1, v3 p2, v2 u, float* pdf) {
    v2 b = uniformSampleTriangle(u);
    ShapeSample it;
    it.p = vadd(vadd(sv(b.x, p0), sv(b.y, p1)), sv(1.0f - b.x - b.y, p2));
    v3 c = vcross(vsub(p1, p0), vsub(p2, p0));
    it.gn = vnormalize(c);
    float area = vlength(c) * 0.5f;
    *pdf = 1.0f / area;
    return it;
}

/* ======================================================================= */
/* BxDFs: KRN/bxdfs.cl (shading frame: normal = y, tangent = x, binormal = z) */
/* ======================================================================= */
enum {
    BSDF_NONE = 0, BSDF_REFLECTION = 1, BSDF_TRANSMISSION = 2, BSDF_DIFFUSE = 4,
    BSDF_GLOSSY = 8, BSDF_SPECULAR = 16,
    BSDF_SPECULAR_REFLECTION = BSDF_REFLECTION | BSDF_SPECULAR,
    BSDF_SPECULAR_TRANSMISSION = BSDF_TRANSMISSION | BSDF_SPECULAR,
    BSDF_LAMBERTIAN_REFLECTION = BSDF_REFLECTION | BSDF_DIFFUSE,
    BSDF_MICROFACET_REFLECTION = BSDF_REFLECTION | BSDF_GLOSSY,
    BSDF_MICROFACET_TRANSMISSION = BSDF_TRANSMISSION | BSDF_GLOSSY,
    BSDF_ALL = BSDF_DIFFUSE | BSDF_GLOSSY | BSDF_SPECULAR | BSDF_REFLECTION | BSDF_TRANSMISSION
};
#define TRANSPORT_MODE_RADIANCE 0

/* bxdfs.cl:22-59 */
static inline float evalCosTheta(v3 w) { return w.y; }
static inline float evalCosSqTheta(v3 w) { return w.y * w.y; }
static inline float evalAbsCosTheta(v3 w) { return fabsf(w.y); }
static inline float evalSinSqTheta(v3 w) { return fmaxf(0.0f, 1.0f - evalCosSqTheta(w)); }
static inline float evalSinTheta(v3 w) { return sqrtf(evalSinSqTheta(w)); }
static inline float evalTanTheta(v3 w) { return evalSinTheta(w) / evalCosTheta(w); }
static inline float evalTanSqTheta(v3 w) { return evalSinSqTheta(w) / evalCosSqTheta(w); }
static inline float evalCosPhi(v3 w) {
    float st = evalSinTheta(w);
    return st == 0 ? 1.0f : clampf(w.x / st, -1.0f, 1.0f);
}
static inline float evalSinPhi(v3 w) {   /* Q1: `evalSinTheta == 0` is always false */
    float st = evalSinTheta(w);
    return clampf(w.z / st, -1.0f, 1.0f);
}
static inline float evalCosSqPhi(v3 w) { return evalCosPhi(w) * evalCosPhi(w); }
static inline float evalSinSqPhi(v3 w) { return evalSinPhi(w) * evalSinPhi(w); }
static inline int isSameHemisphere(v3 a, v3 b) { return a.y * b.y > 0.0f; }
#define BLACK_EPS 0.000001f
static inline int isBlack(v3 c) { return c.x < BLACK_EPS && c.y < BLACK_EPS && c.z < BLACK_EPS; }
static inline int isNotBlack(v3 c) { return c.x > BLACK_EPS || c.y > BLACK_EPS || c.z > BLACK_EPS; }
static inline int matches(int bxdfType, int flags) { return (bxdfType & flags) == bxdfType; }

/* bxdfs.cl:159-190 */
static float evaluateFresnelDielectric(float cosThetaI, float etaI, float etaT) {
    cosThetaI = clampf(cosThetaI, -1.0f, 1.0f);
    if (cosThetaI <= 0.0f) { float h = etaI; etaI = etaT; etaT = h; cosThetaI = fabsf(cosThetaI); }
    float sinThetaI = sqrtf(fmaxf(0.0f, 1.0f - cosThetaI * cosThetaI));
    float sinThetaT = etaI / etaT * sinThetaI;
    if (sinThetaT >= 1.0f) return 1.0f;
    float cosThetaT = sqrtf(fmaxf(0.0f, 1.0f - sinThetaT * sinThetaT));
    float rparl = ((etaT * cosThetaI) - (etaI * cosThetaT)) / ((etaT * cosThetaI) + (etaI * cosThetaT));
    float rperp = ((etaI * cosThetaI) - (etaT * cosThetaT)) / ((etaI * cosThetaI) + (etaT * cosThetaT));
    return (rparl * rparl + rperp * rperp) * 0.5f;
}
/* bxdfs.cl:228-231 */
static inline v3 reflectv(v3 wo, v3 n) { return vadd(vneg(wo), sv(2.0f * vdot(n, wo), n)); }
/* bxdfs.cl:233-245 */
static int refractv(v3 wi, v3 n, float eta, v3* wt) {
    float cosThetaI = vdot(n, wi);
    float sin2ThetaI = fmaxf(0.0f, 1.0f - cosThetaI * cosThetaI);
    float sin2ThetaT = eta * eta * sin2ThetaI;
    if (sin2ThetaT >= 1.0f) return 0;
    float cosThetaT = sqrtf(1.0f - sin2ThetaT);
    *wt = vadd(sv(-eta, wi), sv(eta * cosThetaI - cosThetaT, n));
    return 1;
}
/* bxdfs.cl:259-268 */
static v3 sampleSpecularReflection_Dielectric(v3 R, float etaI, float etaT, v3 wo, v3* wi, float* pdf) {
    *wi = V3(-wo.x, wo.y, -wo.z);
    *pdf = 1.0f;
    float F = evaluateFresnelDielectric(evalCosTheta(*wi), etaI, etaT);
    return vdivs(sv(F, R), evalAbsCosTheta(*wi));
}
/* bxdfs.cl:288-307 */
static v3 sampleSpecularTransmission(v3 T, float etaA, float etaB, int mode, v3 wo, v3* wi, float* pdf) {
    int isEntering = evalCosTheta(wo) > 0.0f;
    float etaI = isEntering ? etaA : etaB;
    float etaT = isEntering ? etaB : etaA;
    v3 n = vs(V3(0.0f, 1.0f, 0.0f), signf(wo.y));
    if (!refractv(wo, n, etaI / etaT, wi)) return V3(0.0f, 0.0f, 0.0f);
    *pdf = 1.0f;
    v3 ft = vs(T, 1.0f - evaluateFresnelDielectric(evalCosTheta(*wi), etaA, etaB));
    if (mode == TRANSPORT_MODE_RADIANCE) ft = vs(ft, (etaI * etaI) / (etaT * etaT));
    return vdivs(ft, evalAbsCosTheta(*wi));
}
/* bxdfs.cl:317-347 */
static void sampleCosineHemisphere(v2 u, v3 wo, v3* wi, float* pdf) {
    *wi = cosineSampleHemisphere(u);
    if (wo.y < 0.0f) wi->y *= -1.0f;
    *pdf = evalAbsCosTheta(*wi) * PI_INV;
}
static inline float evaluateLambertianReflectionPdf(v3 wo, v3 wi) {
    return isSameHemisphere(wo, wi) ? evalAbsCosTheta(wi) * PI_INV : 0.0f;
}
static inline v3 evaluateLambertianReflection(v3 R) { return vs(R, PI_INV); }
static v3 sampleLambertianReflection(v3 R, v2 u, v3 wo, v3* wi, float* pdf) {
    sampleCosineHemisphere(u, wo, wi, pdf);
    return vs(R, PI_INV);
}
/* bxdfs.cl:385-390 */
float orc_roughness_to_alpha(float roughness) {
    roughness = fmaxf(roughness, 1e-3f);
    float x = logf(roughness);
    return 1.62142f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x +
           0.000640711f * x * x * x * x;
}
/* bxdfs.cl:406-415 */
static float trDistribution(v3 wh, v2 alpha) {
    float tan2Theta = evalTanSqTheta(wh);
    if (isinf(tan2Theta)) return 0.0f;
    const float cos4Theta = evalCosSqTheta(wh) * evalCosSqTheta(wh);
    float e = (evalCosSqPhi(wh) / (alpha.x * alpha.x) + evalSinSqPhi(wh) / (alpha.y * alpha.y)) * tan2Theta;
    return 1.0f / (PI * alpha.x * alpha.y * cos4Theta * (1.0f + e) * (1.0f + e));
}
/* bxdfs.cl:435-445 */
static float trLambda(v3 w, v2 alpha) {
    float absTanTheta = fabsf(evalTanTheta(w));
    if (isinf(absTanTheta)) return 0.0f;
    float alphaW = sqrtf(evalCosSqPhi(w) * alpha.x * alpha.x + evalSinSqPhi(w) * alpha.y * alpha.y);
    float a2t2 = (alphaW * absTanTheta) * (alphaW * absTanTheta);
    return (-1.0f + sqrtf(1.f + a2t2)) / 2.0f;
}
/* bxdfs.cl:461-474 */
static inline float trG(v3 wo, v3 wi, v2 alpha) { return 1.0f / (1.0f + trLambda(wo, alpha) + trLambda(wi, alpha)); }
/* bxdfs.cl:481-500 */
static v3 evalMicrofacetReflection(v3 R, v2 alpha, float etaI, float etaT, v3 wo, v3 wi) {
    float cosThetaO = evalAbsCosTheta(wo);
    float cosThetaI = evalAbsCosTheta(wi);
    v3 wh = vadd(wi, wo);
    if (cosThetaI == 0.0f || cosThetaO == 0.0f) return V3(0, 0, 0);
    if (wh.x == 0.0f && wh.y == 0.0f && wh.z == 0.0f) return V3(0, 0, 0);
    wh = vnormalize(wh);
    float F = evaluateFresnelDielectric(vdot(wi, wh), etaI, etaT);
    /* R * D * G * F / (4 cosI cosO), evaluated left to right on float3 */
    v3 r = vs(R, trDistribution(wh, alpha));
    r = vs(r, trG(wo, wi, alpha));
    r = vs(r, F);
    return vdivs(r, 4.0f * cosThetaI * cosThetaO);
}
/* bxdfs.cl:563-588 */
static v3 evalMicrofacetTransmission(v3 T, int mode, v2 alpha, float etaI, float etaT, v3 wo, v3 wi) {
    if (isSameHemisphere(wo, wi)) return V3(0, 0, 0);
    float cosThetaO = evalCosTheta(wo);
    float cosThetaI = evalCosTheta(wi);
    if (cosThetaI == 0.0f || cosThetaO == 0.0f) return V3(0, 0, 0);
    float eta = evalCosTheta(wo) > 0.0f ? (etaT / etaI) : (etaI / etaT);
    v3 wh = vnormalize(vadd(wo, vs(wi, eta)));
    if (wh.z < 0) wh = vneg(wh);   /* Q4: z, not y */
    float F = evaluateFresnelDielectric(vdot(wo, wh), etaI, etaT);
    float sqrtDenom = vdot(wo, wh) + eta * vdot(wi, wh);
    float factor = (mode == TRANSPORT_MODE_RADIANCE) ? (1.0f / eta) : 1.0f;
    float s = fabsf(trDistribution(wh, alpha) * trG(wo, wi, alpha) * eta * eta * absDot(wi, wh) *
                    absDot(wo, wh) * factor * factor / (cosThetaI * cosThetaO * sqrtDenom * sqrtDenom));
    v3 one_minus_F = V3(1.0f - F, 1.0f - F, 1.0f - F);
    return vs(vmul(one_minus_F, T), s);
}
/* bxdfs.cl:647-675 */
static v3 sampleTRwh(v2 u, v3 wo, v2 alpha) {
    float cosTheta = 0.0f;
    float phi = (2.0f * PI) * u.y;
    if (alpha.x == alpha.y) {
        float tanTheta2 = alpha.x * alpha.x * u.x / (1.0f - u.x);
        cosTheta = 1.0f / sqrtf(1.0f + tanTheta2);
    } else {
        phi = atanf(alpha.y / alpha.x * tanf(2.0f * PI * u.y + 0.5f * PI));
        if (u.y > .5f) phi += PI;
        float sinPhi = sinf(phi);
        float cosPhi = cosf(phi);
        const float ax2 = alpha.x * alpha.x, ay2 = alpha.y * alpha.y;
        const float alpha2 = 1.0f / (cosPhi * cosPhi / ax2 + sinPhi * sinPhi / ay2);
        float tanTheta2 = alpha2 * u.x / (1.0f - u.x);
        cosTheta = 1.0f / sqrtf(1.0f + tanTheta2);
    }
    float sinTheta = sqrtf(fmaxf(0.0f, 1.0f - cosTheta * cosTheta));
    v3 wh = V3(sinTheta * cosf(phi), cosTheta, sinTheta * sinf(phi));   /* math.cl:18-23 */
    if (!isSameHemisphere(wo, wh)) wh = vneg(wh);
    return wh;
}
/* bxdfs.cl:677-680, 695-701 */
static inline float trPdfWh(v3 wh, v2 alpha) { return trDistribution(wh, alpha) * evalAbsCosTheta(wh); }
static inline float mfReflPdf(v3 wo, v3 wi, v3 wh, v2 alpha) {
    if (!isSameHemisphere(wo, wi)) return 0.0f;
    return trPdfWh(wh, alpha) / (4.0f * vdot(wo, wh));
}
/* bxdfs.cl:717-729 */
static float mfTransPdf(v3 wo, v3 wi, v2 alpha, float etaA, float etaB) {
    if (isSameHemisphere(wo, wi)) return 0.0f;
    float eta = evalCosTheta(wo) > 0.0f ? (etaB / etaA) : (etaA / etaB);
    v3 wh = vnormalize(vadd(wo, vs(wi, eta)));
    float sqrtDenom = vdot(wo, wh) + eta * vdot(wi, wh);
    float dwh_dwi = fabsf((eta * eta * vdot(wi, wh)) / (sqrtDenom * sqrtDenom));
    return trPdfWh(wh, alpha) * dwh_dwi;
}
/* bxdfs.cl:731-749 */
static v3 sampleMicrofacetReflection(v2 u, v3 R, v2 alpha, float etaI, float etaT, v3 wo, v3* wi, float* pdf) {
    v3 wh = sampleTRwh(u, wo, alpha);
    *wi = reflectv(wo, wh);
    if (!isSameHemisphere(wo, *wi)) return V3(0, 0, 0);
    *pdf = mfReflPdf(wo, *wi, wh, alpha);
    return evalMicrofacetReflection(R, alpha, etaI, etaT, wo, *wi);
}
/* bxdfs.cl:751-762 */
static v3 sampleMicrofacetTransmission(v2 u, v3 T, int mode, v2 alpha, float etaA, float etaB, v3 wo, v3* wi, float* pdf) {
    v3 wh = sampleTRwh(u, wo, alpha);
    float eta = evalCosTheta(wo) > 0.0f ? (etaA / etaB) : (etaB / etaA);
    if (!refractv(wo, wh, eta, wi)) return V3(0, 0, 0);
    *pdf = mfTransPdf(wo, *wi, alpha, etaA, etaB);
    return evalMicrofacetTransmission(T, mode, alpha, etaA, etaB, wo, *wi);
}

/* Shading frame of an interaction (the RTInteraction fields the BSDF uses). */
typedef struct {
    v3 wo, p, gn, sn, dpdu, dpdv, sdpdu, sdpdv;
    v2 uv;
    float traceErrorOffset;
    int shapeIdx;
} Interaction;

/* bxdfs.cl:104-112 */
static inline v3 toShading(v3 v, const Interaction* si) {
    return V3(vdot(si->sdpdu, v), vdot(si->sn, v), vdot(si->sdpdv, v));
}
static inline v3 fromShading(v3 w, const Interaction* si) {
    v3 t = si->sdpdu, n = si->sn, b = si->sdpdv;
    return V3(t.x * w.x + n.x * w.y + b.x * w.z, t.y * w.x + n.y * w.y + b.y * w.z,
              t.z * w.x + n.z * w.y + b.z * w.z);
}
/* bxdfs.cl:118-121 */
static inline int isReflection(v3 wo, v3 wi, const Interaction* si) {
    return vdot(si->gn, wo) * vdot(si->gn, wi) > 0.0f;
}

typedef struct { v3 Kd, Ks, Kr, opacity; float Kt[4]; v2 roughness; float eta; } UberProps;

/* bxdfs.cl:804-827 */
static v3 evaluateUberBSDF(const UberProps* m, const Interaction* si, v3 woW, v3 wiW, int mode) {
    if (!isReflection(woW, wiW, si)) {
        if (m->Kt[3] < 0.5f) return V3(0, 0, 0);
        v3 wo = toShading(woW, si), wi = toShading(wiW, si);
        v3 kt = vmul(load3a(m->Kt), m->opacity);
        return evalMicrofacetTransmission(kt, mode, m->roughness, 1.0f, m->eta, wo, wi);
    }
    v3 wo = toShading(woW, si), wi = toShading(wiW, si);
    v3 kd = vmul(m->Kd, m->opacity);
    v3 ks = vmul(m->Ks, m->opacity);
    return vadd(evalMicrofacetReflection(ks, m->roughness, 1.0f, m->eta, wo, wi), evaluateLambertianReflection(kd));
}
/* bxdfs.cl:829-880 */
static float evaluateUberBSDF_Pdf(const UberProps* m, const Interaction* si, v3 woW, v3 wiW, int type) {
    v3 wo = toShading(woW, si), wi = toShading(wiW, si);
    if (isNearZero(wo.y)) return 0.0f;
    v3 t = vsub(V3(1, 1, 1), m->opacity);
    int n = 0;
    v3 kd = vmul(m->Kd, m->opacity), ks = vmul(m->Ks, m->opacity);
    v3 kt = vmul(load3a(m->Kt), m->opacity), kr = vmul(m->Kr, m->opacity);
    float pdf = 0.0f;
    if (isNotBlack(t) && matches(BSDF_SPECULAR_TRANSMISSION, type)) ++n;
    if (isNotBlack(kr) && matches(BSDF_SPECULAR_REFLECTION, type)) ++n;
    if (isNotBlack(kt)) {
        if (m->Kt[3] < 0.5f) { if (matches(BSDF_SPECULAR_TRANSMISSION, type)) ++n; }
        else if (matches(BSDF_MICROFACET_TRANSMISSION, type)) {
            pdf += mfTransPdf(wo, wi, m->roughness, 1.0f, m->eta);
            ++n;
        }
    }
    if (isNotBlack(kd) && matches(BSDF_LAMBERTIAN_REFLECTION, type)) { pdf += evaluateLambertianReflectionPdf(wo, wi); ++n; }
    if (isNotBlack(ks) && matches(BSDF_MICROFACET_REFLECTION, type)) {
        pdf += mfReflPdf(wo, wi, vnormalize(vadd(wo, wi)), m->roughness);
        ++n;
    }
    if (n > 1) pdf /= n;
    return pdf;
}
/* bxdfs.cl:892-1053 */
static v3 sampleUberBSDF(const UberProps* m, const Interaction* si, v2 u, int mode, int type, v3 woW,
                         v3* wiW, float* pdf, int* numNonDelta, int* sampledType) {
    v3 t = vsub(V3(1, 1, 1), m->opacity);
    int n = 0;
    v3 kd = vmul(m->Kd, m->opacity), ks = vmul(m->Ks, m->opacity);
    v3 kt = vmul(load3a(m->Kt), m->opacity), kr = vmul(m->Kr, m->opacity);
    v3 wo = toShading(woW, si);
    v3 wi = V3(0.0f, 0.0f, 0.0f);   /* Q3: zero-initialised */
    int isPerfectSpecT = m->Kt[3] < 0.5f;
    *sampledType = BSDF_NONE;
    *numNonDelta = 0;
    if (isNotBlack(t) && matches(BSDF_SPECULAR_TRANSMISSION, type)) ++n;
    if (isNotBlack(kd) && matches(BSDF_LAMBERTIAN_REFLECTION, type)) { (*numNonDelta)++; ++n; }
    if (isNotBlack(ks) && matches(BSDF_MICROFACET_REFLECTION, type)) { (*numNonDelta)++; ++n; }
    if (isNotBlack(kr) && matches(BSDF_SPECULAR_REFLECTION, type)) ++n;
    if (isNotBlack(kt)) {
        if (isPerfectSpecT) { if (matches(BSDF_SPECULAR_TRANSMISSION, type)) ++n; }
        else if (matches(BSDF_MICROFACET_TRANSMISSION, type)) { (*numNonDelta)++; ++n; }
    }
    if (n == 0) return V3(0, 0, 0);   /* pdf left as is (PathTracing terminates on black f) */
    int chosen = (int)floorf(u.x * n);
    if (chosen > n - 1) chosen = n - 1;   /* min(int, int) */
    u.x = u.x * n - chosen;
    v3 f = V3(0, 0, 0);
    *pdf = 0.0f;
    int isSamplingSpecular = 0;
    if (isNotBlack(t) && matches(BSDF_SPECULAR_TRANSMISSION, type)) {
        if (chosen-- == 0) {
            f = vadd(f, sampleSpecularTransmission(t, 1.0f, 1.0f, mode, wo, &wi, pdf));
            *sampledType |= BSDF_SPECULAR_TRANSMISSION;
            isSamplingSpecular = 1;
        }
    }
    if (isPerfectSpecT && isNotBlack(kt) && matches(BSDF_SPECULAR_TRANSMISSION, type)) {
        if (chosen-- == 0) {
            f = vadd(f, sampleSpecularTransmission(kt, 1.0f, m->eta, mode, wo, &wi, pdf));
            *sampledType |= BSDF_SPECULAR_TRANSMISSION;
            isSamplingSpecular = 1;
        }
    }
    if (isNotBlack(kr) && matches(BSDF_SPECULAR_REFLECTION, type)) {
        if (chosen-- == 0) {
            f = vadd(f, sampleSpecularReflection_Dielectric(kr, 1.0f, m->eta, wo, &wi, pdf));
            *sampledType |= BSDF_SPECULAR_REFLECTION;
            isSamplingSpecular = 1;
        }
    }
    /* Q2: tested regardless of Kt.w (bxdfs.cl:1004) */
    if (isNotBlack(kt) && matches(BSDF_MICROFACET_TRANSMISSION, type)) {
        if (chosen-- == 0) {
            f = vadd(f, sampleMicrofacetTransmission(u, kt, mode, m->roughness, 1.0f, m->eta, wo, &wi, pdf));
            *sampledType |= BSDF_MICROFACET_TRANSMISSION;
        }
    }
    int lambertEval = 0;
    if (isNotBlack(kd) && matches(BSDF_LAMBERTIAN_REFLECTION, type)) {
        if (chosen-- == 0) {
            f = vadd(f, sampleLambertianReflection(kd, u, wo, &wi, pdf));
            *sampledType |= BSDF_LAMBERTIAN_REFLECTION;
        } else if (!isSamplingSpecular && isSameHemisphere(wi, wo)) {
            lambertEval = 1;
        }
    }
    if (isNotBlack(ks) && matches(BSDF_MICROFACET_REFLECTION, type)) {
        if (chosen-- == 0) {
            f = vadd(f, sampleMicrofacetReflection(u, ks, m->roughness, 1.0f, m->eta, wo, &wi, pdf));
            *sampledType |= BSDF_MICROFACET_REFLECTION;
        } else if (!isSamplingSpecular && isSameHemisphere(wi, wo)) {
            f = vadd(f, evalMicrofacetReflection(ks, m->roughness, 1.0f, m->eta, wo, wi));
            *pdf += mfReflPdf(wo, wi, vnormalize(vadd(wo, wi)), m->roughness);
        }
    }
    if (lambertEval) {
        f = vadd(f, evaluateLambertianReflection(kd));
        *pdf += evaluateLambertianReflectionPdf(wo, wi);
    }
    *pdf /= n;
    *wiW = fromShading(wi, si);
    return f;
}

/* Unit-level wrappers with an identity shading frame */
static Interaction identityFrame(void) {
    Interaction si;
    memset(&si, 0, sizeof(si));
    si.sdpdu = V3(1, 0, 0); si.sn = V3(0, 1, 0); si.sdpdv = V3(0, 0, 1); si.gn = V3(0, 1, 0);
    return si;
}
static UberProps makeProps(const float kd[3], const float ks[3], const float kr[3], const float kt[4],
                           const float ra[2], const float op[3], float eta) {
    UberProps m;
    m.Kd = load3a(kd); m.Ks = load3a(ks); m.Kr = kr ? load3a(kr) : V3(0, 0, 0);
    memcpy(m.Kt, kt, sizeof(m.Kt));
    m.roughness.x = ra[0]; m.roughness.y = ra[1];
    m.opacity = load3a(op); m.eta = eta;
    return m;
}
void orc_sample_uber(const float kd[3], const float ks[3], const float kr[3], const float kt[4],
                     const float ra[2], const float op[3], float eta, const float wo[3], const float u[2],
                     float out[8]) {
    UberProps m = makeProps(kd, ks, kr, kt, ra, op, eta);
    Interaction si = identityFrame();
    v2 uu = {u[0], u[1]};
    v3 wi = V3(0, 0, 0);
    float pdf = 0.0f;
    int nnd, st;
    v3 f = sampleUberBSDF(&m, &si, uu, TRANSPORT_MODE_RADIANCE, BSDF_ALL, load3a(wo), &wi, &pdf, &nnd, &st);
    out[0] = f.x; out[1] = f.y; out[2] = f.z; out[3] = wi.x; out[4] = wi.y; out[5] = wi.z;
    out[6] = pdf; out[7] = (float)st;
}
void orc_eval_uber(const float kd[3], const float ks[3], const float kt[4], const float ra[2],
                   const float op[3], float eta, const float wo[3], const float wi[3], float out[3]) {
    UberProps m = makeProps(kd, ks, NULL, kt, ra, op, eta);
    Interaction si = identityFrame();
    v3 f = evaluateUberBSDF(&m, &si, load3a(wo), load3a(wi), TRANSPORT_MODE_RADIANCE);
    out[0] = f.x; out[1] = f.y; out[2] = f.z;
}
float orc_pdf_uber(const float kd[3], const float ks[3], const float kr[3], const float kt[4],
                   const float ra[2], const float op[3], float eta, const float wo[3], const float wi[3]) {
    UberProps m = makeProps(kd, ks, kr, kt, ra, op, eta);
    Interaction si = identityFrame();
    return evaluateUberBSDF_Pdf(&m, &si, load3a(wo), load3a(wi), BSDF_ALL);
}

/* ======================================================================= */
/* Scene                                                                   */
/* ======================================================================= */
typedef struct {   /* RR Bvh2::Node, RR/src/accelerator/bvh2.h:186-204 (64 B) */
    float lmin_v0[3]; uint32_t addr_left;
    float lmax_v1[3]; uint32_t mesh_id;
    float rmin_v2[3]; uint32_t addr_right;
    float rmax[3];    uint32_t prim_id;
} RRNode;
#define INVALID_ADDR 0xffffffffu

struct orc_scene {
    mcrt_scene_desc d;
    RRNode* nodes;
    int64_t num_nodes;
    /* world-space triangles for the brute force (RRT/utils.cpp GetTransformedFace) */
    float* tri;      /* 9 floats per triangle */
    int32_t* tri_shape;
    int32_t* tri_prim;
    int64_t num_tris;
    /* optional per-node "touched" marks for the bench's compulsory-traffic roofline (bench.py):
     * [class][node] bytes, class 0 = camera rays, 1 = extension rays, 2 = shadow rays of bounce 0,
     * 3 = shadow rays of later bounces (k_shadow_extend traces classes 1 + 2 together) */
    uint8_t* touched;
    /* optional per-pixel path log (tools/oracle_divergence.py): pathlog_depth records of
     * ORC_PATHLOG_FLOATS floats per pixel, layout in mcrt_oracle.h */
    float* pathlog;
    int pathlog_depth;
};

static inline void markTouched(uint8_t* mark, uint32_t node) {
    if (mark) __atomic_store_n(&mark[node], (uint8_t)1, __ATOMIC_RELAXED);   /* idempotent; races benign */
}

/* RR transform_point (RR/include/math/mathutils.h:111-118 with matrix*float4,
 * RR/include/math/matrix.h:182-193): sequential sum, w = 0, then + translation. */
static v3 rrTransformPoint(const mcrt_mat4* m, v3 p) {
    const mcrt_float4* r[3] = {&m->m0, &m->m1, &m->m2};
    float o[3];
    for (int i = 0; i < 3; ++i) {
        float acc = 0.0f;
        acc += r[i]->x * p.x;
        acc += r[i]->y * p.y;
        acc += r[i]->z * p.z;
        acc += r[i]->w * 0.0f;
        o[i] = acc + r[i]->w;
    }
    return V3(o[0], o[1], o[2]);
}

orc_scene* orc_scene_create(const mcrt_scene_desc* desc) {
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    s->d = *desc;
    int64_t nt = 0;
    for (uint32_t i = 0; i < desc->num_shapes; ++i) nt += desc->shapes[i].numTriangles;
    s->num_tris = nt;
    s->tri = (float*)malloc(sizeof(float) * 9 * (nt ? nt : 1));
    s->tri_shape = (int32_t*)malloc(sizeof(int32_t) * (nt ? nt : 1));
    s->tri_prim = (int32_t*)malloc(sizeof(int32_t) * (nt ? nt : 1));
    int64_t k = 0;
    for (uint32_t sh = 0; sh < desc->num_shapes; ++sh) {
        const mcrt_shape* S = &desc->shapes[sh];
        for (uint32_t f = 0; f < S->numTriangles; ++f, ++k) {
            for (int c = 0; c < 3; ++c) {
                uint32_t vi = S->startVertex + desc->indices[S->startIdx + 3 * f + c];
                v3 w = rrTransformPoint(&S->toWorldTransform, load3(&desc->positions[vi]));
                s->tri[9 * k + 3 * c + 0] = w.x;
                s->tri[9 * k + 3 * c + 1] = w.y;
                s->tri[9 * k + 3 * c + 2] = w.z;
            }
            s->tri_shape[k] = (int32_t)sh;
            s->tri_prim[k] = (int32_t)f;
        }
    }
    return s;
}
void orc_scene_destroy(orc_scene* s) {
    if (!s) return;
    free(s->nodes); free(s->tri); free(s->tri_shape); free(s->tri_prim);
    free(s);
}

/* ======================================================================= */
/* Bvh2 build: RR/src/accelerator/bvh2.h:206-505, bvh2.cpp:144-712.         */
/* SSE operations are restated with the same intrinsics (the reference uses  */
/* _mm_rcp_ps and _mm_dp_ps, whose results the layout depends on).          */
/* ======================================================================= */
typedef struct { __m128 bmin, bmax, cmin, cmax; size_t start, num; uint32_t level, index; } SplitRequest;
typedef struct {
    float* amin; float* amax; float* acen;   /* 4 floats each (x,y,z,w=0) */
    uint32_t* refs;
    int32_t* meta_shape; int32_t* meta_prim;
    RRNode* nodes;
    uint32_t num_bins;
    float traversal_cost;
    int use_sah;
    const orc_scene* s;
} Builder;

/* bvh2.cpp:69-75 */
static inline __m128 aabb_surface_area(__m128 pmin, __m128 pmax) {
    __m128 ext = _mm_sub_ps(pmax, pmin);
    __m128 xxy = _mm_shuffle_ps(ext, ext, _MM_SHUFFLE(3, 1, 0, 0));
    __m128 yzz = _mm_shuffle_ps(ext, ext, _MM_SHUFFLE(3, 2, 2, 1));
    return _mm_mul_ps(_mm_dp_ps(xxy, yzz, 0xff), _mm_set_ps(2.f, 2.f, 2.f, 2.f));
}
/* bvh2.cpp:83-92 */
static inline uint32_t aabb_max_extent_axis(__m128 pmin, __m128 pmax) {
    __m128 xyz = _mm_sub_ps(pmax, pmin);
    __m128 yzx = _mm_shuffle_ps(xyz, xyz, _MM_SHUFFLE(3, 0, 2, 1));
    __m128 m0 = _mm_max_ps(xyz, yzx);
    __m128 m1 = _mm_shuffle_ps(m0, m0, _MM_SHUFFLE(3, 0, 2, 1));
    __m128 m2 = _mm_max_ps(m0, m1);
    __m128 cmp = _mm_cmpeq_ps(xyz, m2);
    return (uint32_t)__builtin_ctz((unsigned)_mm_movemask_ps(cmp));
}
static inline float mm_select(__m128 v, uint32_t i) { float t[4]; _mm_storeu_ps(t, v); return t[i]; }
static inline __m128 L4(const float* p) { return _mm_loadu_ps(p); }

/* bvh2.cpp:331-492 */
static float findSahSplit(const Builder* b, const SplitRequest* rq, uint32_t axis) {
    float sah = FLT_MAX;
    uint32_t nb = b->num_bins;
    uint32_t* bin_count = (uint32_t*)alloca(sizeof(uint32_t) * nb);
    __m128* bin_min = (__m128*)alloca(sizeof(__m128) * nb);
    __m128* bin_max = (__m128*)alloca(sizeof(__m128) * nb);
    const float inf = INFINITY;
    for (uint32_t i = 0; i < nb; ++i) {
        bin_count[i] = 0;
        bin_min[i] = _mm_set_ps(inf, inf, inf, inf);
        bin_max[i] = _mm_set_ps(-inf, -inf, -inf, -inf);
    }
    __m128 cext = _mm_sub_ps(rq->cmax, rq->cmin);
    float cmin_a = mm_select(rq->cmin, axis);
    float cext_a = mm_select(cext, axis);
    __m128 centroid_min = _mm_set1_ps(cmin_a);
    __m128 centroid_extent = _mm_set1_ps(cext_a);
    __m128 centroid_extent_inv = _mm_rcp_ps(centroid_extent);
    float area_inv = mm_select(_mm_rcp_ps(aabb_surface_area(rq->bmin, rq->bmax)), 0);
    size_t full4 = rq->num & ~(size_t)3;
    __m128 num_bins = _mm_set1_ps((float)nb);
    const uint32_t* refs = b->refs;
    for (size_t i = rq->start; i < rq->start + full4; i += 4) {
        uint32_t idx[4] = {refs[i], refs[i + 1], refs[i + 2], refs[i + 3]};
        __m128 c = _mm_set_ps(b->acen[4 * idx[3] + axis], b->acen[4 * idx[2] + axis],
                              b->acen[4 * idx[1] + axis], b->acen[4 * idx[0] + axis]);
        __m128 bin_idx = _mm_mul_ps(_mm_mul_ps(_mm_sub_ps(c, centroid_min), centroid_extent_inv), num_bins);
        uint32_t bi[4];
        for (int k = 0; k < 4; ++k) {
            uint32_t v = (uint32_t)mm_select(bin_idx, (uint32_t)k);
            bi[k] = v < nb - 1 ? v : nb - 1;
        }
        for (int k = 0; k < 4; ++k) ++bin_count[bi[k]];
        for (int k = 0; k < 4; ++k) {
            bin_min[bi[k]] = _mm_min_ps(bin_min[bi[k]], L4(&b->amin[4 * idx[k]]));
            bin_max[bi[k]] = _mm_max_ps(bin_max[bi[k]], L4(&b->amax[4 * idx[k]]));
        }
    }
    float cm = mm_select(centroid_min, 0u);
    float cei = mm_select(centroid_extent_inv, 0u);
    for (size_t i = rq->start + full4; i < rq->start + rq->num; ++i) {
        uint32_t idx = refs[i];
        uint32_t v = (uint32_t)((float)nb * (b->acen[4 * idx + axis] - cm) * cei);
        uint32_t bin = v < nb - 1 ? v : nb - 1;
        ++bin_count[bin];
        bin_min[bin] = _mm_min_ps(bin_min[bin], L4(&b->amin[4 * idx]));
        bin_max[bin] = _mm_max_ps(bin_max[bin], L4(&b->amax[4 * idx]));
    }
    __m128* right_min = (__m128*)alloca(sizeof(__m128) * (nb - 1));
    __m128* right_max = (__m128*)alloca(sizeof(__m128) * (nb - 1));
    __m128 tmp_min = _mm_set_ps(inf, inf, inf, inf);
    __m128 tmp_max = _mm_set_ps(-inf, -inf, -inf, -inf);
    for (uint32_t i = nb - 1; i > 0; --i) {
        tmp_min = _mm_min_ps(tmp_min, bin_min[i]);
        tmp_max = _mm_max_ps(tmp_max, bin_max[i]);
        right_min[i - 1] = tmp_min;
        right_max[i - 1] = tmp_max;
    }
    tmp_min = _mm_set_ps(inf, inf, inf, inf);
    tmp_max = _mm_set_ps(-inf, -inf, -inf, -inf);
    uint32_t lc = 0;
    size_t rc = rq->num;
    int split_idx = -1;
    for (uint32_t i = 0; i < nb - 1; ++i) {
        tmp_min = _mm_min_ps(tmp_min, bin_min[i]);
        tmp_max = _mm_max_ps(tmp_max, bin_max[i]);
        lc += bin_count[i];
        rc -= bin_count[i];
        float lsa = mm_select(aabb_surface_area(tmp_min, tmp_max), 0);
        float rsa = mm_select(aabb_surface_area(right_min[i], right_max[i]), 0);
        float s = b->traversal_cost + ((float)lc * lsa + (float)rc * rsa) * area_inv;
        if (s < sah) { split_idx = (int)i; sah = s; }
    }
    return cm + (float)(split_idx + 1) * (mm_select(centroid_extent, 0u) / (float)nb);
}

/* bvh2.h:345-369 */
static void setPrimitive(Builder* b, RRNode* node, uint32_t ref) {
    const orc_scene* s = b->s;
    int32_t sh = b->meta_shape[ref];
    int32_t f = b->meta_prim[ref];
    int64_t k = ref;   /* refs are global face indices in shape order */
    node->lmin_v0[0] = s->tri[9 * k + 0]; node->lmin_v0[1] = s->tri[9 * k + 1]; node->lmin_v0[2] = s->tri[9 * k + 2];
    node->lmax_v1[0] = s->tri[9 * k + 3]; node->lmax_v1[1] = s->tri[9 * k + 4]; node->lmax_v1[2] = s->tri[9 * k + 5];
    node->rmin_v2[0] = s->tri[9 * k + 6]; node->rmin_v2[1] = s->tri[9 * k + 7]; node->rmin_v2[2] = s->tri[9 * k + 8];
    node->mesh_id = (uint32_t)sh;
    node->prim_id = (uint32_t)f;
}

/* bvh2.cpp:494-712 */
static int handleRequest(Builder* b, const SplitRequest* rq, SplitRequest* rl, SplitRequest* rr) {
    RRNode* nodes = b->nodes;
    uint32_t* refs = b->refs;
    if (rq->num <= 1) {   /* kMaxLeafPrimitives */
        nodes[rq->index].addr_left = INVALID_ADDR;
        nodes[rq->index].addr_right = INVALID_ADDR;
        for (size_t i = 0; i < rq->num; ++i) setPrimitive(b, &nodes[rq->index], refs[rq->start + i]);
        return 0;
    }
    uint32_t split_axis = aabb_max_extent_axis(rq->cmin, rq->cmax);
    float split_axis_extent = mm_select(_mm_sub_ps(rq->cmax, rq->cmin), split_axis);
    float split_value = mm_select(_mm_mul_ps(_mm_set_ps(0.5f, 0.5f, 0.5f, 0.5f), _mm_add_ps(rq->cmax, rq->cmin)), split_axis);
    size_t split_idx = rq->start;
    const float inf = INFINITY;
    __m128 pinf = _mm_set_ps(inf, inf, inf, inf), minf = _mm_set_ps(-inf, -inf, -inf, -inf);
    __m128 lmin = pinf, lmax = minf, rmin = pinf, rmax = minf;
    __m128 lcmin = pinf, lcmax = minf, rcmin = pinf, rcmax = minf;
    const float *amin = b->amin, *amax = b->amax, *acen = b->acen;
#define ADDL(id) do { lmin = _mm_min_ps(lmin, L4(&amin[4*(id)])); lmax = _mm_max_ps(lmax, L4(&amax[4*(id)])); \
        __m128 c_ = L4(&acen[4*(id)]); lcmin = _mm_min_ps(lcmin, c_); lcmax = _mm_max_ps(lcmax, c_); } while (0)
#define ADDR(id) do { rmin = _mm_min_ps(rmin, L4(&amin[4*(id)])); rmax = _mm_max_ps(rmax, L4(&amax[4*(id)])); \
        __m128 c_ = L4(&acen[4*(id)]); rcmin = _mm_min_ps(rcmin, c_); rcmax = _mm_max_ps(rcmax, c_); } while (0)
    if (split_axis_extent > 0.0f) {
        if (b->use_sah && rq->num > 8)   /* kMinSAHPrimitives */
            split_value = findSahSplit(b, rq, split_axis);
        size_t first = rq->start, last = rq->start + rq->num;
        for (;;) {
            while (first != last && acen[4 * refs[first] + split_axis] < split_value) {
                ADDL(refs[first]);
                ++first;
            }
            if (first == last--) break;
            ADDR(refs[first]);
            while (first != last && acen[4 * refs[last] + split_axis] >= split_value) {
                ADDR(refs[last]);
                --last;
            }
            if (first == last) break;
            ADDL(refs[last]);
            uint32_t t = refs[first]; refs[first] = refs[last]; refs[last] = t;
            ++first;
        }
        split_idx = first;
    }
    if (split_idx == rq->start || split_idx == rq->start + rq->num) {
        split_idx = rq->start + (rq->num >> 1);
        lmin = pinf; lmax = minf; rmin = pinf; rmax = minf;
        lcmin = pinf; lcmax = minf; rcmin = pinf; rcmax = minf;
        for (size_t i = rq->start; i < split_idx; ++i) ADDL(refs[i]);
        for (size_t i = split_idx; i < rq->start + rq->num; ++i) ADDR(refs[i]);
    }
#undef ADDL
#undef ADDR
    rl->bmin = lmin; rl->bmax = lmax; rl->cmin = lcmin; rl->cmax = lcmax;
    rl->start = rq->start; rl->num = split_idx - rq->start;
    rl->level = rq->level + 1; rl->index = rq->index + 1;
    rr->bmin = rmin; rr->bmax = rmax; rr->cmin = rcmin; rr->cmax = rcmax;
    rr->start = split_idx; rr->num = rq->num - rl->num;
    rr->level = rq->level + 1; rr->index = (uint32_t)(rq->index + rl->num * 2);
    /* EncodeInternal, bvh2.h:330-343 */
    float t4[4];
    _mm_storeu_ps(t4, rq->bmin); memcpy(nodes[rq->index].lmin_v0, t4, 12);
    _mm_storeu_ps(t4, rq->bmax); memcpy(nodes[rq->index].lmax_v1, t4, 12);
    /* _mm_store_ps also writes lane 3 (w = 0) over addr_left / mesh_id; they are then set/ignored */
    nodes[rq->index].addr_left = rl->index;
    nodes[rq->index].addr_right = rr->index;
    _mm_storeu_ps(t4, rq->bmax);
    memcpy(&nodes[rq->index].mesh_id, &t4[3], 4);
    return 1;
}

/* bvh2.h:385-505 */
static void propagateBounds(RRNode* nodes) {
    uint32_t* stack = (uint32_t*)malloc(sizeof(uint32_t) * 4096);
    size_t cap = 4096, sp = 0;
    stack[sp++] = 0;
    while (sp) {
        uint32_t idx = stack[--sp];
        RRNode* node = &nodes[idx];
        if (node->addr_left == INVALID_ADDR) continue;
        uint32_t i0 = node->addr_left, i1 = node->addr_right;
        RRNode* c0 = &nodes[i0];
        RRNode* c1 = &nodes[i1];
        if (sp + 2 > cap) { cap *= 2; stack = (uint32_t*)realloc(stack, sizeof(uint32_t) * cap); }
        if (c0->addr_left != INVALID_ADDR) {
            memcpy(node->lmin_v0, c0->lmin_v0, 12);
            memcpy(node->lmax_v1, c0->lmax_v1, 12);
            stack[sp++] = i0;
        } else {
            for (int k = 0; k < 3; ++k) {
                float a = c0->lmin_v0[k], bb = c0->lmax_v1[k], c = c0->rmin_v2[k];
                float mn = (c < bb) ? c : bb; node->lmin_v0[k] = (mn < a) ? mn : a;   /* std::min(a, std::min(b, c)) */
                float mx = (bb < c) ? c : bb; node->lmax_v1[k] = (a < mx) ? mx : a;   /* std::max(a, std::max(b, c)) */
            }
        }
        if (c1->addr_left != INVALID_ADDR) {
            memcpy(node->rmin_v2, c1->lmin_v0, 12);
            memcpy(node->rmax, c1->lmax_v1, 12);
            stack[sp++] = i1;
        } else {
            for (int k = 0; k < 3; ++k) {
                float a = c1->lmin_v0[k], bb = c1->lmax_v1[k], c = c1->rmin_v2[k];
                float mn = (c < bb) ? c : bb; node->rmin_v2[k] = (mn < a) ? mn : a;
                float mx = (bb < c) ? c : bb; node->rmax[k] = (a < mx) ? mx : a;
            }
        }
    }
    free(stack);
}

int64_t orc_bvh_build(orc_scene* s, float traversal_cost, int num_bins, int use_sah) {
    int64_t n = s->num_tris;
    if (n <= 0) return -1;
    free(s->nodes);
    Builder b;
    memset(&b, 0, sizeof(b));
    b.s = s; b.num_bins = (uint32_t)num_bins; b.traversal_cost = traversal_cost; b.use_sah = use_sah;
    b.amin = (float*)malloc(sizeof(float) * 4 * n);
    b.amax = (float*)malloc(sizeof(float) * 4 * n);
    b.acen = (float*)malloc(sizeof(float) * 4 * n);
    b.refs = (uint32_t*)malloc(sizeof(uint32_t) * n);
    b.meta_shape = s->tri_shape; b.meta_prim = s->tri_prim;
    const float inf = INFINITY;
    __m128 smin = _mm_set_ps(inf, inf, inf, inf), smax = _mm_set_ps(-inf, -inf, -inf, -inf);
    __m128 csmin = smin, csmax = smax;
    /* bvh2.h:263-294: Mesh::GetFaceBounds (RR/src/primitive/mesh.cpp:130-141):
     * bbox(v0, v1) with vmin/vmax (std::min/max), then grow(v2). */
    for (int64_t k = 0; k < n; ++k) {
        const float* t = &s->tri[9 * k];
        float mn[4], mx[4];
        for (int c = 0; c < 3; ++c) {
            float a = t[c], bb = t[3 + c], cc = t[6 + c];
            float m0 = (bb < a) ? bb : a;       /* std::min(a, b) */
            float x0 = (a < bb) ? bb : a;       /* std::max(a, b) */
            mn[c] = (cc < m0) ? cc : m0;        /* vmin(pmin, p) = std::min(pmin, p) */
            x0 = (x0 < cc) ? cc : x0;
            mx[c] = x0;
        }
        mn[3] = 0.0f; mx[3] = 0.0f;
        __m128 pmin = _mm_loadu_ps(mn), pmax = _mm_loadu_ps(mx);
        __m128 cen = _mm_mul_ps(_mm_add_ps(pmin, pmax), _mm_set_ps(0.5f, 0.5f, 0.5f, 0.5f));
        smin = _mm_min_ps(smin, pmin); smax = _mm_max_ps(smax, pmax);
        csmin = _mm_min_ps(csmin, cen); csmax = _mm_max_ps(csmax, cen);
        _mm_storeu_ps(&b.amin[4 * k], pmin);
        _mm_storeu_ps(&b.amax[4 * k], pmax);
        _mm_storeu_ps(&b.acen[4 * k], cen);
        b.refs[k] = (uint32_t)k;
    }
    int64_t count = 2 * n - 1;
    b.nodes = (RRNode*)malloc(sizeof(RRNode) * count);
    for (int64_t i = 0; i < count; ++i) {
        memset(&b.nodes[i], 0, sizeof(RRNode));
        b.nodes[i].addr_left = b.nodes[i].mesh_id = b.nodes[i].addr_right = b.nodes[i].prim_id = INVALID_ADDR;
    }
    /* depth-first, explicit stack (the layout is independent of processing order) */
    size_t cap = 1024, sp = 0;
    SplitRequest* st = (SplitRequest*)malloc(sizeof(SplitRequest) * cap);
    SplitRequest root = {smin, smax, csmin, csmax, 0, (size_t)n, 0, 0};
    st[sp++] = root;
    while (sp) {
        SplitRequest rq = st[--sp];
        SplitRequest rl, rr;
        if (handleRequest(&b, &rq, &rl, &rr)) {
            if (sp + 2 > cap) { cap *= 2; st = (SplitRequest*)realloc(st, sizeof(SplitRequest) * cap); }
            st[sp++] = rr;
            st[sp++] = rl;
        }
    }
    free(st);
    propagateBounds(b.nodes);
    free(b.amin); free(b.amax); free(b.acen); free(b.refs);
    s->nodes = b.nodes;
    s->num_nodes = count;
    return count;
}

int64_t orc_bvh_nodes(orc_scene* s, void* out, int64_t max_nodes) {
    int64_t n = s->num_nodes < max_nodes ? s->num_nodes : max_nodes;
    if (n > 0) memcpy(out, s->nodes, sizeof(RRNode) * n);
    return s->num_nodes;
}

/* ======================================================================= */
/* Traversal: RR/src/kernels/CL/intersect_bvh2_lds.cl + common.cl           */
/* ======================================================================= */
typedef struct { v3 o, d; float tmax; int mask, active; } Ray;

static inline Ray loadRay(const mcrt_ray* r) {
    Ray R;
    R.o = V3(r->o.x, r->o.y, r->o.z); R.tmax = r->o.w;
    R.d = V3(r->d.x, r->d.y, r->d.z);
    R.mask = r->extra[0]; R.active = r->extra[1];
    return R;
}
/* common.cl:220-232 */
static inline v3 safe_invdir(v3 d) {
    const float ooeps = 1e-8f;
    return V3(1.0f / (fabsf(d.x) > ooeps ? d.x : copysignf(ooeps, d.x)),
              1.0f / (fabsf(d.y) > ooeps ? d.y : copysignf(ooeps, d.y)),
              1.0f / (fabsf(d.z) > ooeps ? d.z : copysignf(ooeps, d.z)));
}
/* intersect_bvh2_lds.cl:54-63 (mad = fused multiply-add) */
static inline void bbox2(const float* pmin, const float* pmax, v3 inv, v3 oxinv, float t_max, float* t0, float* t1) {
    float fx = fmaf(pmax[0], inv.x, oxinv.x), fy = fmaf(pmax[1], inv.y, oxinv.y), fz = fmaf(pmax[2], inv.z, oxinv.z);
    float nx = fmaf(pmin[0], inv.x, oxinv.x), ny = fmaf(pmin[1], inv.y, oxinv.y), nz = fmaf(pmin[2], inv.z, oxinv.z);
    float tmx = fmaxf(fx, nx), tmy = fmaxf(fy, ny), tmz = fmaxf(fz, nz);
    float tnx = fminf(fx, nx), tny = fminf(fy, ny), tnz = fminf(fz, nz);
    *t1 = fminf(fminf(fminf(tmx, tmy), tmz), t_max);
    *t0 = fmaxf(fmaxf(fmaxf(tnx, tny), tnz), 0.f);
}
/* common.cl:177-218 (native_recip restated as 1/x) */
static inline float fastTriangle(const Ray* r, const float* v1, const float* v2, const float* v3p, float t_max) {
    v3 a = load3a(v1), b = load3a(v2), c = load3a(v3p);
    v3 e1 = vsub(b, a), e2 = vsub(c, a);
    v3 s1 = vcross(r->d, e2);
    float denom = vdot(s1, e1);
    if (denom == 0.f) return t_max;
    float invd = 1.0f / denom;
    v3 d = vsub(r->o, a);
    float b1 = vdot(d, s1) * invd;
    v3 s2 = vcross(d, e1);
    float b2 = vdot(r->d, s2) * invd;
    float temp = vdot(e2, s2) * invd;
    if (b1 < 0.f || b1 > 1.f || b2 < 0.f || b1 + b2 > 1.f || temp < 0.f || temp > t_max) return t_max;
    return temp;
}
/* common.cl:249-277 */
static inline void triBarycentrics(v3 p, const float* v1, const float* v2, const float* v3p, float* u, float* v) {
    v3 a = load3a(v1);
    v3 e1 = vsub(load3a(v2), a), e2 = vsub(load3a(v3p), a), e = vsub(p, a);
    float d00 = vdot(e1, e1), d01 = vdot(e1, e2), d11 = vdot(e2, e2), d20 = vdot(e, e1), d21 = vdot(e, e2);
    float denom = (d00 * d11 - d01 * d01);
    if (denom == 0.f) { *u = 0.f; *v = 0.f; return; }
    float inv = 1.0f / denom;
    *u = (d11 * d20 - d01 * d21) * inv;
    *v = (d00 * d21 - d01 * d20) * inv;
}

typedef struct { uint32_t* data; int cap; } Stack;
/* leaf visits of the calling thread's walks (render stats [6], [7]: the traversal's leaf / internal
 * mix, which prices the product's compact records at 48 / 32 B, bench.py gather_ceiling) */
static _Thread_local int64_t tl_leafVisits;

/* intersect_bvh2_lds.cl:66-226 (the LDS short stack + global spill is one LIFO) */
static int traceClosest(const orc_scene* s, const Ray* r, mcrt_intersection* hit, uint32_t* stack, int* visits,
                        uint8_t* mark) {
    const RRNode* nodes = s->nodes;
    v3 inv = safe_invdir(r->d);
    v3 oxinv = V3(-r->o.x * inv.x, -r->o.y * inv.y, -r->o.z * inv.z);
    float closest_t = r->tmax;
    uint32_t addr = 0, closest_addr = INVALID_ADDR;
    int sp = 0, nv = 0;
    stack[sp++] = INVALID_ADDR;
    while (addr != INVALID_ADDR) {
        const RRNode* node = &nodes[addr];
        ++nv;
        markTouched(mark, addr);
        if (node->addr_left != INVALID_ADDR) {
            float a0, a1, b0, b1;
            bbox2(node->lmin_v0, node->lmax_v1, inv, oxinv, closest_t, &a0, &a1);
            bbox2(node->rmin_v2, node->rmax, inv, oxinv, closest_t, &b0, &b1);
            int tc0 = a0 <= a1, tc1 = b0 <= b1;
            int c1first = tc1 && (a0 > b0);
            if (tc0 || tc1) {
                uint32_t deferred;
                if (c1first || !tc0) { addr = node->addr_right; deferred = node->addr_left; }
                else { addr = node->addr_left; deferred = node->addr_right; }
                if (tc0 && tc1) stack[sp++] = deferred;
                continue;
            }
        } else {
            ++tl_leafVisits;
            if (r->mask != (int)node->mesh_id) {   /* RR_RAY_MASK */
                float t = fastTriangle(r, node->lmin_v0, node->lmax_v1, node->rmin_v2, closest_t);
                if (t < closest_t) { closest_t = t; closest_addr = addr; }
            }
        }
        addr = stack[--sp];
    }
    if (visits) *visits = nv;
    if (closest_addr != INVALID_ADDR) {
        const RRNode* node = &nodes[closest_addr];
        v3 p = vadd(r->o, sv(closest_t, r->d));
        float u, v;
        triBarycentrics(p, node->lmin_v0, node->lmax_v1, node->rmin_v2, &u, &v);
        hit->primid = (int32_t)node->prim_id;
        hit->shapeid = (int32_t)node->mesh_id;
        hit->uvwt.x = u; hit->uvwt.y = v; hit->uvwt.z = 0.0f; hit->uvwt.w = closest_t;
        return 1;
    }
    hit->primid = -1;
    hit->shapeid = -1;
    return 0;
}
/* intersect_bvh2_lds.cl:229-363 */
static int traceAny(const orc_scene* s, const Ray* r, uint32_t* stack, int* visits, uint8_t* mark) {
    const RRNode* nodes = s->nodes;
    v3 inv = safe_invdir(r->d);
    v3 oxinv = V3(-r->o.x * inv.x, -r->o.y * inv.y, -r->o.z * inv.z);
    const float closest_t = r->tmax;
    uint32_t addr = 0;
    int sp = 0, nv = 0;
    stack[sp++] = INVALID_ADDR;
    while (addr != INVALID_ADDR) {
        const RRNode* node = &nodes[addr];
        ++nv;
        markTouched(mark, addr);
        if (node->addr_left != INVALID_ADDR) {
            float a0, a1, b0, b1;
            bbox2(node->lmin_v0, node->lmax_v1, inv, oxinv, closest_t, &a0, &a1);
            bbox2(node->rmin_v2, node->rmax, inv, oxinv, closest_t, &b0, &b1);
            int tc0 = a0 <= a1, tc1 = b0 <= b1;
            int c1first = tc1 && (a0 > b0);
            if (tc0 || tc1) {
                uint32_t deferred;
                if (c1first || !tc0) { addr = node->addr_right; deferred = node->addr_left; }
                else { addr = node->addr_left; deferred = node->addr_right; }
                if (tc0 && tc1) stack[sp++] = deferred;
                continue;
            }
        } else {
            ++tl_leafVisits;
            if (r->mask != (int)node->mesh_id) {
                float t = fastTriangle(r, node->lmin_v0, node->lmax_v1, node->rmin_v2, closest_t);
                if (t < closest_t) { if (visits) *visits = nv; return 1; }
            }
        }
        addr = stack[--sp];
    }
    if (visits) *visits = nv;
    return -1;
}

/* ----------------------------------------------------------------------- */
/* simple pthread parallel-for                                              */
/* ----------------------------------------------------------------------- */
typedef void (*work_fn)(void* ctx, int64_t i, uint32_t* stack);
typedef struct { work_fn fn; void* ctx; int64_t n; atomic_llong next; int64_t chunk; } PFor;
static void* pfor_worker(void* arg) {
    PFor* p = (PFor*)arg;
    uint32_t* stack = (uint32_t*)malloc(sizeof(uint32_t) * 4096);
    for (;;) {
        int64_t i0 = atomic_fetch_add(&p->next, p->chunk);
        if (i0 >= p->n) break;
        int64_t i1 = i0 + p->chunk < p->n ? i0 + p->chunk : p->n;
        for (int64_t i = i0; i < i1; ++i) p->fn(p->ctx, i, stack);
    }
    free(stack);
    return NULL;
}
static void parallel_for(int64_t n, int threads, int64_t chunk, work_fn fn, void* ctx) {
    PFor p;
    p.fn = fn; p.ctx = ctx; p.n = n; p.chunk = chunk > 0 ? chunk : 1;
    atomic_init(&p.next, 0);
    if (threads <= 1) { pfor_worker(&p); return; }
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * threads);
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, pfor_worker, &p);
    for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL);
    free(th);
}

typedef struct { const orc_scene* s; const mcrt_ray* rays; mcrt_intersection* hits; int32_t* ihits; int32_t* visits; } TraceCtx;
static void closest_one(void* c, int64_t i, uint32_t* stack) {
    TraceCtx* t = (TraceCtx*)c;
    Ray r = loadRay(&t->rays[i]);
    if (!r.active) { if (t->visits) t->visits[i] = 0; return; }   /* record untouched (Q12) */
    int nv = 0;
    traceClosest(t->s, &r, &t->hits[i], stack, &nv, NULL);
    if (t->visits) t->visits[i] = nv;
}
static void any_one(void* c, int64_t i, uint32_t* stack) {
    TraceCtx* t = (TraceCtx*)c;
    Ray r = loadRay(&t->rays[i]);
    if (!r.active) { if (t->visits) t->visits[i] = 0; return; }
    int nv = 0;
    t->ihits[i] = traceAny(t->s, &r, stack, &nv, NULL);
    if (t->visits) t->visits[i] = nv;
}
void orc_trace_closest(orc_scene* s, const mcrt_ray* rays, int n, mcrt_intersection* hits, int32_t* visits, int threads) {
    TraceCtx t = {s, rays, hits, NULL, visits};
    parallel_for(n, threads, 256, closest_one, &t);
}
void orc_trace_any(orc_scene* s, const mcrt_ray* rays, int n, int32_t* hits, int32_t* visits, int threads) {
    TraceCtx t = {s, rays, NULL, hits, visits};
    parallel_for(n, threads, 256, any_one, &t);
}

/* ----------------------------------------------------------------------- */
/* Premise of the compact walk's near-tie repeat (product: mcrt_traverse.h  */
/* qwalk; checked by tests/test_tie_premise_cpu.py)                         */
/* ----------------------------------------------------------------------- */
/* The reference culls a leaf at its parent when the leaf box's entry (fast_intersect_bbox2,
 * intersect_bvh2_lds.cl:54-63, the box the parent stores) exceeds the closest distance found so
 * far (:128-141), and accepts a triangle when its Moller-Trumbore t (common.cl:177-218) is below it.
 * The two are computed differently, so a triangle X can have t_X < e_X ("irregular"): then a hit Y
 * with t_X < t_Y < e_X, found before X's parent is visited, culls the nearer X, and the answer
 * depends on the visit order -- which the compact walk's outward boxes change.  The near-tie repeat
 * (a hit within alpha = 2^-18 of the final distance sends the ray to the exact records) covers such
 * a pair only when t_Y - t_X <= alpha t_Y.  For every ray this enumerates ALL triangle hits up to
 * twice the reference's distance (padded boxes, no culling) with the product's arithmetic (fma
 * dot / cross as triRaw and cl_dot; v_rcp restated as 1/x) and reports, per ray, 6 floats:
 *   [0] the reference walk's distance t_R (+inf: no hit -- then nothing depends on the order)
 *   [1] the largest (t_Y - t_X) / t_Y over ORDER-DEPENDENT pairs: X with t_X <= t_R (1 + alpha), Y
 *       an acceptable hit with t_X < t_Y < e_X (-1: none); the premise is [1] <= alpha
 *   [2] the largest (e_X - t_X) / t_X over the enumerated hits (0: none irregular)
 *   [3] hits enumerated  [4] irregular hits among them
 *   [5] 1 when the check is incomplete for the ray (a hit list overflow, or some X with e_X beyond
 *       the enumerated range), else 0 */
#define PREMISE_MAXHITS 2048
static inline float dotG(v3 a, v3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
static inline v3 crossG(v3 a, v3 b) {
    return V3(fmaf(a.y, b.z, b.y * -a.z), fmaf(a.z, b.x, b.z * -a.x), fmaf(a.x, b.y, b.x * -a.y));
}
/* the product's triRaw (mcrt_traverse.h): the distance, or +inf */
static float triGpu(const Ray* r, const RRNode* n) {
    v3 a = load3a(n->lmin_v0);
    v3 e1 = vsub(load3a(n->lmax_v1), a), e2 = vsub(load3a(n->rmin_v2), a);
    v3 s1 = crossG(r->d, e2);
    float denom = dotG(s1, e1);
    if (denom == 0.f) return INFINITY;
    float invd = 1.0f / denom;
    v3 d = vsub(r->o, a);
    float b1 = dotG(d, s1) * invd;
    v3 s2 = crossG(d, e1);
    float b2 = dotG(r->d, s2) * invd;
    float temp = dotG(e2, s2) * invd;
    if (b1 < 0.f || b1 > 1.f || b2 < 0.f || b1 + b2 > 1.f || temp < 0.f) return INFINITY;
    return temp;
}
/* the slab interval of a padded box in double (enumeration only: contains every hit point) */
static int paddedOverlap(const float* lo, const float* hi, v3 o, v3 d, double T) {
    const double oo[3] = {o.x, o.y, o.z}, dd[3] = {d.x, d.y, d.z};
    double t0 = 0.0, t1 = T;
    for (int a = 0; a < 3; ++a) {
        const double pad = 1e-4 * (fabs((double)lo[a]) + fabs((double)hi[a])) + 1e-6;
        const double l = lo[a] - pad, h = hi[a] + pad;
        if (fabs(dd[a]) < 1e-30) {
            if (oo[a] < l || oo[a] > h) return 0;
            continue;
        }
        double u0 = (l - oo[a]) / dd[a], u1 = (h - oo[a]) / dd[a];
        if (u0 > u1) { double s = u0; u0 = u1; u1 = s; }
        if (u0 > t0) t0 = u0;
        if (u1 < t1) t1 = u1;
        if (t0 > t1) return 0;
    }
    return 1;
}
typedef struct { float t, e; int ok; } PHit;
static void premise_one(const orc_scene* s, const Ray* r, float alpha, uint32_t* stack, float* out) {
    const RRNode* nodes = s->nodes;
    out[0] = INFINITY; out[1] = -1.0f; out[2] = 0.0f; out[3] = 0.0f; out[4] = 0.0f; out[5] = 0.0f;
    /* 1. the reference walk (traceClosest with the product's triangle arithmetic) */
    v3 inv = safe_invdir(r->d);
    v3 oxinv = V3(-r->o.x * inv.x, -r->o.y * inv.y, -r->o.z * inv.z);
    float tR = r->tmax;
    int found = 0;
    uint32_t addr = 0;
    int sp = 0;
    stack[sp++] = INVALID_ADDR;
    while (addr != INVALID_ADDR) {
        const RRNode* node = &nodes[addr];
        if (node->addr_left != INVALID_ADDR) {
            float a0, a1, b0, b1;
            bbox2(node->lmin_v0, node->lmax_v1, inv, oxinv, tR, &a0, &a1);
            bbox2(node->rmin_v2, node->rmax, inv, oxinv, tR, &b0, &b1);
            int tc0 = a0 <= a1, tc1 = b0 <= b1;
            int c1first = tc1 && (a0 > b0);
            if (tc0 || tc1) {
                uint32_t deferred;
                if (c1first || !tc0) { addr = node->addr_right; deferred = node->addr_left; }
                else { addr = node->addr_left; deferred = node->addr_right; }
                if (tc0 && tc1) stack[sp++] = deferred;
                continue;
            }
        } else if (r->mask != (int)node->mesh_id) {
            float t = triGpu(r, node);
            if (t < tR) { tR = t; found = 1; }
        }
        addr = stack[--sp];
    }
    if (!found) return;   /* no hit: every candidate was culled by tmax alone, in any order */
    out[0] = tR;
    /* 2. every hit up to T: padded boxes, no culling; per hit its leaf box entry e as the
     *    reference computes it at the parent (t0 of fast_intersect_bbox2) */
    const double T = fmin((double)r->tmax, 2.0 * (double)tR + 1e-3);
    PHit hits[PREMISE_MAXHITS];
    int nh = 0, incomplete = 0;
    if (nodes[0].addr_left == INVALID_ADDR) return;   /* a root leaf has no box test */
    sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const RRNode* node = &nodes[stack[--sp]];
        for (int side = 0; side < 2; ++side) {
            const float* lo = side ? node->rmin_v2 : node->lmin_v0;
            const float* hi = side ? node->rmax : node->lmax_v1;
            const uint32_t ch = side ? node->addr_right : node->addr_left;
            if (!paddedOverlap(lo, hi, r->o, r->d, T)) continue;
            const RRNode* c = &nodes[ch];
            if (c->addr_left != INVALID_ADDR) {
                if (sp < 4000) stack[sp++] = ch; else incomplete = 1;
                continue;
            }
            if (r->mask == (int)c->mesh_id) continue;
            const float th = triGpu(r, c);
            if (!(th <= T)) continue;
            float e0, e1;
            bbox2(lo, hi, inv, oxinv, INFINITY, &e0, &e1);
            if (nh == PREMISE_MAXHITS) { incomplete = 1; continue; }
            /* acceptable at all: its box passes at some culling distance <= tmax (the far side and
             * tmax do not depend on the order) */
            hits[nh].t = th;
            hits[nh].e = e0;
            hits[nh].ok = e0 <= e1 && e0 <= r->tmax && th < r->tmax;
            ++nh;
        }
    }
    float worstGap = -1.0f, worstIrr = 0.0f;
    int nirr = 0;
    for (int i = 0; i < nh; ++i) {
        const PHit X = hits[i];
        if (X.e > X.t) {
            ++nirr;
            const float irr = (X.e - X.t) / X.t;
            if (irr > worstIrr) worstIrr = irr;
        }
        if (!(X.t <= tR * (1.0f + alpha)) || !(X.e > X.t)) continue;
        if ((double)X.e > T) incomplete = 1;
        for (int j = 0; j < nh; ++j) {
            const PHit Y = hits[j];
            if (j == i || !Y.ok || !(Y.t > X.t) || !(Y.t < X.e)) continue;
            const float gap = (Y.t - X.t) / Y.t;
            if (gap > worstGap) worstGap = gap;
        }
    }
    out[1] = worstGap;
    out[2] = worstIrr;
    out[3] = (float)nh;
    out[4] = (float)nirr;
    out[5] = (float)incomplete;
}
typedef struct { const orc_scene* s; const mcrt_ray* rays; float* out; float alpha; } PremiseCtx;
static void premise_fn(void* c, int64_t i, uint32_t* stack) {
    PremiseCtx* p = (PremiseCtx*)c;
    Ray r = loadRay(&p->rays[i]);
    float* o = p->out + 6 * i;
    if (!r.active) { o[0] = INFINITY; o[1] = -1.0f; o[2] = o[3] = o[4] = o[5] = 0.0f; return; }
    premise_one(p->s, &r, p->alpha, stack, o);
}
void orc_tie_premise(orc_scene* s, const mcrt_ray* rays, int n, float alpha, float* out, int threads) {
    PremiseCtx p = {s, rays, out, alpha};
    parallel_for(n, threads, 64, premise_fn, &p);
}

/* ----------------------------------------------------------------------- */
/* Brute force: RRT/utils.cpp:44-189 (TestIntersections / TestOcclusions)   */
/* ----------------------------------------------------------------------- */
void orc_brute_closest(orc_scene* s, const mcrt_ray* rays, int n, mcrt_intersection* hits) {
    for (int i = 0; i < n; ++i) {
        Ray r = loadRay(&rays[i]);
        mcrt_intersection h;
        memset(&h, 0, sizeof(h));
        h.shapeid = -1; h.primid = -1;
        h.uvwt.w = FLT_MAX;
        for (int64_t k = 0; k < s->num_tris; ++k) {
            const float* t = &s->tri[9 * k];
            v3 v0 = load3a(t);
            v3 e1 = vsub(load3a(t + 3), v0), e2 = vsub(load3a(t + 6), v0);
            v3 s1 = vcross(r.d, e2);
            float det = vdot(s1, e1);
            float invdet = 1.f / det;
            v3 d = vsub(r.o, v0);
            float b1 = vdot(d, s1) * invdet;
            if (b1 < 0.f || b1 > 1.f) continue;
            v3 s2 = vcross(d, e1);
            float b2 = vdot(r.d, s2) * invdet;
            if (b2 < 0.f || b1 + b2 > 1.f) continue;
            float temp = vdot(e2, s2) * invdet;
            if (temp > 0.f && temp < h.uvwt.w) {
                h.uvwt.x = b1; h.uvwt.y = b2; h.uvwt.z = 0; h.uvwt.w = temp;
                h.shapeid = s->tri_shape[k];
                h.primid = s->tri_prim[k];
            }
        }
        hits[i] = h;
    }
}
void orc_brute_any(orc_scene* s, const mcrt_ray* rays, int n, int32_t* hits) {
    for (int i = 0; i < n; ++i) {
        Ray r = loadRay(&rays[i]);
        int hit = 0;
        for (int64_t k = 0; k < s->num_tris && !hit; ++k) {
            const float* t = &s->tri[9 * k];
            v3 v0 = load3a(t);
            v3 e1 = vsub(load3a(t + 3), v0), e2 = vsub(load3a(t + 6), v0);
            v3 s1 = vcross(r.d, e2);
            float det = vdot(s1, e1);
            float invdet = 1.f / det;
            v3 d = vsub(r.o, v0);
            float b1 = vdot(d, s1) * invdet;
            if (b1 < 0.f || b1 > 1.f) continue;
            v3 s2 = vcross(d, e1);
            float b2 = vdot(r.d, s2) * invdet;
            if (b2 < 0.f || b1 + b2 > 1.f) continue;
            float temp = vdot(e2, s2) * invdet;
            if (temp > 0.f) hit = 1;
        }
        hits[i] = hit ? 1 : -1;
    }
}

/* ======================================================================= */
/* Textures: KRN/textures.cl:70-125 (bilinear, always; readTexture2Df :204-209) */
/* ======================================================================= */
typedef struct { float x, y, z, w; } f4;
static f4 readTex(const orc_scene* s, int texId, v2 uv) {
    const mcrt_texture_desc* tex = &s->d.textures[texId];
    int w = tex->width, h = tex->height;
    uv.x -= 1.0f / (float)w * 0.5f;
    uv.y -= 1.0f / (float)h * 0.5f;
    switch (tex->wrap) {
    case 0: uv.x -= floorf(uv.x); uv.y -= floorf(uv.y); break;           /* REPEAT */
    case 1:                                                               /* MIRRORED_REPEAT */
        if (uv.x > 1.0f || uv.x < 0.0f) uv.x = 1.0f - (uv.x - floorf(uv.x));
        if (uv.y > 1.0f || uv.y < 0.0f) uv.y = 1.0f - (uv.y - floorf(uv.y));
        break;
    case 2: uv.x = clampf(uv.x, 0.0f, 1.0f); uv.y = clampf(uv.y, 0.0f, 1.0f); break;   /* CLAMP_TO_EDGE */
    case 3:                                                               /* CLAMP_TO_BORDER */
        if (uv.x > 1.0f || uv.x < 0.0f || uv.y > 1.0f || uv.y < 0.0f) { f4 z = {0, 0, 0, 0}; return z; }
        break;
    }
    int x0 = ((int)floorf(uv.x * (float)w)) % w;
    int y0 = ((int)floorf(uv.y * (float)h)) % h;
    int x1 = (x0 + 1) % w;
    int y1 = (y0 + 1) % h;
    x0 = x0 < 0 ? 0 : (x0 > w - 1 ? w - 1 : x0);
    y0 = y0 < 0 ? 0 : (y0 > h - 1 ? h - 1 : y0);
    x1 = x1 < 0 ? 0 : (x1 > w - 1 ? w - 1 : x1);
    y1 = y1 < 0 ? 0 : (y1 > h - 1 ? h - 1 : y1);
    float tx = uv.x * (float)w - floorf(uv.x * (float)w);
    float ty = uv.y * (float)h - floorf(uv.y * (float)h);
    const uint8_t* base = s->d.tex_data + tex->memOffset;
    const uint8_t* p00 = base + 4 * (x0 + y0 * w);
    const uint8_t* p10 = base + 4 * (x1 + y0 * w);
    const uint8_t* p01 = base + 4 * (x0 + y1 * w);
    const uint8_t* p11 = base + 4 * (x1 + y1 * w);
    float r[4];
    for (int c = 0; c < 4; ++c) {
        float a = p00[c], b = p10[c], cc = p01[c], d = p11[c];
        float m0 = a + (b - a) * tx;
        float m1 = cc + (d - cc) * tx;
        r[c] = (m0 + (m1 - m0) * ty) * (1.0f / 255.0f);
    }
    f4 o = {r[0], r[1], r[2], r[3]};
    return o;
}

/* KRN/materials.cl:76-91 */
static void getUberProps(const orc_scene* s, int mi, const Interaction* si, UberProps* p) {
    const mcrt_material* m = &s->d.materials[mi];
    f4 kdo = {1.0f, 1.0f, 1.0f, 1.0f};
    if (m->uber_diffuseTexId != -1) kdo = readTex(s, m->uber_diffuseTexId, si->uv);
    p->Kd = vmul(V3(kdo.x, kdo.y, kdo.z), load3(&m->uber_kd));
    v3 t3;
    if (m->uber_glossyTexId != -1) { f4 t = readTex(s, m->uber_glossyTexId, si->uv); t3 = V3(t.x, t.y, t.z); } else t3 = V3(1, 1, 1);
    p->Ks = vmul(t3, load3(&m->uber_ks));
    if (m->uber_specReflectionTexId != -1) { f4 t = readTex(s, m->uber_specReflectionTexId, si->uv); t3 = V3(t.x, t.y, t.z); } else t3 = V3(1, 1, 1);
    p->Kr = vmul(t3, load3(&m->uber_kr));
    if (m->uber_transmissionTexId != -1) { f4 t = readTex(s, m->uber_transmissionTexId, si->uv); t3 = V3(t.x, t.y, t.z); } else t3 = V3(1, 1, 1);
    v3 kt = vmul(t3, load3(&m->uber_kt));
    p->Kt[0] = kt.x; p->Kt[1] = kt.y; p->Kt[2] = kt.z; p->Kt[3] = m->uber_kt.w;
    if (m->uber_opacityTexId != -1) { f4 t = readTex(s, m->uber_opacityTexId, si->uv); t3 = V3(t.x, t.y, t.z); } else t3 = V3(1, 1, 1);
    p->opacity = vs(vmul(t3, load3(&m->uber_opacity)), kdo.w);
    if (m->uber_roughnessTexId != -1) { f4 t = readTex(s, m->uber_roughnessTexId, si->uv); p->roughness.x = t.x; p->roughness.y = t.y; }
    else { p->roughness.x = m->uber_roughness.x; p->roughness.y = m->uber_roughness.y; }
    if (m->uber_iorTexId != -1) { f4 t = readTex(s, m->uber_iorTexId, si->uv); p->eta = t.x; } else p->eta = m->uber_eta;
    p->roughness.x = orc_roughness_to_alpha(p->roughness.x);
    p->roughness.y = orc_roughness_to_alpha(p->roughness.y);
}

/* KRN/materials.cl:14-30 */
static void applyNormalMapping(const orc_scene* s, int mi, Interaction* si) {
    if (mi == -1) return;
    int texId = s->d.materials[mi].uber_normalMapId;
    if (texId == -1) return;
    f4 t = readTex(s, texId, si->uv);
    v3 nm = V3(2.0f * t.x - 1.0f, 2.0f * t.y - 1.0f, 2.0f * t.z - 1.0f);
    si->sn = vnormalize(vadd(vadd(vs(si->sdpdu, nm.x), vs(si->sdpdv, nm.y)), vs(si->sn, nm.z)));
    si->sdpdu = vnormalize(vcross(si->sn, si->sdpdv));
    si->sdpdv = vnormalize(vcross(si->sdpdu, si->sn));
}

/* KRN/geometry.cl:9-28 */
static void triPartials(v2 uv0, v2 uv1, v2 uv2, v3 p0, v3 p1, v3 p2, v3 n, v3* dpdu, v3* dpdv) {
    v2 duv02 = {uv0.x - uv2.x, uv0.y - uv2.y};
    v2 duv12 = {uv1.x - uv2.x, uv1.y - uv2.y};
    v3 dp02 = vsub(p0, p2), dp12 = vsub(p1, p2);
    float det = duv02.x * duv12.y - duv02.y * duv12.x;
    if (isNotNearZero(det)) {
        float invdet = 1.0f / det;
        *dpdu = vs(vsub(sv(duv12.y, dp02), sv(duv02.y, dp12)), invdet);
        *dpdv = vs(vneg(vadd(sv(-duv12.x, dp02), sv(duv02.x, dp12))), invdet);
    } else {
        *dpdu = vnormalize(computeOrthogonalVector(n));
        *dpdv = vnormalize(vcross(n, *dpdu));
    }
}

/* KRN/geometry.cl:177-215 */
static void computeSurfaceInteraction(const orc_scene* s, int shapeId, int primIdx, float bu, float bv, Interaction* si) {
    const mcrt_shape* sh = &s->d.shapes[shapeId];
    const uint32_t* I = s->d.indices;
    uint32_t i0 = I[sh->startIdx + 3 * primIdx], i1 = I[sh->startIdx + 3 * primIdx + 1], i2 = I[sh->startIdx + 3 * primIdx + 2];
    uint32_t sv0 = sh->startVertex;
    v3 p0 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sv0 + i0]));
    v3 p1 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sv0 + i1]));
    v3 p2 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sv0 + i2]));
    v2 uv0 = {s->d.uvs[sv0 + i0].x, s->d.uvs[sv0 + i0].y};
    v2 uv1 = {s->d.uvs[sv0 + i1].x, s->d.uvs[sv0 + i1].y};
    v2 uv2 = {s->d.uvs[sv0 + i2].x, s->d.uvs[sv0 + i2].y};
    v3 n0 = transformVector3(&sh->toWorldInverseTranspose, load3(&s->d.normals[sv0 + i0]));
    v3 n1 = transformVector3(&sh->toWorldInverseTranspose, load3(&s->d.normals[sv0 + i1]));
    v3 n2 = transformVector3(&sh->toWorldInverseTranspose, load3(&s->d.normals[sv0 + i2]));
    float w0 = 1.0f - bu - bv;
    si->p = vadd(vadd(vs(p0, w0), vs(p1, bu)), vs(p2, bv));
    si->uv.x = uv0.x * w0 + uv1.x * bu + uv2.x * bv;
    si->uv.y = uv0.y * w0 + uv1.y * bu + uv2.y * bv;
    si->gn = vnormalize(vcross(vsub(p0, p2), vsub(p1, p2)));
    si->sn = vnormalize(vadd(vadd(vs(n0, w0), vs(n1, bu)), vs(n2, bv)));
    triPartials(uv0, uv1, uv2, p0, p1, p2, si->sn, &si->dpdu, &si->dpdv);
    si->sdpdu = vnormalize(vsub(si->dpdu, sv(vdot(si->sn, si->dpdu), si->sn)));
    si->sdpdv = vnormalize(vsub(vsub(si->dpdv, sv(vdot(si->sn, si->dpdv), si->sn)), sv(vdot(si->sdpdu, si->dpdv), si->sdpdu)));
    si->shapeIdx = shapeId;
}

/* ======================================================================= */
/* Lights: KRN/lights.cl                                                    */
/* ======================================================================= */
/* lights.cl:29-39 */
static v3 evalLightLe(const mcrt_light* L, v3 gn, v3 w) {
    if (L->type == MCRT_DISK_AREA_LIGHT || L->type == MCRT_TRIANGLE_MESH_AREA_LIGHT)
        return vdot(gn, w) > 0.0f ? load3(&L->intensity) : V3(0, 0, 0);
    return V3(0, 0, 0);
}
/* lights.cl:45-146.  Writes the shadow ray (setRay) only where the reference does. */
static v3 sampleLightLi(const orc_scene* s, int li, const Interaction* it, v2 u, v3* wi, float* pdf,
                        Ray* shadow, int* shadowSet) {
    const mcrt_light* L = &s->d.lights[li];
    *shadowSet = 0;
    switch (L->type) {
    case MCRT_DIRECTIONAL_LIGHT: {
        *wi = vneg(load3(&L->d));
        *pdf = 1.0f;
        shadow->o = vadd(it->p, vs(it->gn, it->traceErrorOffset));
        shadow->tmax = 1000.0f; shadow->d = *wi; shadow->mask = -1; shadow->active = -1;
        *shadowSet = 1;
        return load3(&L->intensity);
    }
    case MCRT_POINT_LIGHT: {
        *wi = vsub(load3(&L->p), it->p);
        float distSq = vdot(*wi, *wi);
        if (isNearZero(distSq)) return V3(0, 0, 0);   /* Q13 */
        float dist = sqrtf(distSq);
        *wi = vdivs(*wi, dist);
        *pdf = 1.0f;
        shadow->o = vadd(it->p, vs(it->gn, it->traceErrorOffset));
        shadow->tmax = dist; shadow->d = *wi; shadow->mask = -1; shadow->active = -1;
        *shadowSet = 1;
        return vdivs(load3(&L->intensity), distSq);
    }
    case MCRT_DISK_AREA_LIGHT: {
        ShapeSample si = sampleDisk(load3(&L->p), load3(&L->d), L->radius, u, pdf);
        v3 ro = vadd(it->p, vs(it->gn, it->traceErrorOffset));
        v3 rt = vadd(si.p, vs(si.gn, RT_TRACE_OFFSET));
        *wi = vnormalize(vsub(rt, ro));
        float distSq = distanceSquared(si.p, it->p);
        float c = absDot(si.gn, vneg(*wi));
        if (isNearZero(c)) { *pdf = 0.0f; return V3(0, 0, 0); }
        *pdf *= distSq / c;
        shadow->o = ro; shadow->tmax = vlength(vsub(ro, rt)); shadow->d = *wi; shadow->mask = -1; shadow->active = -1;
        *shadowSet = 1;
        return vdot(si.gn, vneg(*wi)) > 0.0f ? load3(&L->intensity) : V3(0, 0, 0);
    }
    case MCRT_TRIANGLE_MESH_AREA_LIGHT: {
        const mcrt_shape* sh = &s->d.shapes[L->shapeId];
        int tri = (int)((uint32_t)((int)floorf(u.x * (float)sh->numTriangles)) % sh->numTriangles);
        u.x = u.x * (float)sh->numTriangles - (float)tri;
        const uint32_t* I = s->d.indices;
        uint32_t i0 = I[sh->startIdx + 3 * tri], i1 = I[sh->startIdx + 3 * tri + 1], i2 = I[sh->startIdx + 3 * tri + 2];
        v3 p0 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i0]));
        v3 p1 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i1]));
        v3 p2 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i2]));
        ShapeSample si = sampleTriangle(p0, p1, p2, u, pdf);
        *pdf = 1.0f / L->area;
        v3 ro = vadd(it->p, vs(it->gn, it->traceErrorOffset));
        v3 rt = vadd(si.p, vs(si.gn, RT_TRACE_OFFSET));
        *wi = vnormalize(vsub(si.p, it->p));
        float distSq = distanceSquared(si.p, it->p);
        float c = absDot(si.gn, vneg(*wi));
        if (isNearZero(c)) { *pdf = 0.0f; return V3(0, 0, 0); }
        *pdf *= distSq / c;
        shadow->o = ro; shadow->tmax = vlength(vsub(ro, rt)); shadow->d = *wi; shadow->mask = -1; shadow->active = -1;
        *shadowSet = 1;
        return vdot(si.gn, vneg(*wi)) > 0.0f ? load3(&L->intensity) : V3(0, 0, 0);
    }
    default:
        return V3(0, 0, 0);
    }
}

/* ======================================================================= */
/* Path tracing: KRN/PathTracing.cl + host loop RTPathTracingPass.cpp:71-86 */
/* ======================================================================= */
typedef struct {
    const orc_scene* s; const mcrt_camera* cam;
    int frame, maxDepth, sampler, W, H;
    float* radiance;
    const int32_t* rows;
    atomic_llong stats[8];
} RenderCtx;

static void renderPixel(RenderCtx* rc, int x, int y, uint32_t* stack) {
    const orc_scene* s = rc->s;
    const mcrt_camera* cam = rc->cam;
    int W = rc->W, H = rc->H;
    uint32_t bufferIdx = (uint32_t)(y * W + x);
    /* GeneratePerspectiveRays, PathTracing.cl:13-35 */
    float rx = 1.0f / (float)cam->width, ry = 1.0f / (float)cam->height;
    float u = (float)x * rx, v = (float)y * ry;
    Ray ray;
    ray.o = load3(&cam->pos); ray.tmax = 1000.0f;
    ray.d = lerpDirection(load3(&cam->r00), load3(&cam->r10), load3(&cam->r11), load3(&cam->r01), u, v);
    ray.mask = -1; ray.active = -1;
    v3 throughput = V3(1, 1, 1);
    int prevBsdfFlags = 0;
    v3 radianceAcc = V3(0, 0, 0);
    mcrt_intersection isect;
    int nv = 0;
    int64_t nprim = 0, vprim = 0, nclosest = 0, nany = 0, vclosest = 0, vany = 0, lclosest = 0, lany = 0;
    /* RTPrimaryRaysPass: first closest hit */
    uint8_t* const tch = s->touched;
    const int64_t NN = s->num_nodes;
    traceClosest(s, &ray, &isect, stack, &nv, tch);
    nprim++; vprim += nv;
    float* plog = s->pathlog ? s->pathlog + (size_t)bufferIdx * s->pathlog_depth * ORC_PATHLOG_FLOATS : NULL;
    for (int b = 0; b < rc->maxDepth; ++b) {
        float* L = (plog && b < s->pathlog_depth) ? plog + (size_t)b * ORC_PATHLOG_FLOATS : NULL;
        if (L) {
            int32_t iv[2] = {ray.active ? isect.shapeid : -2, isect.primid};
            memcpy(&L[0], iv, 8);
            L[2] = isect.uvwt.x; L[3] = isect.uvwt.y; L[4] = isect.uvwt.w;
            L[24] = ray.o.x; L[25] = ray.o.y; L[26] = ray.o.z;
            L[27] = ray.d.x; L[28] = ray.d.y; L[29] = ray.d.z; L[30] = ray.tmax; L[31] = 0.0f;
            int32_t none[3] = {-1, -1, -2};
            memcpy(&L[5], none, 12);
            L[21] = 0.0f;
        }
        v3 temp = V3(0, 0, 0);
        int ignoreOcclusion = 0;
        Ray shadow; shadow.active = 0; int shadowSet = 0;
        int shapeIdx = isect.shapeid, primIdx = isect.primid;
        if (ray.active && shapeIdx != -1 && primIdx != -1 && s->d.num_lights > 0) {
            Interaction si;
            computeSurfaceInteraction(s, shapeIdx, primIdx, isect.uvwt.x, isect.uvwt.y, &si);
            si.wo = vneg(ray.d);
            int isBackfacing = vdot(si.gn, si.wo) < 0.0f;
            si.traceErrorOffset = isBackfacing ? -RT_TRACE_OFFSET : RT_TRACE_OFFSET;
            const mcrt_shape* sh = &s->d.shapes[shapeIdx];
            applyNormalMapping(s, sh->materialId, &si);
            if (b == 0) throughput = V3(1, 1, 1);
            int isEmitter = sh->lightID != -1;
            int sampledSpecular = (BSDF_SPECULAR & prevBsdfFlags) == BSDF_SPECULAR;
            if (isEmitter && (b == 0 || sampledSpecular)) {
                v3 Le = evalLightLe(&s->d.lights[sh->lightID], si.gn, si.wo);
                temp = vadd(temp, vmul(throughput, Le));
                ray.active = 0;
                ignoreOcclusion = 1;
            } else {
                Sampler smp;
                makeSampler(&smp, rc->sampler, bufferIdx, rc->frame, b, W, H, s->d.sobol_matrices);
                ignoreOcclusion = 0;
                {
                    float lightPdf = 0.0f;   /* Q13 */
                    uint32_t lightIdx = (uint32_t)floorf(getSample1D(&smp) * (float)s->d.num_lights);
                    lightIdx %= s->d.num_lights;
                    v3 wi = V3(0, 0, 0);
                    v2 uL = getSample2D(&smp);
                    v3 Li = sampleLightLi(s, (int)lightIdx, &si, uL, &wi, &lightPdf, &shadow, &shadowSet);
                    if (L) { int32_t li = (int32_t)lightIdx; memcpy(&L[6], &li, 4); }
                    lightPdf *= s->d.lights[lightIdx].choicePdf;
                    v3 L = V3(0, 0, 0);
                    int mid = sh->materialId;
                    if (mid != -1) {
                        UberProps um;
                        getUberProps(s, mid, &si, &um);
                        v3 bsdf = evaluateUberBSDF(&um, &si, si.wo, wi, TRANSPORT_MODE_RADIANCE);
                        bsdf = vs(bsdf, absDot(wi, si.sn));
                        if (!isNearZero(lightPdf)) L = vdivs(vmul(Li, bsdf), lightPdf);
                    }
                    temp = vadd(temp, vmul(throughput, L));
                }
                if (b + 1 < rc->maxDepth) {
                    v2 bs = getSample2D(&smp);
                    float pdf = 0.0f;
                    if (sh->materialId != -1) {
                        int sampledType = 0, unused = 0;
                        v3 wi = V3(0, 0, 0);
                        UberProps um;
                        getUberProps(s, sh->materialId, &si, &um);
                        v3 f = sampleUberBSDF(&um, &si, bs, TRANSPORT_MODE_RADIANCE, BSDF_ALL, si.wo, &wi, &pdf, &unused, &sampledType);
                        prevBsdfFlags = sampledType;
                        if (L) { int32_t st = sampledType; memcpy(&L[5], &st, 4); L[22] = bs.x; L[23] = bs.y; }
                        if (isNearZero(pdf) || isBlack(f)) {
                            ray.active = 0;
                        } else {
                            f = vdivs(f, pdf);
                            v3 tp = vs(f, absDot(wi, si.sn));
                            throughput = vmul(throughput, tp);
                            float off = si.traceErrorOffset;
                            if ((sampledType & BSDF_TRANSMISSION) != 0 && vdot(si.gn, wi) * signf(off) < 0.0f) off *= -1.0f;
                            ray.o = vadd(si.p, vs(si.gn, off));
                            ray.tmax = RT_MAX_TRACE_DISTANCE;
                            ray.d = wi; ray.mask = -1; ray.active = -1;
                            if (L) {
                                L[15] = ray.o.x; L[16] = ray.o.y; L[17] = ray.o.z;
                                L[18] = ray.d.x; L[19] = ray.d.y; L[20] = ray.d.z; L[21] = 1.0f;
                            }
                        }
                    } else {
                        ray.active = 0;
                    }
                }
            }
        } else {
            ray.active = 0;
        }
        /* occluded query (applyVisibilityTest) + ShadowPass, PathTracing.cl:186-217 */
        int occl = -1;
        if (shadowSet && shadow.active) {
            int anv = 0;
            const int64_t l0 = tl_leafVisits;
            occl = traceAny(s, &shadow, stack, &anv, tch ? tch + (b == 0 ? 2 : 3) * NN : NULL);
            nany++; vany += anv; lany += tl_leafVisits - l0;
            if (L) {
                int32_t oc = occl; memcpy(&L[7], &oc, 4);
                L[8] = shadow.o.x; L[9] = shadow.o.y; L[10] = shadow.o.z;
                L[11] = shadow.d.x; L[12] = shadow.d.y; L[13] = shadow.d.z; L[14] = shadow.tmax;
            }
        }
        if (!ignoreOcclusion) {
            float V = (!shadowSet || occl != -1) ? 0.0f : 1.0f;
            temp = vs(temp, V);
        }
        radianceAcc = (b == 0) ? temp : vadd(radianceAcc, temp);
        if (b + 1 < rc->maxDepth && ray.active) {
            const int64_t l0 = tl_leafVisits;
            traceClosest(s, &ray, &isect, stack, &nv, tch ? tch + NN : NULL);
            nclosest++; vclosest += nv; lclosest += tl_leafVisits - l0;
        }
    }
    float* out = &rc->radiance[4 * (size_t)bufferIdx];
    out[0] = radianceAcc.x; out[1] = radianceAcc.y; out[2] = radianceAcc.z; out[3] = 0.0f;
    atomic_fetch_add(&rc->stats[0], nprim);
    atomic_fetch_add(&rc->stats[1], vprim);
    atomic_fetch_add(&rc->stats[2], nclosest);
    atomic_fetch_add(&rc->stats[3], vclosest);
    atomic_fetch_add(&rc->stats[4], nany);
    atomic_fetch_add(&rc->stats[5], vany);
    atomic_fetch_add(&rc->stats[6], lclosest);
    atomic_fetch_add(&rc->stats[7], lany);
}

static void render_row(void* c, int64_t i, uint32_t* stack) {
    RenderCtx* rc = (RenderCtx*)c;
    int y = rc->rows ? rc->rows[i] : (int)i;
    for (int x = 0; x < rc->W; ++x) renderPixel(rc, x, y, stack);
}

static void render_common(orc_scene* s, const mcrt_camera* cam, int frame, int max_depth, int sampler,
                          const int32_t* rows, int64_t nrows, int y0, int threads, float* radiance, int64_t* stats) {
    RenderCtx rc;
    rc.s = s; rc.cam = cam; rc.frame = frame; rc.maxDepth = max_depth; rc.sampler = sampler;
    rc.W = (int)cam->width; rc.H = (int)cam->height; rc.radiance = radiance;
    for (int k = 0; k < 8; ++k) atomic_init(&rc.stats[k], 0);
    if (rows) {
        rc.rows = rows;
        parallel_for(nrows, threads, 1, render_row, &rc);
    } else {
        int32_t* r = (int32_t*)malloc(sizeof(int32_t) * (nrows > 0 ? nrows : 1));
        for (int64_t i = 0; i < nrows; ++i) r[i] = (int32_t)(y0 + i);
        rc.rows = r;
        parallel_for(nrows, threads, 1, render_row, &rc);
        free(r);
    }
    if (stats) for (int k = 0; k < 8; ++k) stats[k] = atomic_load(&rc.stats[k]);
}

void orc_render_frame(orc_scene* s, const mcrt_camera* cam, int frame, int max_depth, int sampler,
                      int y0, int y1, int threads, float* radiance, int64_t* stats) {
    if (!s->nodes || s->d.num_lights == 0) {   /* RTPathTracingPass.cpp:42: no lights -> pass skipped */
        if (stats) memset(stats, 0, sizeof(int64_t) * 6);
        if (s->d.num_lights == 0) {
            for (int y = y0; y < y1; ++y)
                for (uint32_t x = 0; x < cam->width; ++x)
                    memset(&radiance[4 * ((size_t)y * cam->width + x)], 0, 16);
        }
        return;
    }
    render_common(s, cam, frame, max_depth, sampler, NULL, y1 - y0, y0, threads, radiance, stats);
}
/* touched: NULL (off) or 4 x num_nodes bytes the renders mark (camera / extension / shadow of
 * bounce 0 / later shadow rays) */
void orc_set_touched(orc_scene* s, uint8_t* touched) { s->touched = touched; }
void orc_set_pathlog(orc_scene* s, float* log, int depth) { s->pathlog = log; s->pathlog_depth = log ? depth : 0; }

void orc_render_rows(orc_scene* s, const mcrt_camera* cam, int frame, int max_depth, int sampler,
                     const int32_t* rows, int nrows, int threads, float* radiance, int64_t* stats) {
    render_common(s, cam, frame, max_depth, sampler, rows, nrows, 0, threads, radiance, stats);
}

/* ======================================================================= */
/* Reconstruction: KRN/reconstruction.cl:6-60 + KRN/filters.cl:12-69         */
/* ======================================================================= */
static float mitchell1D(float x, float B, float C) {
    x = fabsf(2.0f * x);
    if (x > 1.0f)
        return ((-B - 6 * C) * x * x * x + (6 * B + 30 * C) * x * x + (-12 * B - 48 * C) * x + (8 * B + 24 * C)) * (1.f / 6.f);
    return ((12 - 9 * B - 6 * C) * x * x * x + (-18 + 12 * B + 6 * C) * x * x + (6 - 2 * B)) * (1.f / 6.f);
}
static float sincf_(float x) { x = fabsf(x); if (x < 1e-5) return 1.0f; return sinf(PI * x) / (PI * x); }
static float windowedSinc(float x, float radius, float tau) {
    x = fabsf(x);
    if (x > radius) return 0.0f;
    return sincf_(x) * sincf_(x / tau);
}
static float filterWeight(const mcrt_filter* f) {
    v2 p = {f->pixelOffset.x, f->pixelOffset.y};
    switch (f->filterType) {
    case MCRT_BOX_FILTER: return 1.0f;
    case MCRT_TRIANGLE_FILTER:
        return fmaxf(0.0f, f->radius.x - fabsf(p.x)) * fmaxf(0.0f, f->radius.y - fabsf(p.y));
    case MCRT_GAUSSIAN_FILTER:
        return fmaxf(0.0f, expf(-f->gaussianAlpha * p.x * p.x) - f->gaussianExpX) *
               fmaxf(0.0f, expf(-f->gaussianAlpha * p.y * p.y) - f->gaussianExpY);
    case MCRT_MITCHELL_FILTER:
        return mitchell1D(p.x / f->radius.x, f->mitchellB, f->mitchellC) * mitchell1D(p.y / f->radius.y, f->mitchellB, f->mitchellC);
    case MCRT_LANCZOS_SINC_FILTER:
        return windowedSinc(p.x, f->radius.x, f->lanczosSincTau) * windowedSinc(p.y, f->radius.y, f->lanczosSincTau);
    }
    return 1.0f;
}
/* KRN/Denoise.cl:6-47 (BilateralDenoise); the reference writes nothing when a parameter is
 * non-positive (the output keeps its previous content: here, left untouched). */
void orc_denoise(int W, int H, int radius, float ss, float sr, const float* in, float* out) {
    if (radius <= 0 || ss <= 0.0f || sr <= 0.0f) return;
    const float sdSq = ss * ss, srSq = sr * sr;
    for (int gy = 0; gy < H; ++gy)
        for (int gx = 0; gx < W; ++gx) {
            const float* o = &in[4 * ((size_t)gy * W + gx)];
            float fc[4] = {0, 0, 0, 0}, wsum = 0.0f;
            for (int rx = -radius; rx <= radius; ++rx) {
                const int x = rx + gx < 0 ? 0 : (rx + gx > W - 1 ? W - 1 : rx + gx);
                for (int ry = -radius; ry <= radius; ++ry) {
                    const int y = ry + gy < 0 ? 0 : (ry + gy > H - 1 ? H - 1 : ry + gy);
                    const float* k = &in[4 * ((size_t)y * W + x)];
                    float d2 = 0.0f;
                    for (int c = 0; c < 4; ++c) d2 += (o[c] - k[c]) * (o[c] - k[c]);
                    const int sp = (gx - x) * (gx - x) + (gy - y) * (gy - y);
                    const float w = expf((float)(-sp) / (2.0f * sdSq) - d2 / (2.0f * srSq));
                    wsum += w;
                    for (int c = 0; c < 4; ++c) fc[c] += w * k[c];
                }
            }
            for (int c = 0; c < 4; ++c) out[4 * ((size_t)gy * W + gx) + c] = fc[c] / wsum;
        }
}

/* KRN/ToneMapping.cl:42-63 with computeLuminanceFromRGB (KRN/colors.cl:19-22) and
 * toneMapControlled (ToneMapping.cl:37-40); alpha passes through. */
void orc_tonemap(int W, int H, float Lwhite, const float* in, float* out) {
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        const float* p = &in[4 * i];
        const float L = 0.212671f * p[0] + 0.715160f * p[1] + 0.072169f * p[2];
        const float tL = L * (1.0f + L / (Lwhite * Lwhite)) / (1.0f + L);
        const float s = tL / L;
        for (int c = 0; c < 3; ++c) out[4 * i + c] = p[c] * s;
        out[4 * i + 3] = p[3];
    }
}

/* KRN/reconstruction.cl:20-57 for one frame with filter weight w.  `weighted += radiance * w`
 * (reconstruction.cl:50) is contracted to an fma by the reference's OpenCL compiler (FP_CONTRACT
 * ON is the OpenCL default), so it is fmaf here; the final division is IEEE (the reference GPU
 * build uses the 2.5-ulp OpenCL division, tests allow 3 ulp on the image). */
void orc_accumulate_w(int W, int H, int frame, float w, const float* radiance, float* wsum, float* wts, float* image) {
    for (int64_t i = 0; i < (int64_t)W * H; ++i) {
        float r[4];
        for (int c = 0; c < 4; ++c) r[c] = clampf(radiance[4 * i + c], 0.0f, 1000.0f);
        if (frame == 0) {
            for (int c = 0; c < 4; ++c) wsum[4 * i + c] = r[c] * w;
            wts[i] = w;
        } else {
            for (int c = 0; c < 4; ++c) wsum[4 * i + c] = fmaf(r[c], w, wsum[4 * i + c]);
            wts[i] += w;
        }
        for (int c = 0; c < 4; ++c) image[4 * i + c] = wsum[4 * i + c] / wts[i];
    }
}
void orc_accumulate(int W, int H, int frame, const mcrt_filter* f, const float* radiance,
                    float* wsum, float* wts, float* image) {
    orc_accumulate_w(W, H, frame, filterWeight(f), radiance, wsum, wts, image);
}

/* ======================================================================= */
/* BDPT: KRN/BDPT.cl (GenerateStartVertices :240-312, GenerateSecondaryVertices :317-458,  */
/* PrepareConnections :460-646, ConnectVertices :671-913, CopyBuffer :916-931) in the host */
/* pass order of RTBDPTPass::update (RTBDPTPass.cpp:67-128), one pixel per work item.      */
/* Camera model KRN/cameras.cl; light emission sampling KRN/lights.cl:148-252.             */
/* IEEE fp32 without contraction, like the PT restatement above.                           */
/* ======================================================================= */
enum { BV_CAMERA = 0, BV_LIGHT = 1, BV_SURFACE = 2 };                 /* kernel_data.h:202-207 */
enum { BVF_CONNECTIBLE = 1, BVF_DELTA_LIGHT = 2, BVF_DELTA = 4, BVF_INFINITE_LIGHT = 8 };   /* :209-218 */
#define TRANSPORT_MODE_IMPORTANCE_ 1

typedef struct {            /* RTBDPTVertex (kernel_data.h:220-244) */
    v3 throughput;
    Interaction in;
    int type, flags, lightIdx, materialIdx;
    float pdfFwd, pdfRev, pdfPos;
    int radianceBufferIdx;
} BVert;

static inline int bvOnSurface(const BVert* v) {   /* BDPT.cl:40-43 */
    return isNotNearZero(v->in.gn.x) || isNotNearZero(v->in.gn.y) || isNotNearZero(v->in.gn.z);
}
static inline int bvLight(const BVert* v) { return v->type == BV_LIGHT || v->lightIdx != -1; }   /* kernel_data.h:457-460 */

/* KRN/matrix.cl:62-70 (transformVector4): row dots */
static inline float dot4(const mcrt_float4* r, const float v[4]) { return r->x * v[0] + r->y * v[1] + r->z * v[2] + r->w * v[3]; }

/* cameras.cl:8-32 */
static v3 evalPinholeCameraWe(const mcrt_camera* c, v3 ro, v3 rd, v2* nip) {
    float cosTheta = vdot(rd, load3(&c->direction));
    if (cosTheta <= 0.0f) return V3(0, 0, 0);
    v3 pf = vadd(ro, vdivs(rd, cosTheta));
    float p4[4] = {pf.x, pf.y, pf.z, 1.0f};
    float ic[4] = {dot4(&c->worldToClip.m0, p4), dot4(&c->worldToClip.m1, p4), dot4(&c->worldToClip.m2, p4),
                   dot4(&c->worldToClip.m3, p4)};
    if (ic[0] < -ic[3] || ic[0] > ic[3] || ic[1] < -ic[3] || ic[1] > ic[3]) return V3(0, 0, 0);
    if (nip) { nip->x = (ic[0] / ic[3] + 1.0f) * 0.5f; nip->y = (ic[1] / ic[3] + 1.0f) * 0.5f; }
    float w = 1.0f / (c->area * cosTheta * cosTheta * cosTheta);
    return V3(w, w, w);
}
/* cameras.cl:34-57 */
static void evalPinholeCameraPdfWe(const mcrt_camera* c, v3 ro, v3 rd, float* pdfPos, float* pdfDir) {
    float cosTheta = vdot(rd, load3(&c->direction));
    if (cosTheta <= 0.0f) { *pdfPos = 0.0f; *pdfDir = 0.0f; return; }
    v3 pf = vadd(ro, vs(rd, 1.0f / cosTheta));
    float p4[4] = {pf.x, pf.y, pf.z, 1.0f};
    float ic[4] = {dot4(&c->worldToClip.m0, p4), dot4(&c->worldToClip.m1, p4), dot4(&c->worldToClip.m2, p4),
                   dot4(&c->worldToClip.m3, p4)};
    if (ic[0] < -ic[3] || ic[0] > ic[3] || ic[1] < -ic[3] || ic[1] > ic[3]) { *pdfPos = 0.0f; *pdfDir = 0.0f; return; }
    *pdfPos = 1.0f;
    *pdfDir = 1.0f / (c->area * cosTheta * cosTheta * cosTheta);
}
/* cameras.cl:59-69 */
static v3 samplePinholeCameraWi(const mcrt_camera* c, const Interaction* si, v3* wi, float* pdf, v2* nip) {
    *wi = vsub(load3(&c->pos), si->p);
    float dist = vlength(*wi);
    *wi = vdivs(*wi, dist);
    *pdf = (dist * dist) / absDot(load3(&c->direction), *wi);
    return evalPinholeCameraWe(c, load3(&c->pos), vneg(*wi), nip);
}

/* samplers.cl:143-149, 200-203 */
static v3 uniformSampleSphere(v2 u) {
    float y = 1.0f - 2.0f * u.x;
    float r = sqrtf(fmaxf(0.0f, 1.0f - y * y));
    float phi = 2.0f * PI * u.y;
    return V3(r * cosf(phi), y, r * sinf(phi));
}
static inline float cosineHemispherePdf(float cosTheta) { return cosTheta * PI_INV; }

/* lights.cl:148-225 */
static v3 sampleLightLe(const orc_scene* s, int li, v2 u1, v2 u2, v3* ro, v3* rd, v3* ln, float* pdfPos, float* pdfDir) {
    const mcrt_light* L = &s->d.lights[li];
    switch (L->type) {
    case MCRT_DIRECTIONAL_LIGHT: {
        ShapeSample si = sampleDisk(load3(&L->p), load3(&L->d), L->radius, u1, pdfPos);
        *ln = load3(&L->d);
        *pdfDir = 1.0f;
        *ro = si.p;
        *rd = load3(&L->d);
        return load3(&L->intensity);
    }
    case MCRT_POINT_LIGHT:
        *rd = uniformSampleSphere(u1);
        *ro = load3(&L->p);
        *ln = *rd;
        *pdfPos = 1.0f;
        *pdfDir = PI4_INV;
        return load3(&L->intensity);
    case MCRT_DISK_AREA_LIGHT: {
        ShapeSample si = sampleDisk(load3(&L->p), load3(&L->d), L->radius, u1, pdfPos);
        *ln = si.gn;
        v3 w = cosineSampleHemisphere(u2);
        *pdfDir = cosineHemispherePdf(w.y);
        v3 v0 = computeOrthogonalVector(si.gn);
        v3 v1 = vcross(v0, si.gn);
        *rd = vadd(vadd(sv(w.x, v0), sv(w.y, si.gn)), sv(w.z, v1));
        *ro = vadd(si.p, vs(si.gn, RT_TRACE_OFFSET));
        return load3(&L->intensity);
    }
    case MCRT_TRIANGLE_MESH_AREA_LIGHT: {
        const mcrt_shape* sh = &s->d.shapes[L->shapeId];
        int tri = ((int)floorf(u1.x * (float)sh->numTriangles)) % (int)sh->numTriangles;
        u1.x = u1.x * (float)sh->numTriangles - (float)tri;
        const uint32_t* I = s->d.indices;
        uint32_t i0 = I[sh->startIdx + 3 * tri], i1 = I[sh->startIdx + 3 * tri + 1], i2 = I[sh->startIdx + 3 * tri + 2];
        v3 p0 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i0]));
        v3 p1 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i1]));
        v3 p2 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i2]));
        ShapeSample si = sampleTriangle(p0, p1, p2, u1, pdfPos);
        *pdfPos = 1.0f / L->area;
        *ln = si.gn;
        v3 w = cosineSampleHemisphere(u2);
        *pdfDir = cosineHemispherePdf(w.y);
        v3 v0 = computeOrthogonalVector(si.gn);
        v3 v1 = vcross(v0, si.gn);
        *rd = vadd(vadd(sv(w.x, v0), sv(w.y, si.gn)), sv(w.z, v1));
        *ro = vadd(si.p, vs(si.gn, RT_TRACE_OFFSET));
        return load3(&L->intensity);
    }
    }
    return V3(0, 0, 0);
}
/* lights.cl:227-252 (the output pdfs are left unset for unknown types, as the reference) */
static void evalLightPdfLe(const orc_scene* s, int li, v3 rd, v3 ln, float* pdfPos, float* pdfDir) {
    const mcrt_light* L = &s->d.lights[li];
    switch (L->type) {
    case MCRT_DIRECTIONAL_LIGHT: *pdfPos = 1.0f / L->area; *pdfDir = 0.0f; break;
    case MCRT_POINT_LIGHT: *pdfPos = 0.0f; *pdfDir = PI4_INV; break;
    case MCRT_DISK_AREA_LIGHT:
    case MCRT_TRIANGLE_MESH_AREA_LIGHT: *pdfPos = 1.0f / L->area; *pdfDir = cosineHemispherePdf(vdot(ln, rd)); break;
    }
}
/* lights.cl:45-146 with the light position / normal outputs the BDPT s = 1 strategy uses */
static v3 sampleLightLiPos(const orc_scene* s, int li, const Interaction* it, v2 u, v3* lpos, v3* lnrm, v3* wi,
                           float* pdf, Ray* shadow, int* shadowSet) {
    const mcrt_light* L = &s->d.lights[li];
    *shadowSet = 0;
    switch (L->type) {
    case MCRT_DIRECTIONAL_LIGHT:
        *wi = vneg(load3(&L->d));
        *lnrm = V3(0, 0, 0);
        *lpos = vadd(it->p, vs(vs(*wi, L->radius), 2.0f));
        *pdf = 1.0f;
        shadow->o = vadd(it->p, vs(it->gn, it->traceErrorOffset));
        shadow->tmax = 1000.0f; shadow->d = *wi; shadow->mask = -1; shadow->active = -1;
        *shadowSet = 1;
        return load3(&L->intensity);
    case MCRT_POINT_LIGHT: {
        *wi = vsub(load3(&L->p), it->p);
        float distSq = vdot(*wi, *wi);
        if (isNearZero(distSq)) return V3(0, 0, 0);   /* Q13: pdf, position and ray unset */
        float dist = sqrtf(distSq);
        *wi = vdivs(*wi, dist);
        *lnrm = V3(0, 0, 0);
        *pdf = 1.0f;
        shadow->o = vadd(it->p, vs(it->gn, it->traceErrorOffset));
        *lpos = load3(&L->p);
        shadow->tmax = dist; shadow->d = *wi; shadow->mask = -1; shadow->active = -1;
        *shadowSet = 1;
        return vdivs(load3(&L->intensity), distSq);
    }
    case MCRT_DISK_AREA_LIGHT: {
        ShapeSample si = sampleDisk(load3(&L->p), load3(&L->d), L->radius, u, pdf);
        *lnrm = si.gn;
        *lpos = si.p;
        v3 ro = vadd(it->p, vs(it->gn, it->traceErrorOffset));
        v3 rt = vadd(si.p, vs(si.gn, RT_TRACE_OFFSET));
        *wi = vnormalize(vsub(rt, ro));
        float distSq = distanceSquared(si.p, it->p);
        float c = absDot(si.gn, vneg(*wi));
        if (isNearZero(c)) { *pdf = 0.0f; return V3(0, 0, 0); }
        *pdf *= distSq / c;
        shadow->o = ro; shadow->tmax = vlength(vsub(ro, rt)); shadow->d = *wi; shadow->mask = -1; shadow->active = -1;
        *shadowSet = 1;
        return vdot(si.gn, vneg(*wi)) > 0.0f ? load3(&L->intensity) : V3(0, 0, 0);
    }
    case MCRT_TRIANGLE_MESH_AREA_LIGHT: {
        const mcrt_shape* sh = &s->d.shapes[L->shapeId];
        int tri = ((int)floorf(u.x * (float)sh->numTriangles)) % (int)sh->numTriangles;
        u.x = u.x * (float)sh->numTriangles - (float)tri;
        const uint32_t* I = s->d.indices;
        uint32_t i0 = I[sh->startIdx + 3 * tri], i1 = I[sh->startIdx + 3 * tri + 1], i2 = I[sh->startIdx + 3 * tri + 2];
        v3 p0 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i0]));
        v3 p1 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i1]));
        v3 p2 = transformPoint3(&sh->toWorldTransform, load3(&s->d.positions[sh->startVertex + i2]));
        ShapeSample si = sampleTriangle(p0, p1, p2, u, pdf);
        *lnrm = si.gn;
        *lpos = si.p;
        *pdf = 1.0f / L->area;
        v3 ro = vadd(it->p, vs(it->gn, it->traceErrorOffset));
        v3 rt = vadd(si.p, vs(si.gn, RT_TRACE_OFFSET));
        *wi = vnormalize(vsub(si.p, it->p));
        float distSq = distanceSquared(si.p, it->p);
        float c = absDot(si.gn, vneg(*wi));
        if (isNearZero(c)) { *pdf = 0.0f; return V3(0, 0, 0); }
        *pdf *= distSq / c;
        shadow->o = ro; shadow->tmax = vlength(vsub(ro, rt)); shadow->d = *wi; shadow->mask = -1; shadow->active = -1;
        *shadowSet = 1;
        return vdot(si.gn, vneg(*wi)) > 0.0f ? load3(&L->intensity) : V3(0, 0, 0);
    }
    }
    return V3(0, 0, 0);
}

/* materials.cl:93-179 (uber only; other material types evaluate to zero) */
static int isUberMat(const orc_scene* s, int mi) { return s->d.materials[mi].type == 0; }
static float evaluateMaterialPdf(const orc_scene* s, int mi, v3 wo, v3 wi, const Interaction* si) {
    if (!isUberMat(s, mi)) return 0.0f;
    UberProps um;
    getUberProps(s, mi, si, &um);
    return evaluateUberBSDF_Pdf(&um, si, wo, wi, BSDF_ALL);
}
static v3 evaluateMaterial(const orc_scene* s, int mi, v3 wo, v3 wi, const Interaction* si, int mode) {
    if (!isUberMat(s, mi)) return V3(0, 0, 0);
    UberProps um;
    getUberProps(s, mi, si, &um);
    return evaluateUberBSDF(&um, si, wo, wi, mode);
}
static int hasMaterialNonDeltaComponents(const orc_scene* s, int mi, const Interaction* si) {
    const mcrt_material* m = &s->d.materials[mi];
    if (m->type != 0) return 0;
    v3 Kd = load3(&m->uber_kd), Ks = load3(&m->uber_ks), op = load3(&m->uber_opacity);
    if (m->uber_diffuseTexId != -1) { f4 t = readTex(s, m->uber_diffuseTexId, si->uv); Kd = V3(t.x, t.y, t.z); }
    if (m->uber_glossyTexId != -1) { f4 t = readTex(s, m->uber_glossyTexId, si->uv); Ks = V3(t.x, t.y, t.z); }
    if (m->uber_opacityTexId != -1) { f4 t = readTex(s, m->uber_opacityTexId, si->uv); op = V3(t.x, t.y, t.z); }
    return !isBlack(vmul(Kd, op)) || !isBlack(vmul(Ks, op));
}

/* BDPT.cl:22-35 */
static float computeShadingNormalCorrection(const Interaction* in, v3 wo, v3 wi, int mode) {
    if (mode == TRANSPORT_MODE_IMPORTANCE_) {
        float denom = absDot(wo, in->gn) * absDot(wi, in->sn);
        if (isNearZero(denom)) return 0.0f;
        return (absDot(wo, in->sn) * absDot(wi, in->gn)) / denom;
    }
    return 1.0f;
}
/* BDPT.cl:45-60 */
static float convertVertexDensity(float pdf, const BVert* th, const BVert* nx) {
    if (nx->flags & BVF_INFINITE_LIGHT) return pdf;
    v3 w = vsub(nx->in.p, th->in.p);
    float lenSq = vdot(w, w);
    if (isNearZero(lenSq)) return 0.0f;
    float invDistSq = 1.0f / lenSq;
    if (bvOnSurface(nx)) pdf *= absDot(nx->in.gn, vs(w, sqrtf(invDistSq)));
    return pdf * invDistSq;
}
/* BDPT.cl:62-91 */
static float evalVertexPdfLight(const orc_scene* s, const BVert* th, const BVert* v) {
    v3 w = vsub(v->in.p, th->in.p);
    float lenSq = vdot(w, w);
    if (isNearZero(lenSq)) return 0.0f;
    float invDistSq = 1.0f / lenSq;
    w = vs(w, sqrtf(invDistSq));
    float pdf;
    if (th->flags & BVF_INFINITE_LIGHT) {
        float radius = s->d.lights[th->lightIdx].radius;
        pdf = 1.0f / (PI * radius * radius);
    } else {
        float pdfPos = 0.0f, pdfDir = 0.0f;
        evalLightPdfLe(s, th->lightIdx, w, th->in.gn, &pdfPos, &pdfDir);
        pdf = pdfDir * invDistSq;
    }
    if (bvOnSurface(v)) pdf *= absDot(v->in.gn, w);
    return pdf;
}
/* BDPT.cl:93-132 */
static float evalVertexPdf(const orc_scene* s, const mcrt_camera* cam, const BVert* th, const BVert* prev, const BVert* next) {
    if (th->type == BV_LIGHT) return evalVertexPdfLight(s, th, next);
    v3 wn = vsub(next->in.p, th->in.p);
    float lenSq = vdot(wn, wn);
    if (isNearZero(lenSq)) return 0.0f;
    wn = vdivs(wn, sqrtf(lenSq));
    float pdf = 0.0f, unused;
    if (th->type == BV_CAMERA) {
        evalPinholeCameraPdfWe(cam, th->in.p, wn, &unused, &pdf);
    } else if (th->type == BV_SURFACE) {
        v3 wp = V3(0, 0, 0);
        if (prev) {
            wp = vsub(prev->in.p, th->in.p);
            lenSq = vdot(wp, wp);
            if (isNearZero(lenSq)) return 0.0f;
            wp = vdivs(wp, sqrtf(lenSq));
        }
        Interaction in = th->in;
        pdf = evaluateMaterialPdf(s, th->materialIdx, wp, wn, &in);
    }
    return convertVertexDensity(pdf, th, next);
}
/* BDPT.cl:135-152 */
static float evalVertexPdfLightOrigin(const orc_scene* s, const BVert* th, v3 nextPos) {
    v3 w = vsub(nextPos, th->in.p);
    float lenSq = vdot(w, w);
    if (isNearZero(lenSq)) return 0.0f;
    w = vs(w, sqrtf(1.0f / lenSq));
    if (th->flags & BVF_INFINITE_LIGHT) return 0.0f;
    float pdfPos = 0.0f, pdfDir = 0.0f;
    evalLightPdfLe(s, th->lightIdx, w, th->in.gn, &pdfPos, &pdfDir);
    return pdfPos * s->d.lights[th->lightIdx].choicePdf;
}
/* BDPT.cl:157-174 */
static BVert createCameraVertex(v3 p, v3 throughput) {
    BVert v;
    memset(&v, 0, sizeof(v));
    v.throughput = throughput;
    v.in.p = p;
    v.in.gn = V3(0, 0, 0);
    v.type = BV_CAMERA;
    v.flags = BVF_CONNECTIBLE;
    v.lightIdx = -1;
    return v;
}
/* BDPT.cl:176-203 */
static BVert createLightVertex(int li, v3 p, v3 ln, v3 throughput, float pdfFwd, int lightFlags) {
    BVert v;
    memset(&v, 0, sizeof(v));
    v.throughput = throughput;
    v.in.p = p;
    v.in.gn = ln;
    v.in.sn = ln;
    v.in.traceErrorOffset = RT_TRACE_OFFSET;
    v.type = BV_LIGHT;
    v.lightIdx = li;
    v.pdfFwd = pdfFwd;
    if (lightFlags & MCRT_LIGHT_FLAG_DELTA_DIRECTION) v.flags = BVF_DELTA_LIGHT | BVF_INFINITE_LIGHT;
    else {
        v.flags = BVF_CONNECTIBLE;
        if (lightFlags & MCRT_LIGHT_FLAG_DELTA_POSITION) v.flags |= BVF_DELTA_LIGHT;
    }
    return v;
}
/* BDPT.cl:214-234 */
static v3 evalVertex_f(const orc_scene* s, const BVert* th, const BVert* nx, int mode) {
    v3 wi = vsub(nx->in.p, th->in.p);
    float lenSq = vdot(wi, wi);
    if (isNearZero(lenSq)) return V3(0, 0, 0);
    wi = vdivs(wi, sqrtf(lenSq));
    if (th->type == BV_SURFACE) {
        Interaction si = th->in;
        v3 f = evaluateMaterial(s, th->materialIdx, si.wo, wi, &si, mode);
        return vs(f, computeShadingNormalCorrection(&si, si.wo, wi, mode));
    }
    return V3(1.0f, 0.0784f, 0.5765f);
}
static inline float remap0(float f) { return f == 0.0f ? 1.0f : f; }   /* BDPT.cl:650-653 */

/* atomicAdd_f (BDPT.cl:655-669): CAS loop on the float bits */
static void atomicAddF(float* addr, float val) {
    _Atomic uint32_t* a = (_Atomic uint32_t*)addr;
    uint32_t cur = atomic_load_explicit(a, memory_order_relaxed);
    for (;;) {
        float f;
        memcpy(&f, &cur, 4);
        f += val;
        uint32_t nx;
        memcpy(&nx, &f, 4);
        if (atomic_compare_exchange_weak_explicit(a, &cur, nx, memory_order_relaxed, memory_order_relaxed)) return;
    }
}

struct orc_bdpt {
    int W, H, D;
    BVert* sampledLight;   /* W*H*D, persistent across frames (read before it is overwritten, BDPT.cl:585-586) */
    float* final3;         /* finalRadianceBuffer, 3 floats per pixel */
    int32_t* camCount;
    int32_t* lightCount;
};
orc_bdpt* orc_bdpt_create(int W, int H, int D) {
    orc_bdpt* b = (orc_bdpt*)calloc(1, sizeof(orc_bdpt));
    b->W = W; b->H = H; b->D = D;
    const size_t N = (size_t)W * H;
    b->sampledLight = (BVert*)calloc(N * (size_t)D, sizeof(BVert));   /* zero-filled like the clref runner */
    b->final3 = (float*)calloc(3 * N, sizeof(float));
    b->camCount = (int32_t*)calloc(N, sizeof(int32_t));
    b->lightCount = (int32_t*)calloc(N, sizeof(int32_t));
    return b;
}
void orc_bdpt_destroy(orc_bdpt* b) {
    if (!b) return;
    free(b->sampledLight); free(b->final3); free(b->camCount); free(b->lightCount);
    free(b);
}

typedef struct {
    const orc_scene* s; orc_bdpt* b; const mcrt_camera* cam;
    int frame, sampler;
    const int32_t* rows;
    atomic_llong stats[4];   /* subpath rays traced, their node visits, connection rays traced, their visits */
} BdptCtx;

/* GenerateSecondaryVertices (BDPT.cl:317-458) for one pixel and depth */
static void bdptSecondary(BdptCtx* c, uint32_t bufferIdx, int isCam, int curDepth, BVert* verts, int* count, Ray* ray,
                          const mcrt_intersection* isect, v3* throughput, float* fwdPdf) {
    const orc_scene* s = c->s;
    const int D = c->b->D, W = c->b->W, H = c->b->H;
    Sampler smp;
    makeSampler(&smp, c->sampler, bufferIdx, c->frame, curDepth + (D + 1) * isCam, W, H, s->d.sobol_matrices);
    const int shapeIdx = isect->shapeid, prim = isect->primid;
    if (!ray->active || shapeIdx == -1 || prim == -1 || s->d.shapes[shapeIdx].materialId == -1) { ray->active = 0; return; }
    (*count)++;
    Interaction si;
    computeSurfaceInteraction(s, shapeIdx, prim, isect->uvwt.x, isect->uvwt.y, &si);
    si.wo = vneg(ray->d);
    si.traceErrorOffset = vdot(si.gn, si.wo) < 0.0f ? -RT_TRACE_OFFSET : RT_TRACE_OFFSET;
    const int mi = s->d.shapes[shapeIdx].materialId;
    applyNormalMapping(s, mi, &si);
    BVert* cur = &verts[curDepth];
    BVert* prev = &verts[curDepth - 1];
    const int mode = isCam ? TRANSPORT_MODE_RADIANCE : TRANSPORT_MODE_IMPORTANCE_;
    float pdfFwd = *fwdPdf;
    /* setSurfaceVertex (BDPT.cl:205-212) */
    cur->throughput = *throughput;
    cur->in = si;
    cur->type = BV_SURFACE;
    cur->materialIdx = mi;
    cur->flags = 0;
    cur->pdfRev = 0.0f;
    cur->pdfFwd = convertVertexDensity(pdfFwd, prev, cur);
    cur->lightIdx = s->d.shapes[shapeIdx].lightID;
    if (!isCam && curDepth == 1 && (prev->flags & BVF_INFINITE_LIGHT)) {
        cur->pdfFwd = prev->pdfPos;
        if (bvOnSurface(cur)) cur->pdfFwd *= absDot(ray->d, si.gn);
        prev->pdfFwd = 0.0f;
    }
    if (curDepth == D + isCam) {
        if (hasMaterialNonDeltaComponents(s, mi, &si)) cur->flags |= BVF_CONNECTIBLE;
        ray->active = 0;
        return;
    }
    v3 wi = V3(0, 0, 0), wo = si.wo;
    int sampledType = 0, numNonDelta = 0;
    v2 bs = getSample2D(&smp);
    v3 f = V3(0, 0, 0);
    if (isUberMat(s, mi)) {
        UberProps um;
        getUberProps(s, mi, &si, &um);
        f = sampleUberBSDF(&um, &si, bs, mode, BSDF_ALL, wo, &wi, &pdfFwd, &numNonDelta, &sampledType);
    }
    cur->in = si;
    if (numNonDelta > 0) cur->flags |= BVF_CONNECTIBLE;
    if (isBlack(f) || isNearZero(pdfFwd)) { ray->active = 0; return; }
    *throughput = vmul(*throughput, vdivs(vs(f, absDot(wi, si.sn)), pdfFwd));
    float pdfRev;
    if (sampledType & BSDF_SPECULAR) {
        cur->flags |= BVF_DELTA;
        pdfFwd = 0.0f;
        pdfRev = 0.0f;
    } else {
        pdfRev = evaluateMaterialPdf(s, mi, wi, wo, &si);
    }
    float off = si.traceErrorOffset;
    if ((sampledType & BSDF_TRANSMISSION) != 0 && vdot(si.gn, wi) * signf(off) < 0.0f) off *= -1.0f;
    ray->o = vadd(si.p, vs(si.gn, off));
    ray->tmax = RT_MAX_TRACE_DISTANCE;
    ray->d = wi;
    ray->mask = -1;
    ray->active = -1;
    *throughput = vs(*throughput, computeShadingNormalCorrection(&si, wo, wi, mode));
    prev->pdfRev = convertVertexDensity(pdfRev, cur, prev);
    *fwdPdf = pdfFwd;
}

static void bdptPixel(void* vc, int64_t i, uint32_t* stack) {
    BdptCtx* c = (BdptCtx*)vc;
    const orc_scene* s = c->s;
    orc_bdpt* b = c->b;
    const mcrt_camera* cam = c->cam;
    const int W = b->W, H = b->H, D = b->D;
    const int y = c->rows ? c->rows[i / W] : (int)(i / W), x = (int)(i % W);
    const uint32_t bufferIdx = (uint32_t)(x + y * W);
    const int maxCam = D + 2, maxLight = D + 1;
    const int C = maxCam * (maxCam + 1) / 2 - 2;
    BVert cv[34], lv[33];
    int64_t nSub = 0, vSub = 0, nConn = 0, vConn = 0;
    uint8_t* const tch = s->touched;
    const int64_t NN = s->num_nodes;
    /* ---- GenerateStartVertices (BDPT.cl:240-312) ---- */
    Sampler smp;
    makeSampler(&smp, c->sampler, bufferIdx, c->frame, 0, W, H, s->d.sobol_matrices);
    int camCount = 1, lightCount = 1;
    float rx = 1.0f / (float)W, ry = 1.0f / (float)H;
    Ray cray;
    cray.o = load3(&cam->pos); cray.tmax = RT_MAX_TRACE_DISTANCE;
    cray.d = lerpDirection(load3(&cam->r00), load3(&cam->r10), load3(&cam->r11), load3(&cam->r01), (float)x * rx, (float)y * ry);
    cray.mask = -1; cray.active = -1;
    cv[0] = createCameraVertex(load3(&cam->pos), V3(1, 1, 1));
    v3 camT = cv[0].throughput;
    float pdfPos = 0.0f, pdfDir = 0.0f;
    evalPinholeCameraPdfWe(cam, load3(&cam->pos), cray.d, &pdfPos, &pdfDir);
    float camFwd = pdfDir;
    const int nl = (int)s->d.num_lights;
    int chosen = (int)((uint32_t)floorf(getSample1D(&smp) * (float)nl) % (uint32_t)nl);
    float lightPdf = s->d.lights[chosen].choicePdf;
    v2 u1 = getSample2D(&smp);
    v2 u2 = getSample2D(&smp);
    v3 ro = V3(0, 0, 0), rd = V3(0, 0, 0), ln = V3(0, 0, 0);
    v3 Le = sampleLightLe(s, chosen, u1, u2, &ro, &rd, &ln, &pdfPos, &pdfDir);
    Ray lray;
    lray.o = ro; lray.tmax = RT_MAX_TRACE_DISTANCE; lray.d = rd; lray.mask = -1; lray.active = -1;
    lv[0] = createLightVertex(chosen, ro, ln, Le, pdfPos * lightPdf, s->d.lights[chosen].flags);
    lv[0].pdfPos = pdfPos;
    v3 lightT = vdivs(vs(Le, absDot(ln, rd)), lightPdf * pdfPos * pdfDir);
    float lightFwd = pdfDir;
    /* ---- camera subpath, then light subpath: RR QueryIntersection + GenerateSecondaryVertices ---- */
    mcrt_intersection isect;
    isect.shapeid = isect.primid = -1;
    for (int d = 1; d <= D + 1; ++d) {
        if (cray.active) {
            int nv = 0;
            traceClosest(s, &cray, &isect, stack, &nv, tch ? tch + NN : NULL);
            nSub++; vSub += nv;
        }
        bdptSecondary(c, bufferIdx, 1, d, cv, &camCount, &cray, &isect, &camT, &camFwd);
    }
    isect.shapeid = isect.primid = -1;
    for (int d = 1; d <= D; ++d) {
        if (lray.active) {
            int nv = 0;
            traceClosest(s, &lray, &isect, stack, &nv, tch ? tch + NN : NULL);
            nSub++; vSub += nv;
        }
        bdptSecondary(c, bufferIdx, 0, d, lv, &lightCount, &lray, &isect, &lightT, &lightFwd);
    }
    b->camCount[bufferIdx] = camCount;
    b->lightCount[bufferIdx] = lightCount;
    /* ---- PrepareConnections (BDPT.cl:460-646) ---- */
    makeSampler(&smp, c->sampler, bufferIdx, c->frame, maxLight + maxCam, W, H, s->d.sobol_matrices);
    v3 rad[40];
    Ray conn[40];
    BVert sampledCam[32];
    int slot = 0;
    for (int t = 1; t <= camCount; ++t)
        for (int sI = 0; sI <= lightCount; ++sI) {
            const int depth = t + sI - 2;
            if ((t == 1 && sI == 1) || depth < 0 || depth > D) continue;
            BVert* cvx = &cv[t - 1];
            rad[slot] = V3(0, 0, 0);
            conn[slot].active = 0;
            if (sI == 0) {
                /* nothing: the connection ray keeps what the buffer held (inactive in ConnectVertices' use) */
            } else if (t == 1) {
                BVert* lvx = &lv[sI - 1];
                if (lvx->flags & BVF_CONNECTIBLE) {
                    Interaction li = lvx->in;
                    v3 wi;
                    float pdf;
                    v2 nip = {(float)x / (float)W, (float)y / (float)H};
                    v3 imp = samplePinholeCameraWi(cam, &li, &wi, &pdf, &nip);
                    if (pdf > 0.0f && isNotBlack(imp)) {
                        BVert* sc = &sampledCam[sI - 2];
                        *sc = createCameraVertex(load3(&cam->pos), vdivs(imp, pdf));
                        int ix = (int)floorf(nip.x * (float)W + 0.5f), iy = (int)floorf(nip.y * (float)H + 0.5f);
                        ix = ix < 0 ? 0 : (ix > W - 1 ? W - 1 : ix);
                        iy = iy < 0 ? 0 : (iy > H - 1 ? H - 1 : iy);
                        sc->radianceBufferIdx = ix + iy * W;
                        rad[slot] = vmul(vmul(lvx->throughput, sc->throughput), evalVertex_f(s, lvx, sc, TRANSPORT_MODE_IMPORTANCE_));
                        if (bvOnSurface(lvx)) rad[slot] = vs(rad[slot], absDot(wi, li.sn));
                        v3 o = vadd(li.p, vs(li.gn, lvx->in.traceErrorOffset));
                        float dist = vlength(vsub(o, load3(&cam->pos)));
                        conn[slot].o = o; conn[slot].tmax = dist; conn[slot].d = vdivs(vsub(load3(&cam->pos), o), dist);
                        conn[slot].mask = -1; conn[slot].active = -1;
                    }
                }
            } else if (sI == 1) {
                if (cvx->flags & BVF_CONNECTIBLE) {
                    v3 wi = V3(0, 0, 0), lpos = V3(0, 0, 0), lnrm = V3(0, 0, 0);
                    float pdf = 0.0f;
                    int ch = (int)floorf(getSample1D(&smp) * (float)nl);
                    if (ch > nl - 1) ch = nl - 1;
                    float lp = s->d.lights[ch].choicePdf;
                    Interaction ci = cvx->in;
                    Ray shadow;
                    shadow.active = 0;
                    int shadowSet = 0;
                    v2 u = getSample2D(&smp);
                    v3 Li = sampleLightLiPos(s, ch, &ci, u, &lpos, &lnrm, &wi, &pdf, &shadow, &shadowSet);
                    if (shadowSet) conn[slot] = shadow;
                    if (isNotNearZero(pdf) && isNotBlack(Li)) {
                        BVert* sl = &b->sampledLight[(size_t)bufferIdx * D + t - 2];
                        float pf = evalVertexPdfLightOrigin(s, sl, cvx->in.p);   /* the previous content (BDPT.cl:585) */
                        *sl = createLightVertex(ch, lpos, lnrm, vdivs(Li, lp * pdf), pf, s->d.lights[ch].flags);
                        v3 f = evaluateMaterial(s, cvx->materialIdx, ci.wo, wi, &ci, TRANSPORT_MODE_RADIANCE);
                        rad[slot] = vmul(vmul(cvx->throughput, sl->throughput), f);
                        if (bvOnSurface(cvx)) rad[slot] = vs(rad[slot], absDot(wi, ci.sn));
                    } else {
                        conn[slot].active = 0;
                    }
                }
            } else {
                BVert* lvx = &lv[sI - 1];
                if ((cvx->flags & BVF_CONNECTIBLE) && (lvx->flags & BVF_CONNECTIBLE)) {
                    v3 lvf = evalVertex_f(s, lvx, cvx, TRANSPORT_MODE_IMPORTANCE_);
                    v3 cvf = evalVertex_f(s, cvx, lvx, TRANSPORT_MODE_RADIANCE);
                    v3 lp = vadd(lvx->in.p, vs(lvx->in.gn, lvx->in.traceErrorOffset));
                    v3 cp = vadd(cvx->in.p, vs(cvx->in.gn, cvx->in.traceErrorOffset));
                    v3 w = vsub(cp, lp);
                    float sqDist = vdot(w, w);
                    float dist = sqrtf(sqDist);
                    w = vdivs(w, dist);
                    if (isNotNearZero(sqDist)) {
                        float g = absDot(cvx->in.sn, w) * absDot(lvx->in.sn, w) / sqDist;
                        rad[slot] = vs(vmul(vmul(vmul(lvx->throughput, cvx->throughput), lvf), cvf), g);
                    }
                    if (isNotBlack(rad[slot])) {
                        conn[slot].o = lp; conn[slot].tmax = dist; conn[slot].d = w; conn[slot].mask = -1; conn[slot].active = -1;
                    }
                }
            }
            ++slot;
        }
    (void)C;
    /* ---- RR QueryOcclusion over the connection rays + ConnectVertices (BDPT.cl:671-913) ---- */
    float* out = b->final3;
    slot = 0;
    for (int t = 1; t <= camCount; ++t)
        for (int sI = 0; sI <= lightCount; ++sI) {
            const int depth = t + sI - 2;
            if ((t == 1 && sI == 1) || depth < 0 || depth > D) continue;
            BVert* pt0 = &cv[t - 1];
            if (sI == 0) {
                if (bvLight(pt0)) rad[slot] = vmul(evalLightLe(&s->d.lights[pt0->lightIdx], pt0->in.gn, pt0->in.wo), pt0->throughput);
            } else {
                float vis = 0.0f;
                if (conn[slot].active) {
                    int anv = 0;
                    int occ = traceAny(s, &conn[slot], stack, &anv, tch ? tch + 2 * NN : NULL);
                    nConn++; vConn += anv;
                    vis = occ != -1 ? 0.0f : 1.0f;
                }
                rad[slot] = vs(rad[slot], vis);
            }
            float mis = 1.0f;
            if (isBlack(rad[slot])) mis = 0.0f;
            else if (sI + t == 2) mis = 1.0f;
            else {
                float sumRi = 0.0f;
                BVert* qs = sI > 0 ? &lv[sI - 1] : NULL;
                BVert* pt = t > 0 ? &cv[t - 1] : NULL;
                BVert* qsPrev = sI > 1 ? &lv[sI - 2] : NULL;
                BVert* ptPrev = t > 1 ? &cv[t - 2] : NULL;
                BVert backup;
                if (sI == 1) { backup = *qs; *qs = b->sampledLight[(size_t)bufferIdx * D + t - 2]; }
                else if (t == 1) { backup = *pt; *pt = sampledCam[sI - 2]; }
                int ptFlags = 0, qsFlags = 0;
                float ptRev = 0, qsRev = 0, ptPrevRev = 0, qsPrevRev = 0;
                if (pt) { ptFlags = pt->flags; pt->flags &= ~BVF_DELTA; }
                if (qs) { qsFlags = qs->flags; qs->flags &= ~BVF_DELTA; }
                if (pt) { ptRev = pt->pdfRev; pt->pdfRev = sI > 0 ? evalVertexPdf(s, cam, qs, qsPrev, pt) : evalVertexPdfLightOrigin(s, pt, ptPrev->in.p); }
                if (ptPrev) { ptPrevRev = ptPrev->pdfRev; ptPrev->pdfRev = sI > 0 ? evalVertexPdf(s, cam, pt, qs, ptPrev) : evalVertexPdfLight(s, pt, ptPrev); }
                if (qs) { qsRev = qs->pdfRev; qs->pdfRev = evalVertexPdf(s, cam, pt, ptPrev, qs); }
                if (qsPrev) { qsPrevRev = qsPrev->pdfRev; qsPrev->pdfRev = evalVertexPdf(s, cam, qs, pt, qsPrev); }
                float ri = 1.0f;
                for (int k = t - 1; k > 0; --k) {
                    ri *= remap0(cv[k].pdfRev) / remap0(cv[k].pdfFwd);
                    if (!(cv[k].flags & BVF_DELTA) && !(cv[k - 1].flags & BVF_DELTA)) sumRi += ri;
                }
                ri = 1.0f;
                for (int k = sI - 1; k >= 0; --k) {
                    ri *= remap0(lv[k].pdfRev) / remap0(lv[k].pdfFwd);
                    int deltaLight = k > 0 ? (lv[k - 1].flags & BVF_DELTA) != 0 : (lv[0].flags & BVF_DELTA_LIGHT) != 0;
                    if (!(lv[k].flags & BVF_DELTA) && !deltaLight) sumRi += ri;
                }
                if (pt) { pt->flags = ptFlags; pt->pdfRev = ptRev; }
                if (qs) { qs->flags = qsFlags; qs->pdfRev = qsRev; }
                if (ptPrev) ptPrev->pdfRev = ptPrevRev;
                if (qsPrev) qsPrev->pdfRev = qsPrevRev;
                if (sI == 1) *qs = backup;
                else if (t == 1) *pt = backup;
                mis = 1.0f / (1.0f + sumRi);
            }
            if (t == 1) {
                if (isNotBlack(rad[slot])) {
                    const size_t ri3 = (size_t)sampledCam[sI - 2].radianceBufferIdx * 3;
                    atomicAddF(out + ri3, rad[slot].x * mis);
                    atomicAddF(out + ri3 + 1, rad[slot].y * mis);
                    atomicAddF(out + ri3 + 2, rad[slot].z * mis);
                }
            } else {
                const size_t ri3 = (size_t)bufferIdx * 3;
                atomicAddF(out + ri3, rad[slot].x * mis);
                atomicAddF(out + ri3 + 1, rad[slot].y * mis);
                atomicAddF(out + ri3 + 2, rad[slot].z * mis);
            }
            ++slot;
        }
    atomic_fetch_add(&c->stats[0], nSub);
    atomic_fetch_add(&c->stats[1], vSub);
    atomic_fetch_add(&c->stats[2], nConn);
    atomic_fetch_add(&c->stats[3], vConn);
}

/* One RTBDPTPass::update frame over `rows` (NULL = all rows); radiance = CopyBuffer output
 * (float4 per pixel, W*H*4) -- splats from the rendered rows land in any row.  stats[4]:
 * subpath rays traced, their node visits, connection rays traced, their node visits. */
void orc_bdpt_render(orc_scene* s, orc_bdpt* b, const mcrt_camera* cam, int frame, int sampler, const int32_t* rows,
                     int nrows, int threads, float* radiance, int32_t* camCounts, int32_t* lightCounts, int64_t* stats) {
    const size_t N = (size_t)b->W * b->H;
    if (stats) memset(stats, 0, 4 * sizeof(int64_t));
    memset(b->final3, 0, 3 * N * sizeof(float));   /* GenerateStartVertices clears the pixel (BDPT.cl:264-267) */
    if (s->nodes && s->d.num_lights > 0) {          /* RTBDPTPass.cpp:69: no lights -> pass skipped */
        BdptCtx c;
        c.s = s; c.b = b; c.cam = cam; c.frame = frame; c.sampler = sampler; c.rows = rows;
        for (int k = 0; k < 4; ++k) atomic_init(&c.stats[k], 0);
        const int64_t n = rows ? (int64_t)nrows * b->W : (int64_t)N;
        parallel_for(n, threads, b->W, bdptPixel, &c);
        if (stats) for (int k = 0; k < 4; ++k) stats[k] = atomic_load(&c.stats[k]);
    }
    for (size_t i = 0; i < N; ++i) {   /* CopyBuffer (BDPT.cl:916-931) */
        radiance[4 * i] = b->final3[3 * i];
        radiance[4 * i + 1] = b->final3[3 * i + 1];
        radiance[4 * i + 2] = b->final3[3 * i + 2];
        radiance[4 * i + 3] = 0.0f;
    }
    if (camCounts) memcpy(camCounts, b->camCount, N * sizeof(int32_t));
    if (lightCounts) memcpy(lightCounts, b->lightCount, N * sizeof(int32_t));
}

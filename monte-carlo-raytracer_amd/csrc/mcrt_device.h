// mcrt_device.h -- device-side building blocks of the MI355X path-tracing core.
//
// Semantics follow the reference OpenCL kernels (paths: KRN = assets/kernels,
// RR = third_party/RadeonRays/RadeonRays); the data layout and control flow are
// our own (SoA path queues, wave64 compaction, 64-B BVH nodes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mcrt_capi.h"

#define MCRT_DEV __device__ __forceinline__

// ---------------------------------------------------------------------------
// small vector type (OpenCL float3 semantics)
// ---------------------------------------------------------------------------
struct v3 {
    float x, y, z;
};
MCRT_DEV v3 mk3(float x, float y, float z) { return v3{x, y, z}; }
MCRT_DEV v3 operator+(v3 a, v3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
MCRT_DEV v3 operator-(v3 a, v3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
MCRT_DEV v3 operator*(v3 a, v3 b) { return mk3(a.x * b.x, a.y * b.y, a.z * b.z); }
MCRT_DEV v3 operator*(v3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
MCRT_DEV v3 operator*(float s, v3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
MCRT_DEV v3 operator/(v3 a, float s) { return mk3(a.x / s, a.y / s, a.z / s); }
MCRT_DEV v3 operator-(v3 a) { return mk3(-a.x, -a.y, -a.z); }
MCRT_DEV float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
MCRT_DEV v3 cross(v3 a, v3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
MCRT_DEV v3 normalize(v3 p) {
    float l2 = dot(p, p);
    if (l2 < 1.17549435e-38f) { p = p * 0x1.0p+86f; l2 = dot(p, p); }
    else if (__builtin_isinf(l2)) { p = p * 0x1.0p-65f; l2 = dot(p, p); }
    if (l2 == 0.0f) return p;
    return p * (1.0f / sqrtf(l2));
}
MCRT_DEV float length(v3 p) { return sqrtf(dot(p, p)); }
MCRT_DEV v3 mix(v3 a, v3 b, float t) { return a + (b - a) * t; }
MCRT_DEV float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }
MCRT_DEV float signf(float x) {
    if (x > 0.0f) return 1.0f;
    if (x < 0.0f) return -1.0f;
    if (x == 0.0f) return x;
    return 0.0f;
}
MCRT_DEV v3 ld3(const mcrt_float4& p) { return mk3(p.x, p.y, p.z); }
MCRT_DEV v3 ld3(const float4& p) { return mk3(p.x, p.y, p.z); }
MCRT_DEV float absDot(v3 a, v3 b) { return fabsf(dot(a, b)); }
MCRT_DEV bool isNearZero(float v) { return fabsf(v) < 1e-8f; }
MCRT_DEV bool isNotNearZero(float v) { return fabsf(v) > 1e-8f; }

#define PI_F 3.14159265359f   // KRN/math.cl:8
#define PI_INV_F 0.31830988618f
#define PI_DIV_4_F 0.78539816339f
#define PI_DIV_2_F 1.57079632679f
#define RT_TRACE_OFFSET_F 0.00001f
#define RT_MAX_TRACE_F 1000.0f

// KRN/math.cl:53-66
MCRT_DEV v3 orthogonalVector(v3 n) {
    if (fabsf(n.z) > 0.0f) {
        float d = sqrtf(n.z * n.z + n.x * n.x);
        return mk3(-n.z / d, 0.0f, n.x / d);
    }
    float d = sqrtf(n.y * n.y + n.x * n.x);
    return mk3(n.y / d, -n.x / d, 0.0f);
}
// KRN/matrix.cl:44-60 (row-major mat4)
MCRT_DEV v3 xformVec(const mcrt_mat4& m, v3 v) { return mk3(dot(ld3(m.m0), v), dot(ld3(m.m1), v), dot(ld3(m.m2), v)); }
MCRT_DEV v3 xformPt(const mcrt_mat4& m, v3 v) {
    return mk3(dot(ld3(m.m0), v) + m.m0.w, dot(ld3(m.m1), v) + m.m1.w, dot(ld3(m.m2), v) + m.m2.w);
}

// ---------------------------------------------------------------------------
// RNG + samplers (KRN/rng.cl:48-107, KRN/samplers.cl:64-122)
// ---------------------------------------------------------------------------
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
MCRT_DEV float sample1D(Sampler& s) {
    if (s.mats) {
        uint32_t v = s.scramble;
        uint32_t idx = s.idx;
        const uint32_t* C = s.mats + s.dim * 52u;
        for (int i = 0; idx != 0; idx >>= 1, ++i)
            if (idx & 1u) v ^= C[i];
        s.dim++;
        return (float)v * 0x1p-32f;
    }
    return (float)xorshift(s.idx) * 0x1p-32f;   // rng.cl:104-107 (/0xffffffff == /2^32 in float)
}
struct v2 {
    float x, y;
};
MCRT_DEV v2 sample2D(Sampler& s) {
    v2 u;
    u.x = sample1D(s);
    u.y = sample1D(s);
    return u;
}

// KRN/samplers.cl:169-198
MCRT_DEV v2 concentricDisc(v2 u) {
    float ox = 2.0f * u.x - 1.0f, oy = 2.0f * u.y - 1.0f;
    if (u.x < 1e-8f && u.y < 1e-8f) return v2{0.0f, 0.0f};
    float theta, r;
    if (fabsf(ox) > fabsf(oy)) { r = ox; theta = PI_DIV_4_F * (oy / ox); }
    else { r = oy; theta = PI_DIV_2_F - PI_DIV_4_F * (ox / oy); }
    float s, c;
    sincosf(theta, &s, &c);
    return v2{r * c, r * s};
}
MCRT_DEV v3 cosineHemisphere(v2 u) {
    v2 d = concentricDisc(u);
    float y = sqrtf(fmaxf(0.0f, 1.0f - d.x * d.x - d.y * d.y));
    return mk3(d.x, y, d.y);
}

// ---------------------------------------------------------------------------
// Uber BSDF (KRN/bxdfs.cl); shading frame: normal = y, tangent = x, binormal = z
// ---------------------------------------------------------------------------
enum : int {
    BSDF_REFLECTION = 1, BSDF_TRANSMISSION = 2, BSDF_DIFFUSE = 4, BSDF_GLOSSY = 8, BSDF_SPECULAR = 16,
    BSDF_SPEC_REFL = 17, BSDF_SPEC_TRANS = 18, BSDF_LAMBERT = 5, BSDF_MF_REFL = 9, BSDF_MF_TRANS = 10,
};
MCRT_DEV float cosT(v3 w) { return w.y; }
MCRT_DEV float cos2T(v3 w) { return w.y * w.y; }
MCRT_DEV float absCosT(v3 w) { return fabsf(w.y); }
MCRT_DEV float sin2T(v3 w) { return fmaxf(0.0f, 1.0f - cos2T(w)); }
MCRT_DEV float sinT(v3 w) { return sqrtf(sin2T(w)); }
MCRT_DEV float tanT(v3 w) { return sinT(w) / cosT(w); }
MCRT_DEV float tan2T(v3 w) { return sin2T(w) / cos2T(w); }
MCRT_DEV float cosP(v3 w) { float st = sinT(w); return st == 0 ? 1.0f : clampf(w.x / st, -1.0f, 1.0f); }
MCRT_DEV float sinP(v3 w) { float st = sinT(w); return clampf(w.z / st, -1.0f, 1.0f); }   // bxdfs.cl:38 (always clamps)
MCRT_DEV bool sameHemi(v3 a, v3 b) { return a.y * b.y > 0.0f; }
MCRT_DEV bool isBlack(v3 c) { return c.x < 0.000001f && c.y < 0.000001f && c.z < 0.000001f; }
MCRT_DEV bool notBlack(v3 c) { return c.x > 0.000001f || c.y > 0.000001f || c.z > 0.000001f; }

// bxdfs.cl:159-190
MCRT_DEV float fresnelDielectric(float cosI, float etaI, float etaT) {
    cosI = clampf(cosI, -1.0f, 1.0f);
    if (cosI <= 0.0f) { float h = etaI; etaI = etaT; etaT = h; cosI = fabsf(cosI); }
    float sinI = sqrtf(fmaxf(0.0f, 1.0f - cosI * cosI));
    float sinT_ = etaI / etaT * sinI;
    if (sinT_ >= 1.0f) return 1.0f;
    float cosT_ = sqrtf(fmaxf(0.0f, 1.0f - sinT_ * sinT_));
    float rparl = ((etaT * cosI) - (etaI * cosT_)) / ((etaT * cosI) + (etaI * cosT_));
    float rperp = ((etaI * cosI) - (etaT * cosT_)) / ((etaI * cosI) + (etaT * cosT_));
    return (rparl * rparl + rperp * rperp) * 0.5f;
}
MCRT_DEV bool refractDir(v3 wi, v3 n, float eta, v3& wt) {   // bxdfs.cl:233-245
    float cI = dot(n, wi);
    float s2I = fmaxf(0.0f, 1.0f - cI * cI);
    float s2T = eta * eta * s2I;
    if (s2T >= 1.0f) return false;
    float cT = sqrtf(1.0f - s2T);
    wt = (-eta) * wi + (eta * cI - cT) * n;
    return true;
}
MCRT_DEV float roughnessToAlpha(float r) {   // bxdfs.cl:385-390
    r = fmaxf(r, 1e-3f);
    float x = logf(r);
    return 1.62142f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
}
MCRT_DEV float trD(v3 wh, v2 a) {   // bxdfs.cl:406-415
    float t2 = tan2T(wh);
    if (__builtin_isinf(t2)) return 0.0f;
    float c4 = cos2T(wh) * cos2T(wh);
    float cp = cosP(wh), sp = sinP(wh);
    float e = (cp * cp / (a.x * a.x) + sp * sp / (a.y * a.y)) * t2;
    return 1.0f / (PI_F * a.x * a.y * c4 * (1.0f + e) * (1.0f + e));
}
MCRT_DEV float trLambda(v3 w, v2 a) {   // bxdfs.cl:435-445
    float at = fabsf(tanT(w));
    if (__builtin_isinf(at)) return 0.0f;
    float cp = cosP(w), sp = sinP(w);
    float aw = sqrtf(cp * cp * a.x * a.x + sp * sp * a.y * a.y);
    float x = (aw * at) * (aw * at);
    return (-1.0f + sqrtf(1.f + x)) / 2.0f;
}
MCRT_DEV float trG(v3 wo, v3 wi, v2 a) { return 1.0f / (1.0f + trLambda(wo, a) + trLambda(wi, a)); }
// bxdfs.cl:481-500
MCRT_DEV v3 mfReflEval(v3 R, v2 a, float etaI, float etaT, v3 wo, v3 wi) {
    float cO = absCosT(wo), cI = absCosT(wi);
    v3 wh = wi + wo;
    if (cI == 0.0f || cO == 0.0f) return mk3(0, 0, 0);
    if (wh.x == 0.0f && wh.y == 0.0f && wh.z == 0.0f) return mk3(0, 0, 0);
    wh = normalize(wh);
    float F = fresnelDielectric(dot(wi, wh), etaI, etaT);
    return R * trD(wh, a) * trG(wo, wi, a) * F / (4.0f * cI * cO);
}
// bxdfs.cl:563-588
MCRT_DEV v3 mfTransEval(v3 T, v2 a, float etaI, float etaT, v3 wo, v3 wi) {
    if (sameHemi(wo, wi)) return mk3(0, 0, 0);
    float cO = cosT(wo), cI = cosT(wi);
    if (cI == 0.0f || cO == 0.0f) return mk3(0, 0, 0);
    float eta = cosT(wo) > 0.0f ? (etaT / etaI) : (etaI / etaT);
    v3 wh = normalize(wo + wi * eta);
    if (wh.z < 0) wh = -wh;
    float F = fresnelDielectric(dot(wo, wh), etaI, etaT);
    float sd = dot(wo, wh) + eta * dot(wi, wh);
    float factor = 1.0f / eta;   // TRANSPORT_MODE_RADIANCE
    float s = fabsf(trD(wh, a) * trG(wo, wi, a) * eta * eta * absDot(wi, wh) * absDot(wo, wh) * factor * factor /
                    (cI * cO * sd * sd));
    return (mk3(1.0f - F, 1.0f - F, 1.0f - F) * T) * s;
}
// bxdfs.cl:647-675
MCRT_DEV v3 trSampleWh(v2 u, v3 wo, v2 a) {
    float cosTh;
    float phi = (2.0f * PI_F) * u.y;
    if (a.x == a.y) {
        float t2 = a.x * a.x * u.x / (1.0f - u.x);
        cosTh = 1.0f / sqrtf(1.0f + t2);
    } else {
        phi = atanf(a.y / a.x * tanf(2.0f * PI_F * u.y + 0.5f * PI_F));
        if (u.y > .5f) phi += PI_F;
        float sp, cp;
        sincosf(phi, &sp, &cp);
        float a2 = 1.0f / (cp * cp / (a.x * a.x) + sp * sp / (a.y * a.y));
        float t2 = a2 * u.x / (1.0f - u.x);
        cosTh = 1.0f / sqrtf(1.0f + t2);
    }
    float sinTh = sqrtf(fmaxf(0.0f, 1.0f - cosTh * cosTh));
    float sp, cp;
    sincosf(phi, &sp, &cp);
    v3 wh = mk3(sinTh * cp, cosTh, sinTh * sp);
    if (!sameHemi(wo, wh)) wh = -wh;
    return wh;
}
MCRT_DEV float mfReflPdf(v3 wo, v3 wi, v3 wh, v2 a) {   // bxdfs.cl:695-701
    if (!sameHemi(wo, wi)) return 0.0f;
    return trD(wh, a) * absCosT(wh) / (4.0f * dot(wo, wh));
}
MCRT_DEV float mfTransPdf(v3 wo, v3 wi, v2 a, float etaA, float etaB) {   // bxdfs.cl:717-729
    if (sameHemi(wo, wi)) return 0.0f;
    float eta = cosT(wo) > 0.0f ? (etaB / etaA) : (etaA / etaB);
    v3 wh = normalize(wo + wi * eta);
    float sd = dot(wo, wh) + eta * dot(wi, wh);
    float dwh = fabsf((eta * eta * dot(wi, wh)) / (sd * sd));
    return trD(wh, a) * absCosT(wh) * dwh;
}

struct Frame {   // the RTInteraction fields the shading uses
    v3 p, gn, sn, t, b;   // t = sdpdu, b = sdpdv
    v2 uv;
};
MCRT_DEV v3 toLocal(v3 v, const Frame& f) { return mk3(dot(f.t, v), dot(f.sn, v), dot(f.b, v)); }
MCRT_DEV v3 toWorld(v3 w, const Frame& f) {
    return mk3(f.t.x * w.x + f.sn.x * w.y + f.b.x * w.z, f.t.y * w.x + f.sn.y * w.y + f.b.y * w.z,
               f.t.z * w.x + f.sn.z * w.y + f.b.z * w.z);
}

struct Uber {   // RTUberMaterialProperties (materials.cl:67-74)
    v3 kd, ks, kr, kt, op;
    float ktw;
    v2 a;
    float eta;
};

// bxdfs.cl:804-827
MCRT_DEV v3 uberEval(const Uber& m, const Frame& f, v3 woW, v3 wiW) {
    if (!(dot(f.gn, woW) * dot(f.gn, wiW) > 0.0f)) {
        if (m.ktw < 0.5f) return mk3(0, 0, 0);
        return mfTransEval(m.kt * m.op, m.a, 1.0f, m.eta, toLocal(woW, f), toLocal(wiW, f));
    }
    v3 wo = toLocal(woW, f), wi = toLocal(wiW, f);
    return mfReflEval(m.ks * m.op, m.a, 1.0f, m.eta, wo, wi) + (m.kd * m.op) * PI_INV_F;
}

// bxdfs.cl:892-1053 (wi zero-initialised: SURVEY.md App. A Q3)
MCRT_DEV v3 uberSample(const Uber& m, const Frame& f, v2 u, v3 woW, v3& wiW, float& pdf, int& sampledType) {
    v3 t = mk3(1.0f - m.op.x, 1.0f - m.op.y, 1.0f - m.op.z);
    v3 kd = m.kd * m.op, ks = m.ks * m.op, kt = m.kt * m.op, kr = m.kr * m.op;
    v3 wo = toLocal(woW, f);
    v3 wi = mk3(0, 0, 0);
    bool perfT = m.ktw < 0.5f;
    bool hasT = notBlack(t), hasKd = notBlack(kd), hasKs = notBlack(ks), hasKr = notBlack(kr), hasKt = notBlack(kt);
    sampledType = 0;
    int n = (int)hasT + (int)hasKd + (int)hasKs + (int)hasKr + (int)hasKt;   // hasKt counts as spec or glossy
    if (n == 0) return mk3(0, 0, 0);
    int chosen = min((int)floorf(u.x * n), n - 1);
    u.x = u.x * n - chosen;
    v3 fr = mk3(0, 0, 0);
    pdf = 0.0f;
    bool spec = false;
    if (hasT) {
        if (chosen-- == 0) {   // specular transmission of the transparency (eta 1 / 1)
            // sampleSpecularTransmission(t, 1, 1): etaI == etaT => refract never fails
            float sg = signf(wo.y);
            v3 nn = mk3(0.0f, 1.0f, 0.0f) * sg;
            if (refractDir(wo, nn, 1.0f, wi)) {
                pdf = 1.0f;
                v3 ft = t * (1.0f - fresnelDielectric(cosT(wi), 1.0f, 1.0f));
                ft = ft * ((1.0f * 1.0f) / (1.0f * 1.0f));
                fr = fr + ft / absCosT(wi);
            }
            sampledType |= BSDF_SPEC_TRANS;
            spec = true;
        }
    }
    if (perfT && hasKt) {
        if (chosen-- == 0) {   // sampleSpecularTransmission(kt, 1, eta), bxdfs.cl:288-307
            bool entering = cosT(wo) > 0.0f;
            float etaI = entering ? 1.0f : m.eta, etaT = entering ? m.eta : 1.0f;
            v3 nn = mk3(0.0f, 1.0f, 0.0f) * signf(wo.y);
            if (refractDir(wo, nn, etaI / etaT, wi)) {
                pdf = 1.0f;
                v3 ft = kt * (1.0f - fresnelDielectric(cosT(wi), 1.0f, m.eta));
                ft = ft * ((etaI * etaI) / (etaT * etaT));
                fr = fr + ft / absCosT(wi);
            }
            sampledType |= BSDF_SPEC_TRANS;
            spec = true;
        }
    }
    if (hasKr) {
        if (chosen-- == 0) {   // bxdfs.cl:259-268
            wi = mk3(-wo.x, wo.y, -wo.z);
            pdf = 1.0f;
            float F = fresnelDielectric(cosT(wi), 1.0f, m.eta);
            fr = fr + (F * kr) / absCosT(wi);
            sampledType |= BSDF_SPEC_REFL;
            spec = true;
        }
    }
    if (hasKt) {   // bxdfs.cl:1004: tested regardless of Kt.w (Q2)
        if (chosen-- == 0) {   // bxdfs.cl:751-762
            v3 wh = trSampleWh(u, wo, m.a);
            float eta = cosT(wo) > 0.0f ? (1.0f / m.eta) : (m.eta / 1.0f);
            if (refractDir(wo, wh, eta, wi)) {
                pdf = mfTransPdf(wo, wi, m.a, 1.0f, m.eta);
                fr = fr + mfTransEval(kt, m.a, 1.0f, m.eta, wo, wi);
            }
            sampledType |= BSDF_MF_TRANS;
        }
    }
    bool lambertEval = false;
    if (hasKd) {
        if (chosen-- == 0) {   // bxdfs.cl:317-347
            wi = cosineHemisphere(u);
            if (wo.y < 0.0f) wi.y *= -1.0f;
            pdf = absCosT(wi) * PI_INV_F;
            fr = fr + kd * PI_INV_F;
            sampledType |= BSDF_LAMBERT;
        } else if (!spec && sameHemi(wi, wo)) {
            lambertEval = true;
        }
    }
    if (hasKs) {
        if (chosen-- == 0) {   // bxdfs.cl:731-749
            v3 wh = trSampleWh(u, wo, m.a);
            wi = -wo + (2.0f * dot(wh, wo)) * wh;
            if (sameHemi(wo, wi)) {
                pdf = mfReflPdf(wo, wi, wh, m.a);
                fr = fr + mfReflEval(ks, m.a, 1.0f, m.eta, wo, wi);
            }
            sampledType |= BSDF_MF_REFL;
        } else if (!spec && sameHemi(wi, wo)) {
            fr = fr + mfReflEval(ks, m.a, 1.0f, m.eta, wo, wi);
            pdf += mfReflPdf(wo, wi, normalize(wo + wi), m.a);
        }
    }
    if (lambertEval) {
        fr = fr + kd * PI_INV_F;
        pdf += sameHemi(wo, wi) ? absCosT(wi) * PI_INV_F : 0.0f;
    }
    pdf /= (float)n;
    wiW = toWorld(wi, f);
    return fr;
}

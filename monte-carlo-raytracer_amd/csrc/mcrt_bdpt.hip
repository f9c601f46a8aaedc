// mcrt_bdpt.hip -- bidirectional path tracing (KRN/BDPT.cl, host pass RTBDPTPass.cpp:67-488) on gfx950.
//
// One frame (1 sample per pixel, maxDepth D) is, per rank band:
//   k_bdpt_start          camera vertex 0 + light vertex 0 of every pixel (GenerateStartVertices,
//                         BDPT.cl:240-312); the first camera rays and light rays go to two queues
//                         (d = 1: one k_extend_pair launch, the camera rays as wave packets,
//                         then k_bdpt_vertex once per queue)
//   for d in 1..D+1:
//     k_extend            closest hit over the queue (camera and light rays together)
//     k_bdpt_vertex       GenerateSecondaryVertices (BDPT.cl:317-458) for every queued ray: the
//                         surface vertex at depth d and, unless the subpath is done, its next ray;
//                         for a light vertex also its light-tracing strategy (t = 1, below) from the
//                         registers that store it (BdptArgs::lightInVertex)
//   k_bdpt_connect        PrepareConnections (BDPT.cl:460-646) fused with the visibility-independent
//                         part of ConnectVertices (BDPT.cl:671-913): every other (t, s) strategy's
//                         unweighted contribution AND its MIS weight, so only strategies with a
//                         non-zero weighted contribution emit a connection ray (compacted queue)
//   k_bdpt_vis            any hit over the connection queue: an occluded own strategy is zeroed
//                         in its slot; an unoccluded t = 1 strategy (light tracing) is splatted
//                         with a float atomic into the splat buffer of the pixel it projects to
//   k_bdpt_gather         radiance = (own strategies summed in the reference's (t, s) order) + splats
//
// HBM layout (N = W*H pixels; all planes are float4 x N, so every access is coalesced):
//   camera vertices  (D+2) depths x 13 planes, light vertices (D+1) x 13 planes:
//     0 p.xyz|traceErrorOffset  1 gn.xyz|pdfFwd  2 sn.xyz|pdfRev  3 wo.xyz|pdfPos
//     4 sdpdu.xyz|uv.x  5 sdpdv.xyz|uv.y  6 throughput.xyz|-  7 int4(type, flags, lightIdx, materialIdx)
//     8-12 the vertex's uber-material properties (getUberMaterialProperties at its uv, computed
//     once by k_bdpt_vertex): Kd|eta, Ks|Kt.w, Kr|alpha.x, Kt.xyz|alpha.y, opacity|material type --
//     written only where a connection strategy fetches them (not for camera depth D + 1, nor for
//     light depth D while the light-tracing strategies run in the vertex launch).
//   (the reference's 240-B RTBDPTVertex holds the first 8 planes' fields plus unused
//   differentials, and re-reads up to 8 textures per material evaluation instead of plane 8-12).
//   vertex counts: int x N per subpath.  sampled light vertex of the s = 1 strategy, persistent across
//   frames (the reference reads it before overwriting it, BDPT.cl:585-586): D planes of float4
//   (p.xyz | flags<<16 | lightIdx).  own-strategy slots: (C - D) planes of float4 (C = maxConnections).
//   splat buffer: float4 x N (zero between frames).
//
// Arithmetic mirrors the reference expressions (mcrt_device.h conventions: cl_div = the 2.5-ulp
// OpenCL division, contraction as ROCm clang does at -O3 with FP_CONTRACT ON).
#include <rocprim/device/device_radix_sort.hpp>

#include "mcrt_device.h"
#include "mcrt_internal.h"
#include "mcrt_traverse.h"
#include "mcrt_shading.h"

#define BDPT_BLOCK 256
// (register caps for more resident waves spill and lose: k_bdpt_vertex at 5 waves +8 %,
// k_bdpt_connect's GENERAL / NEE classes at 4 waves +20 %; profiles/r04/ab/README.txt item 15)
#define BDPT_LIGHT_KEY_BITS 13
#define BDPT_LIGHT_KEY_NONE ((1u << BDPT_LIGHT_KEY_BITS) - 1)
#define BDPT_BOUNCE_KEY_BITS 16

// RTBDPTVertexType / RTBDPTVertexFlag (kernel_data.h:202-218)
enum { RT_BDPT_CAMERA_VERTEX = 0, RT_BDPT_LIGHT_VERTEX = 1, RT_BDPT_SURFACE_VERTEX = 2 };
enum {
    VF_CONNECTIBLE = 1,
    VF_DELTA_LIGHT = 1 << 1,
    VF_DELTA = 1 << 2,
    VF_INFINITE_LIGHT = 1 << 3,
};
#define MCRT_LIGHT_FLAG_DELTA_LIGHT (MCRT_LIGHT_FLAG_DELTA_POSITION | MCRT_LIGHT_FLAG_DELTA_DIRECTION)

struct BVertex {
    Frame fr;   // p, gn, sn, sdpdu, sdpdv, uv
    f3 wo, throughput;
    float traceErrorOffset, pdfFwd, pdfRev, pdfPos;
    int type, flags, lightIdx, materialIdx;
    const float4* planes;   // where a surface vertex's material properties live (loadUber)
    int depth;
    Uber um;      // planes 8-12 when loaded with the vertex (loadVertexU, hasUm)
    int umType;
    bool hasUm;
};

// --- plane addressing ---------------------------------------------------------------------
MCRT_DEV float4* vplane(float4* base, int depth, int k, int N) {
    return base + (size_t)(depth * BDPT_VERTEX_PLANES + k) * N;
}
MCRT_DEV const float4* vplane(const float4* base, int depth, int k, int N) {
    return base + (size_t)(depth * BDPT_VERTEX_PLANES + k) * N;
}
// material properties of a surface vertex (planes 8-12); matType = RTMaterial::type
MCRT_DEV void storeUber(float4* base, int depth, int pix, int N, const Uber& u, int matType) {
    vplane(base, depth, 8, N)[pix] = make_float4(u.Kd.x, u.Kd.y, u.Kd.z, u.eta);
    vplane(base, depth, 9, N)[pix] = make_float4(u.Ks.x, u.Ks.y, u.Ks.z, u.Kt.w);
    vplane(base, depth, 10, N)[pix] = make_float4(u.Kr.x, u.Kr.y, u.Kr.z, u.roughness.x);
    vplane(base, depth, 11, N)[pix] = make_float4(u.Kt.x, u.Kt.y, u.Kt.z, u.roughness.y);
    vplane(base, depth, 12, N)[pix] = make_float4(u.opacity.x, u.opacity.y, u.opacity.z, __int_as_float(matType));
}
MCRT_DEV Uber loadUber(const float4* base, int depth, int pix, int N, int* matType) {
    const float4 a = vplane(base, depth, 8, N)[pix], b = vplane(base, depth, 9, N)[pix];
    const float4 c = vplane(base, depth, 10, N)[pix], d = vplane(base, depth, 11, N)[pix];
    const float4 e = vplane(base, depth, 12, N)[pix];
    Uber u;
    u.Kd = ld3(a);
    u.eta = a.w;
    u.Ks = ld3(b);
    u.Kt = f4{d.x, d.y, d.z, b.w};
    u.Kr = ld3(c);
    u.roughness = f2{c.w, d.w};
    u.opacity = ld3(e);
    *matType = __float_as_int(e.w);
    return u;
}

MCRT_DEV BVertex loadVertex(const float4* base, int depth, int pix, int N) {
    BVertex v;
    const float4 a = vplane(base, depth, 0, N)[pix], b = vplane(base, depth, 1, N)[pix];
    const float4 c = vplane(base, depth, 2, N)[pix], d = vplane(base, depth, 3, N)[pix];
    const float4 e = vplane(base, depth, 4, N)[pix], f = vplane(base, depth, 5, N)[pix];
    const float4 g = vplane(base, depth, 6, N)[pix];
    const int4 h = *reinterpret_cast<const int4*>(&vplane(base, depth, 7, N)[pix]);
    v.fr.p = ld3(a);
    v.traceErrorOffset = a.w;
    v.fr.gn = ld3(b);
    v.pdfFwd = b.w;
    v.fr.sn = ld3(c);
    v.pdfRev = c.w;
    v.wo = ld3(d);
    v.pdfPos = d.w;
    v.fr.sdpdu = ld3(e);
    v.fr.sdpdv = ld3(f);
    v.fr.uv = f2{e.w, f.w};
    v.throughput = ld3(g);
    v.type = h.x;
    v.flags = h.y;
    v.lightIdx = h.z;
    v.materialIdx = h.w;
    v.planes = base;
    v.depth = depth;
    v.hasUm = false;
    return v;
}
// The vertex with its material properties, all 13 planes in one round trip (the connection kernels:
// a strategy evaluates its vertices' BSDF and pdf several times)
MCRT_DEV BVertex loadVertexU(const float4* base, int depth, int pix, int N) {
    BVertex v = loadVertex(base, depth, pix, N);
    v.um = loadUber(base, depth, pix, N, &v.umType);
    v.hasUm = true;
    return v;
}
// Position / geometric normal / flags only (the "next" or "prev" vertex of a pdf evaluation)
struct BVertexPos {
    f3 p, gn;
    int flags;
};
MCRT_DEV BVertexPos loadVertexPos(const float4* base, int depth, int pix, int N) {
    BVertexPos v;
    v.p = ld3(vplane(base, depth, 0, N)[pix]);
    v.gn = ld3(vplane(base, depth, 1, N)[pix]);
    v.flags = reinterpret_cast<const int4*>(&vplane(base, depth, 7, N)[pix])->y;
    return v;
}
MCRT_DEV BVertexPos posOf(const BVertex& v) { return BVertexPos{v.fr.p, v.fr.gn, v.flags}; }

MCRT_DEV void storeVertex(float4* base, int depth, int pix, int N, const BVertex& v) {
    vplane(base, depth, 0, N)[pix] = make_float4(v.fr.p.x, v.fr.p.y, v.fr.p.z, v.traceErrorOffset);
    vplane(base, depth, 1, N)[pix] = make_float4(v.fr.gn.x, v.fr.gn.y, v.fr.gn.z, v.pdfFwd);
    vplane(base, depth, 2, N)[pix] = make_float4(v.fr.sn.x, v.fr.sn.y, v.fr.sn.z, v.pdfRev);
    vplane(base, depth, 3, N)[pix] = make_float4(v.wo.x, v.wo.y, v.wo.z, v.pdfPos);
    vplane(base, depth, 4, N)[pix] = make_float4(v.fr.sdpdu.x, v.fr.sdpdu.y, v.fr.sdpdu.z, v.fr.uv.x);
    vplane(base, depth, 5, N)[pix] = make_float4(v.fr.sdpdv.x, v.fr.sdpdv.y, v.fr.sdpdv.z, v.fr.uv.y);
    vplane(base, depth, 6, N)[pix] = make_float4(v.throughput.x, v.throughput.y, v.throughput.z, 0.0f);
    *reinterpret_cast<int4*>(&vplane(base, depth, 7, N)[pix]) = make_int4(v.type, v.flags, v.lightIdx, v.materialIdx);
}
MCRT_DEV void storePdfFwd(float4* base, int depth, int pix, int N, float x) {
    reinterpret_cast<float*>(&vplane(base, depth, 1, N)[pix])[3] = x;
}
MCRT_DEV void storePdfRev(float4* base, int depth, int pix, int N, float x) {
    reinterpret_cast<float*>(&vplane(base, depth, 2, N)[pix])[3] = x;
}

// --- kernel_data.h:447-474 vertex predicates ----------------------------------------------
MCRT_DEV bool isVertexOnSurface(f3 gn) {   // BDPT.cl:39-42
    return isNotNearZero(gn.x) || isNotNearZero(gn.y) || isNotNearZero(gn.z);
}
MCRT_DEV bool isInfinite(int flags) { return (flags & VF_INFINITE_LIGHT) != 0; }
MCRT_DEV bool isDeltaV(int flags) { return (flags & VF_DELTA) != 0; }
MCRT_DEV bool isConnectible(int flags) { return (flags & VF_CONNECTIBLE) != 0; }
MCRT_DEV bool isDeltaLightV(int flags) { return (flags & VF_DELTA_LIGHT) != 0; }
MCRT_DEV float remap0(float f) { return f == 0.0f ? 1.0f : f; }   // BDPT.cl:649-652

MCRT_DEV float dot4(float4 a, float4 b) {   // OpenCL dot(float4): fma chain
    return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}
MCRT_DEV float4 transformVector4(const mcrt_mat4& m, float4 v) {   // matrix.cl:62-70
    const float4 m0 = make_float4(m.m0.x, m.m0.y, m.m0.z, m.m0.w), m1 = make_float4(m.m1.x, m.m1.y, m.m1.z, m.m1.w);
    const float4 m2 = make_float4(m.m2.x, m.m2.y, m.m2.z, m.m2.w), m3 = make_float4(m.m3.x, m.m3.y, m.m3.z, m.m3.w);
    return make_float4(dot4(m0, v), dot4(m1, v), dot4(m2, v), dot4(m3, v));
}

// --- cameras.cl ------------------------------------------------------------------------
// evalPinholeCameraPdfWe (cameras.cl:34-59): returns pdfDir (pdfPos is 1 or 0 alongside it)
MCRT_DEV float evalPinholeCameraPdfWe(const mcrt_camera& cam, f3 o, f3 d) {
    const float cosTheta = cl_dot(d, ld3(cam.direction));
    if (cosTheta <= 0.0f) return 0.0f;
    const float r = cl_div(1.0f, cosTheta);
    const f3 pf = o + d * r;
    const float4 img = transformVector4(cam.worldToClip, make_float4(pf.x, pf.y, pf.z, 1.0f));
    if (img.x < -img.w || img.x > img.w || img.y < -img.w || img.y > img.w) return 0.0f;
    return cl_div(1.0f, (cam.area * cosTheta * cosTheta * cosTheta));
}
// evalPinholeCameraWe (cameras.cl:8-32); *nip written only when inside the image.
// `rayDirection / cosTheta` is correctly rounded in the reference's PrepareConnections.
MCRT_DEV float evalPinholeCameraWe(const mcrt_camera& cam, f3 o, f3 d, f2* nip) {
    const float cosTheta = cl_dot(d, ld3(cam.direction));
    if (cosTheta <= 0.0f) return 0.0f;
    const f3 q = f3{cr_div(d.x, cosTheta), cr_div(d.y, cosTheta), cr_div(d.z, cosTheta)};
    const f3 pf = o + q;
    const float4 img = transformVector4(cam.worldToClip, make_float4(pf.x, pf.y, pf.z, 1.0f));
    if (img.x < -img.w || img.x > img.w || img.y < -img.w || img.y > img.w) return 0.0f;
    const f2 ndc = f2{cl_div(img.x, img.w), cl_div(img.y, img.w)};
    *nip = (ndc + f2{1.0f, 1.0f}) * 0.5f;
    return cl_div(1.0f, (cam.area * cosTheta * cosTheta * cosTheta));
}

// --- lights.cl -------------------------------------------------------------------------
// evalLightPdfLe (lights.cl:227-252)
MCRT_DEV void evalLightPdfLe(const mcrt_light& light, f3 rayDirection, f3 lightNormal, float* pdfPos, float* pdfDir) {
    if (light.type == MCRT_DIRECTIONAL_LIGHT) {
        *pdfPos = cl_div(1.0f, light.area);
        *pdfDir = 0.0f;
    } else if (light.type == MCRT_POINT_LIGHT) {
        *pdfPos = 0.0f;
        *pdfDir = 0.07957747154f;   // PI4_INV
    } else {
        *pdfPos = cl_div(1.0f, light.area);
        *pdfDir = cl_dot(lightNormal, rayDirection) * PI_INV_F;   // cosineHemispherePdf
    }
}
// evalLightLe (lights.cl:26-35)
MCRT_DEV f3 evalLightLe(const mcrt_light& light, f3 gn, f3 w) {
    if (light.type == MCRT_DISK_AREA_LIGHT || light.type == MCRT_TRIANGLE_MESH_AREA_LIGHT)
        return cl_dot(gn, w) > 0.0f ? ld3(light.intensity) : splat3(0.0f);
    return splat3(0.0f);
}
// sampleLightLe (lights.cl:148-225)
struct LightLe {
    f3 Le, origin, dir, normal;
    float pdfPos, pdfDir;
};
MCRT_DEV LightLe sampleLightLe(const SceneArgs& s, const mcrt_light& light, f2 u1, f2 u2) {
    LightLe r;
    r.Le = splat3(0.0f);
    r.origin = r.dir = r.normal = splat3(0.0f);
    r.pdfPos = r.pdfDir = 0.0f;
    if (light.type == MCRT_DIRECTIONAL_LIGHT) {
        r.origin = sampleDisk(ld3(light.p), ld3(light.d), light.radius, u1, &r.pdfPos);
        r.normal = ld3(light.d);
        r.pdfDir = 1.0f;
        r.dir = ld3(light.d);
        r.Le = ld3(light.intensity);
    } else if (light.type == MCRT_POINT_LIGHT) {
        const float y = 1.0f - 2.0f * u1.x;   // uniformSampleSphere (samplers.cl:143-149)
        const float rr = cl_sqrt(fmaxf(0.0f, 1.0f - y * y));
        const float phi = 2.0f * PI_F * u1.y;
        r.dir = f3{rr * cosf(phi), y, rr * sinf(phi)};
        r.origin = ld3(light.p);
        r.normal = r.dir;
        r.pdfPos = 1.0f;
        r.pdfDir = 0.07957747154f;
        r.Le = ld3(light.intensity);
    } else if (light.type == MCRT_DISK_AREA_LIGHT || light.type == MCRT_TRIANGLE_MESH_AREA_LIGHT) {
        f3 sp, gn;
        if (light.type == MCRT_DISK_AREA_LIGHT) {
            sp = sampleDisk(ld3(light.p), ld3(light.d), light.radius, u1, &r.pdfPos);
            gn = ld3(light.d);
        } else {
            const mcrt_shape shape = s.shapes[light.shapeId];
            const int triangleIdx = ((int)floorf(u1.x * shape.numTriangles)) % (int)shape.numTriangles;
            u1.x = u1.x * shape.numTriangles - triangleIdx;
            const uint32_t i0 = s.indices[shape.startIdx + 3 * triangleIdx];
            const uint32_t i1 = s.indices[shape.startIdx + 3 * triangleIdx + 1];
            const uint32_t i2 = s.indices[shape.startIdx + 3 * triangleIdx + 2];
            const f3 p0 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i0]));
            const f3 p1 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i1]));
            const f3 p2 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i2]));
            sp = sampleTriangle(p0, p1, p2, u1, &gn);
            r.pdfPos = cl_div(1.0f, light.area);
        }
        r.normal = gn;
        const f3 w = cosineSampleHemisphere(u2);
        r.pdfDir = w.y * PI_INV_F;
        const f3 v0 = computeOrthogonalVector(gn);
        const f3 v1 = cl_cross(v0, gn);
        r.dir = w.x * v0 + w.y * gn + w.z * v1;
        r.origin = sp + gn * RT_TRACE_OFFSET_F;
        r.Le = ld3(light.intensity);
    }
    return r;
}

// --- materials.cl with transport modes ----------------------------------------------------
// evaluateMaterial / evaluateMaterialPdf (materials.cl:120-142) of a stored surface vertex: the
// uber properties come from the vertex's planes 8-12 (the same getUberMaterialProperties values
// the reference recomputes from the textures at every call).  Non-uber materials evaluate to 0.
MCRT_DEV f3 evaluateMaterialV(const BVertex& v, int pix, int N, f3 wo, f3 wi, int mode) {
    int type = v.umType;
    const Uber um = v.hasUm ? v.um : loadUber(v.planes, v.depth, pix, N, &type);
    if (type != 0) return splat3(0.0f);
    return evaluateUberBSDF(um, v.fr, wo, wi, mode);
}
MCRT_DEV float evaluateMaterialPdfV(const BVertex& v, int pix, int N, f3 wo, f3 wi) {
    int type = v.umType;
    const Uber um = v.hasUm ? v.um : loadUber(v.planes, v.depth, pix, N, &type);
    if (type != 0) return 0.0f;
    return evaluateUberBSDF_Pdf(um, v.fr, wo, wi);
}
// computeShadingNormalCorrection (BDPT.cl:23-36).  The reference's compiled kernels evaluate
// this division correctly rounded (its accuracy metadata is dropped when the select of the
// three return values is folded), in GenerateSecondaryVertices and PrepareConnections alike.
MCRT_DEV float shadingNormalCorrection(const Frame& si, f3 wo, f3 wi, int mode) {
    if (mode == TRANSPORT_MODE_IMPORTANCE) {
        const float denom = absDot(wo, si.gn) * absDot(wi, si.sn);
        if (isNearZero(denom)) return 0.0f;
        return cr_div((absDot(wo, si.sn) * absDot(wi, si.gn)), denom);
    }
    return 1.0f;
}

// --- vertex densities (BDPT.cl:44-154) -------------------------------------------------------
// convertVertexDensity(pdf, this, next)
MCRT_DEV float convertVertexDensity(float pdf, f3 thisP, const BVertexPos& next) {
    if (isInfinite(next.flags)) return pdf;
    const f3 w = next.p - thisP;
    const float lenSq = cl_dot(w, w);
    if (isNearZero(lenSq)) return 0.0f;
    const float invDistSq = cl_div(1.0f, lenSq);
    if (isVertexOnSurface(next.gn)) pdf *= absDot(next.gn, w * cl_sqrt(invDistSq));
    return pdf * invDistSq;
}
// evalVertexPdfLight(this = light-like vertex, v)
MCRT_DEV float evalVertexPdfLight(const SceneArgs& s, f3 thisP, f3 thisGn, int thisFlags, int thisLight,
                                  const BVertexPos& v) {
    f3 w = v.p - thisP;
    const float lenSq = cl_dot(w, w);
    if (isNearZero(lenSq)) return 0.0f;
    const float invDistSq = cl_div(1.0f, lenSq);
    w *= cl_sqrt(invDistSq);
    float pdf;
    if (isInfinite(thisFlags)) {
        const float radius = s.lights[thisLight].radius;
        pdf = cl_div(1.0f, (PI_F * radius * radius));
    } else {
        float pdfPos, pdfDir;
        evalLightPdfLe(s.lights[thisLight], w, thisGn, &pdfPos, &pdfDir);
        pdf = pdfDir * invDistSq;
    }
    if (isVertexOnSurface(v.gn)) pdf *= absDot(v.gn, w);
    return pdf;
}
// evalVertexPdfLightOrigin(this, nextVertexPos)
MCRT_DEV float evalVertexPdfLightOrigin(const SceneArgs& s, f3 thisP, f3 thisGn, int thisFlags, int thisLight, f3 nextP) {
    f3 w = nextP - thisP;
    const float lenSq = cl_dot(w, w);
    if (isNearZero(lenSq)) return 0.0f;
    w *= cl_sqrt(cl_div(1.0f, lenSq));
    if (isInfinite(thisFlags)) return 0.0f;
    float pdfPos, pdfDir;
    const mcrt_light light = s.lights[thisLight];
    evalLightPdfLe(light, w, thisGn, &pdfPos, &pdfDir);
    return pdfPos * light.choicePdf;
}
// evalVertexPdf(this, prev (may be null), next)
MCRT_DEV float evalVertexPdf(const SceneArgs& s, const mcrt_camera& cam, const BVertex& v, int pix, int N, bool hasPrev,
                             f3 prevP, const BVertexPos& next) {
    if (v.type == RT_BDPT_LIGHT_VERTEX) return evalVertexPdfLight(s, v.fr.p, v.fr.gn, v.flags, v.lightIdx, next);
    f3 wn = next.p - v.fr.p;
    float lenSq = cl_dot(wn, wn);
    if (isNearZero(lenSq)) return 0.0f;
    wn = cl_div(wn, cl_sqrt(lenSq));
    float pdf = 0.0f;
    if (v.type == RT_BDPT_CAMERA_VERTEX) {
        pdf = evalPinholeCameraPdfWe(cam, v.fr.p, wn);
    } else if (v.type == RT_BDPT_SURFACE_VERTEX) {
        f3 wp = splat3(0.0f);
        if (hasPrev) {
            wp = prevP - v.fr.p;
            lenSq = cl_dot(wp, wp);
            if (isNearZero(lenSq)) return 0.0f;
            wp = cl_div(wp, cl_sqrt(lenSq));
        }
        pdf = evaluateMaterialPdfV(v, pix, N, wp, wn);
    }
    return convertVertexDensity(pdf, v.fr.p, next);
}
// evalVertex_f(this, next, mode) (BDPT.cl:215-235)
MCRT_DEV f3 evalVertex_f(const BVertex& v, int pix, int N, f3 nextP, int mode) {
    f3 wi = nextP - v.fr.p;
    const float lenSq = cl_dot(wi, wi);
    if (isNearZero(lenSq)) return splat3(0.0f);
    wi = cl_div(wi, cl_sqrt(lenSq));
    if (v.type == RT_BDPT_SURFACE_VERTEX) {
        const f3 f = evaluateMaterialV(v, pix, N, v.wo, wi, mode);
        return f * shadingNormalCorrection(v.fr, v.wo, wi, mode);
    }
    return f3{1.0f, 0.0784f, 0.5765f};
}

MCRT_DEV BVertex createCameraVertex(f3 p, f3 throughput) {   // BDPT.cl:159-174
    BVertex v;
    v.fr.p = p;
    v.fr.gn = v.fr.sn = v.fr.sdpdu = v.fr.sdpdv = splat3(0.0f);
    v.fr.uv = f2{0.0f, 0.0f};
    v.wo = splat3(0.0f);
    v.throughput = throughput;
    v.traceErrorOffset = 0.0f;
    v.type = RT_BDPT_CAMERA_VERTEX;
    v.hasUm = false;
    v.flags = VF_CONNECTIBLE;
    v.lightIdx = -1;
    v.materialIdx = -1;
    v.pdfRev = v.pdfFwd = v.pdfPos = 0.0f;
    return v;
}
MCRT_DEV BVertex createLightVertex(int lightIdx, f3 p, f3 n, f3 throughput, float pdfFwd, int lightFlags) {
    BVertex v;   // BDPT.cl:176-202
    v.fr.p = p;
    v.fr.gn = n;
    v.fr.sn = n;
    v.fr.sdpdu = v.fr.sdpdv = splat3(0.0f);
    v.fr.uv = f2{0.0f, 0.0f};
    v.wo = splat3(0.0f);
    v.throughput = throughput;
    v.traceErrorOffset = RT_TRACE_OFFSET_F;
    v.type = RT_BDPT_LIGHT_VERTEX;
    v.hasUm = false;
    v.lightIdx = lightIdx;
    v.materialIdx = -1;
    v.pdfRev = 0.0f;
    v.pdfFwd = pdfFwd;
    v.pdfPos = 0.0f;
    if ((lightFlags & MCRT_LIGHT_FLAG_DELTA_DIRECTION) != 0) {
        v.flags = VF_DELTA_LIGHT | VF_INFINITE_LIGHT;
    } else {
        v.flags = VF_CONNECTIBLE;
        if ((lightFlags & MCRT_LIGHT_FLAG_DELTA_POSITION) != 0) v.flags |= VF_DELTA_LIGHT;
    }
    return v;
}

// --- kernels --------------------------------------------------------------------------------
// Ray-queue record (3 float4): (o.xyz, tag = 2*pix + isLight), (d.xyz, fwdPdf), (throughput.xyz, 0)
MCRT_DEV void pushRay(const BdptQueue& q, int slot, f3 o, int tag, f3 d, float fwdPdf, f3 tp) {
    q.o[slot] = make_float4(o.x, o.y, o.z, __int_as_float(tag));
    q.d[slot] = make_float4(d.x, d.y, d.z, fwdPdf);
    q.t[slot] = make_float4(tp.x, tp.y, tp.z, 0.0f);
}

// Batched frames (mcrt_render_frames, f.batch = B): frame k of the batch is path p = k * N + pixel
// in every per-frame plane (vertices, counts, slots, splats: plane stride NB = N * B), samples with
// frame index f.frame + k and camera camp[k]; launches over (tile, frame) walk a tile's frames
// back to back (their jittered camera rays share nodes).
MCRT_DEV void tileFrame(const FrameArgs& f, int tileAll, int& tile, int& k) {
    tile = tileAll / f.batch;
    k = tileAll - tile * f.batch;
}

// GenerateStartVertices (BDPT.cl:240-312) over the rank's 8x8 tiles x batch frames; the first
// camera rays go to camQ (tile order: coherent, traced as wave packets), the
// light rays to lightQ.
__global__ __launch_bounds__(BDPT_BLOCK) void k_bdpt_start(SceneArgs s, FrameArgs f, BdptArgs b,
                                                           const mcrt_camera* __restrict__ camp, BdptQueue camQ,
                                                           BdptQueue lightQ) {
    const int lane = threadIdx.x & 63;
    const int tileAll = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int tile, k;
    tileFrame(f, tileAll, tile, k);
    int x = 0, y = 0;
    const bool valid = tile < f.numTiles && tilePixel(f, tile, lane, x, y) && s.numLights > 0;
    const int N = (int)(f.W * f.H), NB = N * f.batch;
    const int px = y * (int)f.W + x, pix = k * N + px;   // pix: the path (plane index)
    f3 camDir = splat3(0.0f), camPos = splat3(0.0f), lo = splat3(0.0f), ld = splat3(0.0f), lt = splat3(0.0f);
    float camPdf = 0.0f, lightPdfDir = 0.0f;
    uint32_t key = BDPT_LIGHT_KEY_NONE;   // the light ray's cell (b.lightKey): invalid slots sort last
    if (valid) {
        const mcrt_camera& cam = camp[k];
        b.splat[pix] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        b.camCount[pix] = 1;
        b.lightCount[pix] = 1;
        // camera (BDPT.cl:280-292)
        const f2 r = f2{cl_div(1.0f, (float)f.W), cl_div(1.0f, (float)f.H)};
        const f2 uv = f2{(float)x * r.x, (float)y * r.y};
        camDir = lerpDirection(ld3(cam.r00), ld3(cam.r10), ld3(cam.r11), ld3(cam.r01), uv.x, uv.y);
        camPos = ld3(cam.pos);
        // camera vertex 0 (createCameraVertex): only its position and pdfRev (reset; the depth-1
        // vertex launch may set it) change from frame to frame -- the other 6 planes are constants
        // written once per plane stride
        if (b.depth0Const) {
            vplane(b.camV, 0, 0, NB)[pix] = make_float4(camPos.x, camPos.y, camPos.z, 0.0f);
            vplane(b.camV, 0, 2, NB)[pix] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        } else {
            storeVertex(b.camV, 0, pix, NB, createCameraVertex(camPos, splat3(1.0f)));
        }
        camPdf = evalPinholeCameraPdfWe(cam, camPos, camDir);
        // light (BDPT.cl:294-311)
        Sampler sampler = makeSampler(f.sampler, (uint32_t)px, f.frame + k, 0, f.W, f.H, s.sobol);
        const int chosen = (int)(((uint32_t)floorf(getSample1D(sampler) * s.numLights)) % (uint32_t)s.numLights);
        const mcrt_light light = s.lights[chosen];
        const float lightPdf = light.choicePdf;
        const f2 u1 = getSample2D(sampler);
        const f2 u2 = getSample2D(sampler);
        const LightLe le = sampleLightLe(s, light, u1, u2);
        // cell of the ray for the light-queue sort: a directional light's rays are parallel, so
        // the 64 x 64 grid of its disk sample u1 (concentricSampleDisc keeps cells compact) groups
        // rays that walk the same nodes; other lights by light and a 4 x 4 grid of the direction
        // sample u2
        if (light.type == MCRT_DIRECTIONAL_LIGHT)
            key = (uint32_t)min((int)(u1.y * 64.0f), 63) * 64u + (uint32_t)min((int)(u1.x * 64.0f), 63);
        else
            key = 4096u + (((uint32_t)chosen * 16u + (uint32_t)min((int)(u2.y * 4.0f), 3) * 4u +
                            (uint32_t)min((int)(u2.x * 4.0f), 3)) & 1023u);
        BVertex lv = createLightVertex(chosen, le.origin, le.normal, le.Le, le.pdfPos * lightPdf, light.flags);
        lv.pdfPos = le.pdfPos;
        if (b.depth0Const) {   // planes 4-5 (sdpdu|uv.x, sdpdv|uv.y) of a light vertex are always zero
            vplane(b.lightV, 0, 0, NB)[pix] = make_float4(lv.fr.p.x, lv.fr.p.y, lv.fr.p.z, lv.traceErrorOffset);
            vplane(b.lightV, 0, 1, NB)[pix] = make_float4(lv.fr.gn.x, lv.fr.gn.y, lv.fr.gn.z, lv.pdfFwd);
            vplane(b.lightV, 0, 2, NB)[pix] = make_float4(lv.fr.sn.x, lv.fr.sn.y, lv.fr.sn.z, lv.pdfRev);
            vplane(b.lightV, 0, 3, NB)[pix] = make_float4(lv.wo.x, lv.wo.y, lv.wo.z, lv.pdfPos);
            vplane(b.lightV, 0, 6, NB)[pix] = make_float4(lv.throughput.x, lv.throughput.y, lv.throughput.z, 0.0f);
            *reinterpret_cast<int4*>(&vplane(b.lightV, 0, 7, NB)[pix]) =
                make_int4(lv.type, lv.flags, lv.lightIdx, lv.materialIdx);
        } else {
            storeVertex(b.lightV, 0, pix, NB, lv);
        }
        lo = le.origin;
        ld = le.dir;
        lt = cl_div(le.Le * absDot(le.normal, le.dir), (lightPdf * le.pdfPos * le.pdfDir));
        lightPdfDir = le.pdfDir;
    }
    // slot = the lane's place in the tile walk, so both queues keep tile order (a lane outside the
    // image queues a harmless ray with tag -1, skipped by k_bdpt_vertex)
    if (tile < f.numTiles) {
        const int slot = tileAll * 64 + lane;
        const f3 up = f3{0.0f, 1.0f, 0.0f};
        pushRay(camQ, slot, camPos, valid ? 2 * pix : -1, valid ? camDir : up, camPdf, splat3(1.0f));
        pushRay(lightQ, slot, lo, valid ? 2 * pix + 1 : -1, valid ? ld : up, lightPdfDir, lt);
        if (b.lightKey) {
            b.lightKey[slot] = key;
            b.lightSlot[slot] = (uint32_t)slot;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) camQ.count[0] = lightQ.count[0] = f.numTiles * f.batch * 64;
}

// GenerateSecondaryVertices (BDPT.cl:317-458) for every queued subpath ray at depth d.
// Sort key of a bounce ray (BDPT_BOUNCE_KEY_BITS = 16, the same two 8-bit radix passes as 13): direction
// octant, then a 32 x 8 x 32 grid cell of its origin over the scene bounds (y is up), so a wave of
// the sorted queue holds rays that leave one region in one octant: they share nodes and take the
// octant-specialised loop.
MCRT_DEV uint32_t bounceKey(const BdptArgs& b, f3 o, f3 d) {
    const uint32_t oct = (__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 31) << 1) |
                         ((__float_as_uint(d.z) >> 31) << 2);
    const int cx = min(max((int)((o.x - b.keyLo[0]) * b.keyScale[0]), 0), 31);
    const int cy = min(max((int)((o.y - b.keyLo[1]) * b.keyScale[1]), 0), 7);
    const int cz = min(max((int)((o.z - b.keyLo[2]) * b.keyScale[2]), 0), 31);
    return (oct << 13) | (uint32_t)((cx << 8) | (cy << 5) | cz);
}

// (connectOne below; the vertex launch runs the light-tracing strategy of each light vertex it makes)
struct WaveStage;
struct LightPre {   // a light vertex in registers (with its material properties) and its predecessor
    BVertex lv;
    BVertexPos qsPrev;
};
struct ConnOut {   // a strategy's connection ray, appended by the caller (the vertex launch: per workgroup)
    bool push;
    f3 o, d, L;
    float t;
    int code;
};
template <int CLS>
MCRT_DEV void connectOne(const SceneArgs& s, const FrameArgs& f, const BdptArgs& b, const mcrt_camera* camp,
                         const BdptQueue& qOut, int t, int sI, int k, int x, int y, bool valid,
                         WaveStage* ws = nullptr, const LightPre* lpre = nullptr, ConnOut* cout = nullptr);
MCRT_DEV void pushConn(const BdptQueue& q, int slot, f3 o, float tmax, f3 d, int code, f3 c);
enum { CONN_EMIT = 0, CONN_LIGHT = 1, CONN_NEE = 2, CONN_GENERAL = 3 };

// FINAL: the launch of depth D + 1, whose queue holds camera rays only and whose vertices all end
// their subpath -- no BSDF sampling, so its instantiation carries far fewer registers.
template <bool FINAL>
__global__ __launch_bounds__(BDPT_BLOCK) void k_bdpt_vertex(SceneArgs s, FrameArgs f, BdptArgs b, int depth,
                                                            BdptQueue qIn, const float4* __restrict__ hits,
                                                            BdptQueue qOut) {
    const int n = *qIn.count;
    __shared__ int ldsWave[BDPT_BLOCK / 64 + 1];
    if ((int)blockIdx.x * BDPT_BLOCK >= n) return;
    // (queue = slot order: walking the light-start rays in their sorted order here made this launch
    // 37 % slower for 1 % on the next traversal -- its plane writes follow the pixel order;
    // profiles/r04/ab/README.txt)
    const int i = xcdRemap(blockIdx.x, (n + BDPT_BLOCK - 1) / BDPT_BLOCK) * BDPT_BLOCK + threadIdx.x;
    const int N = (int)(f.W * f.H) * f.batch;   // plane stride (NB)
    const int D = f.maxDepth;
    bool push = false;
    f3 no = splat3(0.0f), nd = splat3(0.0f), ntp = splat3(0.0f);
    float nPdf = 0.0f;
    int tag = 0;
    ConnOut lightRay;   // this light vertex's t = 1 connection ray (appended after the bounce ray)
    lightRay.push = false;
    const float4 O = i < n ? qIn.o[i] : make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
    tag = __float_as_int(O.w);
    if (tag >= 0) {   // tag -1: a start-queue slot outside the image
        const float4 Dd = qIn.d[i], Tp = qIn.t[i];
        const int pix = tag >> 1;   // path k * (W*H) + pixel
        const int kf = pix / (int)(f.W * f.H), px = pix - kf * (int)(f.W * f.H);
        const bool isCamera = (tag & 1) == 0;
        float4* V = isCamera ? b.camV : b.lightV;
        const float4 hit = hits[i];
        const int shapeIdx = __float_as_int(hit.z), primIdx = __float_as_int(hit.w);
        mcrt_shape shp;
        if (shapeIdx >= 0) shp = tableEntry(s.shapes, shapeIdx);
        if (shapeIdx >= 0 && shp.materialId != -1) {
            (isCamera ? b.camCount : b.lightCount)[pix] = depth + 1;
            const f3 rayD = ld3(Dd);
            BVertex cur;
            cur.fr = computeSurfaceInteraction(s, shp, shapeIdx, primIdx, f2{hit.x, hit.y});
            cur.wo = -rayD;
            const bool isBackfacing = cl_dot(cur.fr.gn, cur.wo) < 0.0f;
            cur.traceErrorOffset = isBackfacing ? -RT_TRACE_OFFSET_F : RT_TRACE_OFFSET_F;
            const int materialIdx = shp.materialId;
            const mcrt_material mat = tableEntry(s.materials, materialIdx);
            if (mat.uber_normalMapId != -1) applyNormalMapping(s, mat.uber_normalMapId, cur.fr);
            Uber um;
            bool nonDelta = false;   // hasMaterialNonDeltaComponents, from uberProps' texture reads
            if (mat.type == 0) {
                um = uberProps(s, mat, cur.fr.uv, TexLod{{0, 0}, {0, 0}, false}, &nonDelta);
            } else {
                um.Kd = um.Ks = um.Kr = um.opacity = splat3(0.0f);
                um.Kt = f4{0.0f, 0.0f, 0.0f, 0.0f};
                um.roughness = f2{0.0f, 0.0f};
                um.eta = 0.0f;
            }
            // the material planes are read only by connection strategies that fetch this vertex: none
            // fetches a camera vertex of depth D + 1, nor -- with the light-tracing strategies evaluated
            // here -- a light vertex of depth D (a (t >= 2, s = D + 1) strategy would exceed the depth)
            if (!FINAL && !(b.lightInVertex && !isCamera && depth == D)) storeUber(V, depth, pix, N, um, mat.type);
            const int mode = isCamera ? TRANSPORT_MODE_RADIANCE : TRANSPORT_MODE_IMPORTANCE;
            const BVertexPos prev = loadVertexPos(V, depth - 1, pix, N);
            float pdfFwd = Dd.w;
            f3 throughput = ld3(Tp);
            // setSurfaceVertex (BDPT.cl:204-213)
            cur.throughput = throughput;
            cur.type = RT_BDPT_SURFACE_VERTEX;
            cur.materialIdx = materialIdx;
            cur.flags = 0;
            cur.pdfRev = 0.0f;
            cur.pdfPos = 0.0f;
            cur.pdfFwd = convertVertexDensity(pdfFwd, prev.p, posOf(cur));
            cur.lightIdx = shp.lightID;
            // infinite-light correction of the first light-subpath vertex (BDPT.cl:383-393)
            if (!isCamera && depth == 1 && isInfinite(prev.flags)) {
                const float prevPdfPos = vplane(V, 0, 3, N)[pix].w;
                cur.pdfFwd = prevPdfPos;
                if (isVertexOnSurface(cur.fr.gn)) cur.pdfFwd *= absDot(rayD, cur.fr.gn);
                storePdfFwd(V, 0, pix, N, 0.0f);
            }
            if (FINAL || depth == D + (isCamera ? 1 : 0)) {   // subpath complete (BDPT.cl:395-403)
                if (nonDelta) cur.flags |= VF_CONNECTIBLE;
                storeVertex(V, depth, pix, N, cur);
            } else {
                Sampler sampler = makeSampler(f.sampler, (uint32_t)px, f.frame + kf, depth + (D + 1) * (isCamera ? 1 : 0),
                                              f.W, f.H, s.sobol);
                const f3 wo = cur.wo;
                const f2 bsdfSample = getSample2D(sampler);
                f3 wi = splat3(0.0f), fv = splat3(0.0f);
                int sampledType = 0, numNonDelta = 0;
                if (mat.type == 0)
                    fv = sampleUberBSDF(um, cur.fr, bsdfSample, wo, &wi, &pdfFwd, &sampledType, mode, &numNonDelta);
                if (numNonDelta > 0) cur.flags |= VF_CONNECTIBLE;
                if (isBlack(fv) || isNearZero(pdfFwd)) {
                    storeVertex(V, depth, pix, N, cur);
                } else {
                    throughput = throughput * cl_div(fv * absDot(wi, cur.fr.sn), pdfFwd);
                    float pdfRev;
                    if ((sampledType & BSDF_SPECULAR) != 0) {
                        cur.flags |= VF_DELTA;
                        pdfFwd = 0.0f;
                        pdfRev = 0.0f;
                    } else {
                        pdfRev = mat.type == 0 ? evaluateUberBSDF_Pdf(um, cur.fr, wi, wo) : 0.0f;
                    }
                    float off = cur.traceErrorOffset;
                    if ((sampledType & BSDF_TRANSMISSION) != 0 && cl_dot(cur.fr.gn, wi) * cl_sign(off) < 0.0f) off *= -1.0f;
                    no = cur.fr.p + cur.fr.gn * off;
                    nd = wi;
                    throughput *= shadingNormalCorrection(cur.fr, wo, wi, mode);
                    storePdfRev(V, depth - 1, pix, N, convertVertexDensity(pdfRev, cur.fr.p, prev));
                    storeVertex(V, depth, pix, N, cur);
                    ntp = throughput;
                    nPdf = pdfFwd;
                    push = true;
                }
            }
            // the light-tracing strategy (t = 1, s = depth + 1) of this light vertex, from the registers
            // that just stored it (PrepareConnections + ConnectVertices for t = 1, BDPT.cl:460-913): every
            // input is final here -- the vertex itself, its predecessor, the pdfs below it (earlier
            // launches) -- and nothing it reads changes later, so it equals the connection launch's
            if (!FINAL && !isCamera && b.lightInVertex) {
                LightPre lp;
                lp.lv = cur;
                lp.lv.um = um;
                lp.lv.umType = mat.type;
                lp.lv.hasUm = true;
                lp.lv.planes = V;
                lp.lv.depth = depth;
                lp.qsPrev = prev;
                const BdptQueue cq{b.connCount, b.connO, b.connD, b.connL};
                connectOne<CONN_LIGHT>(s, f, b, b.cams, cq, 1, depth + 1, kf, px % (int)f.W, px / (int)f.W, true,
                                       nullptr, &lp, &lightRay);
            }
        }
    }
    // (queue order = the block's ray order: grouping the next rays by direction as the PT first
    // shading does made this kernel 11 % slower -- its plane reads and writes follow the queue --
    // for 1 % on k_extend; profiles/r04/ab/README.txt)
    if (FINAL) return;
    const int slot = blockAppend<BDPT_BLOCK / 64>(qOut.count, push, ldsWave);
    if (push) {
        pushRay(qOut, slot, no, tag, nd, nPdf, ntp);
        if (b.extKey) {   // the traversal walks the queue sorted by this key (render_bdpt)
            b.extKey[slot] = bounceKey(b, no, nd);
            b.extSlot[slot] = (uint32_t)slot;
        }
    }
    // the light-tracing connection rays: one append per workgroup (a per-wave append on the queue's
    // one counter serialises across the XCDs)
    if (b.lightInVertex) {
        const int cs = blockAppend<BDPT_BLOCK / 64>(b.connCount, lightRay.push, ldsWave);
        if (lightRay.push)
            pushConn(BdptQueue{b.connCount, b.connO, b.connD, b.connL}, cs, lightRay.o, lightRay.t, lightRay.d,
                     lightRay.code, lightRay.L);
    }
}

// Connection-ray record (3 float4): (o.xyz, tmax), (d.xyz, code), (c.xyz, 0) where code >= 0 is an
// own-strategy slot index (slot * N + pix) and code < 0 a splat target pixel (~code).
MCRT_DEV void pushConn(const BdptQueue& q, int slot, f3 o, float tmax, f3 d, int code, f3 c) {
    q.o[slot] = make_float4(o.x, o.y, o.z, tmax);
    q.d[slot] = make_float4(d.x, d.y, d.z, __int_as_float(code));
    q.t[slot] = make_float4(c.x, c.y, c.z, 0.0f);
}

// PrepareConnections (BDPT.cl:460-646) + the MIS weights of ConnectVertices (BDPT.cl:739-876),
// one thread per (pixel, strategy).  The reference walks a pixel's strategies serially in (t, s)
// order; only two things tie them together, and both are restated per strategy here:
//   * the sampler: each s = 1 strategy whose camera vertex is live and connectible draws 3 values
//     (light choice + 2D) from the pixel's connection stream, so strategy (t, 1) starts that stream
//     3 draws later per such earlier strategy (t' < t, counted from the camera vertices' flags);
//   * the stale sampled-light slot (BDPT.cl:585-586): strategy (t, 1) alone reads and rewrites
//     slot t - 2, so its frame-to-frame read-before-write order is kept.
// Strategies are split into four classes, one launch each, so every kernel carries only its own
// registers: EMIT (s = 0), LIGHT (t = 1, light tracing), NEE (s = 1), GENERAL (t, s >= 2).  LIGHT
// runs in k_bdpt_vertex by default, from the registers that store its light vertex (lpre;
// BdptArgs::lightInVertex, profiles/r06/ab/bdpt_connect/README.txt); moving (2, 2) into the depth-1
// light launch as well measured slower there (its own instantiation at 150 VGPRs).  A wave
// holds one strategy of one 8x8 tile for all the call's frames (wave-uniform branches); the waves
// of a tile are adjacent, so its vertex planes are re-read from L2.  Own strategies (t >= 2) write
// their slot (zero when absent, not connectible or contributing nothing); strategies with a
// non-zero weighted contribution that need visibility are queued.  (One workgroup per tile running
// every strategy of its pixels, so each path's planes come from HBM once, measured slower: 1.02
// against 0.74 ms per frame -- all its waves carry the heaviest class's registers, 2-3 waves per
// SIMD, where the light classes run at 4-8; tools/experiments/bdpt_connect_tile_mispre.patch.)
MCRT_DEV int ownSlotOf(int t, int sI, int D) {   // index among the t >= 2 strategies in (t, s) order
    int k = sI;
    for (int u = 2; u < t; ++u) k += D + 3 - u;
    return k;
}
template <int CLS>
MCRT_DEV void strategyOf(int k, int D, int& t, int& sI) {
    if (CLS == CONN_EMIT) { t = k + 2; sI = 0; }
    else if (CLS == CONN_LIGHT) { t = 1; sI = k + 2; }
    else if (CLS == CONN_NEE) { t = k + 2; sI = 1; }
    else {
        t = 2;
        sI = 2;
        for (int u = 2; u <= D; ++u) {
            const int n = D + 1 - u;   // s = 2 .. D + 2 - u
            if (k < n) { t = u; sI = k + 2; break; }
            k -= n;
        }
    }
}

// Connection rays staged in LDS, a segment per wave (no wave waits for another): one global append
// per CONN_STAGE rays of a wave's frame loop instead of one per workgroup, frame and strategy (an
// append to the queue's one counter sits on the appending wave's critical path: with one per wave
// and strategy the connection launches took 1.78 ms per frame; staged, 0.836 against the
// workgroup appends' 0.85, profiles/r06/ab/bdpt_connect).
#define CONN_STAGE 128
struct WaveStage {
    float4 *o, *d, *t;   // this wave's LDS segment
    int n;               // staged rays (wave-uniform)
};
MCRT_DEV void flushStage(WaveStage& ws, const BdptQueue& q) {
    if (ws.n == 0) return;
    const int lane = threadIdx.x & 63;
    __builtin_amdgcn_wave_barrier();
    int base = 0;
    if (lane == 0) base = atomicAdd(q.count, ws.n);
    base = __shfl(base, 0);
    for (int i = lane; i < ws.n; i += 64) {
        q.o[base + i] = ws.o[i];
        q.d[base + i] = ws.d[i];
        q.t[base + i] = ws.t[i];
    }
    __builtin_amdgcn_wave_barrier();
    ws.n = 0;
}

// One strategy (t, sI) of class CLS for batch frame k of the lane's pixel (x, y): PrepareConnections
// + the MIS weight of ConnectVertices, the own-strategy slot, and the connection ray -- appended to
// the wave's LDS stage (ws) or with one global atomic per wave (the queue's order only decides the
// order of the splats' float atomics).
template <int CLS>
MCRT_DEV void connectOne(const SceneArgs& s, const FrameArgs& f, const BdptArgs& b, const mcrt_camera* camp,
                         const BdptQueue& qOut, int t, int sI, int k, int x, int y, bool valid,
                         WaveStage* ws, const LightPre* lpre, ConnOut* cout) {
    const int N0 = (int)(f.W * f.H);
    const int N = N0 * f.batch;   // plane stride
    const int D = f.maxDepth;
    const int px = y * (int)f.W + x;
    const int pix = k * N0 + px;   // the path (plane index)
    const mcrt_camera& cam = camp[k];
    const int camCount = valid ? b.camCount[pix] : 0;
    const int lightCount = valid ? b.lightCount[pix] : 0;
    const bool live = valid && t <= camCount && sI <= lightCount;
    bool push = false, needRay = false;
    f3 L = splat3(0.0f), rayO = splat3(0.0f), rayD = splat3(0.0f);
    float rayT = 0.0f;
    int code = 0;
    if (live) {
        // the strategy's camera / light vertex WITH its material properties (loadVertexU) and the
        // MIS walk's previous vertices in one round trip: the kernel is bound by its chains of
        // dependent fetches (the BSDF and pdf evaluations re-read the material planes otherwise;
        // 0.85 -> 0.74 ms per frame).  Fetching them before the subpath lengths are known, or the
        // MIS walks' pdf planes with them as well, measured slower (lanes of absent strategies
        // fetch for nothing; profiles/r06/ab/bdpt_connect)
        BVertex cv, lv, samp;   // samp: the sampled vertex of a t = 1 / s = 1 strategy (pt / qs in the MIS)
        BVertexPos ptPrev, qsPrev;
        if (CLS != CONN_LIGHT && CLS != CONN_EMIT) {
            cv = loadVertexU(b.camV, t - 1, pix, N);
            ptPrev = loadVertexPos(b.camV, t - 2, pix, N);
        }
        if (CLS == CONN_LIGHT && lpre) {   // the vertex launch's registers
            lv = lpre->lv;
            qsPrev = lpre->qsPrev;
        } else if (CLS == CONN_LIGHT || CLS == CONN_GENERAL) {
            lv = loadVertexU(b.lightV, sI - 1, pix, N);
            qsPrev = loadVertexPos(b.lightV, sI - 2, pix, N);
        }
        if (CLS == CONN_EMIT) {
            // ConnectVertices (BDPT.cl:723-731): emission of a camera vertex that is a light.  Only
            // the type word is read first: for the (many) vertices that are not lights the strategy
            // contributes nothing and the other 7 planes are never needed.
            const int4 h = *reinterpret_cast<const int4*>(&vplane(b.camV, t - 1, 7, N)[pix]);
            if (h.x == RT_BDPT_LIGHT_VERTEX || h.z != -1) {
                cv = loadVertex(b.camV, t - 1, pix, N);
                const f3 Le = evalLightLe(s.lights[cv.lightIdx], cv.fr.gn, cv.wo);
                L = Le * cv.throughput;
            }
        } else if (CLS == CONN_LIGHT) {
            if (isConnectible(lv.flags)) {
                // samplePinholeCameraWi (cameras.cl:61-69)
                f3 wi = ld3(cam.pos) - lv.fr.p;
                const float dist = cl_length(wi);
                wi = cl_div(wi, dist);
                const float pdf = cl_div((dist * dist), absDot(ld3(cam.direction), wi));
                f2 nip = f2{cl_div((float)x, (float)f.W), cl_div((float)y, (float)f.H)};
                const float imp = evalPinholeCameraWe(cam, ld3(cam.pos), -wi, &nip);
                const f3 importance = splat3(imp);
                if (pdf > 0.0f && isNotBlack(importance)) {
                    samp = createCameraVertex(ld3(cam.pos), cl_div(importance, pdf));
                    int ix = (int)floorf(nip.x * f.W + 0.5f), iy = (int)floorf(nip.y * f.H + 0.5f);
                    ix = min(max(ix, 0), (int)f.W - 1);
                    iy = min(max(iy, 0), (int)f.H - 1);
                    code = ~(k * N0 + ix + iy * (int)f.W);   // frame k's splat plane
                    L = lv.throughput * samp.throughput * evalVertex_f(lv, pix, N, samp.fr.p, TRANSPORT_MODE_IMPORTANCE);
                    if (isVertexOnSurface(lv.fr.gn)) L *= absDot(wi, lv.fr.sn);
                    rayO = lv.fr.p + lv.fr.gn * lv.traceErrorOffset;
                    rayT = cl_distance(rayO, ld3(cam.pos));
                    rayD = cl_div(ld3(cam.pos) - rayO, rayT);
                    needRay = true;
                }
            }
        } else if (CLS == CONN_NEE) {
            if (isConnectible(cv.flags)) {
                // the pixel's connection stream, past the draws of the earlier s = 1 strategies
                Sampler sampler = makeSampler(f.sampler, (uint32_t)px, f.frame + k, (D + 1) + (D + 2), f.W, f.H, s.sobol);
                int skip = 0;
                for (int u = 2; u < t; ++u)
                    if (u <= camCount && isConnectible(reinterpret_cast<const int4*>(&vplane(b.camV, u - 1, 7, N)[pix])->y))
                        skip += 3;
                if (sampler.mats) sampler.dim += (uint32_t)skip;
                else
                    for (int u = 0; u < skip; ++u) xorshift(sampler.idx);
                const int chosen = min((int)floorf(getSample1D(sampler) * s.numLights), s.numLights - 1);
                const mcrt_light light = s.lights[chosen];
                const float lightPdf = light.choicePdf;
                const f2 u = getSample2D(sampler);
                const LightSample ls = sampleLightLi(s, light, cv.fr, cv.traceErrorOffset, u);
                if (isNotNearZero(ls.pdf) && isNotBlack(ls.Li)) {
                    // the reference evaluates pdfFwd on the PREVIOUS content of the sampled
                    // vertex slot before overwriting it (BDPT.cl:585-586)
                    float4* stale = b.sampLight + (size_t)(t - 2) * N0 + px;   // per pixel, across frames
                    const float4 st = *stale;
                    const int stBits = __float_as_int(st.w);
                    const int stFlags = stBits >> 16, stLight = (int)(short)(stBits & 0xffff);
                    const float pdfFwdS = evalVertexPdfLightOrigin(s, ld3(st), splat3(0.0f), stFlags, stLight, cv.fr.p);
                    samp = createLightVertex(chosen, ls.lightPos, ls.lightNormal, cl_div(ls.Li, (lightPdf * ls.pdf)),
                                             pdfFwdS, light.flags);
                    *stale = make_float4(samp.fr.p.x, samp.fr.p.y, samp.fr.p.z,
                                         __int_as_float((samp.flags << 16) | (chosen & 0xffff)));
                    const f3 fm = evaluateMaterialV(cv, pix, N, cv.wo, ls.wi, TRANSPORT_MODE_RADIANCE);
                    L = cv.throughput * samp.throughput * fm;
                    if (isVertexOnSurface(cv.fr.gn)) L *= absDot(ls.wi, cv.fr.sn);
                    if (ls.shadowSet) {
                        rayO = ls.shadowO;
                        rayT = ls.shadowT;
                        rayD = ls.wi;
                        needRay = true;
                    }
                }
            }
        } else {
            if (isConnectible(cv.flags) && isConnectible(lv.flags)) {
                const f3 lvf = evalVertex_f(lv, pix, N, cv.fr.p, TRANSPORT_MODE_IMPORTANCE);
                const f3 cvf = evalVertex_f(cv, pix, N, lv.fr.p, TRANSPORT_MODE_RADIANCE);
                const f3 lp = lv.fr.p + lv.fr.gn * lv.traceErrorOffset;
                const f3 cp = cv.fr.p + cv.fr.gn * cv.traceErrorOffset;
                f3 w = cp - lp;
                const float sqDist = cl_dot(w, w);
                const float dist = cl_sqrt(sqDist);
                w = cl_div(w, dist);
                if (isNotNearZero(sqDist)) {
                    const float g = cl_div(absDot(cv.fr.sn, w) * absDot(lv.fr.sn, w), sqDist);
                    L = lv.throughput * cv.throughput * lvf * cvf * g;
                }
                if (isNotBlack(L)) {
                    rayO = lp;
                    rayT = dist;
                    rayD = w;
                    needRay = true;
                }
            }
        }
        // MIS weight (BDPT.cl:739-876), independent of visibility
        float misWeight = 1.0f;
        if (isBlack(L)) {
            misWeight = 0.0f;
        } else if (sI + t != 2) {
            // pt = camera vertex t-1 (or the sampled camera vertex), qs = light vertex s-1 (or the
            // sampled light vertex), with their delta flags cleared and pdfRev re-evaluated
            BVertex pt = CLS == CONN_LIGHT ? samp : cv;
            BVertex qs;
            if (CLS == CONN_NEE) qs = samp;
            else if (CLS == CONN_LIGHT || CLS == CONN_GENERAL) qs = lv;
            if (CLS == CONN_EMIT) ptPrev = loadVertexPos(b.camV, t - 2, pix, N);
            pt.flags &= ~VF_DELTA;
            if (CLS != CONN_EMIT) qs.flags &= ~VF_DELTA;
            const float ptRev = CLS != CONN_EMIT ? evalVertexPdf(s, cam, qs, pix, N, sI > 1, qsPrev.p, posOf(pt))
                                                 : evalVertexPdfLightOrigin(s, pt.fr.p, pt.fr.gn, pt.flags, pt.lightIdx, ptPrev.p);
            float ptPrevRev = 0.0f, qsRev = 0.0f, qsPrevRev = 0.0f;
            if (CLS != CONN_LIGHT)
                ptPrevRev = CLS != CONN_EMIT ? evalVertexPdf(s, cam, pt, pix, N, true, qs.fr.p, ptPrev)
                                             : evalVertexPdfLight(s, pt.fr.p, pt.fr.gn, pt.flags, pt.lightIdx, ptPrev);
            if (CLS != CONN_EMIT) qsRev = evalVertexPdf(s, cam, pt, pix, N, t > 1, ptPrev.p, posOf(qs));
            if (CLS == CONN_LIGHT || CLS == CONN_GENERAL) qsPrevRev = evalVertexPdf(s, cam, qs, pix, N, true, pt.fr.p, qsPrev);
            float sumRi = 0.0f;
            // camera subpath (BDPT.cl:819-827)
            float ri = 1.0f;
            int flagsHi = pt.flags;   // flags of vertex i (walking down from t-1)
            for (int i = t - 1; i > 0; --i) {
                float rev, fwd;
                int fl, flLo;
                if (i == t - 1) {
                    rev = ptRev;
                    fwd = pt.pdfFwd;
                    fl = pt.flags;
                } else {
                    const float4 pb = vplane(b.camV, i, 1, N)[pix];
                    const float4 pc = vplane(b.camV, i, 2, N)[pix];
                    fwd = pb.w;
                    rev = (i == t - 2) ? ptPrevRev : pc.w;
                    fl = flagsHi;
                }
                flLo = reinterpret_cast<const int4*>(&vplane(b.camV, i - 1, 7, N)[pix])->y;
                ri *= cl_div(remap0(rev), remap0(fwd));
                if (!isDeltaV(fl) && !isDeltaV(flLo)) sumRi += ri;
                flagsHi = flLo;
            }
            // light subpath (BDPT.cl:829-838)
            ri = 1.0f;
            for (int i = sI - 1; i >= 0; --i) {
                float rev, fwd;
                int fl;
                if (i == sI - 1) {
                    rev = qsRev;
                    fwd = qs.pdfFwd;
                    fl = qs.flags;
                } else {
                    const float4 pb = vplane(b.lightV, i, 1, N)[pix];
                    const float4 pc = vplane(b.lightV, i, 2, N)[pix];
                    fwd = pb.w;
                    rev = (i == sI - 2) ? qsPrevRev : pc.w;
                    fl = reinterpret_cast<const int4*>(&vplane(b.lightV, i, 7, N)[pix])->y;
                }
                ri *= cl_div(remap0(rev), remap0(fwd));
                bool deltaLightVertex;
                if (i > 0) {
                    deltaLightVertex = isDeltaV(reinterpret_cast<const int4*>(&vplane(b.lightV, i - 1, 7, N)[pix])->y);
                } else {
                    const int f0 = (sI == 1) ? qs.flags : reinterpret_cast<const int4*>(&vplane(b.lightV, 0, 7, N)[pix])->y;
                    deltaLightVertex = isDeltaLightV(f0);
                }
                if (!isDeltaV(fl) && !deltaLightVertex) sumRi += ri;
            }
            misWeight = cl_div(1.0f, (1.0f + sumRi));
        }
        const f3 c = L * misWeight;
        const bool nonzero = c.x != 0.0f || c.y != 0.0f || c.z != 0.0f;
        if (CLS != CONN_EMIT && nonzero) push = needRay;   // no connection ray = not visible (contributes 0)
        if (CLS != CONN_LIGHT) {
            const int own = ownSlotOf(t, sI, D);
            const f3 o = (CLS == CONN_EMIT || push) ? c : splat3(0.0f);
            b.slots[(size_t)own * N + pix] = make_float4(o.x, o.y, o.z, 0.0f);
            if (push) code = own * N + pix;
        }
        L = c;
    } else if (valid && CLS != CONN_LIGHT) {
        b.slots[(size_t)ownSlotOf(t, sI, D) * N + pix] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // strategy absent
    }
    if (cout) {   // the caller appends
        cout->push = push;
        cout->o = rayO;
        cout->d = rayD;
        cout->L = L;
        cout->t = rayT;
        cout->code = code;
        return;
    }
    if (CLS != CONN_EMIT) {   // emission needs no connection ray (class-uniform: the whole wave)
        const uint64_t m = __ballot(push);
        if (m) {
            const int lane = threadIdx.x & 63, leader = __builtin_ctzll(m), cnt = __popcll(m);
            const int pre = __popcll(m & ((1ull << lane) - 1));
            bool staged = false;
            if (ws) {
                if (ws->n + cnt > CONN_STAGE) flushStage(*ws, qOut);
                if (push) {
                    ws->o[ws->n + pre] = make_float4(rayO.x, rayO.y, rayO.z, rayT);
                    ws->d[ws->n + pre] = make_float4(rayD.x, rayD.y, rayD.z, __int_as_float(code));
                    ws->t[ws->n + pre] = make_float4(L.x, L.y, L.z, 0.0f);
                }
                ws->n += cnt;
                staged = true;
            }
            if (!staged) {
                int at = 0;
                if (lane == leader) at = atomicAdd(qOut.count, cnt);
                at = __shfl(at, leader) + pre;
                if (push) pushConn(qOut, at, rayO, rayT, rayD, code, L);
            }
        }
    }
}

// The four class launches: a wave = (tile, strategy), walking the batch's frames in order (frame
// k's s = 1 strategy reads the sampled-light slot frame k - 1 wrote), strategies fastest, so the
// strategies of one tile run in one workgroup or its neighbours at about the same frame; each class
// kernel carries only its own registers.  Connection rays are staged per wave in LDS.
template <int CLS>
__global__ __launch_bounds__(BDPT_BLOCK) void k_bdpt_connect(SceneArgs s, FrameArgs f, BdptArgs b,
                                                             const mcrt_camera* __restrict__ camp, BdptQueue qOut,
                                                             int numStrat) {
    constexpr int NW = BDPT_BLOCK / 64;
    constexpr int SEG = CLS == CONN_EMIT ? 1 : CONN_STAGE;   // emission strategies queue no rays
    __shared__ float4 so[NW][SEG], sd[NW][SEG], st[NW][SEG];
    const int lane = threadIdx.x & 63;
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int wave = xcdRemap((int)blockIdx.x, (int)gridDim.x) * NW + wv;
    const int tile = wave / numStrat;
    const int si = wave - tile * numStrat;
    int t, sI;
    strategyOf<CLS>(si, f.maxDepth, t, sI);
    int x = 0, y = 0;
    const bool valid = tile < f.numTiles && tilePixel(f, tile, lane, x, y) && s.numLights > 0;
    if (tile >= f.numTiles) return;
    WaveStage ws{so[wv], sd[wv], st[wv], 0};
    for (int k = 0; k < f.batch; ++k)
        connectOne<CLS>(s, f, b, camp, qOut, t, sI, k, x, y, valid, CLS == CONN_EMIT ? nullptr : &ws);
    if (CLS != CONN_EMIT) flushStage(ws, qOut);
}

// Any hit over the connection queue (RR occluded_main semantics): occluded own strategies are
// zeroed in their slot, unoccluded light-tracing strategies splatted (BDPT.cl:888-899).
template <int LAY>
__global__ __launch_bounds__(64) void k_bdpt_vis(TraceCtx c, BdptArgs b, const int* __restrict__ count,
                                                 const float4* __restrict__ sO, const float4* __restrict__ sD,
                                                 const float4* __restrict__ sL) {
    // grid-stride over the queue (a batch's C x N slots would need one spill column per slot)
    __shared__ uint32_t lds[STACK_LDS * 64];
    const int n = *count;
    const int lane = threadIdx.x;
    for (int base = blockIdx.x * 64; base < n; base += gridDim.x * 64) {
        const int i = base + lane;
        if (i >= n) return;
        const float4 o = sO[i], d = sD[i];
        TraceRay r;
        r.o = ld3(o);
        r.d = ld3(d);
        r.tmax = o.w;
        r.mask = -1;
        // occluder hints by origin cell (c.hint when on): the NEE rays to a directional light and the
        // light-tracing rays toward the camera leave one cell nearly parallel
        const bool occluded = shadowOccluded<LAY>(c, r, 0, lds + lane, raySpill(c, blockIdx.x, lane));
        const int code = __float_as_int(d.w);
        bool listIt = false;
        float4 rec = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (code >= 0) {
            if (occluded) b.slots[code] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        } else if (!occluded) {
            const float4 L = sL[i];
            const int target = ~code;
            if (b.splatList) {   // band split, sparse exchange: another rank's row -> the list
                const int y = (target % b.splatN0) / b.splatW;
                listIt = ((y >> 3) / b.splatBpb) % b.splatBands != b.splatBand;
                rec = make_float4(__int_as_float(target), L.x, L.y, L.z);
            }
            if (!listIt) {
                float* dst = reinterpret_cast<float*>(&b.splat[target]);
                atomicAdd(dst + 0, L.x);
                atomicAdd(dst + 1, L.y);
                atomicAdd(dst + 2, L.z);
            }
        }
        // the list's entries: ONE atomic per wave (a per-lane append on one counter serialises in L2)
        const uint64_t m = __ballot(listIt);
        if (m) {
            const int leader = __builtin_ctzll(m);
            int at = 0;
            if (lane == leader) at = atomicAdd(b.splatListCount, __popcll(m));
            at = __shfl(at, leader) + __popcll(m & ((1ull << lane) - 1));
            if (listIt && at < b.splatListCap) b.splatList[at] = rec;   // at most D per path: never full
        }
    }
}

// Own strategies summed in (t, s) order (the reference's per-thread atomicAdd_f order), then the
// splats; radiance = float4(sum, 0) as CopyBuffer (BDPT.cl:916-932), frame k of a batch at
// radiance[k * W*H + pixel].  chunk (band split): this rank's rows of the ranks' summed splats in
// the rank-major layout of k_bdpt_splat_pack (frame k's rows at k * chunkPixels, the rank's local
// 8-row block tb at rows 8 tb .. 8 tb + 7), instead of the rank's own splat planes.
__global__ __launch_bounds__(256) void k_bdpt_gather(FrameArgs f, BdptArgs b, float4* __restrict__ radiance,
                                                     const float* __restrict__ chunk, size_t chunkPixels) {
    const int lane = threadIdx.x & 63;
    const int tileAll = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int tile, k;
    tileFrame(f, tileAll, tile, k);
    int x, y;
    if (tile >= f.numTiles || !tilePixel(f, tile, lane, x, y)) return;
    const int N0 = (int)(f.W * f.H), N = N0 * f.batch;
    const int pix = k * N0 + y * (int)f.W + x;
    float rx = 0.0f, ry = 0.0f, rz = 0.0f;
    for (int j = 0; j < b.ownSlots; ++j) {
        const float4 c = b.slots[(size_t)j * N + pix];
        rx += c.x;
        ry += c.y;
        rz += c.z;
    }
    const int tb = tile / f.tilesX;
    float4 sp;
    if (chunk) {   // MCRT_SPLAT_CHANNELS floats per pixel
        const float* c = chunk + 3 * ((size_t)k * chunkPixels + (size_t)(tb * 8 + (lane >> 3)) * f.W + x);
        sp = make_float4(c[0], c[1], c[2], 0.0f);
    } else {
        sp = b.splat[pix];
    }
    radiance[pix] = make_float4(rx + sp.x, ry + sp.y, rz + sp.z, 0.0f);
}

// Band split: the splat planes (W x H per batch frame, any pixel) in rank-major order -- chunk r
// (batch x chunkPixels pixels of 3 floats, r g b: the reference's splat buffer, BDPT.cl:654-669;
// the exchange moves 12 B per pixel, not the splat plane's 16) holds, frame after frame, the rows of rank r's bands, its local 8-row
// block tb (tilePixel's numbering) at rows 8 tb .. 8 tb + 7 -- so ONE reduce-scatter hands every
// rank the summed splats of exactly its own rows (mcrt.dist.exchange_splats).  Rows past a rank's
// last block stay zero (memset).
__global__ __launch_bounds__(256) void k_bdpt_splat_pack(int W, int H, int batch, int bpb, int numBands,
                                                         size_t chunkPixels, const float4* __restrict__ splat,
                                                         float* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const size_t N0 = (size_t)W * H;
    if (i >= N0 * batch) return;
    const int k = (int)(i / N0);
    const size_t q = i - (size_t)k * N0;
    const int y = (int)(q / W), x = (int)(q - (size_t)y * W);
    const int gb = y >> 3;
    const int r = (gb / bpb) % numBands, tb = (gb / (bpb * numBands)) * bpb + gb % bpb;
    const float4 v = splat[i];
    float* o = out + 3 * ((size_t)r * batch * chunkPixels + (size_t)k * chunkPixels + (size_t)(tb * 8 + (y & 7)) * W + x);
    o[0] = v.x;
    o[1] = v.y;
    o[2] = v.z;
}

// Sparse splat exchange (band split): the list's records per owner rank, then grouped by owner
// (any order inside a group: the owner adds them with float atomics, like the reference's splats)
__global__ __launch_bounds__(256) void k_splat_hist(BdptArgs b, int* __restrict__ hist) {
    const int n = min(*b.splatListCount, b.splatListCap);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const int y = (__float_as_int(b.splatList[i].x) % b.splatN0) / b.splatW;
        atomicAdd(&hist[((y >> 3) / b.splatBpb) % b.splatBands], 1);
    }
}
__global__ __launch_bounds__(256) void k_splat_group(BdptArgs b, mcrt::SplatOffsets off, int* __restrict__ cursor,
                                                     float4* __restrict__ dst) {
    const int n = min(*b.splatListCount, b.splatListCap);
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const float4 r = b.splatList[i];
        const int y = (__float_as_int(r.x) % b.splatN0) / b.splatW;
        const int o = ((y >> 3) / b.splatBpb) % b.splatBands;
        dst[off.off[o] + atomicAdd(&cursor[o], 1)] = r;
    }
}
// received records (targets in this rank's rows) into its splat plane
__global__ __launch_bounds__(256) void k_splat_unpack(const float4* __restrict__ recv, int n, float4* __restrict__ splat) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 r = recv[i];
    float* d = reinterpret_cast<float*>(&splat[__float_as_int(r.x)]);
    atomicAdd(d + 0, r.y);
    atomicAdd(d + 1, r.z);
    atomicAdd(d + 2, r.w);
}

// Splats that land outside the rank's bands (multi-GPU band split): added by the rank that owns
// the pixel after the all-reduce of the splat buffers (mcrt_capi.cpp).
__global__ __launch_bounds__(256) void k_bdpt_clear_splat(int n, float4* __restrict__ splat) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) splat[i] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

namespace mcrt {
// The light-start queue in cell order (k_bdpt_start's keys): rocPRIM radix sort of (key, slot)
// over the key's 13 bits; perm[j] = the slot traced j-th.  The queue itself stays in slot (tile)
// order for the vertex launch; only the traversal walks it sorted (k_extend_pair).
size_t bdpt_light_sort_temp_bytes(int n) {
    size_t bytes = 0;
    uint32_t* k = nullptr;
    // a size query: no launch, and a failure leaves bytes = 0 (the caller's allocation then fails loudly)
    (void)rocprim::radix_sort_pairs(nullptr, bytes, k, k, k, k, (size_t)n, 0, BDPT_BOUNCE_KEY_BITS, (hipStream_t)0);
    return bytes;
}
hipError_t bdpt_light_sort(uint32_t* keys, uint32_t* keys2, uint32_t* slots, uint32_t* perm, int n, void* tmp,
                           size_t tmpBytes, hipStream_t st, int bits) {
    return rocprim::radix_sort_pairs(tmp, tmpBytes, keys, keys2, slots, perm, (size_t)n, 0, bits, st);
}

void launch_bdpt_start(const SceneArgs& s, const FrameArgs& f, const BdptArgs& b, const mcrt_camera* cam,
                       const BdptQueue& camQ, const BdptQueue& lightQ, hipStream_t st) {
    const int blocks = (f.numTiles * f.batch * 64 + BDPT_BLOCK - 1) / BDPT_BLOCK;
    hipLaunchKernelGGL(k_bdpt_start, dim3(blocks), dim3(BDPT_BLOCK), 0, st, s, f, b, cam, camQ, lightQ);
}
void launch_bdpt_vertex(const SceneArgs& s, const FrameArgs& f, const BdptArgs& b, int depth, const BdptQueue& qIn,
                        const float4* hits, const BdptQueue& qOut, int maxCount, hipStream_t st) {
    const int blocks = (maxCount + BDPT_BLOCK - 1) / BDPT_BLOCK;
    // depth D + 1 (the round after the light subpaths ended at depth D): camera vertices that all end
    const bool fin = depth >= 2 && depth == f.maxDepth + 1;
    hipLaunchKernelGGL(fin ? k_bdpt_vertex<true> : k_bdpt_vertex<false>, dim3(blocks > 0 ? blocks : 1),
                       dim3(BDPT_BLOCK), 0, st, s, f, b, depth, qIn, hits, qOut);
}
void launch_bdpt_connect(const SceneArgs& s, const FrameArgs& f, const BdptArgs& b, const mcrt_camera* cam,
                         const BdptQueue& q, hipStream_t st) {
    // strategies per class for maxDepth D (C = (D+2)(D+3)/2 - 2 in all): s = 0: D+1, t = 1: D,
    // s = 1: D, t, s >= 2: the rest
    const int D = f.maxDepth;
    const int C = (D + 2) * (D + 3) / 2 - 2;
    const int counts[4] = {D + 1, D, D, C - 3 * D - 1};
    void (*kern[4])(SceneArgs, FrameArgs, BdptArgs, const mcrt_camera*, BdptQueue, int) = {
        k_bdpt_connect<CONN_EMIT>, k_bdpt_connect<CONN_LIGHT>, k_bdpt_connect<CONN_NEE>, k_bdpt_connect<CONN_GENERAL>};
    for (int c = 0; c < 4; ++c) {
        if (counts[c] <= 0 || (c == CONN_LIGHT && b.lightInVertex)) continue;   // (done by the vertex launches)
        const int64_t waves = (int64_t)f.numTiles * counts[c];
        const int blocks = (int)((waves * 64 + BDPT_BLOCK - 1) / BDPT_BLOCK);
        hipLaunchKernelGGL(kern[c], dim3(blocks), dim3(BDPT_BLOCK), 0, st, s, f, b, cam, q, counts[c]);
    }
}
void launch_bdpt_vis(const TraceCtx& c, const BdptArgs& b, const BdptQueue& q, int maxCount, hipStream_t st) {
    const int blocks = std::max(1, std::min((maxCount + 63) / 64, BDPT_VIS_MAX_WAVES));
    hipLaunchKernelGGL(pickLayout(c, k_bdpt_vis<LAY_TWO_LEVEL>, k_bdpt_vis<LAY_QUANT>, k_bdpt_vis<LAY_PLAIN>), dim3(blocks),
                       dim3(64), 0, st, c, b, q.count,
                       q.o, q.d, q.t);
}
void launch_bdpt_gather(const FrameArgs& f, const BdptArgs& b, float4* radiance, const float* chunk,
                        size_t chunkPixels, hipStream_t st) {
    const int blocks = (f.numTiles * f.batch * 64 + 255) / 256;
    hipLaunchKernelGGL(k_bdpt_gather, dim3(blocks), dim3(256), 0, st, f, b, radiance, chunk, chunkPixels);
}
void launch_bdpt_splat_pack(const FrameArgs& f, size_t chunkPixels, const float4* splat, float* out, hipStream_t st) {
    const size_t n = (size_t)f.W * f.H * f.batch;
    hipLaunchKernelGGL(k_bdpt_splat_pack, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, (int)f.W, (int)f.H,
                       f.batch, f.bandRows >> 3, f.numBands, chunkPixels, splat, out);
}
void launch_splat_hist(const BdptArgs& b, int* hist, hipStream_t st) {
    hipLaunchKernelGGL(k_splat_hist, dim3(1024), dim3(256), 0, st, b, hist);
}
void launch_splat_group(const BdptArgs& b, SplatOffsets off, int* cursor, float4* dst, hipStream_t st) {
    hipLaunchKernelGGL(k_splat_group, dim3(1024), dim3(256), 0, st, b, off, cursor, dst);
}
void launch_splat_unpack(const float4* recv, int n, float4* splat, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_splat_unpack, dim3((n + 255) / 256), dim3(256), 0, st, recv, n, splat);
}
void launch_bdpt_clear_splat(int n, float4* splat, hipStream_t st) {
    hipLaunchKernelGGL(k_bdpt_clear_splat, dim3((n + 255) / 256), dim3(256), 0, st, n, splat);
}
}  // namespace mcrt

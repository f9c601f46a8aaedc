// mcrt_camera.cpp -- host camera setup of the reference, restated in float32 in glm's operation
// order so the RTPinholeCamera is bit-identical to the one the reference host builds:
//   CameraComponent::setPerspective/setViewport/updateViewMatrix (source/engine/camera/
//   CameraComponent.cpp:61-134), ndcToCameraPoint / screenToNDC (:149-165), RTUtil::screenToRay
//   (source/application/PathTracer/raytracing/util/RTUtil.cpp:9-41), the corner rays and camera
//   area of RTPrimaryRaysPass::generatePrimaryRays / RTBDPTPass (RTPrimaryRaysPass.cpp:81-104,
//   RTBDPTPass.cpp:138-166) and the TAA jitter (PathTracingApp.cpp:208-215).
// glm (third_party/glm, GLM_FORCE_LEFT_HANDED, depth -1..1) pieces restated: perspectiveLH,
// mat4 * mat4, mat4 * vec4, inverse(mat4) (detail/func_matrix.inl:297-354), translate, dot,
// cross, normalize = v * (1 / sqrt(dot(v, v))).  Compiled with -ffp-contract=off: no FMA, like
// the reference's /fp:precise build.  Pinned bit for bit against the reference's own glm by
// tests/test_camera_cpu.py (oracle/_ref/libcamref.so, tests/golden/camera_ref.npz).
#include <cmath>
#include <cstdint>
#include <cstring>

#include "mcrt_internal.h"

namespace {

struct V3 { float x, y, z; };
struct V4 { float v[4]; };
struct M4 { V4 c[4]; };   // column major, c[col].v[row] = glm m[col][row]

V4 v4(float a, float b, float c, float d) { V4 r; r.v[0] = a; r.v[1] = b; r.v[2] = c; r.v[3] = d; return r; }
V4 add(const V4& a, const V4& b) { return v4(a.v[0] + b.v[0], a.v[1] + b.v[1], a.v[2] + b.v[2], a.v[3] + b.v[3]); }
V4 sub(const V4& a, const V4& b) { return v4(a.v[0] - b.v[0], a.v[1] - b.v[1], a.v[2] - b.v[2], a.v[3] - b.v[3]); }
V4 mul(const V4& a, const V4& b) { return v4(a.v[0] * b.v[0], a.v[1] * b.v[1], a.v[2] * b.v[2], a.v[3] * b.v[3]); }
V4 mul(const V4& a, float s) { return v4(a.v[0] * s, a.v[1] * s, a.v[2] * s, a.v[3] * s); }

float dot3(V3 a, V3 b) {   // func_geometric.inl:54-61: tmp = x * y; tmp.x + tmp.y + tmp.z
    const float tx = a.x * b.x, ty = a.y * b.y, tz = a.z * b.z;
    return tx + ty + tz;
}
V3 cross3(V3 x, V3 y) { return V3{x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y}; }
V3 normalize3(V3 v) {      // v * inversesqrt(dot(v, v)), inversesqrt = 1 / sqrt
    const float s = 1.0f / std::sqrt(dot3(v, v));
    return V3{v.x * s, v.y * s, v.z * s};
}

M4 zero() { M4 m; std::memset(&m, 0, sizeof(m)); return m; }
M4 identity() { M4 m = zero(); for (int i = 0; i < 4; ++i) m.c[i].v[i] = 1.0f; return m; }

// type_mat4x4.inl:595-613: Result[j] = A0 * B[j][0] + A1 * B[j][1] + A2 * B[j][2] + A3 * B[j][3]
M4 mmul(const M4& a, const M4& b) {
    M4 r;
    for (int j = 0; j < 4; ++j)
        r.c[j] = add(add(add(mul(a.c[0], b.c[j].v[0]), mul(a.c[1], b.c[j].v[1])), mul(a.c[2], b.c[j].v[2])),
                     mul(a.c[3], b.c[j].v[3]));
    return r;
}
// type_mat4x4.inl:501-537: (m0 v0 + m1 v1) + (m2 v2 + m3 v3)
V4 mvec(const M4& m, const V4& v) {
    return add(add(mul(m.c[0], v.v[0]), mul(m.c[1], v.v[1])), add(mul(m.c[2], v.v[2]), mul(m.c[3], v.v[3])));
}

// detail/func_matrix.inl:297-354 (compute_inverse<tmat4x4>)
M4 inverse(const M4& M) {
    auto m = [&](int c, int r) { return M.c[c].v[r]; };
    const float Coef00 = m(2, 2) * m(3, 3) - m(3, 2) * m(2, 3);
    const float Coef02 = m(1, 2) * m(3, 3) - m(3, 2) * m(1, 3);
    const float Coef03 = m(1, 2) * m(2, 3) - m(2, 2) * m(1, 3);
    const float Coef04 = m(2, 1) * m(3, 3) - m(3, 1) * m(2, 3);
    const float Coef06 = m(1, 1) * m(3, 3) - m(3, 1) * m(1, 3);
    const float Coef07 = m(1, 1) * m(2, 3) - m(2, 1) * m(1, 3);
    const float Coef08 = m(2, 1) * m(3, 2) - m(3, 1) * m(2, 2);
    const float Coef10 = m(1, 1) * m(3, 2) - m(3, 1) * m(1, 2);
    const float Coef11 = m(1, 1) * m(2, 2) - m(2, 1) * m(1, 2);
    const float Coef12 = m(2, 0) * m(3, 3) - m(3, 0) * m(2, 3);
    const float Coef14 = m(1, 0) * m(3, 3) - m(3, 0) * m(1, 3);
    const float Coef15 = m(1, 0) * m(2, 3) - m(2, 0) * m(1, 3);
    const float Coef16 = m(2, 0) * m(3, 2) - m(3, 0) * m(2, 2);
    const float Coef18 = m(1, 0) * m(3, 2) - m(3, 0) * m(1, 2);
    const float Coef19 = m(1, 0) * m(2, 2) - m(2, 0) * m(1, 2);
    const float Coef20 = m(2, 0) * m(3, 1) - m(3, 0) * m(2, 1);
    const float Coef22 = m(1, 0) * m(3, 1) - m(3, 0) * m(1, 1);
    const float Coef23 = m(1, 0) * m(2, 1) - m(2, 0) * m(1, 1);
    const V4 Fac0 = v4(Coef00, Coef00, Coef02, Coef03), Fac1 = v4(Coef04, Coef04, Coef06, Coef07);
    const V4 Fac2 = v4(Coef08, Coef08, Coef10, Coef11), Fac3 = v4(Coef12, Coef12, Coef14, Coef15);
    const V4 Fac4 = v4(Coef16, Coef16, Coef18, Coef19), Fac5 = v4(Coef20, Coef20, Coef22, Coef23);
    const V4 Vec0 = v4(m(1, 0), m(0, 0), m(0, 0), m(0, 0)), Vec1 = v4(m(1, 1), m(0, 1), m(0, 1), m(0, 1));
    const V4 Vec2 = v4(m(1, 2), m(0, 2), m(0, 2), m(0, 2)), Vec3 = v4(m(1, 3), m(0, 3), m(0, 3), m(0, 3));
    const V4 Inv0 = add(sub(mul(Vec1, Fac0), mul(Vec2, Fac1)), mul(Vec3, Fac2));
    const V4 Inv1 = add(sub(mul(Vec0, Fac0), mul(Vec2, Fac3)), mul(Vec3, Fac4));
    const V4 Inv2 = add(sub(mul(Vec0, Fac1), mul(Vec1, Fac3)), mul(Vec3, Fac5));
    const V4 Inv3 = add(sub(mul(Vec0, Fac2), mul(Vec1, Fac4)), mul(Vec2, Fac5));
    const V4 SignA = v4(+1, -1, +1, -1), SignB = v4(-1, +1, -1, +1);
    M4 inv;
    inv.c[0] = mul(Inv0, SignA);
    inv.c[1] = mul(Inv1, SignB);
    inv.c[2] = mul(Inv2, SignA);
    inv.c[3] = mul(Inv3, SignB);
    const V4 Row0 = v4(inv.c[0].v[0], inv.c[1].v[0], inv.c[2].v[0], inv.c[3].v[0]);
    const V4 Dot0 = mul(M.c[0], Row0);
    const float Dot1 = (Dot0.v[0] + Dot0.v[1]) + (Dot0.v[2] + Dot0.v[3]);
    const float OneOverDeterminant = 1.0f / Dot1;
    for (int i = 0; i < 4; ++i) inv.c[i] = mul(inv.c[i], OneOverDeterminant);
    return inv;
}

// gtc/matrix_transform.inl:281-300 (perspectiveLH, depth -1..1)
M4 perspectiveLH(float fovy, float aspect, float zNear, float zFar) {
    const float tanHalfFovy = std::tan(fovy / 2.0f);
    M4 r = zero();
    r.c[0].v[0] = 1.0f / (aspect * tanHalfFovy);
    r.c[1].v[1] = 1.0f / (tanHalfFovy);
    r.c[2].v[3] = 1.0f;
    r.c[2].v[2] = (zFar + zNear) / (zFar - zNear);
    r.c[3].v[2] = -(2.0f * zFar * zNear) / (zFar - zNear);
    return r;
}

// gtx/transform.inl:7-10 + gtc/matrix_transform.inl:11-17: translate(identity, v)
M4 translate(V3 v) {
    M4 m = identity(), r = identity();
    r.c[3] = add(add(add(mul(m.c[0], v.x), mul(m.c[1], v.y)), mul(m.c[2], v.z)), m.c[3]);
    return r;
}

struct Cam {
    float W, H, nearZ, farZ;
    M4 proj, projInv, viewProj;
};

V3 screenToNDC(const Cam& c, V3 p) {   // CameraComponent.cpp:158-165
    return V3{p.x / c.W * 2.0f - 1.0f, p.y / c.H * 2.0f - 1.0f, (p.z - c.nearZ) / (c.farZ - c.nearZ) * 2.0f - 1.0f};
}

V3 screenToRayDir(const Cam& c, V3 p, float offx, float offy) {   // RTUtil.cpp:9-41
    const V3 n = screenToNDC(c, p);
    V4 start = v4(n.x, n.y, n.z, 1.0f), end = v4(n.x, n.y, 1.0f, 1.0f);
    offx /= c.W;
    offy /= c.H;
    const M4 inv = inverse(mmul(translate(V3{offx, offy, 0.0f}), c.viewProj));
    start = mvec(inv, start);
    { const float w = start.v[3]; for (int i = 0; i < 4; ++i) start.v[i] /= w; }
    end = mvec(inv, end);
    { const float w = end.v[3]; for (int i = 0; i < 4; ++i) end.v[i] /= w; }
    const V4 d = sub(end, start);
    return normalize3(V3{d.v[0], d.v[1], d.v[2]});
}

void put(mcrt_float4& o, V3 v) { o.x = v.x; o.y = v.y; o.z = v.z; o.w = 0.0f; }

}  // namespace

extern "C" {

MCRT_API mcrt_status mcrt_make_pinhole_camera_axes(const float pos[3], const float right[3], const float up[3],
                                                   const float look[3], float fov_y, float near_z, float far_z,
                                                   uint32_t width, uint32_t height, const float pixel_offset[2],
                                                   mcrt_camera* out) {
    if (!pos || !right || !up || !look || !out || width == 0 || height == 0 || !(far_z > near_z) || !(fov_y > 0.0f))
        return MCRT_ERROR_INVALID_ARG;
    Cam c;
    c.W = static_cast<float>(width);
    c.H = static_cast<float>(height);
    c.nearZ = near_z;
    c.farZ = far_z;
    // setViewport(0, 0, W, H): Rect(x, y, x + w, y + h), aspect = width() / height()
    const float aspect = ((0.0f + c.W) - 0.0f) / ((0.0f + c.H) - 0.0f);
    c.proj = perspectiveLH(fov_y, aspect, near_z, far_z);
    c.projInv = inverse(c.proj);
    const V3 p{pos[0], pos[1], pos[2]}, r{right[0], right[1], right[2]}, u{up[0], up[1], up[2]},
        l{look[0], look[1], look[2]};
    const float x = -dot3(p, r), y = -dot3(p, u), z = -dot3(p, l);
    M4 view;   // updateViewMatrix (CameraComponent.cpp:106-130)
    view.c[0] = v4(r.x, u.x, l.x, 0.0f);
    view.c[1] = v4(r.y, u.y, l.y, 0.0f);
    view.c[2] = v4(r.z, u.z, l.z, 0.0f);
    view.c[3] = v4(x, y, z, 1.0f);
    c.viewProj = mmul(c.proj, view);
    const float ox = pixel_offset ? pixel_offset[0] : 0.0f, oy = pixel_offset ? pixel_offset[1] : 0.0f;
    std::memset(out, 0, sizeof(*out));
    float* wc = &out->worldToClip.m0.x;   // CLHelper::toMatrix: row major
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) wc[4 * i + j] = c.viewProj.c[j].v[i];
    const float nc = near_z;
    put(out->r00, screenToRayDir(c, V3{0.0f, 0.0f, nc}, ox, oy));
    put(out->r10, screenToRayDir(c, V3{c.W, 0.0f, nc}, ox, oy));
    put(out->r11, screenToRayDir(c, V3{c.W, c.H, nc}, ox, oy));
    put(out->r01, screenToRayDir(c, V3{0.0f, c.H, nc}, ox, oy));
    put(out->pos, p);
    put(out->direction, l);
    out->width = width;
    out->height = height;
    // RTBDPTPass.cpp:158-164: image-plane area at z = 1 from ndcToCameraPoint of the near corners
    V4 a = mvec(c.projInv, v4(-1.0f, -1.0f, -1.0f, 1.0f)), b = mvec(c.projInv, v4(1.0f, 1.0f, -1.0f, 1.0f));
    { const float w = a.v[3]; for (int i = 0; i < 4; ++i) a.v[i] /= w; }
    { const float w = b.v[3]; for (int i = 0; i < 4; ++i) b.v[i] /= w; }
    const float az = a.v[2], bz = b.v[2];
    for (int i = 0; i < 3; ++i) { a.v[i] /= az; b.v[i] /= bz; }
    out->area = std::fabs((b.v[0] - a.v[0]) * (b.v[1] - a.v[1]));
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_make_pinhole_camera(const float pos[3], const float forward[3], const float up[3],
                                              float fov_y_deg, float near_z, float far_z, uint32_t width,
                                              uint32_t height, const float pixel_offset[2], mcrt_camera* out) {
    if (!pos || !forward || !up || !out) return MCRT_ERROR_INVALID_ARG;
    // Camera::lookAt (source/engine/camera/Camera.cpp:58-63) with forward = target - position
    const V3 l = normalize3(V3{forward[0], forward[1], forward[2]});
    const V3 r = normalize3(cross3(V3{up[0], up[1], up[2]}, l));
    const V3 u = cross3(l, r);
    const float R[3] = {r.x, r.y, r.z}, U[3] = {u.x, u.y, u.z}, L[3] = {l.x, l.y, l.z};
    // glm::radians (detail/func_trigonometric.inl): degrees * 0.01745329251994329576923690768489
    const float fovy = fov_y_deg * static_cast<float>(0.01745329251994329576923690768489);
    return mcrt_make_pinhole_camera_axes(pos, R, U, L, fovy, near_z, far_z, width, height, pixel_offset, out);
}

MCRT_API mcrt_status mcrt_taa_pixel_offset(const uint32_t* sobol_matrices, uint32_t frame, float radius_x,
                                           float radius_y, float out[2]) {
    if (!sobol_matrices || !out) return MCRT_ERROR_INVALID_ARG;
    // Sampler::sobolSample (raytracing/sampling/sampling.h:7-15) for dimensions 0 and 1, scramble 0
    auto sobol = [&](uint32_t idx, uint32_t dim) {
        uint32_t v = 0;
        for (uint32_t i = dim * 52; idx != 0; idx >>= 1, ++i)
            if (idx & 1) v ^= sobol_matrices[i];
        return v * 0x1p-32f;
    };
    // math::lerp(start, end, t) = (1 - t) * start + t * end (source/engine/util/math.h:38)
    auto lerp = [](float s, float e, float t) { return (1 - t) * s + t * e; };
    out[0] = lerp(-radius_x, radius_x, sobol(frame, 0));
    out[1] = lerp(-radius_y, radius_y, sobol(frame, 1));
    return MCRT_OK;
}

}  // extern "C"

// TEST INFRASTRUCTURE ONLY (oracle/_ref/libcamref.so): the reference's host camera path --
// CameraComponent (source/engine/camera/CameraComponent.cpp:61-134, 149-165), RTUtil::screenToRay
// (source/application/PathTracer/raytracing/util/RTUtil.cpp:9-41), the corner rays of
// RTPrimaryRaysPass::generatePrimaryRays / RTBDPTPass (RTPrimaryRaysPass.cpp:81-104,
// RTBDPTPass.cpp:138-166) and the TAA jitter (PathTracingApp.cpp:208-215) -- computed with the
// reference's own vendored glm (third_party/glm, whose glm.hpp forces GLM_FORCE_LEFT_HANDED) and its
// Sampler::sobolSample (raytracing/sampling/sampling.h + sobol.h), compiled from where they lie.
// Only the member plumbing of the engine classes (which need the ECS, SDL and GL) is spelled out
// here, call for call; every arithmetic step is a glm call or the reference's own expression.
// Built without FMA (no -mfma; MSVC /fp:precise does not contract either).
#include <cmath>
#include <cstdint>
#include <cstring>

#include <glm/glm.hpp>
#include <glm/ext.hpp>
#include <glm/gtx/transform.hpp>

#include "engine/util/math.h"   // math::lerp (math.h:38), math::PI_* for sampling.h
using math::PI;                  // sampling.h:44 (uniformSampleDisc, unused here) names it unqualified
#include "sampling.h"

namespace {
using math::lerp;

struct RefCamera {   // CameraComponent state
    float screenW, screenH, fovY, aspect, nearZ, farZ;
    glm::mat4 view, proj, projInv, viewProj, viewInv, viewProjInv;
    glm::vec3 pos, look;
};

// CameraComponent::setPerspective + setViewport (CameraComponent.cpp:61-87) and
// updateViewMatrix (:96-134) with rotation columns right / up / look (glm::toMat3 of the transform)
void setup(RefCamera& c, const float* pos, const float* right, const float* up, const float* look, float fovY,
           float W, float H, float zn, float zf) {
    c.screenW = W;
    c.screenH = H;
    c.fovY = fovY;
    c.nearZ = zn;
    c.farZ = zf;
    // Rect(x, y, x + width, y + height) with x = y = 0: width() = maxX - minX
    const float vw = (0.0f + W) - 0.0f, vh = (0.0f + H) - 0.0f;
    c.aspect = vw / vh;
    c.proj = glm::perspective(c.fovY, c.aspect, c.nearZ, c.farZ);
    c.projInv = glm::inverse(c.proj);
    const glm::vec3 p(pos[0], pos[1], pos[2]), r(right[0], right[1], right[2]), u(up[0], up[1], up[2]),
        l(look[0], look[1], look[2]);
    const float x = -glm::dot(p, r), y = -glm::dot(p, u), z = -glm::dot(p, l);
    c.view[0][0] = r.x; c.view[1][0] = r.y; c.view[2][0] = r.z; c.view[3][0] = x;
    c.view[0][1] = u.x; c.view[1][1] = u.y; c.view[2][1] = u.z; c.view[3][1] = y;
    c.view[0][2] = l.x; c.view[1][2] = l.y; c.view[2][2] = l.z; c.view[3][2] = z;
    c.view[0][3] = 0.0f; c.view[1][3] = 0.0f; c.view[2][3] = 0.0f; c.view[3][3] = 1.0f;
    c.viewProj = c.proj * c.view;
    c.viewInv = glm::inverse(c.view);
    c.viewProjInv = c.viewInv * c.projInv;
    c.pos = p;
    c.look = l;
}

glm::vec3 screenToNDC(const RefCamera& c, const glm::vec3& p) {   // CameraComponent.cpp:158-165
    return glm::vec3(p.x / c.screenW * 2.0f - 1.0f, p.y / c.screenH * 2.0f - 1.0f,
                     (p.z - c.nearZ) / (c.farZ - c.nearZ) * 2.0f - 1.0f);
}

glm::vec3 ndcToCameraPoint(const RefCamera& c, const glm::vec3& p) {   // CameraComponent.cpp:149-156
    glm::vec4 point(p, 1.0f);
    point = c.projInv * point;
    point /= point.w;
    return glm::vec3(point);
}

// RTUtil::screenToRay (RTUtil.cpp:9-41); pixelOffset = GI.filterSettings.curPixelOffset
glm::vec3 screenToRayDir(const RefCamera& c, const glm::vec3& p, glm::vec2 pixelOffset) {
    glm::vec3 ndcP = screenToNDC(c, p);
    glm::vec4 start(ndcP, 1.f);
    glm::vec4 end(ndcP.x, ndcP.y, 1.0f, 1.f);
    pixelOffset.x /= c.screenW;   // Screen::getWidth()
    pixelOffset.y /= c.screenH;
    glm::mat4 inv = glm::inverse(glm::translate(glm::vec3(pixelOffset.x, pixelOffset.y, 0.0f)) * c.viewProj);
    start = inv * start;
    start /= start.w;
    end = inv * end;
    end /= end.w;
    return glm::normalize(glm::vec3(end - start));
}

void put3(float* o, const glm::vec3& v) { o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = 0.0f; }
}  // namespace

extern "C" {

// Camera::lookAt (source/engine/camera/Camera.cpp:58-63): the rotation axes of a look-at camera
__attribute__((visibility("default"))) void camref_lookat_axes(const float* pos, const float* target,
                                                               const float* worldUp, float* right, float* up,
                                                               float* look) {
    const glm::vec3 p(pos[0], pos[1], pos[2]), t(target[0], target[1], target[2]), w(worldUp[0], worldUp[1], worldUp[2]);
    const glm::vec3 l = glm::normalize(t - p);
    const glm::vec3 r = glm::normalize(glm::cross(w, l));
    const glm::vec3 u = glm::cross(l, r);
    for (int i = 0; i < 3; ++i) { right[i] = r[i]; up[i] = u[i]; look[i] = l[i]; }
}

// PathTracingApp.cpp:208-215 (filter radius r, frame index g_frameIndex)
__attribute__((visibility("default"))) void camref_taa_offset(uint32_t frame, float rx, float ry, float* out) {
    const glm::vec2 r(rx, ry);
    out[0] = lerp(-r.x, r.x, Sampler::sobolSample(frame, 0, 0));
    out[1] = lerp(-r.y, r.y, Sampler::sobolSample(frame, 1, 0));
}

// The RTPinholeCamera (kernel_data.h:246-264, 176 B = 44 floats) the BDPT pass uploads
// (RTBDPTPass.cpp:138-166; the PT pass sets the same corner rays, position, direction and size):
// worldToClip @0 (row major, CLHelper::toMatrix), r00 @16, r10 @20, r11 @24, r01 @28, pos @32,
// direction @36, width/height @40/41 (uint32 bits), area @42.
__attribute__((visibility("default"))) void camref_camera(const float* pos, const float* right, const float* up,
                                                          const float* look, float fovY, float zn, float zf,
                                                          uint32_t width, uint32_t height,
                                                          const float* pixelOffset, float* out) {
    RefCamera c;
    const float w = static_cast<float>(width), h = static_cast<float>(height);
    setup(c, pos, right, up, look, fovY, w, h, zn, zf);
    const glm::vec2 off(pixelOffset[0], pixelOffset[1]);
    const float nc = c.nearZ;
    std::memset(out, 0, 44 * sizeof(float));
    const glm::mat4& m = c.viewProj;   // CLHelper::toMatrix: transpose into row major
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out[4 * i + j] = m[j][i];
    put3(out + 16, screenToRayDir(c, glm::vec3(0.0f, 0.0f, nc), off));
    put3(out + 20, screenToRayDir(c, glm::vec3(w, 0.0f, nc), off));
    put3(out + 24, screenToRayDir(c, glm::vec3(w, h, nc), off));
    put3(out + 28, screenToRayDir(c, glm::vec3(0.0f, h, nc), off));
    put3(out + 32, c.pos);
    put3(out + 36, c.look);   // getForward()
    std::memcpy(out + 40, &width, 4);
    std::memcpy(out + 41, &height, 4);
    glm::vec3 pMin = ndcToCameraPoint(c, glm::vec3(-1.0f, -1.0f, -1.0f));
    glm::vec3 pMax = ndcToCameraPoint(c, glm::vec3(1.0f, 1.0f, -1.0f));
    pMin /= pMin.z;
    pMax /= pMax.z;
    out[42] = std::abs((pMax.x - pMin.x) * (pMax.y - pMin.y));
}

}  // extern "C"

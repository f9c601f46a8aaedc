"""RTPinholeCamera construction (host side, once per frame).

Restates RTPrimaryRaysPass::generatePrimaryRays
(source/application/PathTracer/raytracing/renderPasses/RTPrimaryRaysPass.cpp:81-104),
RTUtil::screenToRay (raytracing/util/RTUtil.cpp:9-41), Camera::screenToNDC
(source/engine/camera/Camera.cpp:139-145) and the TAA jitter
(PathTracingApp.cpp:208-215) for a left-handed glm camera
(x right, y up, z forward; math.cl:4-6).
"""
import math

import numpy as np

from . import types as T


def look_at_lh(eye, target, up):
    eye, target, up = (np.asarray(v, np.float64) for v in (eye, target, up))
    f = target - eye
    f /= np.linalg.norm(f)
    s = np.cross(up, f)
    s /= np.linalg.norm(s)
    u = np.cross(f, s)
    M = np.eye(4)
    M[0, :3], M[1, :3], M[2, :3] = s, u, f
    M[0, 3], M[1, 3], M[2, 3] = -s @ eye, -u @ eye, -f @ eye
    return M


def perspective_lh(fovy_deg, aspect, near, far):
    t = math.tan(math.radians(fovy_deg) / 2.0)
    P = np.zeros((4, 4))
    P[0, 0] = 1.0 / (aspect * t)
    P[1, 1] = 1.0 / t
    P[2, 2] = (far + near) / (far - near)
    P[2, 3] = -(2.0 * far * near) / (far - near)
    P[3, 2] = 1.0
    return P


def make_camera(pos, target, width, height, fovy=45.0, near=0.3, far=30.0, up=(0.0, 1.0, 0.0),
                pixel_offset=(0.0, 0.0)):
    view = look_at_lh(pos, target, up)
    proj = perspective_lh(fovy, width / height, near, far)
    view_proj = proj @ view
    # glm::translate(vec3(offset / screen, 0)) * viewProj, then inverse (RTUtil.cpp:27-30)
    Tm = np.eye(4)
    Tm[0, 3] = pixel_offset[0] / width
    Tm[1, 3] = pixel_offset[1] / height
    inv = np.linalg.inv(Tm @ view_proj)

    def screen_to_ray(sx, sy):
        ndc = np.array([sx / width * 2.0 - 1.0, sy / height * 2.0 - 1.0, (near - near) / (far - near) * 2.0 - 1.0])
        start = inv @ np.array([ndc[0], ndc[1], ndc[2], 1.0])
        end = inv @ np.array([ndc[0], ndc[1], 1.0, 1.0])
        start, end = start / start[3], end / end[3]
        d = end[:3] - start[:3]
        return d / np.linalg.norm(d)

    cam = np.zeros(1, T.CAMERA_DTYPE)
    cam["worldToClip"] = view_proj.astype(np.float32)
    cam["r00"][0, :3] = screen_to_ray(0.0, 0.0)
    cam["r10"][0, :3] = screen_to_ray(width, 0.0)
    cam["r11"][0, :3] = screen_to_ray(width, height)
    cam["r01"][0, :3] = screen_to_ray(0.0, height)
    cam["pos"][0, :3] = pos
    f = np.asarray(target, np.float64) - np.asarray(pos, np.float64)
    cam["direction"][0, :3] = f / np.linalg.norm(f)
    cam["width"] = width
    cam["height"] = height
    # image-plane area at distance 1 (BDPT camera importance, cameras.cl:8-32)
    t = math.tan(math.radians(fovy) / 2.0)
    cam["area"] = np.float32((2.0 * t * width / height) * (2.0 * t))
    return cam


def sobol_1d(idx, dim, mats, scramble=0):
    """Sampler::sobolSample (raytracing/sampling/sampling.h:7-15)."""
    v = scramble
    i = dim * 52
    while idx:
        if idx & 1:
            v ^= int(mats[i])
        idx >>= 1
        i += 1
    return np.float32(v) * np.float32(2.0 ** -32)


def taa_jitter(frame, radius=(2.0, 2.0), mats=None):
    """PathTracingApp.cpp:208-215: lerp(-r, r, sobol(frame, dim 0/1, scramble 0)); mats defaults to
    the Sobol matrices shipped with the package (g_SobolMatrices32)."""
    if mats is None:
        from . import sobol_matrices
        mats = sobol_matrices()
    u = sobol_1d(frame, 0, mats)
    v = sobol_1d(frame, 1, mats)
    f32 = np.float32

    def lerp(s, e, t):   # math::lerp (source/engine/util/math.h:38) in float32
        return float(f32(f32(1) - t) * f32(s) + t * f32(e))
    return (lerp(-radius[0], radius[0], u), lerp(-radius[1], radius[1], v))


def scene_camera(name, width, height, frame=0, mats=None, jitter=False):
    from .scenes import CAMERAS
    pos, target, fov = CAMERAS[name]
    off = taa_jitter(frame, mats=mats) if jitter else (0.0, 0.0)
    return make_camera(pos, target, width, height, fovy=fov, pixel_offset=off)


def scene_camera_at(name, width, height, offset, frame=0, mats=None, jitter=False):
    """scene_camera of a scene moved by `offset` (mcrt.scenes.translated)."""
    from .scenes import CAMERAS
    pos, target, fov = CAMERAS[name]
    off = taa_jitter(frame, mats=mats) if jitter else (0.0, 0.0)
    o = np.asarray(offset, np.float64)
    return make_camera(tuple(np.asarray(pos) + o), tuple(np.asarray(target) + o), width, height, fovy=fov,
                       pixel_offset=off)

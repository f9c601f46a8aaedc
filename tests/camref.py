"""Bindings of oracle/_ref/libcamref.so (TEST INFRASTRUCTURE: the reference's host camera path with
its own vendored glm and Sobol sampler, oracle/refbuild/camref_driver.cpp) and the camera cases the
golden fixture tests/golden/camera_ref.npz holds (regenerate: python tests/camref.py)."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_ref", "libcamref.so")
FIXTURE = os.path.join(ROOT, "tests", "golden", "camera_ref.npz")
_vp = ctypes.c_void_p


def available():
    return os.path.exists(LIB)


def _lib():
    L = ctypes.CDLL(LIB)
    L.camref_lookat_axes.argtypes = [_vp] * 6
    L.camref_taa_offset.argtypes = [ctypes.c_uint32, ctypes.c_float, ctypes.c_float, _vp]
    L.camref_camera.argtypes = [_vp, _vp, _vp, _vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_uint32,
                                ctypes.c_uint32, _vp, _vp]
    return L


def cases(n=48, seed=7):
    """Random look-at cameras: position, target, fov (degrees), near, far, size, TAA frame."""
    rng = np.random.default_rng(seed)
    pos = rng.uniform(-20, 20, (n, 3)).astype(np.float32)
    tgt = (pos + rng.normal(size=(n, 3)) * rng.uniform(0.5, 10, (n, 1))).astype(np.float32)
    fov = rng.uniform(20, 100, n).astype(np.float32)
    fov[:4] = 45.0
    near = rng.choice([0.3, 0.1, 1.0], n).astype(np.float32)
    far = rng.choice([30.0, 100.0, 1000.0], n).astype(np.float32)
    sizes = np.array([(1920, 1080), (3840, 2160), (512, 512), (96, 64), (1280, 720), (640, 480)], np.uint32)
    wh = sizes[rng.integers(0, len(sizes), n)]
    frame = rng.integers(0, 5000, n).astype(np.uint32)
    frame[:8] = np.arange(8)
    return dict(pos=pos, target=tgt, fov_deg=fov, near=near, far=far, wh=wh, frame=frame)


def reference(c, radius=(2.0, 2.0)):
    """Per case: the TAA pixel offset (PathTracingApp.cpp:208-215) and the 176-B RTPinholeCamera
    (44 float32 words) the reference host builds for it, computed by libcamref.so."""
    L = _lib()
    n = len(c["pos"])
    cams = np.zeros((n, 44), np.float32)
    offs = np.zeros((n, 2), np.float32)
    up = np.array([0, 1, 0], np.float32)
    for i in range(n):
        r, u, l = (np.zeros(3, np.float32) for _ in range(3))
        p = np.ascontiguousarray(c["pos"][i])
        t = np.ascontiguousarray(c["target"][i])
        L.camref_lookat_axes(p.ctypes.data, t.ctypes.data, up.ctypes.data, r.ctypes.data, u.ctypes.data, l.ctypes.data)
        L.camref_taa_offset(int(c["frame"][i]), radius[0], radius[1], offs[i].ctypes.data)
        fovy = np.float32(c["fov_deg"][i]) * np.float32(0.01745329251994329576923690768489)   # glm::radians
        out = np.zeros(44, np.float32)
        L.camref_camera(p.ctypes.data, r.ctypes.data, u.ctypes.data, l.ctypes.data, float(fovy), float(c["near"][i]),
                        float(c["far"][i]), int(c["wh"][i][0]), int(c["wh"][i][1]), offs[i].ctypes.data, out.ctypes.data)
        cams[i] = out
    return offs, cams


if __name__ == "__main__":
    c = cases()
    offs, cams = reference(c)
    np.savez_compressed(FIXTURE, **c, taa_offset=offs, camera=cams)
    print(f"{len(cams)} reference cameras -> {FIXTURE}")

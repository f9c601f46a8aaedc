"""SURVEY.md §8 a1 (host camera): the product's C-ABI camera helpers against the reference's own
host camera path -- CameraComponent + RTUtil::screenToRay + RTBDPTPass camera area, with the
reference's vendored glm, and the PathTracingApp TAA jitter with its Sobol sampler -- compiled
from the reference sources (oracle/_ref/libcamref.so, tests/camref.py).  Bit-exact: every one of
the 44 words of the RTPinholeCamera and both jitter components.  Runs on the CPU (host-only math)."""
import numpy as np
import pytest

import camref
from mcrt import lib, sobol_matrices
from mcrt import types as T


def product(c, offs):
    n = len(c["pos"])
    out = np.zeros((n, 44), np.float32)
    for i in range(n):
        fwd = c["target"][i] - c["pos"][i]   # float32, as glm's target - m_pos
        cam = lib.make_pinhole_camera(c["pos"][i], fwd, (0, 1, 0), float(c["fov_deg"][i]), float(c["near"][i]),
                                      float(c["far"][i]), int(c["wh"][i][0]), int(c["wh"][i][1]), offs[i])
        out[i] = cam.view(np.float32).reshape(-1)
    return out


def product_taa(c, radius=(2.0, 2.0)):
    m = sobol_matrices()
    return np.stack([lib.taa_pixel_offset(m, int(f), radius) for f in c["frame"]])


def _bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


def test_camera_matches_reference_fixture():
    z = np.load(camref.FIXTURE, allow_pickle=False)
    c = {k: z[k] for k in ("pos", "target", "fov_deg", "near", "far", "wh", "frame")}
    offs = product_taa(c)
    np.testing.assert_array_equal(_bits(offs), _bits(z["taa_offset"]))
    cams = product(c, offs)
    np.testing.assert_array_equal(_bits(cams), _bits(z["camera"]))
    # the fixture cameras are real cameras: unit corner rays spanning the view
    d = z["camera"][:, 16:32].reshape(-1, 4, 4)[..., :3]
    np.testing.assert_allclose(np.linalg.norm(d, axis=-1), 1.0, atol=1e-6)


@pytest.mark.skipif(not camref.available(), reason="oracle/_ref/libcamref.so not built (no /root/reference)")
def test_camera_matches_reference_live():
    c = camref.cases(n=200, seed=11)
    offs_ref, cams_ref = camref.reference(c)
    offs = product_taa(c)
    np.testing.assert_array_equal(_bits(offs), _bits(offs_ref))
    np.testing.assert_array_equal(_bits(product(c, offs)), _bits(cams_ref))


def test_python_taa_restatement_matches_reference():
    from mcrt.camera import taa_jitter
    z = np.load(camref.FIXTURE, allow_pickle=False)
    got = np.array([taa_jitter(int(f)) for f in z["frame"]], np.float32)
    np.testing.assert_array_equal(_bits(got), _bits(z["taa_offset"]))


def test_axes_form_and_errors():
    """mcrt_make_pinhole_camera_axes with the look-at axes equals the look-at form; bad input fails."""
    z = np.load(camref.FIXTURE, allow_pickle=False)
    cam = z["camera"][0]
    look = cam[36:39]
    up0 = np.array([0, 1, 0], np.float32)
    r = np.cross(up0, look).astype(np.float32)   # float32 cross, then glm normalize
    r = (r * (np.float32(1) / np.sqrt(np.float32((r * r)[0] + (r * r)[1] + (r * r)[2])))).astype(np.float32)
    u = np.cross(look, r).astype(np.float32)
    fovy = np.float32(z["fov_deg"][0]) * np.float32(0.01745329251994329576923690768489)
    a = lib.make_pinhole_camera_axes(z["pos"][0], r, u, look, float(fovy), float(z["near"][0]), float(z["far"][0]),
                                     int(z["wh"][0][0]), int(z["wh"][0][1]), z["taa_offset"][0])
    np.testing.assert_allclose(a.view(np.float32).reshape(-1)[16:32], cam[16:32], atol=2e-7)
    with pytest.raises(lib.MCRTError):
        lib.make_pinhole_camera_axes((0, 0, 0), (1, 0, 0), (0, 1, 0), (0, 0, 1), 0.0, 0.3, 30.0, 64, 64)
    assert T.CAMERA_DTYPE.itemsize == 176

"""GPU tests of the optional mip-mapped texture path (mcrt_frame_params.texture_lod).

The reference carries this path but never calls it (textures.cl:204-209 keeps the bilinear
level-0 read).  Its pieces -- ray differentials of the camera ray (PathTracing.cl:29-33), the
pixel's uv footprint (computeSurfaceInteractionWithDifferentials, geometry.cl:92-175), the mip
level (computeMipmapLOD, textures.cl:198-202) and the trilinear read (readTexture2Df_lod,
textures.cl:148-196) -- are compiled from the reference into a probe kernel
(oracle/refbuild/clprobe_lod.cl) and run live at the reference's own primary hits; the product's
MCRT_AOV_TEXTURE_LOD output (the same device functions k_shade0<LOD> uses) must match it bit for
bit.  Frames with the path on differ from the default frames only where a camera ray hits a
textured surface."""
import os
import subprocess
import sys

import numpy as np
import pytest

from clref_job import LOD_CASES, build_scene
from mcrt import types as T
from mcrt.camera import scene_camera
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def clref_lod(tmp_path_factory):
    if not po.clref_available():
        pytest.skip("oracle/_ref/clref_runner.so not built")
    out = str(tmp_path_factory.mktemp("clref") / "clref_lod.npz")
    r = subprocess.run([sys.executable, os.path.join(HERE, "clref_job.py"), out, "ieee", "lod"],
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        pytest.fail("reference LOD probe job failed:\n" + r.stdout + r.stderr)
    return np.load(out, allow_pickle=False)


@pytest.mark.parametrize("case", LOD_CASES, ids=[c[0] for c in LOD_CASES])
def test_texture_footprint_matches_reference_functions(hip_ctx, clref_lod, case):
    from mcrt import lib
    name, W, H = case
    ds = lib.DeviceScene(hip_ctx, build_scene(name))
    fb = lib.FrameBuffer(hip_ctx, W, H)
    ours = fb.render_aov(ds, scene_camera(name, W, H), T.AOV_TEXTURE_LOD)
    ref = clref_lod[f"lod_{name}_{W}x{H}"]
    hit = ref[..., 1, 1].view(np.int32) != 0   # shape id bits (0 = a miss or shape 0)
    same_shape = ours[..., 1, 1].view(np.int32) == ref[..., 1, 1].view(np.int32)
    assert same_shape.all()
    ne = (ours.view(np.uint32) != ref.view(np.uint32)) & ~(np.isnan(ours) & np.isnan(ref))
    bad = ne.any(-1).any(-1)
    print(name, "pixels", hit.sum(), "differing", int(bad.sum()),
          "lod range", float(np.nanmin(ref[..., 1, 0])), float(np.nanmax(ref[..., 1, 0])))
    assert not bad.any(), [(k, int(ne[..., k, :].any(-1).sum())) for k in range(3)]
    fb.close()
    ds.close()


def test_lod_frames(hip_ctx):
    """texture_lod = 1 changes only pixels whose camera ray hits a textured surface, and only
    where that surface is minified; the image mean stays close (mip averages are unbiased)."""
    from mcrt import lib
    sc = build_scene("lod_test")
    W, H = 160, 120
    cam = scene_camera("lod_test", W, H)
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    fb.render(ds, cam, frame=0, max_depth=2)
    off = fb.read(0)[..., :3].copy()
    fb.render(ds, cam, frame=0, max_depth=2, texture_lod=True)
    on = fb.read(0)[..., :3].copy()
    fp = fb.render_aov(ds, cam, T.AOV_TEXTURE_LOD)
    lod = fp[..., 1, 0]
    textured = np.zeros((H, W), bool)
    shape = fp[..., 1, 1].view(np.int32)
    mats = sc.shapes["materialId"][shape]
    textured = (sc.materials["uber_diffuseTexId"][mats] != -1) | (sc.materials["uber_normalMapId"][mats] != -1)
    hitmask = (fp[..., 0, :] != 0).any(-1) | (fp[..., 1, 2:] != 0).any(-1)
    diff = (on.view(np.uint32) != off.view(np.uint32)).any(-1)
    assert not (diff & ~(textured & hitmask)).any(), int((diff & ~(textured & hitmask)).sum())
    assert diff[(lod > 1.0) & textured].mean() > 0.5   # minified texels are filtered
    assert abs(on.mean() / off.mean() - 1.0) < 0.05, (on.mean(), off.mean())
    # albedo AOV: level-0 vs mip-mapped reads of the same hits
    a0 = fb.render_aov(ds, cam, T.AOV_ALBEDO)
    a1 = fb.render_aov(ds, cam, T.AOV_ALBEDO, texture_lod=True)
    far = (lod > 3.0) & textured
    assert far.any()
    # far away the checker averages out: the mip-mapped albedo varies much less between neighbours
    v0 = np.abs(np.diff(a0[..., 0], axis=1))[far[:, 1:]].mean()
    v1 = np.abs(np.diff(a1[..., 0], axis=1))[far[:, 1:]].mean()
    assert v1 < 0.5 * v0, (v0, v1)
    fb.close()
    ds.close()

"""Dynamic scene updates (RTScene::update, RTScene.cpp:317-391 -> mcrt_scene_update_materials /
_shapes / _lights, a moved shape followed by mcrt_accel_build as RR's Commit) against the
REFERENCE kernels run live on the scene built fresh with the same arrays (tests/clref_job.py
... updates): after every cumulative update the product's frames are bit-exact."""
import os
import subprocess
import sys

import numpy as np
import pytest

from clref_job import build_scene, update_steps
from mcrt.camera import scene_camera
from oracle import pyoracle as po

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_updates_match_reference(hip_ctx, tmp_path):
    from mcrt import lib
    if not po.clref_available():
        pytest.skip("oracle/_ref/clref_runner.so not built")
    out = str(tmp_path / "updates.npz")
    r = subprocess.run([sys.executable, os.path.join(HERE, "clref_job.py"), out, "ieee", "updates"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    ref = np.load(out, allow_pickle=False)
    sc = build_scene("mixed")
    steps = update_steps(build_scene("mixed"))
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, 96, 64)
    cam = scene_camera("mixed", 96, 64)
    fb.render(ds, cam, frame=0, max_depth=3)
    before = fb.read(0)
    for i, (kind, arr) in enumerate(steps):
        if kind == "materials":
            ds.update_materials(arr)
        elif kind == "lights":
            ds.update_lights(arr)
        else:
            ds.update_shapes(arr)
            ds.build()                     # a moved shape needs the BVH rebuilt (RR Commit)
        for f in (0, 1):
            fb.render(ds, cam, frame=f, max_depth=3)
            g = fb.read(0)
            want = ref[f"update{i}_{kind}_f{f}"]
            diff = (g[..., :3].view(np.uint32) != want[..., :3].view(np.uint32)).any(-1)
            assert not diff.any(), (i, kind, f, int(diff.sum()))
        if i == 0:
            assert (g != before).any()
    fb.close()
    ds.close()

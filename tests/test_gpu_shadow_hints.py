"""Occluder hints of the shadow rays (mcrt_traverse.h hintOccludes): a shadow ray first tests the
leaf its pixel's bounce-0 ray (or its origin cell's rays) last found occluding, with the walk's own
triangle and box arithmetic, and skips the walk when both pass.  The answer must be the walk's for
ANY hint content, so every frame is compared bit for bit with hints off (MCRT_SHADOW_HINTS=0):
the pixel hints (bounce 0, wave packets and per ray), the cell hints (later bounces, D = 2 and 3),
hints carried over from earlier calls, and tables filled with random leaf indices
(MCRT_TEST_HINT_FILL); BDPT's connection rays take the cell hints too."""
import os

import numpy as np
import pytest

from mcrt import scenes
from mcrt.camera import scene_camera

pytestmark = pytest.mark.gpu


def _frames(hip_ctx, sc, name, W, H, max_depth, calls=3, batch=4, integrator=None, device_build=False):
    from mcrt import lib
    ds = lib.DeviceScene(hip_ctx, sc, device_build=device_build)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    out = []
    for c in range(calls):   # TAA-jittered cameras, as the bench
        cams = [scene_camera(name, W, H, frame=c * batch + k, jitter=True) for k in range(batch)]
        kw = {} if integrator is None else {"integrator": integrator}
        fb.render_frames(ds, cams, frame=c * batch, max_depth=max_depth, **kw)
        hip_ctx.sync()
        out.append(np.stack([fb.read_frame(k) for k in range(batch)]))
    fb.close()
    ds.close()
    return np.stack(out)


def _with_env(env, fn):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return fn()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def sm_small():
    return scenes.san_miguel_proxy(tris=1_000_000)


CASES = [("mixed", 2, {}), ("mixed", 3, {}), ("sm", 2, {}), ("sm", 3, {}),
         ("sm", 2, {"MCRT_CAMERA_PACKETS": "0"}),          # bounce-0 shadow rays walked per ray
         ("sm", 2, {"MCRT_TEST_HINT_FILL": "7"}),          # tables full of random leaf indices
         ("mixed", 3, {"MCRT_TEST_HINT_FILL": "11"})]


@pytest.mark.parametrize("name,max_depth,env", CASES)
def test_hints_change_no_answer(hip_ctx, sm_small, name, max_depth, env):
    sc, cam_name, W, H = ((scenes.test_scene(), "mixed", 96, 64) if name == "mixed" else
                          (sm_small, "san_miguel_proxy", 256, 144))
    on = _with_env(dict(env, MCRT_SHADOW_HINTS="1"), lambda: _frames(hip_ctx, sc, cam_name, W, H, max_depth))
    off = _with_env(dict(env, MCRT_SHADOW_HINTS="0"), lambda: _frames(hip_ctx, sc, cam_name, W, H, max_depth))
    assert np.isfinite(on).all()
    assert on[..., :3].max() > 0
    diff = on.view(np.uint32) != off.view(np.uint32)
    assert not diff.any(), f"{int(diff.any(-1).sum())} pixels differ"


@pytest.mark.parametrize("build", [1, 4])
def test_hints_change_no_answer_other_builders(hip_ctx, sm_small, build):
    """The device LBVH (1) and the perf tree (4) take the hints too: frames bit-identical with them
    off, with random tables, on trees other than the reference's."""
    args = (hip_ctx, sm_small, "san_miguel_proxy", 256, 144, 3)
    off = _with_env({"MCRT_SHADOW_HINTS": "0"}, lambda: _frames(*args, device_build=build))
    for env in ({}, {"MCRT_TEST_HINT_FILL": "5"}):
        on = _with_env(dict(env, MCRT_SHADOW_HINTS="1"), lambda: _frames(*args, device_build=build))
        assert np.isfinite(on).all() and on[..., :3].max() > 0
        diff = on.view(np.uint32) != off.view(np.uint32)
        assert not diff.any(), (build, env, int(diff.any(-1).sum()))


@pytest.mark.parametrize("build", [1, 2])
def test_device_trees_nest_and_report_depth(hip_ctx, sm_small, build):
    """The hints' premise (test_hint_premise_cpu.py) on the device-built trees, and their reported
    depth (the packet stack's bound) against the deepest leaf."""
    from mcrt import lib
    from test_hint_premise_cpu import check_nesting, leaf_depth
    ds = lib.DeviceScene(hip_ctx, sm_small, device_build=build)
    rec = ds.records()
    depth = ds.layout()["depth"]
    ds.close()
    assert check_nesting(rec) > 0
    assert depth >= leaf_depth(rec), (build, depth, leaf_depth(rec))


def test_bdpt_visibility_hints(hip_ctx, sm_small):
    """k_bdpt_vis takes the origin-cell hints: the same visibility answers, so the frames agree up to
    the order of the light-tracing splats' float atomics (test_gpu_bdpt.py's 4e-6)."""
    from mcrt import types as T
    args = (hip_ctx, sm_small, "san_miguel_proxy", 256, 144, 2)
    on = _with_env({"MCRT_SHADOW_HINTS": "1"}, lambda: _frames(*args, integrator=T.INTEGRATOR_BDPT))
    off = _with_env({"MCRT_SHADOW_HINTS": "0"}, lambda: _frames(*args, integrator=T.INTEGRATOR_BDPT))
    assert np.isfinite(on).all() and on[..., :3].max() > 0
    np.testing.assert_allclose(on[..., :3], off[..., :3], rtol=4e-6, atol=4e-6)


def test_hint_counts(hip_ctx, sm_small):
    """mcrt_framebuffer_hint_counts: the hints answer a large share of the occluded bounce-0 shadow
    rays from the second call on (the pixel table holds the first call's occluders), none when off."""
    from mcrt import lib

    def run():
        ds = lib.DeviceScene(hip_ctx, sm_small)
        fb = lib.FrameBuffer(hip_ctx, 256, 144)
        hip_ctx.set_profiling(2)   # counters on
        got = []
        for c in range(2):
            cams = [scene_camera("san_miguel_proxy", 256, 144, frame=4 * c + k, jitter=True) for k in range(4)]
            fb.render_frames(ds, cams, frame=4 * c, max_depth=2)
            got.append((fb.hint_counts(2), fb.queue_counts(2)[0]))
        hip_ctx.set_profiling(False)
        fb.close()
        ds.close()
        return got

    on = _with_env({"MCRT_SHADOW_HINTS": "1"}, run)
    off = _with_env({"MCRT_SHADOW_HINTS": "0"}, run)
    (h1, q1), (h2, q2) = on
    assert all(0 <= h <= q for h, q in zip(h2, q2))
    assert h2[0] > 0.2 * q2[0], (h2, q2)     # bounce 0: pixel + cell hints of the first call
    assert h2[1] > 0, (h2, q2)                # bounce 1: cell hints
    assert all(h == 0 for h, _ in [(x, None) for x in off[1][0]])

"""The C ABI from compiled C++: tests/capi_consumer/capi_consumer.cpp replays INTEGRATION.md's
reference-side code (RTScene::commit -> mcrt_scene_create + mcrt_accel_build; RTPrimaryRaysPass
with 48-B rays in hipMalloc'd memory through mcrt_trace_closest / mcrt_trace_any;
RTPathTracingPass + RTReconstructionPass -> mcrt_render_frame + mcrt_accumulate +
mcrt_framebuffer_read; errors as std::runtime_error via check()).  It runs as its own process on
the GPU; its outputs must equal the same calls made through the ctypes binding, bit for bit."""
import json
import os
import subprocess

import numpy as np
import pytest

from mcrt import scenes, sobol_matrices
from mcrt import types as T
from mcrt.camera import scene_camera

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
EXE = os.path.join(HERE, "capi_consumer", "capi_consumer")


def write_scene(sc, cam, d):
    os.makedirs(d, exist_ok=True)
    arrays = {"shapes": sc.shapes, "indices": sc.indices, "positions": sc.positions, "uvs": sc.uvs,
              "normals": sc.normals, "tangents": sc.tangents, "binormals": sc.binormals, "textures": sc.textures,
              "texdata": sc.tex_data, "sobol": sc.sobol, "lights": sc.lights, "materials": sc.materials, "camera": cam}
    for k, a in arrays.items():
        np.ascontiguousarray(a).tofile(os.path.join(d, f"{k}.bin"))


def test_cpp_consumer_matches_ctypes(hip_ctx, tmp_path):
    import torch
    from mcrt import lib
    if not os.path.exists(EXE):
        pytest.skip("tests/capi_consumer/capi_consumer not built (make -C tests/capi_consumer)")
    sc = scenes.test_scene()
    sc.sobol = sobol_matrices()
    W, H, frames, D = 96, 64, 4, 3
    cam = scene_camera("mixed", W, H)
    write_scene(sc, cam, str(tmp_path / "scene"))
    os.makedirs(tmp_path / "out")
    r = subprocess.run([EXE, str(tmp_path / "scene"), str(tmp_path / "out"), str(frames), str(D)],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["pixels"] == W * H and info["error_caught"] == 1 and info["closest_hits"] > 0, info
    # device-count queries with events (radeon_rays.h:272-277) = the host-count ones on the first k rays
    assert info["count_queries_match"] == 1, info
    out = lambda n, dt: np.fromfile(str(tmp_path / "out" / f"{n}.bin"), dt)   # noqa: E731
    # the same through ctypes
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    for f in range(frames):
        fb.render(ds, cam, frame=f, max_depth=D)
        fb.accumulate(T.make_filter(T.BOX), f)
    np.testing.assert_array_equal(out("radiance", np.uint32).reshape(H, W, 4), fb.read(0).view(np.uint32))
    np.testing.assert_array_equal(out("image", np.uint32).reshape(H, W, 4), fb.read(2).view(np.uint32))
    rays = out("rays", T.RAY_DTYPE)
    rd = torch.from_numpy(rays.view(np.uint8).copy()).cuda()
    h = torch.full((len(rays) * 32,), 0xff, dtype=torch.uint8, device="cuda")
    o = torch.full((len(rays),), 0x7f7f7f7f, dtype=torch.int32, device="cuda")
    ds.trace_closest(rd.data_ptr(), len(rays), h.data_ptr())
    ds.trace_any(rd.data_ptr(), len(rays), o.data_ptr())
    hip_ctx.sync()
    np.testing.assert_array_equal(out("hits", np.uint8), h.cpu().numpy())
    np.testing.assert_array_equal(out("occl", np.int32), o.cpu().numpy())
    inactive = rays["extra"][:, 1] == 0
    assert inactive.any() and (out("occl", np.int32)[inactive] == 0x7f7f7f7f).all()   # untouched (Q12)
    fb.close()
    ds.close()


def test_cpp_consumer_obj_scene(hip_ctx, tmp_path):
    """A C++ host loading an OBJ/MTL/PNG scene through mcrt_obj_load (the reference's
    AssetImporter + RTScene step) renders the same frames as the ctypes path over lib.load_obj."""
    from mcrt import lib
    from mcrt.camera import make_camera
    from test_objload_cpu import _write_scene
    if not os.path.exists(EXE):
        pytest.skip("tests/capi_consumer/capi_consumer not built (make -C tests/capi_consumer)")
    _write_scene(str(tmp_path))
    obj = str(tmp_path / "s.obj")
    W, H, frames, D = 48, 40, 3, 3
    cam = make_camera((0.5, 0.5, -3.0), (0.5, 0.5, 0.0), W, H)
    sun = (scenes.euler_forward(45.0, 20.0), (4.0, 4.0, 4.0))
    d = tmp_path / "scene"
    os.makedirs(d)
    np.ascontiguousarray(cam).tofile(str(d / "camera.bin"))
    np.array(list(sun[0]) + list(sun[1]), np.float32).tofile(str(d / "sun.bin"))
    os.makedirs(tmp_path / "out")
    r = subprocess.run([EXE, str(d), str(tmp_path / "out"), str(frames), str(D), obj], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    out = lambda n, dt: np.fromfile(str(tmp_path / "out" / f"{n}.bin"), dt)   # noqa: E731
    sc = lib.load_obj(obj, directional_lights=[sun])
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    for f in range(frames):
        fb.render(ds, cam, frame=f, max_depth=D)
        fb.accumulate(T.make_filter(T.BOX), f)
    img = fb.read(2)
    assert img[..., :3].max() > 0
    np.testing.assert_array_equal(out("radiance", np.uint32).reshape(H, W, 4), fb.read(0).view(np.uint32))
    np.testing.assert_array_equal(out("image", np.uint32).reshape(H, W, 4), img.view(np.uint32))
    fb.close()
    ds.close()


RCCL_EXE = os.path.join(HERE, "capi_consumer", "capi_rccl")


def test_cpp_rccl_end_of_job(hip_ctx, tmp_path):
    """The multi-GPU end of job from C++ (capi_rccl.cpp; INTEGRATION.md "Multi-GPU"): 3 bands on one
    GPU with a 1-rank RCCL communicator -- each band's accumulators packed on the context stream, ONE
    ncclGroupStart/ncclSend/ncclRecv gather, mcrt_framebuffer_bands_unpack; BDPT adds a per-frame
    mcrt_bdpt_splats_copy -> ncclReduceScatter -> mcrt_bdpt_gather.  PT: the whole-image frame bit
    for bit; BDPT: up to the order of the splat sums (rtol 2e-5, as the band-split BDPT tests)."""
    from mcrt import lib
    if not os.path.exists(RCCL_EXE):
        pytest.skip("tests/capi_consumer/capi_rccl not built (make -C tests/capi_consumer)")
    sc = scenes.test_scene()
    sc.sobol = sobol_matrices()
    W, H, frames, D, bands = 96, 72, 3, 2, 3
    cam = scene_camera("mixed", W, H)
    write_scene(sc, cam, str(tmp_path / "scene"))
    os.makedirs(tmp_path / "out")
    env = dict(os.environ, NCCL_DEBUG=os.environ.get("NCCL_DEBUG", "WARN"))
    r = subprocess.run([RCCL_EXE, str(tmp_path / "scene"), str(tmp_path / "out"), str(frames), str(D), str(bands)],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    assert info["world"] == 1 and info["bands"] == bands and info["pixels"] == W * H, info
    assert info["pt_identical"] == 1, info
    assert 0 <= info["bdpt_max_rel"] <= 2e-5, info
    out = lambda n: np.fromfile(str(tmp_path / "out" / f"{n}.bin"), np.float32).reshape(H, W, 4)   # noqa: E731
    np.testing.assert_array_equal(out("pt_split").view(np.uint32), out("pt_plain").view(np.uint32))
    bd = out("bdpt_split")
    assert np.isfinite(bd).all() and bd[..., :3].max() > 0
    np.testing.assert_allclose(bd, out("bdpt_plain"), rtol=2e-5, atol=2e-5)
    # the C++ host's whole-image frames = the ctypes path's
    ds = lib.DeviceScene(hip_ctx, sc)
    fb = lib.FrameBuffer(hip_ctx, W, H)
    for f in range(frames):
        fb.render(ds, cam, frame=f, max_depth=D)
        fb.accumulate(T.make_filter(T.BOX), f)
    np.testing.assert_array_equal(out("pt_plain").view(np.uint32), fb.read(2).view(np.uint32))
    fb.close()
    ds.close()

"""ctypes binding of libmcrt.so (include/mcrt_capi.h) -- the product path.

There is deliberately no fallback: if the HIP library is missing or no GPU is present,
the calls raise.  Device memory for ray queries comes from torch tensors on cuda
(torch is plumbing here), everything else lives inside the library.
"""
import ctypes
import weakref
import os

import numpy as np

from . import PKG_DIR
from . import types as T

# MCRT_LIB_PATH: an alternative in-tree build of the same library (kernel tuning experiments)
_DEFAULT_LIB = os.path.join(os.path.dirname(PKG_DIR), "libmcrt.so")
LIB_PATH = os.environ.get("MCRT_LIB_PATH") or _DEFAULT_LIB
HEADER = os.path.join(os.path.dirname(os.path.dirname(PKG_DIR)), "include", "mcrt_capi.h")

_c = ctypes
_vp = _c.c_void_p
_lib = None

# every entry point of include/mcrt_capi.h: name -> (restype, argtypes)
SIGNATURES = {
    "mcrt_version": (_c.c_char_p, []),
    "mcrt_last_error": (_c.c_char_p, [_vp]),
    "mcrt_ctx_create": (_c.c_int, [_c.c_int, _c.POINTER(_vp)]),
    "mcrt_ctx_destroy": (_c.c_int, [_vp]),
    "mcrt_ctx_synchronize": (_c.c_int, [_vp]),
    "mcrt_ctx_set_stream": (_c.c_int, [_vp, _vp]),
    "mcrt_ctx_set_profiling": (_c.c_int, [_vp, _c.c_int]),
    "mcrt_ctx_kernel_stats": (_c.c_int, [_vp, _c.c_int, _vp, _vp, _vp, _vp, _c.POINTER(_c.c_int)]),
    "mcrt_ctx_reset_stats": (_c.c_int, [_vp]),
    "mcrt_ctx_stream_copy": (_c.c_int, [_vp, _c.c_uint64, _c.c_int, _c.POINTER(_c.c_double)]),
    "mcrt_ctx_get_stream": (_c.c_int, [_vp, _c.POINTER(_vp)]),
    "mcrt_ctx_gather_chase": (_c.c_int, [_vp, _c.c_uint64, _c.c_int, _c.c_int, _c.POINTER(_c.c_double)]),
    "mcrt_ctx_gather_chase_compact": (_c.c_int, [_vp, _c.c_uint64, _c.c_double, _c.c_int, _c.c_int,
                                                 _c.POINTER(_c.c_double)]),
    "mcrt_scene_create": (_c.c_int, [_vp, _vp, _c.POINTER(_vp)]),
    "mcrt_scene_destroy": (_c.c_int, [_vp]),
    "mcrt_scene_update_lights": (_c.c_int, [_vp, _vp, _c.c_uint32]),
    "mcrt_scene_update_materials": (_c.c_int, [_vp, _vp, _c.c_uint32]),
    "mcrt_scene_update_shapes": (_c.c_int, [_vp, _vp, _c.c_uint32]),
    "mcrt_accel_build": (_c.c_int, [_vp, _vp]),
    "mcrt_accel_info": (_c.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "mcrt_accel_layout": (_c.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "mcrt_accel_builder": (_c.c_int, [_vp, _vp]),
    "mcrt_bdpt_splats_copy": (_c.c_int, [_vp, _vp]),
    "mcrt_bdpt_splat_layout": (_c.c_int, [_vp, _c.POINTER(_c.c_uint64), _c.POINTER(_c.c_int32)]),
    "mcrt_framebuffer_stream": (_c.c_int, [_vp, _c.POINTER(_vp)]),
    "mcrt_bdpt_gather": (_c.c_int, [_vp, _vp]),
    "mcrt_framebuffer_set_splat_exchange": (_c.c_int, [_vp, _c.c_int32]),
    "mcrt_bdpt_splats_sparse": (_c.c_int, [_vp, _vp, _c.c_int64, _c.POINTER(_c.c_int64), _c.c_int32]),
    "mcrt_bdpt_gather_sparse": (_c.c_int, [_vp, _vp, _c.c_int64]),
    "mcrt_obj_load": (_c.c_int, [_c.c_char_p, _c.c_uint32, _vp]),
    "mcrt_obj_add_directional_light": (_c.c_int, [_vp, _vp, _vp]),
    "mcrt_obj_add_point_light": (_c.c_int, [_vp, _vp, _vp]),
    "mcrt_obj_scene_desc": (_c.c_int, [_vp, _vp]),
    "mcrt_obj_warnings": (_c.c_char_p, [_vp]),
    "mcrt_obj_free": (None, [_vp]),
    "mcrt_accel_read_records": (_c.c_int, [_vp, _vp, _c.c_uint64, _vp]),
    "mcrt_accel_build_host_records": (_c.c_int, [_vp, _vp, _vp, _c.c_uint64, _c.POINTER(_c.c_uint64), _vp]),
    "mcrt_trace_closest": (_c.c_int, [_vp, _vp, _c.c_int32, _vp]),
    "mcrt_trace_any": (_c.c_int, [_vp, _vp, _c.c_int32, _vp]),
    "mcrt_trace_closest_count": (_c.c_int, [_vp, _vp, _vp, _c.c_int32, _vp, _vp, _c.POINTER(_vp)]),
    "mcrt_trace_any_count": (_c.c_int, [_vp, _vp, _vp, _c.c_int32, _vp, _vp, _c.POINTER(_vp)]),
    "mcrt_event_wait": (_c.c_int, [_vp]),
    "mcrt_event_destroy": (_c.c_int, [_vp]),
    "mcrt_framebuffer_create": (_c.c_int, [_vp, _c.c_uint32, _c.c_uint32, _c.POINTER(_vp)]),
    "mcrt_framebuffer_destroy": (_c.c_int, [_vp]),
    "mcrt_framebuffer_set_frames_in_flight": (_c.c_int, [_vp, _c.c_int32]),
    "mcrt_render_frame": (_c.c_int, [_vp, _vp, _vp, _vp]),
    "mcrt_accumulate": (_c.c_int, [_vp, _vp, _c.c_int32]),
    "mcrt_render_frames": (_c.c_int, [_vp, _vp, _vp, _c.c_int32, _vp]),
    "mcrt_accumulate_frames": (_c.c_int, [_vp, _vp, _c.c_int32, _c.c_int32]),
    "mcrt_framebuffer_device_ptrs": (_c.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "mcrt_framebuffer_read": (_c.c_int, [_vp, _c.c_int, _vp]),
    "mcrt_framebuffer_read_frame": (_c.c_int, [_vp, _c.c_int32, _vp]),
    "mcrt_framebuffer_stats": (_c.c_int, [_vp, _vp, _vp, _vp]),
    "mcrt_framebuffer_copy_device": (_c.c_int, [_vp, _c.c_int, _vp]),
    "mcrt_framebuffer_set_accumulation": (_c.c_int, [_vp, _vp, _vp]),
    "mcrt_framebuffer_bands_pack": (_c.c_int, [_vp, _vp]),
    "mcrt_framebuffer_bands_unpack": (_c.c_int, [_vp, _vp, _c.c_int32]),
    "mcrt_framebuffer_band_layout": (_c.c_int, [_vp, _c.POINTER(_c.c_int32), _c.POINTER(_c.c_int32),
                                                _c.POINTER(_c.c_int32)]),
    "mcrt_framebuffer_read_queue": (_c.c_int, [_vp, _c.c_int, _vp, _c.c_int64, _c.POINTER(_c.c_int32)]),
    "mcrt_framebuffer_queue_counts": (_c.c_int, [_vp, _c.POINTER(_c.c_int32), _c.POINTER(_c.c_int32), _c.c_int]),
    "mcrt_framebuffer_hint_counts": (_c.c_int, [_vp, _c.POINTER(_c.c_int32), _c.c_int]),
    "mcrt_framebuffer_retrace_counts": (_c.c_int, [_vp, _c.POINTER(_c.c_int32), _c.c_int]),
    "mcrt_framebuffer_wave_clock": (_c.c_int, [_vp, _c.c_int, _vp, _c.c_int64, _c.POINTER(_c.c_int64)]),
    "mcrt_postprocess": (_c.c_int, [_vp, _c.POINTER(T.PostprocessParams)]),
    "mcrt_render_aov": (_c.c_int, [_vp, _vp, _vp, _vp, _c.c_int, _vp]),
    "mcrt_framebuffer_read_bdpt": (_c.c_int, [_vp, _c.c_int, _vp, _c.c_uint64, _c.POINTER(_c.c_uint64)]),
    "mcrt_make_pinhole_camera": (_c.c_int, [_vp, _vp, _vp, _c.c_float, _c.c_float, _c.c_float, _c.c_uint32,
                                            _c.c_uint32, _vp, _vp]),
    "mcrt_make_pinhole_camera_axes": (_c.c_int, [_vp, _vp, _vp, _vp, _c.c_float, _c.c_float, _c.c_float,
                                                 _c.c_uint32, _c.c_uint32, _vp, _vp]),
    "mcrt_taa_pixel_offset": (_c.c_int, [_vp, _c.c_uint32, _c.c_float, _c.c_float, _vp]),
}


class MCRTError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MCRTError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                            "(make -C monte-carlo-raytracer_amd/csrc); there is no CPU fallback")
        L = _c.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            try:
                f = getattr(L, name)
            except AttributeError:
                # an older library selected with MCRT_LIB_PATH (A/B runs) may lack a later entry
                # point: it fails when called; the in-tree library exports every one
                # (tests/test_capi_cpu.py)
                if LIB_PATH == _DEFAULT_LIB:
                    raise
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _check(status, ctx=None):
    if status != 0:
        msg = lib().mcrt_last_error(ctx)
        raise MCRTError(f"mcrt status {status}: {msg.decode() if msg else ''}")


def _p(a):
    return None if a is None else a.ctypes.data


def _records(items):
    """Stacks one-record structured arrays into one array of the SAME dtype (np.stack would promote
    a padded dtype such as the 56-B filter layout to a packed one and shift its fields)."""
    first = np.asarray(items[0])
    out = np.empty(len(items), first.dtype)
    for i, a in enumerate(items):
        out[i] = np.asarray(a, first.dtype).reshape(-1)[0]
    return out


class Context:
    def __init__(self, device=0, profiling=False):
        h = _vp()
        _check(lib().mcrt_ctx_create(device, _c.byref(h)))
        self.h = h
        if profiling:
            self.set_profiling(True)

    def _adopt(self, child):
        """Scenes and frame buffers die with their context (closed first on ctx.close())."""
        if not hasattr(self, "_children"):
            self._children = weakref.WeakSet()
        self._children.add(child)

    def close(self):
        if self.h:
            for c in list(getattr(self, "_children", ())):
                c.close()
            lib().mcrt_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        _check(lib().mcrt_ctx_synchronize(self.h), self.h)

    def set_stream(self, stream_ptr):
        _check(lib().mcrt_ctx_set_stream(self.h, stream_ptr), self.h)

    def stream(self):
        """hipStream_t (int) of the context stream (mcrt_ctx_get_stream)."""
        st = _vp()
        _check(lib().mcrt_ctx_get_stream(self.h, _c.byref(st)), self.h)
        return st.value or 0

    def set_profiling(self, on=True):
        """on: True / 1 = per-kernel HIP events; 2 = also the occluder-hint counters."""
        _check(lib().mcrt_ctx_set_profiling(self.h, int(on)), self.h)

    def reset_stats(self):
        _check(lib().mcrt_ctx_reset_stats(self.h), self.h)

    def gather_chase_gsteps(self, records, steps=256, iters=3):
        """Dependent 64-B gather ceiling, G steps/s (mcrt_ctx_gather_chase)."""
        g = _c.c_double()
        _check(lib().mcrt_ctx_gather_chase(self.h, records, steps, iters, _c.byref(g)), self.h)
        return g.value

    def gather_chase_compact_gsteps(self, records, leaf_frac, steps=256, iters=3):
        """The same ceiling over packed 32-B / 48-B records, a share leaf_frac of them 48-B leaves
        (the compact walk's layout; mcrt_ctx_gather_chase_compact), G steps/s."""
        g = _c.c_double()
        _check(lib().mcrt_ctx_gather_chase_compact(self.h, records, float(leaf_frac), steps, iters, _c.byref(g)),
               self.h)
        return g.value

    def stream_copy_gbps(self, nbytes=2 << 30, iters=5):
        """Attainable HBM GB/s of a stream copy (mcrt_ctx_stream_copy)."""
        g = _c.c_double()
        _check(lib().mcrt_ctx_stream_copy(self.h, nbytes, iters, _c.byref(g)), self.h)
        return g.value

    def kernel_stats(self):
        n = 16
        names = (_c.c_char_p * n)()
        ms = np.zeros(n, np.float64)
        launches = np.zeros(n, np.int64)
        items = np.zeros(n, np.int64)
        cnt = _c.c_int()
        _check(lib().mcrt_ctx_kernel_stats(self.h, n, names, _p(ms), _p(launches), _p(items), _c.byref(cnt)), self.h)
        return {names[i].decode(): {"ms": float(ms[i]), "launches": int(launches[i]), "items": int(items[i])}
                for i in range(cnt.value)}


def accel_opts(cost=10.0, bins=64, sah=True, device_build=False, force_2level=False, force_flat=False,
               world_to_local=None):
    """mcrt_accel_opts; device_build: 0/False (default) or 2 the RadeonRays-identical tree built on
    the device, 3 the same tree built on the host, 1/True device LBVH; world_to_local: optional (num_shapes, 4, 4) float32 array (kept alive by
    the caller until the build returns)."""
    w2l = None if world_to_local is None else world_to_local.ctypes.data
    return T.AccelOpts(cost, bins, 1 if sah else 0, int(device_build), 1 if force_2level else 0,
                       1 if force_flat else 0, w2l)


def event_wait(ev):
    _check(lib().mcrt_event_wait(ev))


def event_destroy(ev):
    _check(lib().mcrt_event_destroy(ev))


def build_host_records(scene, **opts):
    """Host-only build (no GPU): (records float32 (n, 16), info dict) of the structure
    mcrt_accel_build would upload for `scene` (mcrt.scenes.Scene)."""
    desc = scene.desc()
    w2l = opts.get("world_to_local")
    if w2l is not None:
        opts["world_to_local"] = np.ascontiguousarray(w2l, np.float32)
    o = accel_opts(**opts)
    n = _c.c_uint64()
    _check(lib().mcrt_accel_build_host_records(_c.byref(desc), _c.byref(o), None, 0, _c.byref(n), None))
    rec = np.zeros((n.value, 16), np.float32)
    info = np.zeros(4, np.int32)
    _check(lib().mcrt_accel_build_host_records(_c.byref(desc), _c.byref(o), _p(rec), n.value, _c.byref(n), _p(info)))
    return rec, {"two_level": int(info[0]), "top_records": int(info[1]), "depth": int(info[2]),
                 "meshes": int(info[3])}


class DeviceScene:
    def __init__(self, ctx, scene, build=True, cost=10.0, bins=64, sah=True, device_build=False,
                 force_2level=False, force_flat=False, world_to_local=None):
        self.ctx = ctx
        self.scene = scene
        self._desc = scene.desc()
        h = _vp()
        _check(lib().mcrt_scene_create(ctx.h, _c.byref(self._desc), _c.byref(h)), ctx.h)
        self.h = h
        ctx._adopt(self)
        if build:
            self.build(cost, bins, sah, device_build, force_2level, force_flat, world_to_local)

    def build(self, cost=10.0, bins=64, sah=True, device_build=False, force_2level=False, force_flat=False,
              world_to_local=None):
        w2l = None if world_to_local is None else np.ascontiguousarray(world_to_local, np.float32)
        opts = accel_opts(cost, bins, sah, device_build, force_2level, force_flat, w2l)
        _check(lib().mcrt_accel_build(self.h, _c.byref(opts)), self.ctx.h)

    def layout(self):
        tl, nm, ni, dp = _c.c_int32(), _c.c_uint32(), _c.c_uint32(), _c.c_int32()
        _check(lib().mcrt_accel_layout(self.h, _c.byref(tl), _c.byref(nm), _c.byref(ni), _c.byref(dp)), self.ctx.h)
        return {"two_level": tl.value, "meshes": nm.value, "instances": ni.value, "depth": dp.value}

    def records(self):
        """The device's BVH records, float32 (n, 16) (mcrt_accel_read_records)."""
        n = _c.c_uint64()
        _check(lib().mcrt_accel_read_records(self.h, None, 0, _c.byref(n)), self.ctx.h)
        rec = np.zeros((n.value, 16), np.float32)
        _check(lib().mcrt_accel_read_records(self.h, _p(rec), n.value, _c.byref(n)), self.ctx.h)
        return rec

    def builder(self):
        """0 host build (or two-level), 1 device LBVH, 2 device SAH (mcrt_accel_builder)."""
        b = _c.c_int32()
        _check(lib().mcrt_accel_builder(self.h, _c.byref(b)), self.ctx.h)
        return b.value

    def info(self):
        nn, nb, ms, nt = _c.c_uint64(), _c.c_uint64(), _c.c_double(), _c.c_uint32()
        _check(lib().mcrt_accel_info(self.h, _c.byref(nn), _c.byref(nb), _c.byref(ms), _c.byref(nt)), self.ctx.h)
        return {"nodes": nn.value, "bytes": nb.value, "build_ms": ms.value, "triangles": nt.value}

    def update_lights(self, lights):
        self._lights = np.ascontiguousarray(lights)
        _check(lib().mcrt_scene_update_lights(self.h, _p(self._lights), len(self._lights)), self.ctx.h)

    def update_materials(self, mats):
        self._mats = np.ascontiguousarray(mats)
        _check(lib().mcrt_scene_update_materials(self.h, _p(self._mats), len(self._mats)), self.ctx.h)

    def update_shapes(self, shapes):
        """mcrt_scene_update_shapes (same topology; call build() after a transform change)."""
        self._shapes = np.ascontiguousarray(shapes)
        _check(lib().mcrt_scene_update_shapes(self.h, _p(self._shapes), len(self._shapes)), self.ctx.h)

    def trace_closest(self, rays_dev_ptr, n, hits_dev_ptr):
        _check(lib().mcrt_trace_closest(self.h, rays_dev_ptr, n, hits_dev_ptr), self.ctx.h)

    def trace_any(self, rays_dev_ptr, n, out_dev_ptr):
        _check(lib().mcrt_trace_any(self.h, rays_dev_ptr, n, out_dev_ptr), self.ctx.h)

    def trace_count(self, any_hit, rays_dev_ptr, count_dev_ptr, maxrays, out_dev_ptr, wait_event=None,
                    want_event=False):
        """mcrt_trace_closest_count / mcrt_trace_any_count: min(*count, maxrays) rays, the count in
        device memory; waits for wait_event; returns the done event (a handle for event_wait /
        event_destroy) when want_event."""
        ev = _vp()
        f = lib().mcrt_trace_any_count if any_hit else lib().mcrt_trace_closest_count
        _check(f(self.h, rays_dev_ptr, count_dev_ptr, maxrays, out_dev_ptr, wait_event,
                 _c.byref(ev) if want_event else None), self.ctx.h)
        return ev.value if want_event else None

    def close(self):
        if self.h:
            lib().mcrt_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FrameBuffer:
    def __init__(self, ctx, width, height):
        self.ctx = ctx
        self.W, self.H = width, height
        h = _vp()
        _check(lib().mcrt_framebuffer_create(ctx.h, width, height, _c.byref(h)), ctx.h)
        self.h = h
        ctx._adopt(self)

    def set_frames_in_flight(self, n):
        """mcrt_framebuffer_set_frames_in_flight: 0 = auto (2 slots)."""
        _check(lib().mcrt_framebuffer_set_frames_in_flight(self.h, n), self.ctx.h)

    def render(self, dscene, cam, frame=0, max_depth=2, sampler=T.SAMPLER_RANDOM, rr=False, rr_start=3,
               band_rows=8, num_bands=1, band_index=0, integrator=T.INTEGRATOR_PT, texture_lod=False):
        p = T.FrameParams(frame, max_depth, sampler, 1 if rr else 0, rr_start, band_rows, num_bands, band_index,
                          integrator, 1 if texture_lod else 0)
        cam = np.ascontiguousarray(cam)
        _check(lib().mcrt_render_frame(dscene.h, self.h, _p(cam), _c.byref(p)), self.ctx.h)

    def render_frames(self, dscene, cams, frame=0, max_depth=2, sampler=T.SAMPLER_RANDOM, rr=False, rr_start=3,
                      band_rows=8, num_bands=1, band_index=0, integrator=T.INTEGRATOR_PT):
        """mcrt_render_frames: len(cams) consecutive frames frame, frame+1, ... in one pass (PT or BDPT)."""
        p = T.FrameParams(frame, max_depth, sampler, 1 if rr else 0, rr_start, band_rows, num_bands, band_index,
                          integrator, 0)
        cams = _records(cams)
        _check(lib().mcrt_render_frames(dscene.h, self.h, _p(cams), len(cams), _c.byref(p)), self.ctx.h)

    def accumulate_frames(self, filters, frame):
        """mcrt_accumulate_frames: one filter per frame of the last render_frames (or one shared)."""
        filters = _records(filters)
        _check(lib().mcrt_accumulate_frames(self.h, _p(filters), len(filters), frame), self.ctx.h)

    def render_aov(self, dscene, cam, aov=T.AOV_ALBEDO, texture_lod=False):
        """mcrt_render_aov: (H, W, 4) albedo or (H, W, 3, 4) texture-footprint records."""
        p = T.FrameParams(0, 1, T.SAMPLER_RANDOM, 0, 3, 8, 1, 0, T.INTEGRATOR_PT, 1 if texture_lod else 0)
        cam = np.ascontiguousarray(cam)
        shape = (self.H, self.W, 3, 4) if aov == T.AOV_TEXTURE_LOD else (self.H, self.W, 4)
        out = np.zeros(shape, np.float32)
        _check(lib().mcrt_render_aov(dscene.h, self.h, _p(cam), _c.byref(p), aov, _p(out)), self.ctx.h)
        return out

    def accumulate(self, filt, frame):
        filt = np.ascontiguousarray(filt)
        _check(lib().mcrt_accumulate(self.h, _p(filt), frame), self.ctx.h)

    def postprocess(self, denoise=False, radius=1, sigma_spatial=1.0, sigma_range=0.1, tonemap=False,
                    min_luminance=2.0):
        """RTDenoisePass + RTToneMappingPass on the accumulated image -> read(3)."""
        p = T.PostprocessParams(1 if denoise else 0, radius, sigma_spatial, sigma_range, 1 if tonemap else 0,
                                min_luminance)
        _check(lib().mcrt_postprocess(self.h, _c.byref(p)), self.ctx.h)

    def read(self, which=0):
        out = np.zeros((self.H, self.W, 4), np.float32)
        _check(lib().mcrt_framebuffer_read(self.h, which, _p(out)), self.ctx.h)
        return out

    def read_frame(self, k):
        """Radiance of frame k of the last render_frames batch (mcrt_framebuffer_read_frame)."""
        out = np.zeros((self.H, self.W, 4), np.float32)
        _check(lib().mcrt_framebuffer_read_frame(self.h, k, _p(out)), self.ctx.h)
        return out

    def device_ptrs(self):
        r, s, w, i = _vp(), _vp(), _vp(), _vp()
        _check(lib().mcrt_framebuffer_device_ptrs(self.h, _c.byref(r), _c.byref(s), _c.byref(w), _c.byref(i)),
               self.ctx.h)
        return r.value, s.value, w.value, i.value

    def copy_device(self, which, dst_ptr):
        _check(lib().mcrt_framebuffer_copy_device(self.h, which, dst_ptr), self.ctx.h)

    def bdpt_splat_layout(self):
        """(chunk_pixels, chunks) of the rank-major splat layout of the last band split."""
        cp, ch = _c.c_uint64(), _c.c_int32()
        _check(lib().mcrt_bdpt_splat_layout(self.h, _c.byref(cp), _c.byref(ch)), self.ctx.h)
        return cp.value, ch.value

    def stream(self):
        """hipStream_t (int) of the last frame's slot (mcrt_framebuffer_stream)."""
        st = _vp()
        _check(lib().mcrt_framebuffer_stream(self.h, _c.byref(st)), self.ctx.h)
        return st.value or 0

    def bdpt_splats_copy(self, dst_ptr):
        """Band-split BDPT: this rank's light-tracing splats, rank-major (chunks x chunk_pixels
        float4), into device memory."""
        _check(lib().mcrt_bdpt_splats_copy(self.h, dst_ptr), self.ctx.h)

    def bdpt_gather(self, own_chunk_ptr=None):
        """Completes a band-split BDPT frame with this rank's chunk of the summed splats (None:
        the rank's own splats)."""
        _check(lib().mcrt_bdpt_gather(self.h, own_chunk_ptr), self.ctx.h)

    def set_splat_exchange(self, sparse):
        """Band-split BDPT: the sparse (record lists, one all-to-all) or the dense (rank-major
        planes, one reduce-scatter) splat exchange for the frames rendered from now on."""
        _check(lib().mcrt_framebuffer_set_splat_exchange(self.h, 1 if sparse else 0), self.ctx.h)

    def bdpt_splats_sparse(self, dst_ptr=None, capacity=0):
        """Sparse exchange: per-rank record counts of this rank's splats into other ranks' rows
        (waits for the frame's visibility pass); with dst_ptr also groups the records (4 floats
        each) by rank into device memory on the frame's stream.  Returns an int64 array."""
        n = self.bands_count()
        counts = (_c.c_int64 * n)()
        _check(lib().mcrt_bdpt_splats_sparse(self.h, dst_ptr, capacity, counts, n), self.ctx.h)
        return np.array(counts, np.int64)

    def bdpt_gather_sparse(self, recv_ptr, records):
        """Sparse exchange: adds the received records and completes the rank's bands."""
        _check(lib().mcrt_bdpt_gather_sparse(self.h, recv_ptr, int(records)), self.ctx.h)

    def bands_count(self):
        """Bands (ranks) of the last frame's split."""
        return int(self.band_layout()[1])

    def set_accumulation(self, wsum_ptr, wts_ptr):
        _check(lib().mcrt_framebuffer_set_accumulation(self.h, wsum_ptr, wts_ptr), self.ctx.h)

    def bands_pack(self, dst_ptr):
        """mcrt_framebuffer_bands_pack: this rank's rows of the accumulators, packed (5 W floats a row)."""
        _check(lib().mcrt_framebuffer_bands_pack(self.h, dst_ptr), self.ctx.h)

    def bands_unpack(self, recv_ptr, max_rows):
        """mcrt_framebuffer_bands_unpack: the other ranks' packed rows into the accumulators + image."""
        _check(lib().mcrt_framebuffer_bands_unpack(self.h, recv_ptr, max_rows), self.ctx.h)

    def band_layout(self):
        """(max_rows, num_bands, band_index) of the last render (mcrt_framebuffer_band_layout)."""
        a, b, c = _c.c_int32(), _c.c_int32(), _c.c_int32()
        _check(lib().mcrt_framebuffer_band_layout(self.h, _c.byref(a), _c.byref(b), _c.byref(c)), self.ctx.h)
        return a.value, b.value, c.value

    def stats(self):
        a, b, c = _c.c_int64(), _c.c_int64(), _c.c_int64()
        _check(lib().mcrt_framebuffer_stats(self.h, _c.byref(a), _c.byref(b), _c.byref(c)), self.ctx.h)
        return {"closest_rays": a.value, "any_rays": b.value, "shaded_paths": c.value}

    def queue_counts(self, max_bounces=8):
        """(shadow[b], extension[b]) queue sizes of the last PT render."""
        sh = (_c.c_int32 * max_bounces)()
        ex = (_c.c_int32 * max_bounces)()
        _check(lib().mcrt_framebuffer_queue_counts(self.h, sh, ex, max_bounces), self.ctx.h)
        return list(sh), list(ex)

    def hint_counts(self, max_bounces=8):
        """hits[b]: shadow rays of bounce b answered by their occluder hint in the last PT render."""
        h = (_c.c_int32 * max_bounces)()
        _check(lib().mcrt_framebuffer_hint_counts(self.h, h, max_bounces), self.ctx.h)
        return list(h)

    def retrace_counts(self, max_bounces=8):
        """retraces[b]: rays traced for bounce b+1 whose compact-record walk ended on a near tie and
        was repeated on the exact records, in the last PT render (counted at profiling level 2)."""
        h = (_c.c_int32 * max_bounces)()
        _check(lib().mcrt_framebuffer_retrace_counts(self.h, h, max_bounces), self.ctx.h)
        return list(h)

    def wave_clock(self, which):
        """(blocks, 2) uint32 (start, end) 100-MHz clocks of the last PT call's launch `which` (0 camera,
        1 shadow + extension, 2 last shadow); needs MCRT_WAVE_CLOCK=1 (diagnostics)."""
        n = _c.c_int64()
        _check(lib().mcrt_framebuffer_wave_clock(self.h, which, None, 0, _c.byref(n)), self.ctx.h)
        out = np.zeros((n.value, 2), np.uint32)
        if n.value:
            _check(lib().mcrt_framebuffer_wave_clock(self.h, which, _p(out), n.value, _c.byref(n)), self.ctx.h)
        return out

    def read_queue(self, which):
        """(a, b, c) float4 arrays of the last bounce's shadow (0) / extension (1) queue."""
        cnt = _c.c_int32()
        _check(lib().mcrt_framebuffer_read_queue(self.h, which, None, 0, _c.byref(cnt)), self.ctx.h)
        n = cnt.value
        out = np.zeros((3, max(n, 1), 4), np.float32)
        _check(lib().mcrt_framebuffer_read_queue(self.h, which, _p(out), max(n, 1), _c.byref(cnt)), self.ctx.h)
        return out[0, :n], out[1, :n], out[2, :n]

    BDPT_READ = {"camera_vertices": 0, "light_vertices": 1, "camera_counts": 2, "light_counts": 3,
                 "slots": 4, "sampled_light": 5, "splat": 6}

    def read_bdpt(self, which):
        """Raw bytes of a BDPT state array of the last BDPT frame (mcrt_framebuffer_read_bdpt)."""
        need = _c.c_uint64()
        idx = self.BDPT_READ[which]
        _check(lib().mcrt_framebuffer_read_bdpt(self.h, idx, None, 0, _c.byref(need)), self.ctx.h)
        out = np.zeros(need.value, np.uint8)
        _check(lib().mcrt_framebuffer_read_bdpt(self.h, idx, _p(out), need.value, _c.byref(need)), self.ctx.h)
        return out

    def close(self):
        if self.h:
            lib().mcrt_framebuffer_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def load_obj(path, mips=True, emissive_lights=True, directional_lights=(), point_lights=()):
    """Scene ingestion through the C ABI (mcrt_obj_load, csrc/mcrt_objload.cpp): returns a
    mcrt.scenes.Scene holding copies of the loader's arrays and the loader's warnings.
    directional_lights / point_lights: [(direction or position, intensity)] added after the
    emissive-material lights, as a host adds the demo sun."""
    from .scenes import Scene
    h = _vp()
    flags = (T.OBJ_MIPS if mips else 0) | (T.OBJ_EMISSIVE_LIGHTS if emissive_lights else 0)
    _check(lib().mcrt_obj_load(os.fsencode(path), flags, _c.byref(h)))
    try:
        f3 = lambda v: (_c.c_float * 3)(*[float(x) for x in v])   # noqa: E731
        for d, it in directional_lights:
            _check(lib().mcrt_obj_add_directional_light(h, f3(d), f3(it)))
        for p, it in point_lights:
            _check(lib().mcrt_obj_add_point_light(h, f3(p), f3(it)))
        d = T.SceneDesc()
        _check(lib().mcrt_obj_scene_desc(h, _c.byref(d)))

        def arr(ptr, n, dtype, shape=None):
            dtype = np.dtype(dtype)
            if not n or not ptr:
                return np.zeros((0,) + (shape or ()), dtype)
            a = np.frombuffer(_c.string_at(ptr, n * dtype.itemsize), dtype).copy()
            return a.reshape((n,) + shape) if shape else a
        nv = d.num_vertices
        sc = Scene(arr(d.shapes, d.num_shapes, T.SHAPE_DTYPE), arr(d.indices, d.num_indices, np.uint32),
                   arr(d.positions, nv * 4, np.float32).reshape(-1, 4), arr(d.uvs, nv * 2, np.float32).reshape(-1, 2),
                   arr(d.normals, nv * 4, np.float32).reshape(-1, 4), arr(d.tangents, nv * 4, np.float32).reshape(-1, 4),
                   arr(d.binormals, nv * 4, np.float32).reshape(-1, 4), None,
                   arr(d.textures, d.num_textures, T.TEXDESC_DTYPE), arr(d.tex_data, d.tex_data_bytes, np.uint8),
                   arr(d.lights, d.num_lights, T.LIGHT_DTYPE), arr(d.materials, d.num_materials, T.MATERIAL_DTYPE),
                   name=os.path.splitext(os.path.basename(path))[0])
        sc.warnings = lib().mcrt_obj_warnings(h).decode()
        return sc
    finally:
        lib().mcrt_obj_free(h)


def make_pinhole_camera(pos, forward, up, fovy, near, far, width, height, pixel_offset=(0.0, 0.0)):
    cam = np.zeros(1, T.CAMERA_DTYPE)
    a = [np.asarray(v, np.float32) for v in (pos, forward, up, pixel_offset)]
    _check(lib().mcrt_make_pinhole_camera(_p(a[0]), _p(a[1]), _p(a[2]), fovy, near, far, width, height, _p(a[3]),
                                          _p(cam)))
    return cam


def make_pinhole_camera_axes(pos, right, up, look, fovy_rad, near, far, width, height, pixel_offset=(0.0, 0.0)):
    """mcrt_make_pinhole_camera_axes: the reference host's RTPinholeCamera, bit for bit."""
    cam = np.zeros(1, T.CAMERA_DTYPE)
    a = [np.asarray(v, np.float32) for v in (pos, right, up, look, pixel_offset)]
    _check(lib().mcrt_make_pinhole_camera_axes(_p(a[0]), _p(a[1]), _p(a[2]), _p(a[3]), fovy_rad, near, far, width,
                                               height, _p(a[4]), _p(cam)))
    return cam


def taa_pixel_offset(sobol_matrices, frame, radius=(2.0, 2.0)):
    """mcrt_taa_pixel_offset: the reference's per-frame TAA jitter in pixels."""
    m = np.ascontiguousarray(sobol_matrices, np.uint32)
    out = np.zeros(2, np.float32)
    _check(lib().mcrt_taa_pixel_offset(_p(m), frame, radius[0], radius[1], _p(out)))
    return out


def header_symbols():
    """Entry points declared in include/mcrt_capi.h (MCRT_API lines)."""
    import re
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"MCRT_API\s+[\w\s\*]+?\b(mcrt_\w+)\s*\(", txt)))

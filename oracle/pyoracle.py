"""TEST INFRASTRUCTURE ONLY: ctypes bindings of the oracle (CPU restatement,
oracle/libmcrt_oracle.so) and of oracle/_ref (the reference's own RadeonRays
sources compiled in place, oracle/_ref/librrref.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_c = ctypes
_vp = _c.c_void_p


def _load(path):
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} not built (run __graft_entry__.build() or make -C oracle)")
    return _c.CDLL(path)


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = _load(os.path.join(HERE, "libmcrt_oracle.so"))
        L.orc_wang_hash.restype = _c.c_uint32
        L.orc_wang_hash.argtypes = [_c.c_uint32]
        L.orc_xorshift.restype = _c.c_uint32
        L.orc_xorshift.argtypes = [_c.POINTER(_c.c_uint32)]
        L.orc_rand_float.restype = _c.c_float
        L.orc_rand_float.argtypes = [_c.POINTER(_c.c_uint32)]
        L.orc_sobol_sample.restype = _c.c_float
        L.orc_sobol_sample.argtypes = [_c.c_uint32, _c.c_uint32, _c.c_uint32, _vp]
        L.orc_sampler_draws.argtypes = [_c.c_int, _c.c_uint32, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _vp, _vp]
        L.orc_scene_create.restype = _vp
        L.orc_scene_create.argtypes = [_vp]
        L.orc_scene_destroy.argtypes = [_vp]
        L.orc_bvh_build.restype = _c.c_int64
        L.orc_bvh_build.argtypes = [_vp, _c.c_float, _c.c_int, _c.c_int]
        L.orc_bvh_nodes.restype = _c.c_int64
        L.orc_bvh_nodes.argtypes = [_vp, _vp, _c.c_int64]
        L.orc_trace_closest.argtypes = [_vp, _vp, _c.c_int, _vp, _vp, _c.c_int]
        L.orc_trace_any.argtypes = [_vp, _vp, _c.c_int, _vp, _vp, _c.c_int]
        L.orc_brute_closest.argtypes = [_vp, _vp, _c.c_int, _vp]
        L.orc_tie_premise.argtypes = [_vp, _vp, _c.c_int, _c.c_float, _vp, _c.c_int]
        L.orc_brute_any.argtypes = [_vp, _vp, _c.c_int, _vp]
        L.orc_render_frame.argtypes = [_vp, _vp, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _vp, _vp]
        L.orc_set_touched.argtypes = [_vp, _vp]
        L.orc_set_pathlog.argtypes = [_vp, _vp, _c.c_int]
        L.orc_bdpt_create.restype = _vp
        L.orc_bdpt_create.argtypes = [_c.c_int, _c.c_int, _c.c_int]
        L.orc_bdpt_destroy.argtypes = [_vp]
        L.orc_bdpt_render.argtypes = [_vp, _vp, _vp, _c.c_int, _c.c_int, _vp, _c.c_int, _c.c_int, _vp, _vp, _vp, _vp]
        L.orc_render_rows.argtypes = [_vp, _vp, _c.c_int, _c.c_int, _c.c_int, _vp, _c.c_int, _c.c_int, _vp, _vp]
        L.orc_accumulate.argtypes = [_c.c_int, _c.c_int, _c.c_int, _vp, _vp, _vp, _vp, _vp]
        L.orc_accumulate_w.argtypes = [_c.c_int, _c.c_int, _c.c_int, _c.c_float, _vp, _vp, _vp, _vp]
        L.orc_denoise.argtypes = [_c.c_int, _c.c_int, _c.c_int, _c.c_float, _c.c_float, _vp, _vp]
        L.orc_tonemap.argtypes = [_c.c_int, _c.c_int, _c.c_float, _vp, _vp]
        L.orc_sample_uber.argtypes = [_vp] * 6 + [_c.c_float, _vp, _vp, _vp]
        L.orc_eval_uber.argtypes = [_vp] * 5 + [_c.c_float, _vp, _vp, _vp]
        L.orc_pdf_uber.restype = _c.c_float
        L.orc_pdf_uber.argtypes = [_vp] * 6 + [_c.c_float, _vp, _vp]
        L.orc_roughness_to_alpha.restype = _c.c_float
        L.orc_roughness_to_alpha.argtypes = [_c.c_float]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class OracleScene:
    """Oracle view of an mcrt.scenes.Scene (keeps the numpy arrays alive)."""

    def __init__(self, scene):
        self.scene = scene
        self._desc = scene.desc()
        self.h = lib().orc_scene_create(ctypes.byref(self._desc))
        self.num_nodes = 0

    def __del__(self):
        try:
            if self.h:
                lib().orc_scene_destroy(self.h)
        except Exception:
            pass

    def build(self, cost=10.0, bins=64, sah=True):
        self.num_nodes = lib().orc_bvh_build(self.h, cost, bins, 1 if sah else 0)
        return self.num_nodes

    def nodes(self):
        from mcrt.types import RRNODE_DTYPE
        out = np.zeros(self.num_nodes, RRNODE_DTYPE)
        lib().orc_bvh_nodes(self.h, _p(out), self.num_nodes)
        return out

    def closest(self, rays, threads=8, visits=False):
        from mcrt.types import ISECT_DTYPE
        hits = np.zeros(len(rays), ISECT_DTYPE)
        hits["shapeid"] = -7
        hits["primid"] = -7
        v = np.zeros(len(rays), np.int32) if visits else None
        lib().orc_trace_closest(self.h, _p(rays), len(rays), _p(hits), _p(v), threads)
        return (hits, v) if visits else hits

    def any(self, rays, threads=8, visits=False):
        out = np.full(len(rays), -7, np.int32)
        v = np.zeros(len(rays), np.int32) if visits else None
        lib().orc_trace_any(self.h, _p(rays), len(rays), _p(out), _p(v), threads)
        return (out, v) if visits else out

    def tie_premise(self, rays, alpha=2.0 ** -18, threads=8):
        """Per ray (n, 6) float32: the reference walk's distance, the largest relative gap of an
        order-dependent hit pair (-1: none), the largest relative irregularity of a hit's leaf box
        entry, hits enumerated, irregular hits, incomplete flag (orc_tie_premise in mcrt_oracle.c)."""
        out = np.zeros((len(rays), 6), np.float32)
        lib().orc_tie_premise(self.h, _p(rays), len(rays), alpha, _p(out), threads)
        return out

    def brute_closest(self, rays):
        from mcrt.types import ISECT_DTYPE
        hits = np.zeros(len(rays), ISECT_DTYPE)
        lib().orc_brute_closest(self.h, _p(rays), len(rays), _p(hits))
        return hits

    def brute_any(self, rays):
        out = np.zeros(len(rays), np.int32)
        lib().orc_brute_any(self.h, _p(rays), len(rays), _p(out))
        return out

    def render(self, cam, frame=0, max_depth=2, sampler=1, y0=0, y1=None, threads=8, radiance=None):
        W, H = int(cam["width"][0]), int(cam["height"][0])
        if y1 is None:
            y1 = H
        if radiance is None:
            radiance = np.zeros((H, W, 4), np.float32)
        stats = np.zeros(8, np.int64)
        lib().orc_render_frame(self.h, _p(cam), frame, max_depth, sampler, y0, y1, threads, _p(radiance), _p(stats))
        return radiance, stats

    def track_touched(self, on=True):
        """Marks every BVH node later renders visit, per query class (bench.py's compulsory-traffic
        roofline): returns the (4, num_nodes) uint8 array -- rows camera, extension, shadow of
        bounce 0, later shadow rays -- or None when switched off."""
        if not on:
            lib().orc_set_touched(self.h, None)
            self._touched = None
            return None
        self._touched = np.zeros((4, self.num_nodes), np.uint8)
        lib().orc_set_touched(self.h, _p(self._touched))
        return self._touched

    PATHLOG_FLOATS = 32   # ORC_PATHLOG_FLOATS (mcrt_oracle.h)

    def path_log(self, W=None, H=None, depth=2):
        """Per-pixel path records of later PT renders (divergence diagnostics): returns the
        (H*W, depth, 32) float32 array the renders fill (layout in mcrt_oracle.h), or switches the
        log off when W is None."""
        if W is None:
            lib().orc_set_pathlog(self.h, None, 0)
            self._pathlog = None
            return None
        self._pathlog = np.zeros((H * W, depth, self.PATHLOG_FLOATS), np.float32)
        lib().orc_set_pathlog(self.h, _p(self._pathlog), depth)
        return self._pathlog

    def render_rows(self, cam, rows, frame=0, max_depth=2, sampler=1, threads=8, radiance=None):
        W, H = int(cam["width"][0]), int(cam["height"][0])
        rows = np.ascontiguousarray(rows, np.int32)
        if radiance is None:
            radiance = np.zeros((H, W, 4), np.float32)
        stats = np.zeros(8, np.int64)
        lib().orc_render_rows(self.h, _p(cam), frame, max_depth, sampler, _p(rows), len(rows), threads,
                              _p(radiance), _p(stats))
        return radiance, stats


class OracleBDPT:
    """The oracle's BDPT (KRN/BDPT.cl restated in oracle/mcrt_oracle.c) on an OracleScene: keeps
    the per-pixel sampled-light-vertex state the s = 1 strategy carries from frame to frame
    (BDPT.cl:585-586), zero-filled at creation like the reference runner's buffers."""

    def __init__(self, oscene, W, H, max_depth=2):
        self.o, self.W, self.H, self.D = oscene, W, H, max_depth
        self.h = lib().orc_bdpt_create(W, H, max_depth)

    def __del__(self):
        try:
            if self.h:
                lib().orc_bdpt_destroy(self.h)
        except Exception:
            pass

    def render(self, cam, frame=0, sampler=1, rows=None, threads=8):
        """One frame -> (radiance (H, W, 4), camera counts, light counts, stats[4] = subpath rays,
        their node visits, connection rays, their node visits).  rows: render only these rows'
        subpaths (their light-tracing splats still land anywhere)."""
        assert int(cam["width"][0]) == self.W and int(cam["height"][0]) == self.H
        rad = np.zeros((self.H, self.W, 4), np.float32)
        cc = np.zeros(self.W * self.H, np.int32)
        lc = np.zeros(self.W * self.H, np.int32)
        st = np.zeros(4, np.int64)
        r = None if rows is None else np.ascontiguousarray(rows, np.int32)
        lib().orc_bdpt_render(self.o.h, self.h, _p(cam), frame, sampler, _p(r), 0 if r is None else len(r), threads,
                              _p(rad), _p(cc), _p(lc), _p(st))
        return rad, cc, lc, st


def accumulate(radiance, frame, filt, wsum=None, wts=None):
    H, W = radiance.shape[:2]
    if wsum is None:
        wsum = np.zeros((H, W, 4), np.float32)
        wts = np.zeros((H, W), np.float32)
    image = np.zeros((H, W, 4), np.float32)
    lib().orc_accumulate(W, H, frame, _p(filt), _p(radiance), _p(wsum), _p(wts), _p(image))
    return wsum, wts, image


def accumulate_w(radiance, frame, w, wsum=None, wts=None):
    """ReconstructionPass for one frame with an explicit filter weight w (orc_accumulate_w)."""
    radiance = np.ascontiguousarray(radiance, np.float32)
    H, W = radiance.shape[:2]
    if wsum is None:
        wsum = np.zeros((H, W, 4), np.float32)
        wts = np.zeros((H, W), np.float32)
    image = np.zeros((H, W, 4), np.float32)
    lib().orc_accumulate_w(W, H, frame, float(w), _p(radiance), _p(wsum), _p(wts), _p(image))
    return wsum, wts, image


def denoise(img, radius, sigma_spatial, sigma_range):
    """BilateralDenoise (Denoise.cl:6-47) on an (H, W, 4) float32 image."""
    img = np.ascontiguousarray(img, np.float32)
    out = img.copy()
    lib().orc_denoise(img.shape[1], img.shape[0], radius, sigma_spatial, sigma_range, _p(img), _p(out))
    return out


def tonemap(img, l_white):
    """ReinhardToneMapping (ToneMapping.cl:42-63) on an (H, W, 4) float32 image."""
    img = np.ascontiguousarray(img, np.float32)
    out = np.empty_like(img)
    lib().orc_tonemap(img.shape[1], img.shape[0], l_white, _p(img), _p(out))
    return out


def wang_hash(x):
    return lib().orc_wang_hash(x)


def sampler_draws(kind, pix, frame, bounce, W, H, sobol=None):
    out = np.zeros(5, np.float32)
    lib().orc_sampler_draws(kind, pix, frame, bounce, W, H, _p(sobol), _p(out))
    return out


def sample_uber(kd, ks, kr, kt, alpha, opacity, eta, wo, u):
    a = [np.asarray(x, np.float32) for x in (kd, ks, kr, kt, alpha, opacity)]
    wo = np.asarray(wo, np.float32)
    u = np.asarray(u, np.float32)
    out = np.zeros(8, np.float32)
    lib().orc_sample_uber(*[_p(x) for x in a], eta, _p(wo), _p(u), _p(out))
    return out


# --------------------------------------------------------------------------
# oracle/_ref: the reference's own RadeonRays C++ (bvh2.cpp, mesh.cpp, utils.cpp)
# --------------------------------------------------------------------------
REF_LIB = os.path.join(HERE, "_ref", "librrref.so")
_ref = None


def ref_available():
    return os.path.exists(REF_LIB)


def ref():
    global _ref
    if _ref is None:
        L = _load(REF_LIB)
        L.rr_bvh_build.restype = _c.c_int64
        L.rr_bvh_build.argtypes = [_c.c_int, _vp, _vp, _c.c_int, _vp, _vp, _vp, _c.c_float, _c.c_int, _c.c_int,
                                   _vp, _c.c_int64]
        L.rr_test_intersections.argtypes = [_c.c_int, _vp, _vp, _c.c_int, _vp, _vp, _vp, _vp, _c.c_int, _vp]
        L.rr_test_occlusions.argtypes = [_c.c_int, _vp, _vp, _c.c_int, _vp, _vp, _vp, _vp, _c.c_int, _vp]
        L.rr_load_obj.restype = _vp
        L.rr_load_obj.argtypes = [_c.c_char_p, _c.c_char_p]
        L.rr_obj_num_shapes.restype = _c.c_int
        L.rr_obj_num_shapes.argtypes = [_vp]
        L.rr_obj_shape.argtypes = [_vp, _c.c_int, _vp, _vp, _vp, _vp]
        L.rr_obj_free.argtypes = [_vp]
        L.rr2l_build.restype = _vp
        L.rr2l_build.argtypes = [_c.c_int, _vp, _vp, _vp, _vp, _vp, _c.c_float, _c.c_int, _c.c_int]
        L.rr2l_sizes.argtypes = [_vp, _vp]
        L.rr2l_copy.argtypes = [_vp, _vp, _vp, _vp, _vp]
        L.rr2l_free.argtypes = [_vp]
        _ref = L
    return _ref


class _RefShapes:
    """Per-shape arrays of an mcrt.scenes.Scene in the layout RadeonRays' CreateMesh takes."""

    def __init__(self, scene):
        self.P, self.I, self.M = [], [], []
        for s in scene.shapes:
            v0, n = int(s["startVertex"]), 0
            idx = scene.indices[s["startIdx"]: s["startIdx"] + 3 * s["numTriangles"]].astype(np.int32)
            n = int(idx.max()) + 1 if idx.size else 0
            self.P.append(np.ascontiguousarray(scene.positions[v0:v0 + n]))   # stride 16
            self.I.append(np.ascontiguousarray(idx))
            self.M.append(s["toWorldTransform"].astype(np.float32))
        self.nv = np.array([p.shape[0] for p in self.P], np.int32)
        self.nf = np.array([i.size // 3 for i in self.I], np.int32)
        self.pp = (_c.c_void_p * len(self.P))(*[p.ctypes.data for p in self.P])
        self.ip = (_c.c_void_p * len(self.I))(*[i.ctypes.data for i in self.I])
        self.mt = np.ascontiguousarray(np.stack(self.M)) if self.M else np.zeros((0, 4, 4), np.float32)

    def args(self):
        return (len(self.P), self.pp, _p(self.nv), 16, self.ip, _p(self.nf), _p(self.mt))


# IntersectorTwoLevel's buffers (intersect_bvh2level_skiplinks.cl kernel arguments)
RR2L_SHAPE_DTYPE = np.dtype([("id", "<i4"), ("bvhidx", "<i4"), ("shapeDisabled", "<u4"), ("padding1", "<i4"),
                             ("minv", "<f4", (4, 4)), ("lv", "<f4", 4), ("av", "<f4", 4)])
RR2L_FACE_DTYPE = np.dtype([("idx", "<i4", 3), ("shape_id", "<i4"), ("prim_id", "<i4")])


def ref_bvh2l(scene, world_to_local=None, cost=10.0, bins=64, sah=True):
    """The reference's two-level structure for `scene` (oracle/_ref/librrref.so: RR Bvh +
    PlainBvhTranslator run by the Process mirror in rrref_driver.cpp).  world_to_local:
    (S, 4, 4) float32 (default: transpose of toWorldInverseTranspose, as the product's default).
    Returns dict(nodes (K, 8) float32 = bbox pmin/pmax xyzw, vertices (V, 4), faces, shapes, root,
    meshes, instances)."""
    sh = scene.shapes
    keys = np.ascontiguousarray(np.stack([sh["startIdx"], sh["startVertex"], sh["numTriangles"]], 1).astype(np.uint32))
    m = np.ascontiguousarray(sh["toWorldTransform"].astype(np.float32))
    if world_to_local is None:
        world_to_local = np.transpose(sh["toWorldInverseTranspose"], (0, 2, 1))
    minv = np.ascontiguousarray(world_to_local, np.float32)
    idx = np.ascontiguousarray(scene.indices, np.uint32)
    pos = np.ascontiguousarray(scene.positions, np.float32)
    L = ref()
    h = L.rr2l_build(len(sh), _p(keys), _p(m), _p(minv), _p(idx), _p(pos), cost, bins, 1 if sah else 0)
    try:
        sz = np.zeros(7, np.int64)
        L.rr2l_sizes(h, _p(sz))
        nodes = np.zeros((sz[0], 8), np.float32)
        verts = np.zeros((sz[1], 4), np.float32)
        faces = np.zeros(sz[2], RR2L_FACE_DTYPE)
        shapes = np.zeros(sz[3], RR2L_SHAPE_DTYPE)
        L.rr2l_copy(h, _p(nodes), _p(verts), _p(faces), _p(shapes))
    finally:
        L.rr2l_free(h)
    return {"nodes": nodes, "vertices": verts, "faces": faces, "shapes": shapes, "root": int(sz[4]),
            "meshes": int(sz[5]), "instances": int(sz[6])}


def ref_bvh_nodes(scene, cost=10.0, bins=64, sah=True):
    from mcrt.types import RRNODE_DTYPE
    sh = _RefShapes(scene)
    n = ref().rr_bvh_build(*sh.args(), cost, bins, 1 if sah else 0, None, 0)
    out = np.zeros(n, RRNODE_DTYPE)
    ref().rr_bvh_build(*sh.args(), cost, bins, 1 if sah else 0, _p(out), n)
    return out


def ref_brute_closest(scene, rays):
    from mcrt.types import ISECT_DTYPE
    sh = _RefShapes(scene)
    out = np.zeros(len(rays), ISECT_DTYPE)
    ref().rr_test_intersections(*sh.args(), _p(rays), len(rays), _p(out))
    return out


def ref_brute_any(scene, rays):
    sh = _RefShapes(scene)
    out = np.zeros(len(rays), np.int32)
    ref().rr_test_occlusions(*sh.args(), _p(rays), len(rays), _p(out))
    return out


def ref_load_obj(path):
    L = ref()
    base = os.path.dirname(path) + "/"
    h = L.rr_load_obj(path.encode(), base.encode())
    if not h:
        raise RuntimeError(f"tinyobj failed on {path}")
    shapes = []
    for i in range(L.rr_obj_num_shapes(h)):
        pp, npf, ip, ni = _c.c_void_p(), _c.c_int(), _c.c_void_p(), _c.c_int()
        L.rr_obj_shape(h, i, _c.byref(pp), _c.byref(npf), _c.byref(ip), _c.byref(ni))
        P = np.ctypeslib.as_array(_c.cast(pp, _c.POINTER(_c.c_float)), (npf.value,)).copy().reshape(-1, 3)
        I = np.ctypeslib.as_array(_c.cast(ip, _c.POINTER(_c.c_int)), (ni.value,)).copy().reshape(-1, 3)
        shapes.append((P, I))
    L.rr_obj_free(h)
    return shapes


# --------------------------------------------------------------------------
# oracle/_ref on the GPU box: the reference's OpenCL kernels (PathTracing.cl,
# reconstruction.cl, RadeonRays intersect_bvh2_lds.cl) compiled for gfx950,
# run through the ROCm OpenCL runtime by oracle/_ref/clref_runner.so.
# --------------------------------------------------------------------------
CLREF_LIB = os.path.join(HERE, "_ref", "clref_runner.so")

# RTBDPTVertex (KRN/kernel_data.h:162-244): 240 B, RTInteraction at offset 16
REF_VERTEX_DTYPE = np.dtype([
    ("throughput", "<f4", 4), ("wo", "<f4", 4), ("p", "<f4", 4), ("uv", "<f4", 2), ("traceErrorOffset", "<f4"),
    ("shapeIdx", "<i4"), ("gn", "<f4", 4), ("sn", "<f4", 4), ("dpdu", "<f4", 4), ("dpdv", "<f4", 4),
    ("sdpdu", "<f4", 4), ("sdpdv", "<f4", 4), ("dpdx", "<f4", 4), ("dpdy", "<f4", 4), ("duvdx", "<f4", 2),
    ("duvdy", "<f4", 2), ("type", "<i4"), ("flags", "<i4"), ("lightIdx", "<i4"), ("materialIdx", "<i4"),
    ("pdfFwd", "<f4"), ("pdfRev", "<f4"), ("pdfPos", "<f4"), ("radianceBufferIdx", "<i4")])
assert REF_VERTEX_DTYPE.itemsize == 240
_clref = None


def clref_available():
    return os.path.exists(CLREF_LIB)


def clref(variant="ieee"):
    global _clref
    if _clref is None:
        L = _load(CLREF_LIB)
        L.clref_error.restype = _c.c_char_p
        L.clref_device.restype = _c.c_char_p
        L.clref_init.argtypes = [_c.c_char_p, _c.c_char_p]
        L.clref_scene_create.restype = _vp
        L.clref_scene_create.argtypes = [_vp, _vp, _c.c_int64]
        L.clref_render.argtypes = [_vp, _vp, _c.c_int, _c.c_int, _vp, _vp]
        L.clref_accumulate.argtypes = [_vp, _c.c_int, _vp, _vp]
        L.clref_trace.argtypes = [_vp, _vp, _c.c_int, _vp, _c.c_int]
        L.clref_read.argtypes = [_vp, _c.c_int, _vp]
        L.clref_bdpt_render.argtypes = [_vp, _vp, _c.c_int, _c.c_int, _vp]
        L.clref_bdpt_read.restype = _c.c_int64
        L.clref_bdpt_read.argtypes = [_vp, _c.c_int, _vp]
        L.clref_probe_lod.argtypes = [_vp, _c.c_char_p, _vp, _vp, _c.c_int, _c.c_int, _vp]
        L.clref_probe_filters.argtypes = [_c.c_char_p, _vp, _c.c_int, _vp]
        L.clref_probe_tonemap.argtypes = [_c.c_char_p, _vp, _c.c_int, _c.c_float, _vp]
        L.clref_scene_set_two_level.argtypes = [_vp, _vp, _c.c_int64, _vp, _c.c_int64, _vp, _c.c_int64, _vp,
                                                _c.c_int64, _c.c_int]
        st = L.clref_init(os.path.join(HERE, "_ref").encode(), variant.encode())
        if st != 0:
            raise RuntimeError(f"clref_init({variant}) = {st}: {L.clref_error().decode()}")
        _clref = L
    return _clref


def clref_filter_weights(filters, variant="ieee"):
    """The reference's filter weights (filters.cl via oracle/refbuild/clprobe_filters.cl, run live)
    for an array of mcrt.types.FILTER_DTYPE records (the 56-B device layout)."""
    L = clref(variant)
    f = np.ascontiguousarray(filters)
    out = np.zeros(len(f), np.float32)
    st = L.clref_probe_filters(os.path.join(HERE, "_ref", "clref_probe_filters.hsaco").encode(), _p(f), len(f), _p(out))
    if st != 0:
        raise RuntimeError(f"clref_probe_filters {st}: {L.clref_error().decode()}")
    return out


def clref_tonemap(img, Lwhite, variant="ieee"):
    """The reference's Reinhard tone mapping (computeLuminanceFromRGB + toneMapControlled of
    ToneMapping.cl / colors.cl via oracle/refbuild/clprobe_tonemap.cl, run live) of a float32
    (..., 4) image."""
    L = clref(variant)
    a = np.ascontiguousarray(img, np.float32)
    out = np.zeros_like(a)
    n = a.size // 4
    st = L.clref_probe_tonemap(os.path.join(HERE, "_ref", "clref_probe_tonemap.hsaco").encode(), _p(a), n,
                               float(Lwhite), _p(out))
    if st != 0:
        raise RuntimeError(f"clref_probe_tonemap {st}: {L.clref_error().decode()}")
    return out


class CLRefScene:
    """A scene on the reference OpenCL pipeline; BVH nodes from the reference Bvh2 builder
    (librrref.so) when available, else from the oracle's bit-identical restatement."""

    def __init__(self, scene, variant="ieee", nodes=None, two_level=False, world_to_local=None):
        """two_level: ray queries go through RadeonRays' IntersectorTwoLevel kernels over the
        reference's own two-level build (ref_bvh2l), as RR does for instanced scenes."""
        self.L = clref(variant)
        self.scene = scene
        self._desc = scene.desc()
        if two_level and nodes is None:
            nodes = np.zeros((1, 16), np.float32)   # flat structure unused
        if nodes is None:
            o = OracleScene(scene)
            o.build()
            nodes = o.nodes()
        self.nodes = np.ascontiguousarray(nodes)
        self.h = self.L.clref_scene_create(ctypes.byref(self._desc), _p(self.nodes), len(self.nodes))
        if not self.h:
            raise RuntimeError(self.L.clref_error().decode())
        if two_level:
            r = self.two_level = ref_bvh2l(scene, world_to_local=world_to_local)
            st = self.L.clref_scene_set_two_level(self.h, _p(r["nodes"]), len(r["nodes"]), _p(r["vertices"]),
                                                  len(r["vertices"]), _p(r["faces"]), len(r["faces"]),
                                                  _p(r["shapes"]), len(r["shapes"]), r["root"])
            if st != 0:
                raise RuntimeError(f"clref_scene_set_two_level {st}: {self.L.clref_error().decode()}")

    def render(self, cam, frame=0, max_depth=2):
        W, H = int(cam["width"][0]), int(cam["height"][0])
        out = np.zeros((H, W, 4), np.float32)
        st = self.L.clref_render(self.h, _p(cam), frame, max_depth, _p(out), None)
        if st != 0:
            raise RuntimeError(f"clref_render {st}: {self.L.clref_error().decode()}")
        return out

    def accumulate(self, frame, filt, H, W):
        img = np.zeros((H, W, 4), np.float32)
        st = self.L.clref_accumulate(self.h, frame, _p(filt), _p(img))
        if st != 0:
            raise RuntimeError(f"clref_accumulate {st}: {self.L.clref_error().decode()}")
        return img

    READ = {"rays": (0, 48), "isect": (1, 32), "shadow_rays": (2, 48), "temp": (3, 16), "throughput": (4, 32),
            "occlusion": (5, 4), "radiance": (6, 16), "ray_differentials": (7, 64)}

    def read(self, which, W, H):
        """Raw bytes of an intermediate buffer of the last frame (diagnostics)."""
        idx, sz = self.READ[which]
        out = np.zeros(W * H * sz, np.uint8)
        st = self.L.clref_read(self.h, idx, _p(out))
        if st != 0:
            raise RuntimeError(f"clref_read {st}: {self.L.clref_error().decode()}")
        return out

    def probe_lod(self, cam):
        """The reference's (unused) texture-LOD functions at its own primary hits: renders one
        depth-1 frame (GeneratePerspectiveRays + intersect), then runs clprobe_lod.cl's ProbeLOD
        on its intersections and ray differentials.  Returns (H, W, 3, 4) float32."""
        W, H = int(cam["width"][0]), int(cam["height"][0])
        self.render(cam, frame=0, max_depth=1)
        isect = self.read("isect", W, H)
        diffs = self.read("ray_differentials", W, H)
        out = np.zeros((H, W, 3, 4), np.float32)
        st = self.L.clref_probe_lod(self.h, os.path.join(HERE, "_ref", "clref_probe_lod.hsaco").encode(), _p(isect),
                                    _p(diffs), W, H, _p(out))
        if st != 0:
            raise RuntimeError(f"clref_probe_lod {st}: {self.L.clref_error().decode()}")
        return out

    def render_bdpt(self, cam, frame=0, max_depth=2):
        """One RTBDPTPass::update frame (BDPT.cl kernels); returns the W*H float4 radiance."""
        W, H = int(cam["width"][0]), int(cam["height"][0])
        out = np.zeros((H, W, 4), np.float32)
        st = self.L.clref_bdpt_render(self.h, _p(cam), frame, max_depth, _p(out))
        if st != 0:
            raise RuntimeError(f"clref_bdpt_render {st}: {self.L.clref_error().decode()}")
        return out

    BDPT_READ = {"camera_vertices": 0, "light_vertices": 1, "camera_counts": 2, "light_counts": 3,
                 "connection_rays": 4, "visibility": 5, "temp_radiance": 6, "sampled_light": 7, "sampled_camera": 8}

    def read_bdpt(self, which):
        """Raw bytes of a BDPT buffer of the last BDPT frame (RTBDPTPass's buffers)."""
        idx = self.BDPT_READ[which]
        n = self.L.clref_bdpt_read(self.h, idx, None)
        if n < 0:
            raise RuntimeError(f"clref_bdpt_read {n}: {self.L.clref_error().decode()}")
        out = np.zeros(n, np.uint8)
        st = self.L.clref_bdpt_read(self.h, idx, _p(out))
        if st < 0:
            raise RuntimeError(f"clref_bdpt_read {st}: {self.L.clref_error().decode()}")
        return out

    def trace(self, rays, any_hit=False, init=-7):
        from mcrt.types import ISECT_DTYPE
        if any_hit:
            out = np.full(len(rays), init, np.int32)
        else:
            out = np.zeros(len(rays), ISECT_DTYPE)
            out["shapeid"] = init
            out["primid"] = init
        st = self.L.clref_trace(self.h, _p(rays), len(rays), _p(out), 1 if any_hit else 0)
        if st != 0:
            raise RuntimeError(f"clref_trace {st}: {self.L.clref_error().decode()}")
        return out

"""numpy dtypes and ctypes mirrors of include/mcrt_capi.h.

Every record dtype is byte-identical to the OpenCL device struct of the reference
(assets/kernels/kernel_data.h; sizes/offsets in SURVEY.md Appendix B), so arrays
built here can be handed to the product (C ABI), to the oracle, and to the
reference's own OpenCL kernels unchanged.
"""
import ctypes

import numpy as np

F4 = (np.float32, (4,))

SHAPE_DTYPE = np.dtype(
    [
        ("toWorldTransform", np.float32, (4, 4)),
        ("toWorldInverseTranspose", np.float32, (4, 4)),
        ("startIdx", np.uint32),
        ("startVertex", np.uint32),
        ("numTriangles", np.uint32),
        ("materialId", np.int32),
        ("lightID", np.int32),
        ("area", np.float32),
        ("pad", np.int32, (2,)),
    ],
    align=True,
)
assert SHAPE_DTYPE.itemsize == 160

MATERIAL_DTYPE = np.dtype(
    {
        "names": [
            "uber_kd", "uber_ks", "uber_kr", "uber_kt", "uber_opacity", "uber_roughness",
            "uber_eta", "type", "uber_normalMapId", "uber_diffuseTexId", "uber_glossyTexId",
            "uber_specReflectionTexId", "uber_transmissionTexId", "uber_opacityTexId",
            "uber_roughnessTexId", "uber_iorTexId",
        ],
        "formats": [F4, F4, F4, F4, F4, (np.float32, (2,)), np.float32, np.int32] + [np.int32] * 8,
        "offsets": [0, 16, 32, 48, 64, 80, 88, 92, 96, 100, 104, 108, 112, 116, 120, 124],
        "itemsize": 128,
    }
)

LIGHT_DTYPE = np.dtype(
    {
        "names": ["d", "p", "intensity", "radius", "area", "choicePdf", "shapeId", "type", "flags", "pad"],
        "formats": [F4, F4, F4, np.float32, np.float32, np.float32, np.int32, np.int32, np.int32, (np.int32, (2,))],
        "offsets": [0, 16, 32, 48, 52, 56, 60, 64, 68, 72],
        "itemsize": 80,
    }
)

CAMERA_DTYPE = np.dtype(
    {
        "names": ["worldToClip", "r00", "r10", "r11", "r01", "pos", "direction", "width", "height", "area", "padding"],
        "formats": [(np.float32, (4, 4)), F4, F4, F4, F4, F4, F4, np.uint32, np.uint32, np.float32, np.int32],
        "offsets": [0, 64, 80, 96, 112, 128, 144, 160, 164, 168, 172],
        "itemsize": 176,
    }
)

TEXDESC_DTYPE = np.dtype(
    [("width", np.uint16), ("height", np.uint16), ("numMipLevels", np.uint16), ("format", np.uint16),
     ("wrap", np.uint16), ("pad", np.uint16), ("memOffset", np.uint32)]
)
assert TEXDESC_DTYPE.itemsize == 16

RAY_DTYPE = np.dtype(
    {
        "names": ["o", "d", "extra", "doBackfaceCulling", "padding"],
        "formats": [F4, F4, (np.int32, (2,)), np.int32, np.int32],
        "offsets": [0, 16, 32, 40, 44],
        "itemsize": 48,
    }
)

ISECT_DTYPE = np.dtype(
    {
        "names": ["shapeid", "primid", "padding", "uvwt"],
        "formats": [np.int32, np.int32, (np.int32, (2,)), F4],
        "offsets": [0, 4, 8, 16],
        "itemsize": 32,
    }
)

FILTER_DTYPE = np.dtype(
    {
        "names": ["filterType", "radius", "mitchellB", "mitchellC", "lanczosSincTau", "gaussianAlpha",
                  "gaussianExpX", "gaussianExpY", "pixelOffset", "pad"],
        "formats": [np.int32, (np.float32, (2,)), np.float32, np.float32, np.float32, np.float32,
                    np.float32, np.float32, (np.float32, (2,)), np.float32],
        "offsets": [0, 8, 16, 20, 24, 28, 32, 36, 40, 48],
        "itemsize": 56,
    }
)

# RadeonRays Bvh2::Node (bvh2.h:186-204), used by the oracle / reference dumps
RRNODE_DTYPE = np.dtype(
    [("lmin_v0", np.float32, (3,)), ("addr_left", np.uint32),
     ("lmax_v1", np.float32, (3,)), ("mesh_id", np.uint32),
     ("rmin_v2", np.float32, (3,)), ("addr_right", np.uint32),
     ("rmax", np.float32, (3,)), ("prim_id", np.uint32)]
)
assert RRNODE_DTYPE.itemsize == 64

DIRECTIONAL, POINT, DISK_AREA, TRIANGLE_MESH_AREA = 0, 1, 2, 3
FLAG_DELTA_POSITION, FLAG_DELTA_DIRECTION, FLAG_AREA = 1 << 1, 1 << 2, 1 << 3
SAMPLER_SOBOL, SAMPLER_RANDOM = 0, 1
BOX, TRIANGLE, GAUSSIAN, MITCHELL, LANCZOS = 0, 1, 2, 3, 4


class SceneDesc(ctypes.Structure):
    """mcrt_scene_desc (include/mcrt_capi.h)."""

    _fields_ = [
        ("shapes", ctypes.c_void_p), ("num_shapes", ctypes.c_uint32),
        ("indices", ctypes.c_void_p), ("num_indices", ctypes.c_uint32),
        ("positions", ctypes.c_void_p), ("num_vertices", ctypes.c_uint32),
        ("uvs", ctypes.c_void_p),
        ("normals", ctypes.c_void_p),
        ("tangents", ctypes.c_void_p),
        ("binormals", ctypes.c_void_p),
        ("colors", ctypes.c_void_p),
        ("textures", ctypes.c_void_p), ("num_textures", ctypes.c_uint32),
        ("tex_data", ctypes.c_void_p), ("tex_data_bytes", ctypes.c_uint64),
        ("sobol_matrices", ctypes.c_void_p), ("num_sobol_words", ctypes.c_uint32),
        ("lights", ctypes.c_void_p), ("num_lights", ctypes.c_uint32),
        ("materials", ctypes.c_void_p), ("num_materials", ctypes.c_uint32),
    ]


class AccelOpts(ctypes.Structure):
    _fields_ = [("traversal_cost", ctypes.c_float), ("num_bins", ctypes.c_int), ("use_sah", ctypes.c_int),
                ("device_build", ctypes.c_int), ("force_2level", ctypes.c_int), ("force_flat", ctypes.c_int),
                ("world_to_local", ctypes.c_void_p)]


class FrameParams(ctypes.Structure):
    _fields_ = [
        ("frame_index", ctypes.c_int32), ("max_depth", ctypes.c_int32), ("sampler", ctypes.c_int32),
        ("russian_roulette", ctypes.c_int32), ("rr_start_depth", ctypes.c_int32),
        ("band_rows", ctypes.c_int32), ("num_bands", ctypes.c_int32), ("band_index", ctypes.c_int32),
        ("integrator", ctypes.c_int32), ("texture_lod", ctypes.c_int32),
    ]


class PostprocessParams(ctypes.Structure):
    _fields_ = [("use_denoise", ctypes.c_int32), ("denoise_radius", ctypes.c_int32),
                ("sigma_spatial", ctypes.c_float), ("sigma_range", ctypes.c_float),
                ("use_tonemapping", ctypes.c_int32), ("min_luminance", ctypes.c_float)]


INTEGRATOR_PT = 0
INTEGRATOR_BDPT = 1


def ptr(a):
    """Raw address of a numpy array (None for None)."""
    if a is None:
        return None
    return a.ctypes.data


def make_filter(kind=BOX, radius=(2.0, 2.0), pixel_offset=(0.0, 0.0), B=1.0 / 3, C=1.0 / 3, tau=3.0,
                alpha=1.0):
    """RTFilterProperties with the device layout (filters.cl); defaults per PathTracingSettings.h."""
    f = np.zeros(1, FILTER_DTYPE)
    f["filterType"] = kind
    f["radius"] = radius
    f["mitchellB"], f["mitchellC"] = B, C
    f["lanczosSincTau"] = tau
    f["gaussianAlpha"] = alpha
    f["gaussianExpX"] = np.exp(-alpha * radius[0] * radius[0])
    f["gaussianExpY"] = np.exp(-alpha * radius[1] * radius[1])
    f["pixelOffset"] = pixel_offset
    return f

AOV_ALBEDO = 0        # MCRT_AOV_ALBEDO
AOV_TEXTURE_LOD = 1   # MCRT_AOV_TEXTURE_LOD

# mcrt_obj_load flags (include/mcrt_capi.h)
OBJ_MIPS = 1
OBJ_EMISSIVE_LIGHTS = 2

"""CPU tests of the C ABI boundary: libmcrt.so loads and exports every entry point that
include/mcrt_capi.h declares; host-only helpers work without a GPU."""
import ctypes

import numpy as np

from mcrt import lib
from mcrt import types as T
from mcrt.camera import make_camera


def test_library_exports_every_header_symbol():
    L = ctypes.CDLL(lib.LIB_PATH)
    declared = lib.header_symbols()
    assert len(declared) >= 25
    missing = [s for s in declared if not hasattr(L, s)]
    assert not missing, missing
    assert set(declared) == set(lib.SIGNATURES), set(declared) ^ set(lib.SIGNATURES)


def test_struct_sizes_match_reference_layouts():
    assert T.SHAPE_DTYPE.itemsize == 160 and T.MATERIAL_DTYPE.itemsize == 128
    assert T.LIGHT_DTYPE.itemsize == 80 and T.CAMERA_DTYPE.itemsize == 176
    assert T.RAY_DTYPE.itemsize == 48 and T.ISECT_DTYPE.itemsize == 32
    assert T.FILTER_DTYPE.itemsize == 56 and T.FILTER_DTYPE.fields["pixelOffset"][1] == 40
    assert T.TEXDESC_DTYPE.itemsize == 16


def test_version_and_error_strings():
    assert b"gfx950" in lib.lib().mcrt_version()
    # no context: last global error string is available and calls fail loudly on bad input
    assert lib.lib().mcrt_trace_closest(None, None, 0, None) == 1


def test_camera_helper_matches_python_restatement():
    pos, target = (1.0, 2.0, -5.0), (0.5, 1.0, 0.0)
    fwd = np.array(target) - np.array(pos)
    c1 = lib.make_pinhole_camera(pos, fwd, (0, 1, 0), 45.0, 0.3, 30.0, 320, 200, (0.25, -0.5))
    c2 = make_camera(pos, target, 320, 200, fovy=45.0, pixel_offset=(0.25, -0.5))
    for k in ("r00", "r10", "r11", "r01", "pos"):
        np.testing.assert_allclose(c1[k], c2[k], atol=1e-5)
    assert int(c1["width"][0]) == 320 and int(c1["height"][0]) == 200

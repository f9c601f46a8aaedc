"""Python side of the MI355X Monte-Carlo path-tracing core.

`mcrt.lib` binds the C ABI (include/mcrt_capi.h) of libmcrt.so (HIP, gfx950);
`mcrt.scenes` / `mcrt.camera` build the reference's scene arrays and camera.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(os.path.dirname(PKG_DIR))

"""Python side of the MI355X Monte-Carlo path-tracing core.

`mcrt.lib` binds the C ABI (include/mcrt_capi.h) of libmcrt.so (HIP, gfx950);
`mcrt.scenes` / `mcrt.camera` build the reference's scene arrays and camera.
"""
import os

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT_DIR = os.path.dirname(os.path.dirname(PKG_DIR))


def sobol_matrices():
    """g_SobolMatrices32 (APP/raytracing/sampling/sobol.h:34): the 1024 x 52 uint32 Sobol generator
    matrices the reference uploads as scene data (RTScene::setSceneArgs, scene_sobolMatrices) for
    its Sobol sampler.  Stored as package data (extracted from sobol.h by
    tests/golden/make_fixtures.py)."""
    import numpy as np
    m = np.load(os.path.join(PKG_DIR, "data", "sobol_1024x52.npy"), allow_pickle=False)
    assert m.dtype == np.uint32 and m.size == 1024 * 52
    return m

"""The premise of the shadow rays' occluder hints (mcrt_traverse.h hintOccludes), on the host-built
records that the device build reproduces byte for byte (test_gpu_sah_build.py): in the flat tree,
every child box an internal record stores contains the child boxes that child's own record
stores, so the box on each root-to-leaf path only shrinks.  With fma's monotone rounding a ray
that passes a leaf's box test then passes every ancestor's (intersect_bvh2_lds.cl:54-63), which is
what lets one leaf test stand for the any-hit walk."""
import numpy as np
import pytest

from mcrt import scenes


def _child_boxes(rec):
    """(n, 2, 2, 3): per record, child k's (lo, hi) as the record stores them."""
    b = np.empty((len(rec), 2, 2, 3), np.float32)
    b[:, 0, 0] = rec[:, [0, 2, 8]]
    b[:, 0, 1] = rec[:, [1, 3, 9]]
    b[:, 1, 0] = rec[:, [4, 6, 10]]
    b[:, 1, 1] = rec[:, [5, 7, 11]]
    return b


@pytest.mark.parametrize("name", ["mixed", "dragon_50k", "sm_200k"])
def test_child_boxes_nest(name):
    from mcrt import lib
    sc = {"mixed": scenes.test_scene, "dragon_50k": lambda: scenes.dragon_proxy(tris=50_000),
          "sm_200k": lambda: scenes.san_miguel_proxy(tris=200_000)}[name]()
    rec, _ = lib.build_host_records(sc, device_build=3)
    rec = np.asarray(rec, np.float32).reshape(-1, 16)
    ids = rec.view(np.int32)[:, 12:14]
    internal = ids[:, 0] >= 0
    box = _child_boxes(rec)
    checked = 0
    for k in range(2):
        par = np.nonzero(internal)[0]
        ch = ids[par, k]
        sub = internal[ch]          # children that are internal records themselves
        par, ch = par[sub], ch[sub]
        outer = box[par, k]         # the child's box as its parent stores it
        for j in range(2):
            inner = box[ch, j]      # the grandchildren's boxes as the child stores them
            assert (outer[:, 0] <= inner[:, 0]).all() and (inner[:, 1] <= outer[:, 1]).all()
            checked += len(ch)
    assert checked > 0

"""The premise of the shadow rays' occluder hints (mcrt_traverse.h hintOccludes), on the host-built
records that the device build reproduces byte for byte (test_gpu_sah_build.py): in the flat tree,
every child box an internal record stores contains the child boxes that child's own record
stores, so the box on each root-to-leaf path only shrinks.  With fma's monotone rounding a ray
that passes a leaf's box test then passes every ancestor's (intersect_bvh2_lds.cl:54-63), which is
what lets one leaf test stand for the any-hit walk.

Checked for every flat builder: the host restatement of the reference's Bvh2 (device_build 3,
which the device SAH build reproduces byte for byte) and the host 3-axis perf tree (4) here; the
device LBVH (1) and the device SAH build (2) on the GPU (test_gpu_shadow_hints.py).  The same
walk checks each builder's reported depth, which bounds the wave-packet stack (2 entries per
level, mcrt_capi.cpp finish_accel): it must not be below the deepest leaf's level."""
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


def check_nesting(rec):
    """Asserts that every stored child box contains its child's stored child boxes; returns the
    number of (parent, grandchild) pairs checked."""
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
    return checked


def leaf_depth(rec):
    """Level of the deepest leaf (root = level 0) of a flat record array."""
    ids = np.asarray(rec, np.float32).reshape(-1, 16).view(np.int32)[:, 12:14]
    level = np.full(len(ids), -1, np.int64)
    level[0] = 0
    frontier = np.array([0])
    while len(frontier):
        inner = frontier[ids[frontier, 0] >= 0]
        nxt = ids[inner].ravel()
        level[nxt] = np.repeat(level[inner] + 1, 2)
        frontier = nxt
    assert (level >= 0).all(), "records unreachable from the root"
    return int(level.max())


@pytest.mark.parametrize("build", [3, 4])
@pytest.mark.parametrize("name", ["mixed", "dragon_50k", "sm_200k"])
def test_child_boxes_nest(name, build):
    from mcrt import lib
    sc = {"mixed": scenes.test_scene, "dragon_50k": lambda: scenes.dragon_proxy(tris=50_000),
          "sm_200k": lambda: scenes.san_miguel_proxy(tris=200_000)}[name]()
    rec, info = lib.build_host_records(sc, device_build=build)
    assert check_nesting(rec) > 0
    assert info["depth"] >= leaf_depth(rec), (info["depth"], leaf_depth(rec))

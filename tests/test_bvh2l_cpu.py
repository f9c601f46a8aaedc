"""CPU tests of the two-level (instanced) acceleration structure build (mcrt_bvh2l.cpp), pinned
node for node against the reference's own RadeonRays Bvh + PlainBvhTranslator (bvh.cpp,
plain_bvh_translator.cpp compiled from /root/reference into oracle/_ref/librrref.so, driven by
the IntersectorTwoLevel::Process mirror in oracle/refbuild/rrref_driver.cpp).

Both layouts number every tree in pre-order, so the reference's node j of a tree is our record
j of the same tree: internal/leaf pattern, child indices, every child box (bit-exact), the
triangle of every leaf (face reordering and object-space vertices) and the instance record of
every top-level leaf (shape id, world-to-local rows, bottom tree) are compared."""
import math

import numpy as np
import pytest

from mcrt import lib, scenes
from oracle import pyoracle as O

pytestmark = pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref/librrref.so not built")


def _ints(rec):
    return rec[:, 12:16].view(np.int32)


def _compare_tree(ref_nodes, rbase, mine, mbase, count):
    """Tree of `count` nodes at reference index rbase / our record mbase."""
    R = ref_nodes[rbase:rbase + count]
    M = mine[mbase:mbase + count]
    mi = _ints(M)
    r_internal = R[:, 3] == -1.0
    m_internal = mi[:, 0] >= 0
    np.testing.assert_array_equal(r_internal, m_internal)
    p = np.nonzero(m_internal)[0]
    # children: left = p + 1 in both; right = the left child's skip link in the reference
    np.testing.assert_array_equal(mi[p, 0] - mbase, p + 1)
    r_right = R[p + 1, 7].astype(np.int64) - rbase
    np.testing.assert_array_equal(mi[p, 1] - mbase, r_right)
    c0, c1 = p + 1, r_right
    # child boxes: our (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y | c1 ... | c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
    got = M[p][:, :12].view(np.uint32)
    want = np.stack([R[c0, 0], R[c0, 4], R[c0, 1], R[c0, 5], R[c1, 0], R[c1, 4], R[c1, 1], R[c1, 5],
                     R[c0, 2], R[c0, 6], R[c1, 2], R[c1, 6]], 1).astype(np.float32).view(np.uint32)
    np.testing.assert_array_equal(got, want)
    leaves = np.nonzero(~m_internal)[0]
    start = R[leaves, 3].astype(np.int64) >> 4
    return leaves, start


def compare_with_reference(scene, **opts):
    ref = O.ref_bvh2l(scene, world_to_local=opts.get("world_to_local"))
    rec, info = lib.build_host_records(scene, force_2level=True, **opts)
    assert info["two_level"] == 1
    assert rec.shape[0] == ref["nodes"].shape[0]
    assert info["meshes"] == ref["meshes"]
    S = ref["meshes"] + ref["instances"]
    top = 2 * S - 1
    assert info["top_records"] == top
    leaves, start = _compare_tree(ref["nodes"], ref["root"], rec, 0, top)
    mi = _ints(rec)
    assert (mi[leaves, 0] == -2).all()
    shp = ref["shapes"][start]
    np.testing.assert_array_equal(mi[leaves, 2], shp["id"])
    np.testing.assert_array_equal(rec[leaves, :12].view(np.uint32),
                                  shp["minv"][:, :3, :].reshape(-1, 12).astype(np.float32).view(np.uint32))
    # bottom trees: one per mesh, reached through the top leaves
    seen = {}
    for k, leaf in enumerate(leaves):
        seen.setdefault(int(mi[leaf, 1]), int(shp["bvhidx"][k]))
    for mroot, rroot in seen.items():
        sid = int(mi[leaves[list(mi[leaves, 1]).index(mroot)], 2])
        nf = int(scene.shapes[sid]["numTriangles"])
        bl, bstart = _compare_tree(ref["nodes"], rroot, rec, mroot, 2 * nf - 1)
        faces = ref["faces"][bstart]
        R = rec[mroot + bl]
        np.testing.assert_array_equal(R[:, 7].view(np.int32), faces["prim_id"])
        v = ref["vertices"][faces["idx"]][..., :3]   # (L, 3, 3)
        np.testing.assert_array_equal(R[:, 0:3].view(np.uint32), v[:, 0].view(np.uint32))
        np.testing.assert_array_equal(R[:, 4:7].view(np.uint32), (v[:, 1] - v[:, 0]).view(np.uint32))
        np.testing.assert_array_equal(R[:, 8:11].view(np.uint32), (v[:, 2] - v[:, 0]).view(np.uint32))
        assert (_ints(R)[:, 0] == -1).all()
    assert len(seen) == ref["meshes"]
    return rec, info, ref


def _mixed_instances(seed=0):
    return scenes.instances_test_scene(seed)


def test_two_level_matches_reference_mixed():
    compare_with_reference(_mixed_instances())


def test_two_level_matches_reference_instanced_proxy():
    sc = scenes.instanced_proxy(grid_n=6, body_tris=150_000)   # > 65536 faces: concurrent subtrees
    rec, info, ref = compare_with_reference(sc)
    assert info["meshes"] == 4 and ref["instances"] == len(sc.shapes) - 4


def test_two_level_explicit_world_to_local():
    sc = _mixed_instances(seed=3)
    w2l = np.linalg.inv(sc.shapes["toWorldTransform"].astype(np.float64)).astype(np.float32)
    w2l[:, :3, 3] += np.float32(1e-3)   # distinguishable from the default
    rec, info, ref = compare_with_reference(sc, world_to_local=w2l)


def test_two_level_median_heavy_geometry():
    """Many coincident / coplanar primitives: the partition degenerates and RR's median
    fallback (which keeps the partition-grown boxes) shapes the tree."""
    b = scenes.SceneBuilder("coincident")
    m = b.add_material()
    P = np.zeros((300, 3), np.float32)
    P[:, 0] = np.repeat(np.arange(100), 3) % 7
    P[1::3, 1] = 1.0
    P[2::3, 2] = 1.0
    tris = np.arange(300).reshape(-1, 3)
    A = b.add_mesh(P, np.tile([0, 0, 1], (300, 1)), np.zeros((300, 2)), tris, m)
    for i in range(5):
        b.add_instance(A, scenes._affine(1.0, 0.0, (0, 0, 0)))   # identical boxes at the top level too
    compare_with_reference(b.build())


def test_auto_selection():
    """RR picks the two-level intersector only when some shape is an instance (or forced)."""
    flat_scene = scenes.test_scene()
    _, info = lib.build_host_records(flat_scene)
    assert info["two_level"] == 0
    _, info = lib.build_host_records(flat_scene, force_2level=True)
    assert info["two_level"] == 1 and info["meshes"] == len(flat_scene.shapes)
    inst = _mixed_instances()
    _, info = lib.build_host_records(inst)
    assert info["two_level"] == 1
    _, info = lib.build_host_records(inst, force_flat=True)
    assert info["two_level"] == 0


def test_scene_builder_instances_share_data():
    sc = _mixed_instances()
    sh = sc.shapes
    key = list(zip(sh["startIdx"], sh["startVertex"], sh["numTriangles"]))
    assert len(set(key)) == 5 and len(key) == 15
    # instance area = base mesh area under its own transform (uniform scale s -> s^2)
    assert math.isclose(float(sh[2]["area"]), float(sh[1]["area"]) * 0.25, rel_tol=1e-4)

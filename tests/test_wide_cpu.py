"""Host restatement of the 4-wide quantized tree (mcrt_wide.cpp via mcrt_accel_build_host_wide):
structural properties, no GPU.

  * every triangle of the scene is in exactly one triangle record, and its record holds the world
    vertices whose v0 and edges are the Bvh2 leaf record's bit for bit;
  * every child reference is in range, internal children are numbered breadth first and
    consecutively per node, triangle records in parent order;
  * every decoded child box (fma(q, 2^e, origin), the traversal's own float) contains the exact
    bounds of all triangles below that child -- the property the traversal's parity rests on;
  * the decode of each plane is the tightest: one quantum further in would cut the child's box.
"""
import numpy as np
import pytest

from helpers import bunny_scene, rr_cornell_scene
from mcrt import lib, scenes

WIDE_K = 4


def plane(q, eb, o):
    """mcrt::wide_plane in float32: fma(q, 2^(eb-127), o) -- exact through float64 (q * 2^e is exact
    and the sum of two floats rounds once to float32 only if done as an fma: use np.float64 then
    round, which equals the fused result because q * 2^e and o are both exactly representable)."""
    s = np.ldexp(1.0, eb.astype(np.int64) - 127)
    return (q.astype(np.float64) * s + o.astype(np.float64)).astype(np.float32)


def decode(nodes):
    o = nodes[:, 0:3].view(np.float32)
    meta = nodes[:, 3]
    eb = np.stack([(meta >> (8 * a)) & 255 for a in range(3)], 1)
    valid = (meta >> 24) & 15
    leaf = (meta >> 28) & 15
    lo = np.zeros((len(nodes), WIDE_K, 3), np.float32)
    hi = np.zeros_like(lo)
    for c in range(WIDE_K):
        for a in range(3):
            ql = (nodes[:, 4 + 2 * a] >> (8 * c)) & 255
            qh = (nodes[:, 5 + 2 * a] >> (8 * c)) & 255
            lo[:, c, a] = plane(ql, eb[:, a], o[:, a])
            hi[:, c, a] = plane(qh, eb[:, a], o[:, a])
    return o, eb, valid, leaf, lo, hi


@pytest.mark.parametrize("name", ["cornell", "bunny", "mixed", "dragon_20k", "sm_50k"])
def test_wide_tree_structure(name):
    sc = {"cornell": lambda: rr_cornell_scene()[0], "bunny": bunny_scene, "mixed": scenes.test_scene,
          "dragon_20k": lambda: scenes.dragon_proxy(tris=20_000),
          "sm_50k": lambda: scenes.san_miguel_proxy(tris=50_000)}[name]()
    nodes, tris = lib.build_host_wide(sc)
    rec, _ = lib.build_host_records(sc)
    n_tri = sc.num_triangles
    assert len(tris) == n_tri
    # (shape, prim) of every triangle exactly once
    key = tris[:, 3].view(np.int32).astype(np.int64) << 32 | tris[:, 7].view(np.int32).astype(np.int64)
    assert len(np.unique(key)) == n_tri
    # the Bvh2 leaf records: v0 and edges bit-identical to the wide record's vertices
    leaves = rec[rec[:, 12].view(np.int32) < 0]
    lkey = leaves[:, 3].view(np.int32).astype(np.int64) << 32 | leaves[:, 7].view(np.int32).astype(np.int64)
    order = np.argsort(lkey)
    pos = np.searchsorted(lkey[order], key)
    L = leaves[order][pos]
    assert (lkey[order][pos] == key).all()
    for a in range(3):
        assert (tris[:, a].view(np.uint32) == L[:, a].view(np.uint32)).all()
        assert ((tris[:, 4 + a] - tris[:, a]).view(np.uint32) == L[:, 4 + a].view(np.uint32)).all()
        assert ((tris[:, 8 + a] - tris[:, a]).view(np.uint32) == L[:, 8 + a].view(np.uint32)).all()
    o, eb, valid, leaf, lo, hi = decode(nodes)
    assert ((valid & leaf) == leaf).all()
    assert (valid[:] != 0).all()
    # references: breadth-first numbering, consecutive internal children, triangle records in order
    nxt, ntri = 1, 0
    for i in range(len(nodes)):
        for c in range(WIDE_K):
            if not (valid[i] >> c) & 1:
                continue
            ref = int(nodes[i, 10 + c])
            if (leaf[i] >> c) & 1:
                assert ref == ntri
                ntri += 1
            else:
                assert ref == nxt
                nxt += 1
    assert nxt == len(nodes) and ntri == n_tri
    # exact bounds of each subtree (children are numbered after their parent: reverse order)
    v = tris[:, [0, 1, 2, 4, 5, 6, 8, 9, 10]].reshape(-1, 3, 3)
    tlo, thi = v.min(1), v.max(1)
    blo = np.zeros((len(nodes), 3), np.float32)
    bhi = np.zeros((len(nodes), 3), np.float32)
    for i in range(len(nodes) - 1, -1, -1):
        cl, ch = [], []
        for c in range(WIDE_K):
            if not (valid[i] >> c) & 1:
                continue
            ref = int(nodes[i, 10 + c])
            el, eh = (tlo[ref], thi[ref]) if (leaf[i] >> c) & 1 else (blo[ref], bhi[ref])
            assert (lo[i, c] <= el).all() and (hi[i, c] >= eh).all(), (i, c)
            # tight: one quantum in from the decoded plane would cut the exact box
            for a in range(3):
                e = int(eb[i, a])
                ql = (int(nodes[i, 4 + 2 * a]) >> (8 * c)) & 255
                qh = (int(nodes[i, 5 + 2 * a]) >> (8 * c)) & 255
                if ql < 255:
                    assert plane(np.array([ql + 1]), np.array([e]), o[i:i + 1, a])[0] > el[a]
                if qh > 0:
                    assert plane(np.array([qh - 1]), np.array([e]), o[i:i + 1, a])[0] < eh[a]
            cl.append(el)
            ch.append(eh)
        blo[i], bhi[i] = np.min(cl, 0), np.max(ch, 0)
    # the root spans the scene
    slo, shi = tlo.min(0), thi.max(0)
    assert (blo[0] == slo).all() and (bhi[0] == shi).all()


def test_wide_single_triangle_and_instanced():
    sc = scenes.SceneBuilder("one")
    m = sc.add_material()
    sc.add_mesh(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], float), np.tile([0, 0, 1], (3, 1)), np.zeros((3, 2)),
                np.array([[0, 1, 2]]), m)
    one = sc.build()
    nodes, tris = lib.build_host_wide(one)   # the root is the triangle record itself
    assert len(nodes) == 0 and len(tris) == 1
    assert (tris[0, [0, 1, 2, 4, 5, 6, 8, 9, 10]] == [0, 0, 0, 1, 0, 0, 0, 1, 0]).all()
    inst = scenes.instances_test_scene()
    with pytest.raises(lib.MCRTError, match="instanced"):
        lib.build_host_wide(inst)

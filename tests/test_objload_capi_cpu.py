"""Scene ingestion through the C ABI (mcrt_obj_load, csrc/mcrt_objload.cpp) for C/C++ hosts,
against the package's Python loader (mcrt/objload.py, the same restatement of the reference's
assimp preset + RTScene conversion) on a synthetic OBJ/MTL/PNG scene and on the reference's own
assets (assets/meshes: the Cornell-box family and bunny.obj, read in place when /root/reference
is present), and against the committed CornellBox-Original fixture (tests/golden, data only).

Integer data, texel data and everything the loaders compute in a single IEEE operation are
compared bit for bit; values the Python side reduces with numpy/BLAS (generated face normals,
tangent frames, shape areas, the directional light's bounding sphere) to within 2 ulp / 1e-6.
Parity with assimp itself is unpinned (assimp is not in the image)."""
import glob
import os

import numpy as np
import pytest

from mcrt import lib, objload
from test_objload_cpu import _write_scene

REF = "/root/reference/assets/meshes"
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _compare(a, b):
    assert a.num_triangles == b.num_triangles
    for f in ("startIdx", "startVertex", "numTriangles", "materialId", "lightID", "toWorldTransform",
              "toWorldInverseTranspose"):
        np.testing.assert_array_equal(a.shapes[f], b.shapes[f], err_msg=f)
    np.testing.assert_allclose(a.shapes["area"], b.shapes["area"], rtol=1e-6)
    np.testing.assert_array_equal(a.indices, b.indices)
    np.testing.assert_array_equal(a.positions, b.positions)
    np.testing.assert_array_equal(a.uvs, b.uvs)
    np.testing.assert_allclose(a.normals, b.normals, rtol=0, atol=2.5e-7)
    np.testing.assert_allclose(a.tangents, b.tangents, rtol=0, atol=2.5e-7)
    np.testing.assert_allclose(a.binormals, b.binormals, rtol=0, atol=5e-7)
    assert a.materials.tobytes() == b.materials.tobytes()
    assert a.textures.tobytes() == b.textures.tobytes()
    np.testing.assert_array_equal(a.tex_data, b.tex_data)
    assert len(a.lights) == len(b.lights)
    for f in ("shapeId", "type", "flags"):
        np.testing.assert_array_equal(a.lights[f], b.lights[f])
    for f in ("d", "p", "intensity", "radius", "area", "choicePdf"):
        np.testing.assert_allclose(a.lights[f], b.lights[f], rtol=2e-7, atol=1e-6, err_msg=f)


def _python(path, sun=None):
    b = objload.load_obj(path)
    if sun is not None:
        b.add_directional_light(*sun)
    return b.build()


def test_synthetic_scene_matches_python_loader(tmp_path):
    _write_scene(str(tmp_path))
    p = str(tmp_path / "s.obj")
    sun = ((0.3, -1.0, 0.2), (40.0, 40.0, 40.0))
    a = lib.load_obj(p, directional_lights=[sun])
    _compare(a, _python(p, sun))
    assert a.warnings == ""


def test_missing_texture_and_mtl_warn(tmp_path):
    open(tmp_path / "m.obj", "w").write("mtllib nope.mtl\nmtllib t.mtl\nv 0 0 0\nv 1 0 0\nv 0 1 0\nusemtl a\nf 1 2 3\n")
    open(tmp_path / "t.mtl", "w").write("newmtl a\nKd 0.1 0.2 0.3\nmap_Kd missing.png\n")
    a = lib.load_obj(str(tmp_path / "m.obj"))
    assert "nope.mtl" in a.warnings and "missing.png" in a.warnings
    assert a.materials["uber_diffuseTexId"][0] == -1 and a.num_triangles == 1
    with pytest.warns(UserWarning):
        b = objload.load_obj(str(tmp_path / "m.obj")).build()
    _compare(a, b)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference assets not present")
@pytest.mark.parametrize("name", sorted(os.path.basename(p) for p in glob.glob(f"{REF}/cornell-box/*.obj")) + ["bunny.obj"])
def test_reference_assets_match_python_loader(name):
    path = f"{REF}/bunny.obj" if name == "bunny.obj" else f"{REF}/cornell-box/{name}"
    sun = ((-0.5, -1.0, 0.3), (40.0, 40.0, 40.0))
    _compare(lib.load_obj(path, directional_lights=[sun]), _python(path, sun))


def test_cornell_fixture():
    """CornellBox-Original as the C++ loader sees it, against the committed fixture (the file's
    vertices and faces, data only): the same set of triangles (z negated, winding reversed), and
    the 'light' group (Ke 17 12 4) as the one mesh light.  The loader splits a group at each
    usemtl (assimp makes one mesh per material); the fixture groups by g, so triangles are
    compared as a set."""
    if not os.path.isdir(REF):
        pytest.skip("reference assets not present")
    z = np.load(f"{GOLD}/cornell_original.npz", allow_pickle=False)
    names = [str(n) for n in z["names"]]
    flip = np.array([1, 1, -1], np.float32)

    def canon(tris):   # (n, 3, 3) -> sorted tuples, rotation-invariant but winding-aware
        out = []
        for t in tris:
            k = min(range(3), key=lambda i: tuple(t[i]))
            out.append(tuple(np.roll(t, -k, axis=0).reshape(-1)))
        return sorted(out)
    want = np.concatenate([(z[f"P{i}"] * flip)[z[f"T{i}"][:, [0, 2, 1]]] for i in range(len(names))])
    a = lib.load_obj(f"{REF}/cornell-box/CornellBox-Original.obj")
    got = np.concatenate([a.positions[s["startVertex"] + a.indices[s["startIdx"]:s["startIdx"] + 3 * s["numTriangles"]], :3]
                          .reshape(-1, 3, 3) for s in a.shapes])
    assert canon(got) == canon(want)
    L = [i for i, n in enumerate(names) if n == "light"][0]
    assert len(a.lights) == 1
    s = a.shapes[a.lights[0]["shapeId"]]
    lt = a.positions[s["startVertex"] + a.indices[s["startIdx"]:s["startIdx"] + 3 * s["numTriangles"]], :3].reshape(-1, 3, 3)
    assert canon(lt) == canon((z[f"P{L}"] * flip)[z[f"T{L}"][:, [0, 2, 1]]])
    np.testing.assert_array_equal(a.lights[0]["intensity"][:3], [17, 12, 4])

"""Scene ingestion (mcrt/objload.py): OBJ/MTL + PNG into the RTScene arrays, following the
reference's assimp preset (MakeLeftHanded, FlipWindingOrder, fan triangulation, GenNormals)
and RTScene's material / texture mapping (RTScene.cpp:680-766, 826-880).  CPU only."""
import math
import os

import numpy as np

from mcrt import objload, scenes


def _write_scene(d):
    tex = np.zeros((8, 4, 4), np.uint8)
    tex[..., 0] = np.arange(8)[:, None] * 30
    tex[..., 1] = np.arange(4)[None, :] * 60
    tex[..., 3] = 255
    objload.write_png(os.path.join(d, "wall.png"), tex)
    open(os.path.join(d, "s.mtl"), "w").write(
        "newmtl wall\nKd 0.5 0.6 0.7\nKs 0.1 0.1 0.1\nNs 98\nmap_Kd wall.png\n"
        "newmtl lamp\nKd 0.8 0.8 0.8\nKs 0 0 0\nKe 17 12 4\n")
    open(os.path.join(d, "s.obj"), "w").write(
        "mtllib s.mtl\n"
        "v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0 0 1\nv 1 0 1\nv 0 1 1\n"
        "vt 0 0\nvt 1 0\nvt 1 1\nvt 0 1\n"
        "vn 0 0 1\n"
        "o quad\nusemtl wall\nf 1/1/1 2/2/1 3/3/1 4/4/1\n"
        "o lamp\nusemtl lamp\nf 5 6 7\n")
    return tex


def test_png_roundtrip(tmp_path):
    img = (np.random.default_rng(1).integers(0, 256, (13, 7, 4))).astype(np.uint8)
    p = str(tmp_path / "x.png")
    objload.write_png(p, img)
    np.testing.assert_array_equal(objload.read_png(p), img)


def test_obj_mapping(tmp_path):
    tex = _write_scene(str(tmp_path))
    sc = objload.load_obj(str(tmp_path / "s.obj")).build()
    assert sc.num_triangles == 3
    assert len(sc.shapes) == 2
    # left-handed: z negated; winding reversed so the geometric normal matches the (flipped) vn
    P = sc.positions[:, :3]
    assert np.allclose(sorted(set(P[:, 2])), [-1.0, 0.0])
    s0 = sc.shapes[0]
    tri = sc.indices[s0["startIdx"]:s0["startIdx"] + 6].reshape(2, 3) + s0["startVertex"]
    for t in tri:
        n = np.cross(P[t[1]] - P[t[0]], P[t[2]] - P[t[0]])
        assert np.dot(n, sc.normals[t[0], :3]) > 0
        assert np.allclose(sc.normals[t[0], :3], (0, 0, -1))
    # the lamp face had no vn: generated face normal, consistent with its winding
    s1 = sc.shapes[1]
    t = sc.indices[s1["startIdx"]:s1["startIdx"] + 3] + s1["startVertex"]
    n = np.cross(P[t[1]] - P[t[0]], P[t[2]] - P[t[0]])
    np.testing.assert_allclose(sc.normals[t[0], :3], n / np.linalg.norm(n), atol=1e-6)
    # materials: RTScene::createUberMaterial
    m = sc.materials[s0["materialId"]]
    np.testing.assert_allclose(m["uber_kd"][:3], (0.5, 0.6, 0.7))
    np.testing.assert_allclose(m["uber_ks"][:3], (0.1, 0.1, 0.1))
    np.testing.assert_allclose(m["uber_roughness"], [math.sqrt(2.0 / 100.0)] * 2, rtol=1e-6)
    assert m["uber_opacity"][:3].tolist() == [1.0, 1.0, 1.0] and m["uber_eta"] == np.float32(1.5)
    assert m["uber_diffuseTexId"] == 0 and m["uber_normalMapId"] == -1
    lamp = sc.materials[s1["materialId"]]
    np.testing.assert_allclose(lamp["uber_roughness"], [1.0, 1.0])   # Ns 0 -> sqrt(2/2) = 1
    # Ke -> triangle-mesh area light on the lamp shape
    assert len(sc.lights) == 1 and sc.lights[0]["shapeId"] == 1 and s1["lightID"] == 0
    np.testing.assert_allclose(sc.lights[0]["intensity"][:3], (17, 12, 4))
    # texture: level 0 + glGenerateMipmap chain 8x4 -> 4x2 -> 2x1 -> 1x1, REPEAT
    d = sc.textures[0]
    assert (d["width"], d["height"], d["numMipLevels"], d["wrap"]) == (4, 8, 4, 0)
    np.testing.assert_array_equal(sc.tex_data[:tex.nbytes].reshape(tex.shape), tex)
    lv1 = sc.tex_data[tex.nbytes:tex.nbytes + 4 * 2 * 4].reshape(4, 2, 4)
    exp = (tex.astype(np.uint32).reshape(4, 2, 2, 2, 4).sum((1, 3)) + 2) // 4
    np.testing.assert_array_equal(lv1, exp)
    assert len(sc.tex_data) == 4 * (32 + 8 + 2 + 1)


def test_obj_scene_renders_on_oracle(tmp_path):
    """The loaded scene goes through the same scene arrays as the generators (oracle frame)."""
    from mcrt.camera import make_camera
    from oracle import pyoracle as po
    _write_scene(str(tmp_path))
    b = objload.load_obj(str(tmp_path / "s.obj"))
    b.add_directional_light(scenes.euler_forward(45.0, 20.0), (4.0, 4.0, 4.0))
    sc = b.build()
    o = po.OracleScene(sc)
    o.build()
    cam = make_camera((0.5, 0.5, -3.0), (0.5, 0.5, 0.0), 16, 16)
    img, _ = o.render(cam, frame=0, max_depth=2)
    assert np.isfinite(img).all() and img[..., :3].max() > 0

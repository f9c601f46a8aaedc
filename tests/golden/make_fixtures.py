"""Regenerates the committed fixtures in tests/golden/ (run HERE, where /root/reference
exists; the GPU box only reads the .npz files).  Fixtures are data: inputs taken from
the reference's own asset/test files and expected outputs computed by the reference's
own C++ (oracle/_ref/librrref.so, built from /root/reference by oracle/refbuild).

  cornell_original.npz  assets/meshes/cornell-box/CornellBox-Original.{obj,mtl}
  rr_cornell.npz        RadeonRays UnitTest conformance fixture Resources/CornellBox/orig.objm
                        (loaded with the reference's tiny_obj_loader) + random rays generated
                        as ExpectClosestRaysOk does (glibc rand(), srand(0xABCDEF12),
                        radeon_rays_conformance_test_cl.h:160,552-556) + brute-force golden hits
                        from the reference's UnitTest/utils.cpp TestIntersections/TestOcclusions
  bunny.npz             assets/meshes/bunny.obj
  sobol_1024x52.npy     the Joe-Kuo Sobol generator matrices uploaded as scene data (written to
                        monte-carlo-raytracer_amd/mcrt/data/, the product's package data)
                        (source/application/PathTracer/raytracing/sampling/sobol.h:34)
  rr_bvh_mixed.npz      node array of the reference Bvh2 (bvh2.cpp) over mcrt.scenes.test_scene()

Generated on the GPU box instead (the reference's OpenCL kernels need the MI355X):
  clref_{ieee,fast}.npz       python tests/clref_job.py OUT VARIANT
  clref_bdpt_{ieee,fast}.npz  python tests/clref_job.py OUT VARIANT bdpt, then
                              tests/clref_job.py:strip_bdpt_golden(OUT, FIXTURE) keeps the
                              radiance frames and vertex counts

usage: python tests/golden/make_fixtures.py
"""
import ctypes
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "monte-carlo-raytracer_amd"))
sys.path.insert(0, ROOT)

REF = "/root/reference"


def parse_obj(path):
    """Minimal OBJ reader: v, f (polygons fan-triangulated), g/o/usemtl groups."""
    V, groups, cur = [], [], None
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "v":
            V.append([float(x) for x in t[1:4]])
        elif t[0] in ("g", "o"):
            cur = {"name": t[1] if len(t) > 1 else "default", "mtl": None, "faces": []}
            groups.append(cur)
        elif t[0] == "usemtl":
            if cur is None:
                cur = {"name": t[1], "mtl": None, "faces": []}
                groups.append(cur)
            cur["mtl"] = t[1]
        elif t[0] == "f":
            if cur is None:
                cur = {"name": "default", "mtl": None, "faces": []}
                groups.append(cur)
            idx = [int(x.split("/")[0]) for x in t[1:]]
            idx = [i - 1 if i > 0 else len(V) + i for i in idx]
            for k in range(1, len(idx) - 1):
                cur["faces"].append((idx[0], idx[k], idx[k + 1]))
    return np.array(V, np.float32), [g for g in groups if g["faces"]]


def parse_mtl(path):
    mats, cur = {}, None
    for line in open(path):
        t = line.split()
        if not t:
            continue
        if t[0] == "newmtl":
            cur = t[1]
            mats[cur] = {}
        elif cur and t[0] in ("Kd", "Ks", "Ke"):
            mats[cur][t[0]] = [float(x) for x in t[1:4]]
    return mats


def cornell():
    d = f"{REF}/assets/meshes/cornell-box"
    V, groups = parse_obj(f"{d}/CornellBox-Original.obj")
    mtl = parse_mtl(f"{d}/CornellBox-Original.mtl")
    out = {"names": np.array([g["name"] for g in groups])}
    for i, g in enumerate(groups):
        F = np.array(g["faces"], np.int64)
        used, inv = np.unique(F, return_inverse=True)
        out[f"P{i}"] = V[used]
        out[f"T{i}"] = inv.reshape(-1, 3).astype(np.int32)
        out[f"kd{i}"] = np.array(mtl.get(g["mtl"], {}).get("Kd", [0.5, 0.5, 0.5]), np.float32)
    np.savez_compressed(os.path.join(HERE, "cornell_original.npz"), **out)


def bunny():
    V, groups = parse_obj(f"{REF}/assets/meshes/bunny.obj")
    F = np.concatenate([np.array(g["faces"], np.int32) for g in groups])
    np.savez_compressed(os.path.join(HERE, "bunny.npz"), P=V, T=F)


def sobol():
    txt = open(f"{REF}/source/application/PathTracer/raytracing/sampling/sobol.h").read()
    body = txt[txt.index("g_SobolMatrices32"):]
    body = body[body.index("{") + 1: body.index("};")]
    vals = np.array([int(x, 16) for x in re.findall(r"0x[0-9A-Fa-f]+", body)], np.uint32)
    assert vals.size == 1024 * 52, vals.size
    # package data: the product uploads it as scene input (scene_sobolMatrices), like the reference
    np.save(os.path.join(HERE, "..", "..", "monte-carlo-raytracer_amd", "mcrt", "data", "sobol_1024x52.npy"), vals)


def rr_conformance(n=10000):
    from oracle import pyoracle as po
    from mcrt import types as T
    from mcrt.scenes import SceneBuilder
    shapes = po.ref_load_obj(f"{REF}/third_party/RadeonRays/Resources/CornellBox/orig.objm")
    b = SceneBuilder("rr_cornell")
    m = b.add_material()
    for P, I in shapes:
        b.add_mesh(P, np.tile([0, 1, 0], (len(P), 1)), np.zeros((len(P), 2)), I, m)
    scene = b.build()
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(0xABCDEF12)
    RAND_MAX = 2147483647

    def rand_float():
        return np.float32(np.float32(libc.rand()) / np.float32(RAND_MAX))

    rays = np.zeros(2 * n, T.RAY_DTYPE)
    for i in range(2 * n):
        o = [rand_float() * np.float32(3.0) - np.float32(1.5) for _ in range(3)]
        d = np.array([rand_float() for _ in range(3)], np.float32)
        d = d / np.float32(np.sqrt(np.float32(d @ d)))
        rays[i]["o"] = o + [1000.0]
        rays[i]["d"][:3] = d
        rays[i]["extra"] = (-1, 1)
    closest = po.ref_brute_closest(scene, rays[:n])
    occl = po.ref_brute_any(scene, rays[n:])
    out = {"rays_closest": rays[:n], "rays_any": rays[n:], "golden_closest": closest, "golden_any": occl}
    for i, (P, I) in enumerate(shapes):
        out[f"P{i}"] = P
        out[f"T{i}"] = I
    out["nshapes"] = np.array(len(shapes))
    np.savez_compressed(os.path.join(HERE, "rr_cornell.npz"), **out)


def rr_bvh_mixed():
    from oracle import pyoracle as po
    from mcrt import scenes
    nodes = po.ref_bvh_nodes(scenes.test_scene())
    np.savez_compressed(os.path.join(HERE, "rr_bvh_mixed.npz"), nodes=nodes.view(np.uint32).reshape(-1, 16))


if __name__ == "__main__":
    cornell()
    bunny()
    sobol()
    rr_conformance()
    rr_bvh_mixed()
    for f in sorted(os.listdir(HERE)):
        if f.endswith((".npz", ".npy")):
            print(f, os.path.getsize(os.path.join(HERE, f)))

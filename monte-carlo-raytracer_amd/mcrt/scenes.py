"""Scene assembly (numpy) and the deterministic synthetic benchmark proxies.

The reference's benchmark scenes (Stanford Dragon, Crytek Sponza, San Miguel) are
not in the container, so BASELINE.json's configs run on seeded
synthetic proxies with the same triangle counts and material mix.
`SceneBuilder` produces exactly the arrays RTScene uploads
(source/application/PathTracer/raytracing/scene/RTScene.cpp:564-809):
shapes, per-shape-local indices, float3 positions/normals/tangents/binormals,
float2 uvs, RGBA8 textures + TextureDesc2D, RTLight, RTMaterial.
"""
import math

import numpy as np

from . import types as T

SEED_BASE = 0x5EED


def _f4(v, w=0.0):
    v = np.asarray(v, np.float32).reshape(-1, 3)
    out = np.zeros((v.shape[0], 4), np.float32)
    out[:, :3] = v
    out[:, 3] = w
    return out


def default_material(**kw):
    """RTMaterial defaults of the reference constructor (kernel_data.h:89-94)."""
    m = np.zeros(1, T.MATERIAL_DTYPE)[0]
    m["uber_kd"] = (0.25, 0.25, 0.25, 0.0)
    m["uber_ks"] = (0.25, 0.25, 0.25, 0.0)
    m["uber_kr"] = (0.0, 0.0, 0.0, 0.0)
    m["uber_kt"] = (0.0, 0.0, 0.0, 0.0)
    m["uber_opacity"] = (1.0, 1.0, 1.0, 0.0)
    m["uber_roughness"] = (0.1, 0.1)
    m["uber_eta"] = 1.5
    m["type"] = 0
    for k in ("uber_normalMapId", "uber_diffuseTexId", "uber_glossyTexId", "uber_specReflectionTexId",
              "uber_transmissionTexId", "uber_opacityTexId", "uber_roughnessTexId", "uber_iorTexId"):
        m[k] = -1
    for k, v in kw.items():
        if k in ("kd", "ks", "kr", "opacity"):
            m["uber_" + k] = tuple(v)[:3] + (0.0,)
        elif k == "kt":
            v = tuple(v)
            m["uber_kt"] = v if len(v) == 4 else v + (0.0,)
        elif k == "roughness":
            m["uber_roughness"] = (v, v) if np.isscalar(v) else tuple(v)
        elif k == "eta":
            m["uber_eta"] = v
        else:
            m[k if k.startswith("uber_") or k == "type" else "uber_" + k] = v
    return m


class Scene:
    """The 15 SCENE_PARAMS arrays (kernel_data.h:338-352) + bookkeeping."""

    def __init__(self, shapes, indices, positions, uvs, normals, tangents, binormals, colors,
                 textures, tex_data, lights, materials, sobol=None, name="scene"):
        self.shapes = shapes
        self.indices = indices
        self.positions = positions
        self.uvs = uvs
        self.normals = normals
        self.tangents = tangents
        self.binormals = binormals
        self.colors = colors
        self.textures = textures
        self.tex_data = tex_data
        self.lights = lights
        self.materials = materials
        self.sobol = sobol
        self.name = name
        self._desc = None

    @property
    def num_triangles(self):
        return int(self.shapes["numTriangles"].sum())

    def desc(self):
        d = T.SceneDesc()
        d.shapes, d.num_shapes = T.ptr(self.shapes), len(self.shapes)
        d.indices, d.num_indices = T.ptr(self.indices), len(self.indices)
        d.positions, d.num_vertices = T.ptr(self.positions), len(self.positions)
        d.uvs = T.ptr(self.uvs)
        d.normals = T.ptr(self.normals)
        d.tangents = T.ptr(self.tangents)
        d.binormals = T.ptr(self.binormals)
        d.colors = T.ptr(self.colors)
        d.textures, d.num_textures = (T.ptr(self.textures), len(self.textures)) if len(self.textures) else (None, 0)
        d.tex_data, d.tex_data_bytes = (T.ptr(self.tex_data), self.tex_data.nbytes) if self.tex_data.nbytes else (None, 0)
        if self.sobol is not None:
            d.sobol_matrices, d.num_sobol_words = T.ptr(self.sobol), self.sobol.size
        d.lights, d.num_lights = (T.ptr(self.lights), len(self.lights)) if len(self.lights) else (None, 0)
        d.materials, d.num_materials = (T.ptr(self.materials), len(self.materials)) if len(self.materials) else (None, 0)
        self._desc = d
        return d

    def world_triangles(self):
        """(T, 3, 3) float32 world-space triangles (identity transforms only)."""
        out = []
        for s in self.shapes:
            idx = self.indices[s["startIdx"]: s["startIdx"] + 3 * s["numTriangles"]].astype(np.int64) + s["startVertex"]
            P = self.positions[idx, :3].reshape(-1, 3, 3)
            M = s["toWorldTransform"]
            if not np.array_equal(M, np.eye(4, dtype=np.float32)):
                P = (P @ M[:3, :3].T) + M[:3, 3]
            out.append(P.astype(np.float32))
        return np.concatenate(out) if out else np.zeros((0, 3, 3), np.float32)

    def bbox(self):
        """World-space bounds of the shapes (transforms applied)."""
        M = self.shapes["toWorldTransform"]
        if np.array_equal(M, np.broadcast_to(np.eye(4, dtype=np.float32), M.shape)):
            P = self.positions[:, :3]
        else:
            P = self.world_triangles().reshape(-1, 3)
        return P.min(0), P.max(0)


class SceneBuilder:
    def __init__(self, name="scene"):
        self.name = name
        self.meshes = []       # (P, N, UV, tris, material, transform, is_light)
        self.materials = []
        self.textures = []     # (rgba uint8 (h, w, 4), wrap)
        self.lights = []       # dicts
        self.sobol = None

    # -- content --------------------------------------------------------
    def add_material(self, **kw):
        self.materials.append(default_material(**kw))
        return len(self.materials) - 1

    def add_texture(self, rgba, wrap=0, mips=False):
        """RGBA8 texture; mips=True stores its glGenerateMipmap chain after level 0 the way
        RTScene::uploadTextures packs it (RTScene.cpp:680-766; only level 0 is sampled, the
        reference's LOD path is disabled at textures.cl:207)."""
        rgba = np.ascontiguousarray(rgba, np.uint8)
        assert rgba.ndim == 3 and rgba.shape[2] == 4
        if mips:
            from .objload import mip_chain
            self.textures.append((mip_chain(rgba), wrap))
        else:
            self.textures.append((rgba, wrap))
        return len(self.textures) - 1

    def add_mesh(self, P, N, UV, tris, material, transform=None):
        P = np.asarray(P, np.float32).reshape(-1, 3)
        N = np.asarray(N, np.float32).reshape(-1, 3)
        UV = np.asarray(UV, np.float32).reshape(-1, 2)
        tris = np.asarray(tris, np.uint32).reshape(-1, 3)
        self.meshes.append((P, N, UV, tris, int(material), transform))
        return len(self.meshes) - 1

    def add_instance(self, mesh, transform, material=None):
        """Another shape that shares mesh `mesh`'s vertex and index data (same startIdx,
        startVertex, numTriangles) under its own transform: what RTScene::attachMesh records for
        every further entity of an already attached mesh (RTScene.cpp:572-596), which makes
        RadeonRays build its two-level structure.  material None = the first entity's material,
        as the reference's instance shapes carry (sharedShapeInfo.materialId)."""
        base = mesh
        while self.meshes[base][0] is None:
            base = self.meshes[base][1]
        mat = self.meshes[base][4] if material is None else int(material)
        self.meshes.append((None, base, None, None, mat, transform))
        return len(self.meshes) - 1

    def add_directional_light(self, direction, intensity):
        self.lights.append({"type": T.DIRECTIONAL, "d": np.asarray(direction, np.float64), "intensity": intensity})
        return len(self.lights) - 1

    def add_point_light(self, p, intensity):
        self.lights.append({"type": T.POINT, "p": p, "intensity": intensity})
        return len(self.lights) - 1

    def add_disk_light(self, p, d, radius, intensity):
        self.lights.append({"type": T.DISK_AREA, "p": p, "d": d, "radius": radius, "intensity": intensity})
        return len(self.lights) - 1

    def add_mesh_light(self, shape, intensity):
        self.lights.append({"type": T.TRIANGLE_MESH_AREA, "shape": shape, "intensity": intensity})
        return len(self.lights) - 1

    # -- assembly -------------------------------------------------------
    def build(self, sobol=None):
        nshape = len(self.meshes)
        shapes = np.zeros(nshape, T.SHAPE_DTYPE)
        nv = sum(m[0].shape[0] for m in self.meshes if m[0] is not None)
        ni = sum(m[3].size for m in self.meshes if m[0] is not None)
        positions = np.zeros((nv, 4), np.float32)
        normals = np.zeros((nv, 4), np.float32)
        tangents = np.zeros((nv, 4), np.float32)
        binormals = np.zeros((nv, 4), np.float32)
        uvs = np.zeros((nv, 2), np.float32)
        indices = np.zeros(ni, np.uint32)
        v0 = i0 = 0
        for k, (P, N, UV, tris, mat, M) in enumerate(self.meshes):
            if P is None:   # instance of shape N (= base mesh index)
                base = self.meshes[N]
                s = shapes[k]
                Mw = np.eye(4, dtype=np.float32) if M is None else np.asarray(M, np.float32)
                s["toWorldTransform"] = Mw
                s["toWorldInverseTranspose"] = np.linalg.inv(Mw.astype(np.float64)).T.astype(np.float32)
                for f in ("startIdx", "startVertex", "numTriangles"):
                    s[f] = shapes[N][f]
                s["materialId"] = mat
                s["lightID"] = -1
                Pw = base[0] @ Mw[:3, :3].T + Mw[:3, 3]
                tri = Pw[base[3].astype(np.int64)]
                s["area"] = 0.5 * np.linalg.norm(np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]), axis=1).sum()
                continue
            n = P.shape[0]
            positions[v0:v0 + n, :3] = P
            normals[v0:v0 + n, :3] = N
            uvs[v0:v0 + n] = UV
            # tangent frame (unused by the PT kernel; RTScene uploads assimp's)
            t = np.cross(N, np.array([0.0, 1.0, 0.0], np.float32))
            bad = np.linalg.norm(t, axis=1) < 1e-4
            t[bad] = np.cross(N[bad], np.array([1.0, 0.0, 0.0], np.float32))
            t /= np.maximum(np.linalg.norm(t, axis=1, keepdims=True), 1e-20)
            tangents[v0:v0 + n, :3] = t
            binormals[v0:v0 + n, :3] = np.cross(N, t)
            indices[i0:i0 + tris.size] = tris.reshape(-1)
            s = shapes[k]
            Mw = np.eye(4, dtype=np.float32) if M is None else np.asarray(M, np.float32)
            s["toWorldTransform"] = Mw
            s["toWorldInverseTranspose"] = np.linalg.inv(Mw.astype(np.float64)).T.astype(np.float32)
            s["startIdx"] = i0
            s["startVertex"] = v0
            s["numTriangles"] = tris.shape[0]
            s["materialId"] = mat
            s["lightID"] = -1
            Pw = P @ Mw[:3, :3].T + Mw[:3, 3]
            tri = Pw[tris.astype(np.int64)]
            s["area"] = 0.5 * np.linalg.norm(np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]), axis=1).sum()
            s["pad"] = 0
            v0 += n
            i0 += tris.size
        # scene bbox (RTScene::m_sceneBBox, used by directional lights: RTScene.cpp:484-489)
        if nv:
            Pw_all = []
            for k, (P, N, UV, tris, mat, M) in enumerate(self.meshes):
                Mw = shapes[k]["toWorldTransform"]
                if P is None:
                    P = self.meshes[N][0]
                Pw_all.append((P @ Mw[:3, :3].T + Mw[:3, 3]).astype(np.float32))
            Pw_all = np.concatenate(Pw_all)
            bmin, bmax = Pw_all.min(0), Pw_all.max(0)
        else:
            bmin = bmax = np.zeros(3, np.float32)
        lights = np.zeros(len(self.lights), T.LIGHT_DTYPE)
        for i, L in enumerate(self.lights):
            l = lights[i]
            l["shapeId"] = -1
            l["intensity"][:3] = L["intensity"]
            l["type"] = L["type"]
            if L["type"] == T.DIRECTIONAL:   # RTScene::setLight, RTScene.cpp:482-494
                d = np.asarray(L["d"], np.float64)
                d = d / np.linalg.norm(d)
                radius = np.float32(np.linalg.norm(bmax - bmin) * 0.5)
                center = (bmin.astype(np.float64) + bmax) * 0.5
                l["d"][:3] = d
                l["radius"] = radius
                l["p"][:3] = center - d * radius
                l["flags"] = T.FLAG_DELTA_DIRECTION
                l["area"] = np.float32(math.pi) * radius * radius
            elif L["type"] == T.POINT:
                l["p"][:3] = L["p"]
                l["flags"] = T.FLAG_DELTA_POSITION
            elif L["type"] == T.DISK_AREA:
                l["p"][:3] = L["p"]
                dd = np.asarray(L["d"], np.float64)
                l["d"][:3] = dd / np.linalg.norm(dd)
                l["radius"] = L["radius"]
                l["area"] = np.float32(math.pi) * np.float32(L["radius"]) ** 2
                l["flags"] = T.FLAG_AREA
            else:                            # RTScene.cpp:525-545
                sh = L["shape"]
                l["shapeId"] = sh
                l["flags"] = T.FLAG_AREA
                l["area"] = shapes[sh]["area"]
                l["p"][:3] = 0.0
                shapes[sh]["lightID"] = i
        if len(lights):
            lights["choicePdf"] = np.float32(1.0) / np.float32(len(lights))   # RTScene.cpp:811-819
        # textures: one RGBA8 byte buffer + TextureDesc2D (RTScene::uploadTextures, RTScene.cpp:680-766)
        descs = np.zeros(len(self.textures), T.TEXDESC_DTYPE)
        chunks, off = [], 0
        for i, (img, wrap) in enumerate(self.textures):
            levels = img if isinstance(img, list) else [img]
            h, w = levels[0].shape[:2]
            descs[i] = (w, h, len(levels), 3, wrap, 0, off)
            for lv in levels:
                chunks.append(lv.reshape(-1))
                off += lv.nbytes
        tex_data = np.concatenate(chunks) if chunks else np.zeros(0, np.uint8)
        materials = np.array(self.materials, T.MATERIAL_DTYPE) if self.materials else np.zeros(0, T.MATERIAL_DTYPE)
        return Scene(shapes, indices, positions, uvs, normals, tangents, binormals, None, descs,
                     tex_data, lights, materials, sobol=sobol, name=self.name)


# --------------------------------------------------------------------------
# geometry primitives
# --------------------------------------------------------------------------
def grid(origin, du, dv, nu, nv, uv_scale=1.0, flip=False):
    """Subdivided parallelogram: nu x nv quads, 2*nu*nv triangles."""
    origin, du, dv = (np.asarray(x, np.float64) for x in (origin, du, dv))
    s = np.linspace(0.0, 1.0, nu + 1)
    t = np.linspace(0.0, 1.0, nv + 1)
    S, Tt = np.meshgrid(s, t, indexing="xy")
    P = origin + S[..., None] * du + Tt[..., None] * dv
    n = np.cross(du, dv)
    n = n / np.linalg.norm(n)
    if flip:
        n = -n
    N = np.broadcast_to(n, P.shape)
    UV = np.stack([S, Tt], -1) * uv_scale
    i = np.arange(nv)[:, None] * (nu + 1) + np.arange(nu)[None, :]
    a, b, c, d = i, i + 1, i + nu + 2, i + nu + 1
    if flip:
        tris = np.concatenate([np.stack([a, c, b], -1).reshape(-1, 3), np.stack([a, d, c], -1).reshape(-1, 3)])
    else:
        tris = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    return P.reshape(-1, 3), N.reshape(-1, 3), UV.reshape(-1, 2), tris


def box(lo, hi, n=1):
    lo, hi = np.asarray(lo, np.float64), np.asarray(hi, np.float64)
    e = hi - lo
    X, Y, Z = np.array([e[0], 0, 0]), np.array([0, e[1], 0]), np.array([0, 0, e[2]])
    faces = [
        (lo, Y, X), (lo + Z, X, Y),           # -z, +z
        (lo, Z, Y), (lo + X, Y, Z),           # -x, +x
        (lo, X, Z), (lo + Y, Z, X),           # -y, +y
    ]
    return merge([grid(o, a, b, n, n) for o, a, b in faces])


def cylinder(base, radius, height, nseg=16, nh=4, cap=False):
    base = np.asarray(base, np.float64)
    th = np.linspace(0, 2 * np.pi, nseg + 1)
    y = np.linspace(0, height, nh + 1)
    TH, Y = np.meshgrid(th, y, indexing="xy")
    P = np.stack([base[0] + radius * np.cos(TH), base[1] + Y, base[2] + radius * np.sin(TH)], -1)
    N = np.stack([np.cos(TH), np.zeros_like(TH), np.sin(TH)], -1)
    UV = np.stack([TH / (2 * np.pi) * 2.0, Y / max(height, 1e-6)], -1)
    i = np.arange(nh)[:, None] * (nseg + 1) + np.arange(nseg)[None, :]
    a, b, c, d = i, i + 1, i + nseg + 2, i + nseg + 1
    tris = np.concatenate([np.stack([a, c, b], -1).reshape(-1, 3), np.stack([a, d, c], -1).reshape(-1, 3)])
    return P.reshape(-1, 3), N.reshape(-1, 3), UV.reshape(-1, 2), tris


def merge(parts):
    Ps, Ns, UVs, Ts, off = [], [], [], [], 0
    for P, N, UV, tris in parts:
        Ps.append(P); Ns.append(N); UVs.append(UV); Ts.append(tris + off)
        off += P.shape[0]
    return np.concatenate(Ps), np.concatenate(Ns), np.concatenate(UVs), np.concatenate(Ts)


def displaced_sphere(center, radius, nu, nv, rng, amp=0.12, octaves=5):
    """Closed, noise-displaced UV sphere (the Dragon proxy body): 2*nu*(nv-1) triangles."""
    th = np.linspace(0.0, 2 * np.pi, nu + 1)[:-1]
    ph = np.linspace(0.0, np.pi, nv + 1)
    TH, PH = np.meshgrid(th, ph, indexing="xy")
    dirs = np.stack([np.sin(PH) * np.cos(TH), np.cos(PH), np.sin(PH) * np.sin(TH)], -1)
    disp = np.zeros(TH.shape)
    for o in range(octaves):
        k = rng.normal(size=3) * (2.0 ** o) * 2.0
        phase = rng.uniform(0, 2 * np.pi)
        disp += np.sin(dirs @ k + phase) * (0.5 ** o)
    r = radius * (1.0 + amp * disp / 2.0)
    r[0, :] = r[0, 0]
    r[-1, :] = r[-1, 0]
    P = center + dirs * r[..., None]
    # normals by finite differences on the grid (periodic in theta)
    dth = np.roll(P, -1, axis=1) - np.roll(P, 1, axis=1)
    dph = np.zeros_like(P)
    dph[1:-1] = P[2:] - P[:-2]
    dph[0] = dph[1]
    dph[-1] = dph[-2]
    N = np.cross(dph, dth)
    ln = np.linalg.norm(N, axis=-1, keepdims=True)
    N = np.where(ln > 1e-12, N / np.maximum(ln, 1e-30), dirs)
    UV = np.stack([TH / (2 * np.pi), PH / np.pi], -1)
    i = np.arange(nv)[:, None] * nu + np.arange(nu)[None, :]
    j = np.arange(nv)[:, None] * nu + (np.arange(nu)[None, :] + 1) % nu
    a, b, c, d = i, j, j + nu, i + nu
    t1 = np.stack([a, c, b], -1)[1:].reshape(-1, 3)    # skip degenerate pole rows
    t2 = np.stack([a, d, c], -1)[:-1].reshape(-1, 3)
    return P.reshape(-1, 3), N.reshape(-1, 3), UV.reshape(-1, 2), np.concatenate([t1, t2])


def foliage(centers, radii, quads_per_crown, leaf_size, rng):
    """Many small randomly oriented quads in spherical crowns (San-Miguel trees)."""
    parts = []
    for c, R in zip(centers, radii):
        k = quads_per_crown
        u = rng.normal(size=(k, 3))
        u /= np.linalg.norm(u, axis=1, keepdims=True)
        rr = R * rng.uniform(0.2, 1.0, size=(k, 1)) ** (1.0 / 3.0)
        ctr = np.asarray(c) + u * rr
        n = rng.normal(size=(k, 3))
        n /= np.linalg.norm(n, axis=1, keepdims=True)
        a = np.cross(n, rng.normal(size=(k, 3)))
        a /= np.linalg.norm(a, axis=1, keepdims=True)
        b = np.cross(n, a)
        s = leaf_size * rng.uniform(0.6, 1.4, size=(k, 1))
        corners = np.stack([ctr - a * s - b * s, ctr + a * s - b * s, ctr + a * s + b * s, ctr - a * s + b * s], 1)
        P = corners.reshape(-1, 3)
        N = np.repeat(n, 4, axis=0)
        UV = np.tile(np.array([[0, 0], [1, 0], [1, 1], [0, 1]], np.float64), (k, 1))
        base = (np.arange(k) * 4)[:, None]
        tris = np.concatenate([base + np.array([0, 1, 2]), base + np.array([0, 2, 3])])
        parts.append((P, N, UV, tris))
    return merge(parts)


# --------------------------------------------------------------------------
# procedural textures (RGBA8)
# --------------------------------------------------------------------------
def tex_checker(n, c0, c1, tiles=8):
    y, x = np.mgrid[0:n, 0:n]
    m = ((x * tiles // n) + (y * tiles // n)) % 2
    img = np.where(m[..., None] == 0, np.array(c0 + (255,), np.uint8), np.array(c1 + (255,), np.uint8))
    return img.astype(np.uint8)


def tex_noise(n, rng, base, var=60):
    img = np.empty((n, n, 4), np.uint8)
    noise = rng.integers(-var, var + 1, size=(n, n, 1))
    img[..., :3] = np.clip(np.asarray(base)[None, None, :] + noise, 0, 255)
    img[..., 3] = 255
    return img


def tex_leaf(n, color=(60, 140, 50)):
    """Leaf cut-out: alpha = 255 inside an ellipse (opacity via Kd.w, materials.cl:80-86)."""
    y, x = (np.mgrid[0:n, 0:n] + 0.5) / n
    inside = ((x - 0.5) / 0.45) ** 2 + ((y - 0.5) / 0.3) ** 2 < 1.0
    img = np.zeros((n, n, 4), np.uint8)
    img[..., 0], img[..., 1], img[..., 2] = color
    img[..., 3] = np.where(inside, 255, 0)
    return img


def tex_bricks(n, mortar=(200, 200, 190), brick=(150, 60, 40)):
    y, x = np.mgrid[0:n, 0:n]
    row = y // (n // 8)
    off = (row % 2) * (n // 8)
    m = (((x + off) % (n // 4)) < 3) | ((y % (n // 8)) < 3)
    img = np.where(m[..., None], np.array(mortar + (255,), np.uint8), np.array(brick + (255,), np.uint8))
    return img.astype(np.uint8)


def tex_normalmap(n, rng, strength=0.3):
    g = rng.normal(size=(n, n, 2)) * strength
    nz = np.sqrt(np.maximum(0.0, 1.0 - (g ** 2).sum(-1)))
    v = np.concatenate([g, nz[..., None]], -1)
    img = np.empty((n, n, 4), np.uint8)
    img[..., :3] = np.clip((v * 0.5 + 0.5) * 255.0, 0, 255)
    img[..., 3] = 255
    return img


# --------------------------------------------------------------------------
# scenes
# --------------------------------------------------------------------------
def euler_forward(pitch_deg, yaw_deg):
    p, y = math.radians(pitch_deg), math.radians(yaw_deg)
    return np.array([math.cos(p) * math.sin(y), -math.sin(p), math.cos(p) * math.cos(y)])


def cornell_box(fixture):
    """CornellBox-Original (assets/meshes/cornell-box/CornellBox-Original.obj), from the
    committed fixture tests/golden/cornell_original.npz (data only), with the demo's
    directional light (PathTracingApp.cpp:395-401) and the 'light' group (Ke 17 12 4)
    as a triangle-mesh area light."""
    z = np.load(fixture, allow_pickle=False)
    b = SceneBuilder("cornell")
    names = [str(n) for n in z["names"]]
    light_shape = None
    for i, name in enumerate(names):
        P = z[f"P{i}"]
        tris = z[f"T{i}"]
        kd = tuple(float(x) for x in z[f"kd{i}"])
        tri = P[tris]
        n = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
        n /= np.linalg.norm(n, axis=1, keepdims=True)
        N = np.zeros_like(P)
        np.add.at(N, tris.reshape(-1), np.repeat(n, 3, axis=0))
        N /= np.maximum(np.linalg.norm(N, axis=1, keepdims=True), 1e-20)
        UV = P[:, [0, 2]] * 0.5
        mat = b.add_material(kd=kd, ks=(0.0, 0.0, 0.0), roughness=0.5)
        sid = b.add_mesh(P, N, UV, tris, mat)
        if name == "light":
            light_shape = sid
    b.add_directional_light(euler_forward(46.0, -14.0), (40.0, 40.0, 40.0))
    if light_shape is not None:
        b.add_mesh_light(light_shape, (17.0, 12.0, 4.0))
    return b.build()


def material_zoo(b, rng, tex):
    """One material per uber-BSDF lobe combination (divergence stress)."""
    mats = []
    mats.append(b.add_material(kd=(0.7, 0.7, 0.7), ks=(0, 0, 0)))                                   # lambert
    mats.append(b.add_material(kd=(0.5, 0.3, 0.2), ks=(0.3, 0.3, 0.3), roughness=0.3))              # plastic
    mats.append(b.add_material(kd=(0.0, 0.0, 0.0), ks=(0.9, 0.8, 0.6), roughness=0.05))             # glossy metal-ish
    mats.append(b.add_material(kd=(0.1, 0.1, 0.1), ks=(0, 0, 0), kr=(0.8, 0.8, 0.8)))               # mirror + diffuse
    mats.append(b.add_material(kd=(0, 0, 0), ks=(0, 0, 0), kt=(0.9, 0.9, 0.9, 1.0), roughness=0.2, eta=1.5))  # glossy glass
    mats.append(b.add_material(kd=(0, 0, 0), ks=(0.2, 0.2, 0.2), kt=(0.9, 0.95, 0.9, 0.0), eta=1.33))  # specular glass
    mats.append(b.add_material(kd=(0.6, 0.6, 0.6), ks=(0.2, 0.2, 0.2), opacity=(0.5, 0.5, 0.5)))    # half-transparent
    mats.append(b.add_material(kd=(1, 1, 1), ks=(0.1, 0.1, 0.1), diffuseTexId=tex["checker"], roughness=(0.1, 0.4)))  # anisotropic
    mats.append(b.add_material(kd=(1, 1, 1), ks=(0, 0, 0), diffuseTexId=tex["leaf"]))               # alpha cut-out
    mats.append(b.add_material(kd=(0.8, 0.8, 0.8), ks=(0.1, 0.1, 0.1), normalMapId=tex["normal"]))  # normal mapped
    return mats


def test_scene(seed=1, n_sphere=40):
    """Small mixed scene (every BSDF lobe, textures, all 4 light types) for parity tests."""
    rng = np.random.default_rng(SEED_BASE + seed)
    b = SceneBuilder("mixed")
    tex = {
        "checker": b.add_texture(tex_checker(64, (220, 220, 220), (40, 40, 160))),
        "leaf": b.add_texture(tex_leaf(32)),
        "normal": b.add_texture(tex_normalmap(32, rng)),
        "bricks": b.add_texture(tex_bricks(64), wrap=2),
    }
    mats = material_zoo(b, rng, tex)
    floor = b.add_material(kd=(1, 1, 1), ks=(0, 0, 0), diffuseTexId=tex["checker"])
    b.add_mesh(*grid((-6, 0, -6), (12, 0, 0), (0, 0, 12), 4, 4, uv_scale=3.0, flip=True), floor)
    wall = b.add_material(kd=(1, 1, 1), ks=(0.05, 0.05, 0.05), diffuseTexId=tex["bricks"])
    b.add_mesh(*grid((-6, 0, 6), (12, 0, 0), (0, 6, 0), 3, 3, uv_scale=1.0, flip=True), wall)
    for i, m in enumerate(mats):
        x = -4.5 + (i % 5) * 2.2
        zc = -1.5 + (i // 5) * 3.0
        b.add_mesh(*displaced_sphere(np.array([x, 0.9, zc]), 0.8, n_sphere, n_sphere // 2, rng, amp=0.1), m)
    lm = b.add_material(kd=(0.8, 0.8, 0.8), ks=(0, 0, 0))
    ls = b.add_mesh(*grid((-1, 5.0, -1), (2, 0, 0), (0, 0, 2), 1, 1, flip=True), lm)
    b.add_directional_light(euler_forward(50.0, 30.0), (4.0, 4.0, 4.0))
    b.add_mesh_light(ls, (12.0, 10.0, 8.0))
    b.add_point_light((3.0, 3.0, -3.0), (6.0, 6.0, 6.0))
    b.add_disk_light((-3.0, 4.0, 0.0), (0.3, -1.0, 0.1), 0.6, (5.0, 5.0, 6.0))
    return b.build()


def dragon_proxy(tris=871_414, seed=2):
    """Stanford-Dragon proxy (config 1/2): one noise-displaced closed mesh on a ground
    quad, the demo's directional light (intensity 40) + a triangle-mesh area light."""
    rng = np.random.default_rng(SEED_BASE + seed)
    b = SceneBuilder("dragon_proxy")
    ground_tex = b.add_texture(tex_checker(256, (200, 200, 200), (90, 90, 90), tiles=16))
    ground = b.add_material(kd=(0.8, 0.8, 0.8), ks=(0.05, 0.05, 0.05), diffuseTexId=ground_tex, roughness=0.4)
    body = b.add_material(kd=(0.55, 0.45, 0.25), ks=(0.35, 0.3, 0.2), roughness=0.25)
    b.add_mesh(*grid((-8, 0, -8), (16, 0, 0), (0, 0, 16), 8, 8, uv_scale=4.0, flip=True), ground)
    body_tris = max(tris - 128 - 2, 64)
    nu = max(8, int(round(math.sqrt(body_tris / 1.0))))
    nv = max(4, int(body_tris // (2 * nu)) + 1)
    b.add_mesh(*displaced_sphere(np.array([0.0, 1.6, 0.0]), 1.5, nu, nv, rng, amp=0.25, octaves=7), body)
    lm = b.add_material(kd=(0.8, 0.8, 0.8), ks=(0, 0, 0))
    ls = b.add_mesh(*grid((-1.5, 6.0, -1.5), (3, 0, 0), (0, 0, 3), 1, 1, flip=True), lm)
    b.add_directional_light(euler_forward(45.5, 87.0), (40.0, 40.0, 40.0))
    b.add_mesh_light(ls, (17.0, 12.0, 4.0))
    return b.build()


def _affine(scale, yaw_deg, t, tilt_deg=0.0):
    """4x4 float32 local-to-world: translate(t) * rotY(yaw) * rotX(tilt) * scale."""
    a, b = math.radians(yaw_deg), math.radians(tilt_deg)
    ry = np.array([[math.cos(a), 0, math.sin(a)], [0, 1, 0], [-math.sin(a), 0, math.cos(a)]])
    rx = np.array([[1, 0, 0], [0, math.cos(b), -math.sin(b)], [0, math.sin(b), math.cos(b)]])
    M = np.eye(4)
    M[:3, :3] = ry @ rx * scale
    M[:3, 3] = t
    return M.astype(np.float32)


def instanced_proxy(grid_n=8, body_tris=60_000, seed=5):
    """Instancing workload: a field of grid_n x grid_n copies of two
    shared meshes (a displaced 'rock' and a column) under rotated / scaled / translated
    transforms, on a ground plane with a mesh light -- the scene shape for which RTScene
    creates RadeonRays instances and RR switches to its two-level intersector.  ~2 x grid_n^2
    x body_tris effective triangles from 2 x body_tris stored."""
    rng = np.random.default_rng(SEED_BASE + seed)
    b = SceneBuilder("instanced_proxy")
    ground_tex = b.add_texture(tex_checker(128, (190, 190, 190), (80, 80, 90), tiles=16))
    ground = b.add_material(kd=(0.8, 0.8, 0.8), ks=(0.05, 0.05, 0.05), diffuseTexId=ground_tex, roughness=0.5)
    rock = b.add_material(kd=(0.5, 0.42, 0.3), ks=(0.3, 0.28, 0.2), roughness=0.3)
    metal = b.add_material(kd=(0.1, 0.1, 0.1), ks=(0.9, 0.85, 0.7), roughness=0.15)
    half = grid_n * 1.5
    b.add_mesh(*grid((-half - 2, 0, -half - 2), (2 * half + 4, 0, 0), (0, 0, 2 * half + 4), 8, 8, uv_scale=6.0,
                     flip=True), ground)
    nu = max(8, int(round(math.sqrt(body_tris))))
    nv = max(4, body_tris // (2 * nu) + 1)
    rock_mesh = None
    col_mesh = None
    for i in range(grid_n):
        for j in range(grid_n):
            x, z = -half + 3.0 * i + 1.5, -half + 3.0 * j + 1.5
            if (i + j) % 2 == 0:
                M = _affine(rng.uniform(0.6, 1.1), rng.uniform(0, 360), (x, 0.9, z), rng.uniform(-20, 20))
                if rock_mesh is None:
                    P, N, UV, tris = displaced_sphere(np.zeros(3), 1.0, nu, nv, rng, amp=0.25, octaves=6)
                    rock_mesh = b.add_mesh(P, N, UV, tris, rock, transform=M)
                else:
                    b.add_instance(rock_mesh, M)
            else:
                M = _affine(rng.uniform(0.8, 1.2), rng.uniform(0, 360), (x, 0.0, z))
                if col_mesh is None:
                    P, N, UV, tris = cylinder(np.zeros(3), 0.5, 2.5, nseg=max(16, body_tris // 64), nh=16, cap=True)
                    col_mesh = b.add_mesh(P, N, UV, tris, metal, transform=M)
                else:
                    b.add_instance(col_mesh, M)
    lm = b.add_material(kd=(0.8, 0.8, 0.8), ks=(0, 0, 0))
    ls = b.add_mesh(*grid((-2.0, 7.0, -2.0), (4, 0, 0), (0, 0, 4), 1, 1, flip=True), lm)
    b.add_directional_light(euler_forward(50.0, 60.0), (6.0, 6.0, 6.0))
    b.add_mesh_light(ls, (20.0, 16.0, 12.0))
    return b.build()


def instances_test_scene(seed=0):
    """Small instancing parity scene: meshes and instances interleaved in attach order (the
    std::partition order of IntersectorTwoLevel::Process matters), a single-triangle mesh
    (bottom tree = one leaf), scaled / rotated / tilted instances with per-instance materials,
    a mesh light and a point light."""
    rng = np.random.default_rng(SEED_BASE + 100 + seed)
    b = SceneBuilder("instances_test")
    tex = b.add_texture(tex_checker(64, (220, 220, 220), (60, 60, 150)))
    m0 = b.add_material(kd=(0.7, 0.6, 0.5), ks=(0.2, 0.2, 0.2), roughness=0.3)
    m1 = b.add_material(kd=(0.2, 0.5, 0.7), ks=(0.6, 0.6, 0.6), roughness=0.1)
    floor = b.add_material(kd=(1, 1, 1), diffuseTexId=tex)
    b.add_mesh(*grid((-9, 0, -9), (18, 0, 0), (0, 0, 18), 4, 4, uv_scale=4.0, flip=True), floor)
    A = b.add_mesh(*displaced_sphere(np.zeros(3), 1.0, 24, 12, rng), m0, transform=_affine(1.0, 10.0, (0, 1, 0)))
    b.add_instance(A, _affine(0.5, 45.0, (3, 1, 0), 30.0))
    B = b.add_mesh(*grid((-1, 0, -1), (2, 0, 0), (0, 0, 2), 3, 3), m1, transform=_affine(1.0, 0.0, (0, 0.01, -4)))
    b.add_instance(A, _affine(2.0, -70.0, (-4, 2, 1)), material=m1)
    b.add_instance(B, _affine(1.0, 90.0, (0, 3, 5), 80.0))
    C = b.add_mesh(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0]], np.float32), np.tile([0, 0, 1], (3, 1)),
                   np.zeros((3, 2)), np.array([[0, 1, 2]]), m0, transform=_affine(1.0, 0.0, (2, 0, -3)))
    b.add_instance(C, _affine(3.0, 33.0, (-2, 0, -3), 12.0))
    for i in range(6):
        b.add_instance(A, _affine(rng.uniform(0.3, 1.5), rng.uniform(0, 360), rng.uniform(-7, 7, 3) * (1, 0, 1)
                                  + (0, 1.2, 0), rng.uniform(-40, 40)))
    lm = b.add_material(kd=(0.8, 0.8, 0.8), ks=(0, 0, 0))
    ls = b.add_mesh(*grid((-1, 6.0, -1), (2, 0, 0), (0, 0, 2), 1, 1, flip=True), lm)
    b.add_mesh_light(ls, (14.0, 12.0, 10.0))
    b.add_point_light((3.0, 5.0, -3.0), (6.0, 6.0, 6.0))
    b.add_directional_light(euler_forward(50.0, 30.0), (3.0, 3.0, 3.0))
    return b.build()


def lod_test_scene(seed=0):
    """Texture-LOD workload: a large checker floor and a brick wall seen at grazing angles
    (strong minification), textured spheres with normal maps, every texture with its full mip
    chain (numMipLevels > 1), plus one untextured sphere."""
    rng = np.random.default_rng(SEED_BASE + 200 + seed)
    b = SceneBuilder("lod_test")
    checker = b.add_texture(tex_checker(256, (230, 230, 230), (30, 30, 120), tiles=32), mips=True)
    bricks = b.add_texture(tex_bricks(128), mips=True)
    normal = b.add_texture(tex_normalmap(64, rng), mips=True)
    leaf = b.add_texture(tex_leaf(64), wrap=2, mips=True)
    floor = b.add_material(kd=(1, 1, 1), ks=(0.04, 0.04, 0.04), roughness=0.4, diffuseTexId=checker)
    wall = b.add_material(kd=(1, 1, 1), diffuseTexId=bricks, normalMapId=normal)
    b.add_mesh(*grid((-40, 0, -10), (80, 0, 0), (0, 0, 120), 8, 8, uv_scale=12.0, flip=True), floor)
    b.add_mesh(*grid((-40, 0, 60), (80, 0, 0), (0, 12, 0), 4, 4, uv_scale=6.0, flip=True), wall)
    for i in range(5):
        m = b.add_material(kd=(0.9, 0.9, 0.9), ks=(0.2, 0.2, 0.2), roughness=0.3,
                           diffuseTexId=(leaf if i % 2 else checker), normalMapId=normal if i == 2 else -1)
        b.add_mesh(*displaced_sphere(np.array([-6.0 + 3.0 * i, 1.0, 4.0 + 2.0 * i]), 1.0, 32, 16, rng, amp=0.05), m)
    plain = b.add_material(kd=(0.7, 0.3, 0.2))
    b.add_mesh(*displaced_sphere(np.array([8.0, 1.0, 2.0]), 1.0, 32, 16, rng, amp=0.05), plain)
    b.add_directional_light(euler_forward(40.0, 20.0), (5.0, 5.0, 5.0))
    b.add_point_light((0.0, 6.0, 0.0), (20.0, 20.0, 20.0))
    return b.build()


def san_miguel_proxy(tris=10_000_000, seed=4, tex_size=512):
    """San-Miguel proxy (configs 4/5 and the headline metric): courtyard with arcades,
    tables, ~70 % of the triangles in foliage quads with alpha cut-out leaves, >= 64
    materials covering every uber-BSDF lobe mix."""
    rng = np.random.default_rng(SEED_BASE + seed)
    b = SceneBuilder("san_miguel_proxy")
    tex = {
        "checker": b.add_texture(tex_checker(tex_size, (210, 200, 180), (120, 90, 70), tiles=16)),
        "leaf": b.add_texture(tex_leaf(64)),
        "normal": b.add_texture(tex_normalmap(128, rng)),
        "bricks": b.add_texture(tex_bricks(tex_size)),
        "plaster": b.add_texture(tex_noise(tex_size, rng, (200, 180, 150), 25)),
        "stone": b.add_texture(tex_noise(tex_size, rng, (140, 140, 130), 40)),
    }
    zoo = material_zoo(b, rng, tex)
    mats = list(zoo)
    while len(mats) < 72:   # >= 64 materials: random variations of the zoo
        k = int(rng.integers(0, 7))
        kd = tuple(rng.uniform(0.1, 0.9, 3))
        if k == 0:
            mats.append(b.add_material(kd=kd, ks=(0, 0, 0), diffuseTexId=tex["plaster"]))
        elif k == 1:
            mats.append(b.add_material(kd=kd, ks=tuple(rng.uniform(0.05, 0.4, 3)), roughness=float(rng.uniform(0.05, 0.5))))
        elif k == 2:
            mats.append(b.add_material(kd=kd, ks=(0.1, 0.1, 0.1), diffuseTexId=tex["stone"], normalMapId=tex["normal"]))
        elif k == 3:
            mats.append(b.add_material(kd=(0.05, 0.05, 0.05), ks=(0, 0, 0), kr=tuple(rng.uniform(0.5, 0.9, 3))))
        elif k == 4:
            mats.append(b.add_material(kd=(0, 0, 0), ks=(0.05, 0.05, 0.05), kt=tuple(rng.uniform(0.7, 1.0, 3)) + (1.0,),
                                       roughness=float(rng.uniform(0.05, 0.4)), eta=1.5))
        elif k == 5:
            mats.append(b.add_material(kd=kd, ks=(0, 0, 0), diffuseTexId=tex["leaf"]))
        else:
            mats.append(b.add_material(kd=kd, ks=(0.2, 0.2, 0.2), opacity=tuple(rng.uniform(0.3, 0.9, 3)),
                                       roughness=float(rng.uniform(0.1, 0.6))))
    leaf_mats = [m for i, m in enumerate(mats) if i >= len(zoo) and (i % 7 == 5)] or [zoo[8]]
    arch_mats = [m for m in mats if m not in leaf_mats]
    budget = int(tris)
    foliage_budget = int(budget * 0.70)
    arch_budget = budget - foliage_budget
    W, D, H = 24.0, 18.0, 9.0
    # ground + walls (architecture): finely tessellated so the arch budget is spent here
    ground = b.add_material(kd=(1, 1, 1), ks=(0.05, 0.05, 0.05), diffuseTexId=tex["checker"], roughness=0.4)
    ng = max(2, int(math.sqrt(arch_budget * 0.25 / 2)))
    b.add_mesh(*grid((-W / 2, 0, -D / 2), (W, 0, 0), (0, 0, D), ng, ng, uv_scale=8.0, flip=True), ground)
    wall_mat = b.add_material(kd=(1, 1, 1), ks=(0.02, 0.02, 0.02), diffuseTexId=tex["bricks"], normalMapId=tex["normal"])
    nw = max(2, int(math.sqrt(arch_budget * 0.25 / 2 / 4)))
    b.add_mesh(*grid((-W / 2, 0, D / 2), (W, 0, 0), (0, H, 0), nw, nw, uv_scale=4.0, flip=True), wall_mat)
    b.add_mesh(*grid((-W / 2, 0, -D / 2), (W, 0, 0), (0, H, 0), nw, nw, uv_scale=4.0), wall_mat)
    b.add_mesh(*grid((-W / 2, 0, -D / 2), (0, 0, D), (0, H, 0), nw, nw, uv_scale=4.0, flip=True), wall_mat)
    b.add_mesh(*grid((W / 2, 0, -D / 2), (0, 0, D), (0, H, 0), nw, nw, uv_scale=4.0), wall_mat)
    used = 2 * ng * ng + 4 * 2 * nw * nw
    # arcade columns + tables/chairs (boxes) fill the rest of the architecture budget
    ncol = 24
    col_tris = max(64, (arch_budget - used) // 3 // ncol)
    nseg = max(8, int(math.sqrt(col_tris / 2)))
    for i in range(ncol):
        side = -1 if i < ncol // 2 else 1
        x = -W / 2 + 1.5 + (i % (ncol // 2)) * (W - 3) / (ncol // 2 - 1)
        b.add_mesh(*cylinder((x, 0, side * (D / 2 - 1.5)), 0.3, 4.0, nseg, nseg), arch_mats[i % len(arch_mats)])
    box_tris = max(12, (arch_budget - used) * 2 // 3)
    nbox = 60
    sub = max(1, int(math.sqrt(box_tris / nbox / 12)))
    for i in range(nbox):
        cx, cz = rng.uniform(-W / 2 + 2, W / 2 - 2), rng.uniform(-D / 2 + 3, D / 2 - 3)
        sx, sy, sz = rng.uniform(0.3, 1.2), rng.uniform(0.3, 1.1), rng.uniform(0.3, 1.2)
        b.add_mesh(*box((cx - sx / 2, 0, cz - sz / 2), (cx + sx / 2, sy, cz + sz / 2), sub), arch_mats[(i * 5) % len(arch_mats)])
    # trees: trunks + leaf crowns (foliage: 70 % of the triangles, high depth complexity)
    ntrees = 16
    quads = max(1, foliage_budget // 2 // ntrees)
    trunk = b.add_material(kd=(0.35, 0.25, 0.15), ks=(0, 0, 0), diffuseTexId=tex["stone"])
    for i in range(ntrees):
        cx, cz = rng.uniform(-W / 2 + 3, W / 2 - 3), rng.uniform(-D / 2 + 3, D / 2 - 3)
        h = rng.uniform(3.0, 5.5)
        b.add_mesh(*cylinder((cx, 0, cz), 0.15, h, 12, 4), trunk)
        b.add_mesh(*foliage([(cx, h + 1.0, cz)], [rng.uniform(1.5, 2.6)], quads, 0.06, rng),
                   leaf_mats[i % len(leaf_mats)])
    # emitters: one triangle-mesh area light + the sun
    lm = b.add_material(kd=(0.8, 0.8, 0.8), ks=(0, 0, 0))
    ls = b.add_mesh(*grid((-2, H - 0.5, -2), (4, 0, 0), (0, 0, 4), 1, 1, flip=True), lm)
    b.add_directional_light(euler_forward(55.0, 35.0), (40.0, 40.0, 40.0))
    b.add_mesh_light(ls, (17.0, 12.0, 4.0))
    return b.build()


def sponza_proxy(tris=262_267, seed=3, tex_size=1024):
    """Crytek-Sponza proxy (config 3): a long atrium with two storeys of
    arcades (columns and beams), hanging drapes, 25 materials and 16 RGBA8 1024^2 textures
    (the reference's Sponza textures are mip-mapped; its LOD path is disabled,
    textures.cl:207, so only level 0 is read).  Sun (intensity 40) + a triangle-mesh area light."""
    rng = np.random.default_rng(SEED_BASE + seed)
    b = SceneBuilder("sponza_proxy")
    gens = [
        lambda: tex_bricks(tex_size), lambda: tex_checker(tex_size, (200, 190, 170), (150, 130, 110), tiles=32),
        lambda: tex_noise(tex_size, rng, (190, 170, 140), 30), lambda: tex_noise(tex_size, rng, (150, 150, 140), 45),
        lambda: tex_noise(tex_size, rng, (160, 40, 40), 30), lambda: tex_noise(tex_size, rng, (40, 80, 150), 30),
        lambda: tex_noise(tex_size, rng, (60, 120, 50), 30), lambda: tex_normalmap(tex_size, rng),
    ]
    texs = [b.add_texture(gens[i % len(gens)]()) for i in range(16)]
    mats = []
    for i in range(25):
        k = i % 5
        kd = tuple(rng.uniform(0.4, 0.9, 3))
        if k == 0:
            mats.append(b.add_material(kd=kd, ks=(0, 0, 0), diffuseTexId=texs[i % 7]))
        elif k == 1:
            mats.append(b.add_material(kd=kd, ks=(0.08, 0.08, 0.08), diffuseTexId=texs[(i + 2) % 7],
                                       normalMapId=texs[7 + (i % 2) * 8], roughness=0.35))
        elif k == 2:
            mats.append(b.add_material(kd=kd, ks=tuple(rng.uniform(0.05, 0.3, 3)), roughness=float(rng.uniform(0.1, 0.5)),
                                       diffuseTexId=texs[8 + (i % 7)]))
        elif k == 3:   # drapes: coloured cloth
            mats.append(b.add_material(kd=kd, ks=(0, 0, 0), diffuseTexId=texs[4 + (i % 3)]))
        else:
            mats.append(b.add_material(kd=kd, ks=(0.04, 0.04, 0.04), diffuseTexId=texs[9 + (i % 6)]))
    budget = int(tris)
    L, Wd, H = 30.0, 12.0, 14.0
    parts_fixed = 0
    # floor, walls, upper walls of the nave
    ng = max(2, int(math.sqrt(budget * 0.10 / 2)))
    b.add_mesh(*grid((-L / 2, 0, -Wd / 2), (L, 0, 0), (0, 0, Wd), ng, ng // 2 + 1, uv_scale=10.0, flip=True), mats[1])
    parts_fixed += 2 * ng * (ng // 2 + 1)
    nw = max(2, int(math.sqrt(budget * 0.12 / 2 / 4)))
    for z, fl in ((-Wd / 2 - 3, False), (Wd / 2 + 3, True)):
        b.add_mesh(*grid((-L / 2, 0, z), (L, 0, 0), (0, H, 0), nw, nw, uv_scale=6.0, flip=fl), mats[0])
    for x, fl in ((-L / 2, True), (L / 2, False)):
        b.add_mesh(*grid((x, 0, -Wd / 2 - 3), (0, 0, Wd + 6), (0, H, 0), nw, nw, uv_scale=4.0, flip=fl), mats[5])
    parts_fixed += 4 * 2 * nw * nw
    # two storeys of arcades on both sides: columns + beams
    ncol = 11
    col_budget = int(budget * 0.45)
    per_col = max(64, col_budget // (2 * 2 * ncol))
    nseg = max(8, int(math.sqrt(per_col / 2)))
    for storey, (y0, hgt, rad) in enumerate(((0.0, 5.0, 0.45), (6.0, 4.0, 0.3))):
        for side in (-1, 1):
            for i in range(ncol):
                x = -L / 2 + 2.0 + i * (L - 4.0) / (ncol - 1)
                b.add_mesh(*cylinder((x, y0, side * Wd / 2), rad, hgt, nseg, nseg), mats[(2 + storey * 3 + i) % 25])
            b.add_mesh(*box((-L / 2, y0 + hgt, side * Wd / 2 - 0.6), (L / 2, y0 + hgt + 1.0, side * Wd / 2 + 0.6), 12),
                       mats[10 + storey])
    # drapes between the upper columns (displaced cloth)
    used = parts_fixed + 2 * 2 * ncol * 2 * nseg * nseg + 4 * 6 * 2 * 144
    nd = 2 * (ncol - 1)
    dr = max(2, int(math.sqrt(max(budget - used, nd * 8) / nd / 2)))
    for side in (-1, 1):
        for i in range(ncol - 1):
            x0 = -L / 2 + 2.0 + i * (L - 4.0) / (ncol - 1) + 0.4
            w = (L - 4.0) / (ncol - 1) - 0.8
            P, N, UV, T_ = grid((x0, 6.2, side * (Wd / 2 - 0.2)), (w, 0, 0), (0, 3.6, 0), dr, dr, flip=side > 0)
            ph = rng.uniform(0, 2 * np.pi)
            P = P.copy()
            P[:, 2] += side * 0.15 * np.sin(P[:, 0] * 6.0 + ph) * (1.0 - (P[:, 1] - 6.2) / 3.6)
            b.add_mesh(P, N, UV, T_, mats[3 + 5 * (i % 4)])
    lm = b.add_material(kd=(0.8, 0.8, 0.8), ks=(0, 0, 0))
    ls = b.add_mesh(*grid((-2, H - 0.3, -1.5), (4, 0, 0), (0, 0, 3), 1, 1, flip=True), lm)
    b.add_directional_light(euler_forward(70.0, 20.0), (40.0, 40.0, 40.0))
    b.add_mesh_light(ls, (17.0, 12.0, 4.0))
    return b.build()


def translated(scene, offset):
    """The same scene moved by `offset` (float32 positions and light anchors; the tests of the
    compact walk's exactness far from the world origin, where a slab test's error scales with
    |o / d| rather than with the hit distance).  Identity shape transforms only."""
    M = scene.shapes["toWorldTransform"]
    if not np.array_equal(M, np.broadcast_to(np.eye(4, dtype=np.float32), M.shape)):
        raise NotImplementedError("translated(): shapes with transforms")
    off = np.asarray(offset, np.float32)
    pos = scene.positions.copy()
    pos[:, :3] += off
    lights = scene.lights.copy()
    if len(lights):
        lights["p"][:, :3] += off   # point / spot positions; a directional light's disk centre
    return Scene(scene.shapes, scene.indices, pos, scene.uvs, scene.normals, scene.tangents, scene.binormals,
                 scene.colors, scene.textures, scene.tex_data, lights, scene.materials, sobol=scene.sobol,
                 name=scene.name)


CAMERAS = {
    # name: (pos, look-at, fov_y) -- perspective 45 deg, near 0.3 (PathTracingApp.cpp:387)
    "cornell": ((0.0, 1.0, 3.4), (0.0, 1.0, 0.0), 45.0),
    "mixed": ((0.0, 3.0, -9.0), (0.0, 1.0, 0.5), 45.0),
    "dragon_proxy": ((-3.3, 3.2, -4.5), (0.0, 1.4, 0.0), 45.0),
    "san_miguel_proxy": ((8.2, 2.56, -6.6), (-2.0, 2.8, 3.0), 45.0),
    "sponza_proxy": ((12.0, 3.0, 0.5), (-4.0, 4.5, -0.5), 45.0),
    "instanced_proxy": ((0.0, 9.0, -17.0), (0.0, 0.5, 0.0), 45.0),
    "instances_test": ((0.0, 5.0, -13.0), (0.0, 1.0, 0.0), 45.0),
    "lod_test": ((0.0, 2.0, -9.0), (0.0, 1.0, 10.0), 45.0),
}

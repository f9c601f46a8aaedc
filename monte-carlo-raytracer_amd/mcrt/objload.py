"""Scene ingestion from OBJ/MTL files.

The reference imports scenes with assimp (source/engine/resource/AssetImporter.cpp:40, preset
aiProcessPreset_TargetRealtime_Fast | aiProcess_MakeLeftHanded | aiProcess_FlipWindingOrder),
then RTScene turns every mesh into an RTShape and every material into an uber RTMaterial
(RTScene.cpp:564-678, createUberMaterial :826-845, updateRTMaterialTextures :859-880) and packs
each texture with its whole mip chain into one RGBA8 buffer (uploadTextures :680-766).
assimp is not available here, so this module restates the parts of that pipeline the hot path
sees:

* faces triangulated as fans, identical (v, vt, vn) corners joined, one shape per (object,
  material) run;
* left-handed conversion: z of positions and normals negated (MakeLeftHanded), triangle
  winding reversed (FlipWindingOrder);
* missing normals generated per face (GenNormals is in the TargetRealtime_Fast preset);
* materials: kd = Kd, ks = Ks, roughness = clamp(sqrt(2 / (Ns + 2)), 1e-5, 1) (RTScene.cpp:840),
  kr = kt = 0, opacity = 1, eta = 1.5 (RTUberMaterialComponent::MaterialData defaults);
  textures map_Kd -> diffuse, map_bump/bump/norm -> normal map, map_d -> opacity,
  map_Ks -> glossy (AssetImporter.cpp:145-150 + updateRTMaterialTextures), wrap REPEAT;
* textures: 8-bit PNG (decoded here with zlib; other formats are skipped with a warning),
  stored with a box-filtered mip chain (glGenerateMipmap-sized levels) like uploadTextures;
* optional: materials with an emission colour Ke become triangle-mesh area lights.
"""
import math
import os
import struct
import warnings
import zlib

import numpy as np

from .scenes import SceneBuilder


# ---------------------------------------------------------------------------------------------
# PNG (8-bit, non-interlaced; colour types 0, 2, 3, 4, 6)
# ---------------------------------------------------------------------------------------------
def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)


def read_png(path):
    """RGBA8 (H, W, 4) array of an 8-bit non-interlaced PNG."""
    data = open(path, "rb").read()
    if data[:8] != b"\x89PNG\r\n\x1a\n":
        raise ValueError("not a PNG")
    pos, idat, plte, trns = 8, [], None, None
    while pos < len(data):
        n, typ = struct.unpack(">I4s", data[pos:pos + 8])
        chunk = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if typ == b"IHDR":
            W, H, depth, ctype, _, _, interlace = struct.unpack(">IIBBBBB", chunk)
        elif typ == b"IDAT":
            idat.append(chunk)
        elif typ == b"PLTE":
            plte = np.frombuffer(chunk, np.uint8).reshape(-1, 3)
        elif typ == b"tRNS":
            trns = np.frombuffer(chunk, np.uint8)
        elif typ == b"IEND":
            break
    if depth != 8 or interlace != 0:
        raise ValueError("only 8-bit non-interlaced PNG is supported")
    ch = {0: 1, 2: 3, 3: 1, 4: 2, 6: 4}[ctype]
    raw = np.frombuffer(zlib.decompress(b"".join(idat)), np.uint8)
    stride = W * ch
    out = np.zeros((H, stride), np.uint8)
    prev = np.zeros(stride, np.int32)
    for y in range(H):
        f = raw[y * (stride + 1)]
        line = raw[y * (stride + 1) + 1:(y + 1) * (stride + 1)].astype(np.int32)
        if f == 0:
            cur = line
        elif f == 2:
            cur = (line + prev) & 255
        else:
            cur = np.zeros(stride, np.int32)
            for x in range(stride):
                a = cur[x - ch] if x >= ch else 0
                b = prev[x]
                c = prev[x - ch] if x >= ch else 0
                if f == 1:
                    cur[x] = (line[x] + a) & 255
                elif f == 3:
                    cur[x] = (line[x] + ((a + b) >> 1)) & 255
                else:
                    cur[x] = (line[x] + _paeth(a, b, c)) & 255
        out[y] = cur
        prev = cur
    px = out.reshape(H, W, ch)
    rgba = np.full((H, W, 4), 255, np.uint8)
    if ctype == 0:
        rgba[..., :3] = px
    elif ctype == 2:
        rgba[..., :3] = px
    elif ctype == 3:
        rgba[..., :3] = plte[px[..., 0]]
        if trns is not None:
            alpha = np.full(256, 255, np.uint8)
            alpha[:len(trns)] = trns
            rgba[..., 3] = alpha[px[..., 0]]
    elif ctype == 4:
        rgba[..., :3] = px[..., :1]
        rgba[..., 3] = px[..., 1]
    else:
        rgba[:] = px
    return rgba


def write_png(path, rgba):
    """Minimal RGBA8 PNG writer (filter 0), for tests and tools."""
    rgba = np.ascontiguousarray(rgba, np.uint8)
    H, W = rgba.shape[:2]
    raw = b"".join(b"\x00" + rgba[y].tobytes() for y in range(H))

    def chunk(t, d):
        return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)
    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, 6, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw)) + chunk(b"IEND", b"")
    open(path, "wb").write(png)


def mip_chain(rgba):
    """Levels of glGenerateMipmap sizes (max(w/2, 1) x max(h/2, 1)), 2x2 box filter."""
    levels = [np.ascontiguousarray(rgba, np.uint8)]
    while levels[-1].shape[0] > 1 or levels[-1].shape[1] > 1:
        a = levels[-1].astype(np.uint32)
        h, w = a.shape[:2]
        nh, nw = max(h // 2, 1), max(w // 2, 1)
        ys = np.minimum(np.arange(nh)[:, None] * 2 + np.array([0, 1])[None, :], h - 1)
        xs = np.minimum(np.arange(nw)[:, None] * 2 + np.array([0, 1])[None, :], w - 1)
        blk = a[ys[:, :, None, None], xs[None, None, :, :]]   # (nh, 2, nw, 2, 4)
        levels.append(((blk.sum((1, 3)) + 2) // 4).astype(np.uint8))
    return levels


# ---------------------------------------------------------------------------------------------
# MTL / OBJ
# ---------------------------------------------------------------------------------------------
def _parse_mtl(path):
    mats, cur = {}, None
    for line in open(path, encoding="utf-8", errors="replace"):
        t = line.split()
        if not t or t[0].startswith("#"):
            continue
        key = t[0]
        if key == "newmtl":
            cur = mats.setdefault(" ".join(t[1:]), {})
        elif cur is None:
            continue
        elif key in ("Kd", "Ks", "Ke", "Ka"):
            cur[key] = tuple(float(x) for x in t[1:4])
        elif key in ("Ns", "d", "Ni"):
            cur[key] = float(t[1])
        elif key in ("map_Kd", "map_Ks", "map_d", "map_bump", "bump", "norm", "map_Bump"):
            cur["bump" if key in ("map_bump", "bump", "norm", "map_Bump") else key] = t[-1]   # last token = file
    return mats


def _obj_index(tok, n):
    i = int(tok)
    return i - 1 if i > 0 else n + i


def load_obj(path, *, name=None, mips=True, emissive_lights=True, builder=None):
    """Parse an OBJ (+ its MTL libraries) into a SceneBuilder (shapes, materials, textures; the
    caller adds the scene's other lights, e.g. the demo sun) following RTScene's mapping."""
    base = os.path.dirname(os.path.abspath(path))
    b = builder or SceneBuilder(name or os.path.splitext(os.path.basename(path))[0])
    V, VT, VN = [], [], []
    runs = []          # [(material name, [faces of [(v, vt, vn), ...]])]
    mtl = {}
    cur_mat, cur_obj = None, None
    for line in open(path, encoding="utf-8", errors="replace"):
        t = line.split()
        if not t or t[0].startswith("#"):
            continue
        k = t[0]
        if k == "v":
            V.append([float(x) for x in t[1:4]])
        elif k == "vt":
            VT.append([float(x) for x in t[1:3]] + ([0.0] if len(t) < 3 else []))
        elif k == "vn":
            VN.append([float(x) for x in t[1:4]])
        elif k == "f":
            corners = []
            for c in t[1:]:
                p = c.split("/")
                vi = _obj_index(p[0], len(V))
                ti = _obj_index(p[1], len(VT)) if len(p) > 1 and p[1] else -1
                ni = _obj_index(p[2], len(VN)) if len(p) > 2 and p[2] else -1
                corners.append((vi, ti, ni))
            if not runs or runs[-1][0] != (cur_obj, cur_mat):
                runs.append(((cur_obj, cur_mat), []))
            runs[-1][1].append(corners)
        elif k == "usemtl":
            cur_mat = " ".join(t[1:])
        elif k in ("o", "g"):
            cur_obj = " ".join(t[1:])
        elif k == "mtllib":
            for lib in t[1:]:
                p = os.path.join(base, lib)
                if os.path.exists(p):
                    mtl.update(_parse_mtl(p))
                else:
                    warnings.warn(f"missing MTL library {p}")
    V = np.asarray(V, np.float64).reshape(-1, 3)
    VT = np.asarray(VT, np.float64).reshape(-1, 2) if VT else np.zeros((0, 2))
    VN = np.asarray(VN, np.float64).reshape(-1, 3) if VN else np.zeros((0, 3))

    tex_cache = {}

    def texture(fname):
        if fname in tex_cache:
            return tex_cache[fname]
        p = os.path.join(base, fname.replace("\\", "/"))
        tid = -1
        try:
            tid = b.add_texture(read_png(p), wrap=0, mips=mips)   # RT_TEX_WRAP_REPEAT (RTScene.cpp:739)
        except (OSError, ValueError, KeyError) as e:
            warnings.warn(f"texture {p} skipped: {e}")
        tex_cache[fname] = tid
        return tid

    mat_ids = {}

    def material(mname):
        if mname in mat_ids:
            return mat_ids[mname]
        m = mtl.get(mname, {})
        ns = m.get("Ns", 0.0)   # assimp: AI_MATKEY_SHININESS default 0 (AssetImporter.cpp:155)
        rough = min(max(math.sqrt(2.0 / (ns + 2.0)), 0.00001), 1.0)   # RTScene.cpp:840
        kw = dict(kd=m.get("Kd", (1.0, 1.0, 1.0)), ks=m.get("Ks", (1.0, 1.0, 1.0)), kr=(0.0, 0.0, 0.0),
                  kt=(0.0, 0.0, 0.0, 0.0), opacity=(1.0, 1.0, 1.0), roughness=rough, eta=1.5)
        for key, field in (("map_Kd", "diffuseTexId"), ("bump", "normalMapId"), ("map_d", "opacityTexId"),
                           ("map_Ks", "glossyTexId")):
            if key in m:
                tid = texture(m[key])
                if tid >= 0:
                    kw[field] = tid
        mat_ids[mname] = b.add_material(**kw)
        return mat_ids[mname]

    flipz = np.array([1.0, 1.0, -1.0])
    for (obj, mname), faces in runs:
        mid = material(mname)
        corner_id, P, N, UV, tris = {}, [], [], [], []
        for corners in faces:
            need_flat = any(c[2] < 0 for c in corners)
            fn = None
            if need_flat:   # GenNormals: face normal of the (left-handed, flipped-winding) polygon
                a, bb, c = (V[corners[0][0]] * flipz, V[corners[2][0]] * flipz, V[corners[1][0]] * flipz)
                fn = np.cross(bb - a, c - a)
                ln = np.linalg.norm(fn)
                fn = fn / ln if ln > 0 else np.array([0.0, 1.0, 0.0])
            ids = []
            for c in corners:
                key = c if not need_flat else (c, tuple(fn))
                if key not in corner_id:
                    corner_id[key] = len(P)
                    P.append(V[c[0]] * flipz)
                    N.append(VN[c[2]] * flipz if c[2] >= 0 else fn)
                    UV.append(VT[c[1]] if c[1] >= 0 else (0.0, 0.0))
                ids.append(corner_id[key])
            for i in range(1, len(ids) - 1):   # fan triangulation, winding reversed
                tris.append((ids[0], ids[i + 1], ids[i]))
        if not tris:
            continue
        shape = b.add_mesh(np.asarray(P), np.asarray(N), np.asarray(UV), np.asarray(tris), mid)
        ke = mtl.get(mname, {}).get("Ke")
        if emissive_lights and ke is not None and max(ke) > 0.0:
            b.add_mesh_light(shape, tuple(ke))
    return b

// mcrt_objload.cpp -- scene ingestion for C/C++ hosts: OBJ + MTL + PNG into the 15 SCENE_PARAMS
// arrays (mcrt_scene_desc), the job the reference does with assimp + RTScene
// (source/engine/resource/AssetImporter.cpp:40 preset aiProcessPreset_TargetRealtime_Fast |
// aiProcess_MakeLeftHanded | aiProcess_FlipWindingOrder; APP/raytracing/scene/RTScene.cpp:564-678
// shapes, :680-766 uploadTextures, :826-845 createUberMaterial, :859-880 material textures).
// Same mapping as the package's Python loader (mcrt/objload.py, whose arrays this reproduces;
// tests/test_objload_capi_cpu.py compares them):
//   * faces as fans, equal (v, vt, vn) corners joined, one shape per (object, material) run;
//   * left-handed: z of positions and normals negated, winding reversed;
//   * faces without normals get their face normal (GenNormals);
//   * materials: Kd, Ks, roughness = clamp(sqrt(2 / (Ns + 2)), 1e-5, 1), kr = kt = 0, opacity 1,
//     eta 1.5; map_Kd -> diffuse, map_bump/bump/norm -> normal map, map_d -> opacity,
//     map_Ks -> glossy; textures RGBA8 with the glGenerateMipmap chain, REPEAT;
//   * materials with an emission Ke become triangle-mesh area lights (flag);
//   * directional lights get RTScene::setLight's bounding-sphere placement (RTScene.cpp:482-494).
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "mcrt_internal.h"

struct mcrt_obj_scene_s {
    std::vector<mcrt_shape> shapes;
    std::vector<uint32_t> indices;
    std::vector<mcrt_float3> positions, normals, tangents, binormals;
    std::vector<mcrt_float2> uvs;
    std::vector<mcrt_texture_desc> textures;
    std::vector<uint8_t> texData;
    std::vector<mcrt_light> lights;
    std::vector<mcrt_material> materials;
    float bmin[3] = {0, 0, 0}, bmax[3] = {0, 0, 0};
    std::string warnings;
    std::string error;
};

namespace {

// ---- PNG (8-bit, non-interlaced; colour types 0, 2, 3, 4, 6) ----
int paeth(int a, int b, int c) {
    const int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}
uint32_t be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

bool readPng(const std::string& path, std::vector<uint8_t>& rgba, int& W, int& H, std::string& why) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { why = "cannot open"; return false; }
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (d.size() < 8 || std::memcmp(d.data(), sig, 8) != 0) { why = "not a PNG"; return false; }
    size_t pos = 8;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte, trns;
    while (pos + 12 <= d.size()) {
        const uint32_t n = be32(&d[pos]);
        if (pos + 12 + n > d.size()) break;
        const char* typ = (const char*)&d[pos + 4];
        const uint8_t* c = &d[pos + 8];
        if (!std::memcmp(typ, "IHDR", 4)) {
            if (n < 13) { why = "truncated IHDR chunk"; return false; }
            W = (int)be32(c); H = (int)be32(c + 4); depth = c[8]; ctype = c[9]; interlace = c[12];
        } else if (!std::memcmp(typ, "IDAT", 4)) {
            idat.insert(idat.end(), c, c + n);
        } else if (!std::memcmp(typ, "PLTE", 4)) {
            plte.assign(c, c + n);
        } else if (!std::memcmp(typ, "tRNS", 4)) {
            trns.assign(c, c + n);
        } else if (!std::memcmp(typ, "IEND", 4)) {
            break;
        }
        pos += 12 + n;
    }
    if (depth != 8 || interlace != 0) { why = "only 8-bit non-interlaced PNG is supported"; return false; }
    const int ch = ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : ctype == 6 ? 4 : 0;
    if (!ch || W <= 0 || H <= 0) { why = "unsupported PNG colour type"; return false; }
    if (W > 65535 || H > 65535) { why = "image larger than a texture descriptor holds (65535)"; return false; }
    const size_t stride = (size_t)W * ch;
    std::vector<uint8_t> raw((stride + 1) * H);
    uLongf rawLen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawLen, idat.data(), (uLong)idat.size()) != Z_OK || rawLen != raw.size()) {
        why = "corrupt image data";
        return false;
    }
    std::vector<uint8_t> px(stride * H), prev(stride, 0);
    for (int y = 0; y < H; ++y) {
        const uint8_t ft = raw[y * (stride + 1)];
        const uint8_t* line = &raw[y * (stride + 1) + 1];
        uint8_t* cur = &px[y * stride];
        for (size_t x = 0; x < stride; ++x) {
            const int a = x >= (size_t)ch ? cur[x - ch] : 0, b = prev[x], c = x >= (size_t)ch ? prev[x - ch] : 0;
            int v = line[x];
            if (ft == 1) v += a;
            else if (ft == 2) v += b;
            else if (ft == 3) v += (a + b) >> 1;
            else if (ft == 4) v += paeth(a, b, c);
            cur[x] = (uint8_t)(v & 255);
        }
        std::memcpy(prev.data(), cur, stride);
    }
    rgba.assign((size_t)W * H * 4, 255);
    for (size_t i = 0; i < (size_t)W * H; ++i) {
        uint8_t* o = &rgba[4 * i];
        const uint8_t* p = &px[i * ch];
        if (ctype == 0) { o[0] = o[1] = o[2] = p[0]; }
        else if (ctype == 2) { o[0] = p[0]; o[1] = p[1]; o[2] = p[2]; }
        else if (ctype == 3) {
            const size_t k = p[0];
            if (3 * k + 2 < plte.size()) { o[0] = plte[3 * k]; o[1] = plte[3 * k + 1]; o[2] = plte[3 * k + 2]; }
            if (k < trns.size()) o[3] = trns[k];
        } else if (ctype == 4) { o[0] = o[1] = o[2] = p[0]; o[3] = p[1]; }
        else { std::memcpy(o, p, 4); }
    }
    return true;
}

// glGenerateMipmap-sized levels, 2x2 box filter ((sum + 2) / 4, edge texels repeated)
void appendMips(std::vector<uint8_t>& out, std::vector<uint8_t> lv, int w, int h, int& levels) {
    levels = 1;
    out.insert(out.end(), lv.begin(), lv.end());
    while (w > 1 || h > 1) {
        const int nw = std::max(w / 2, 1), nh = std::max(h / 2, 1);
        std::vector<uint8_t> nx((size_t)nw * nh * 4);
        for (int y = 0; y < nh; ++y)
            for (int x = 0; x < nw; ++x)
                for (int c = 0; c < 4; ++c) {
                    uint32_t s = 0;
                    for (int dy = 0; dy < 2; ++dy)
                        for (int dx = 0; dx < 2; ++dx) {
                            const int yy = std::min(2 * y + dy, h - 1), xx = std::min(2 * x + dx, w - 1);
                            s += lv[((size_t)yy * w + xx) * 4 + c];
                        }
                    nx[((size_t)y * nw + x) * 4 + c] = (uint8_t)((s + 2) / 4);
                }
        out.insert(out.end(), nx.begin(), nx.end());
        lv.swap(nx);
        w = nw;
        h = nh;
        ++levels;
    }
}

std::vector<std::string> split(const std::string& line) {
    std::vector<std::string> t;
    std::istringstream is(line);
    std::string s;
    while (is >> s) t.push_back(s);
    return t;
}
std::string joinFrom(const std::vector<std::string>& t, size_t i) {
    std::string s;
    for (size_t k = i; k < t.size(); ++k) s += (k > i ? " " : "") + t[k];
    return s;
}

struct Mtl {
    bool hasKd = false, hasKs = false, hasKe = false;
    double Kd[3] = {1, 1, 1}, Ks[3] = {1, 1, 1}, Ke[3] = {0, 0, 0}, Ns = 0.0;
    std::map<std::string, std::string> maps;
};

void parseMtl(const std::string& path, std::map<std::string, Mtl>& mats) {
    std::ifstream f(path);
    std::string line;
    Mtl* cur = nullptr;
    while (std::getline(f, line)) {
        const auto t = split(line);
        if (t.empty() || t[0][0] == '#') continue;
        const std::string& k = t[0];
        if (k == "newmtl") {
            cur = &mats[joinFrom(t, 1)];
        } else if (!cur) {
            continue;
        } else if ((k == "Kd" || k == "Ks" || k == "Ke") && t.size() >= 4) {
            double* dst = k == "Kd" ? cur->Kd : k == "Ks" ? cur->Ks : cur->Ke;
            for (int c = 0; c < 3; ++c) dst[c] = std::strtod(t[1 + c].c_str(), nullptr);
            (k == "Kd" ? cur->hasKd : k == "Ks" ? cur->hasKs : cur->hasKe) = true;
        } else if (k == "Ns" && t.size() >= 2) {
            cur->Ns = std::strtod(t[1].c_str(), nullptr);
        } else if (k == "map_Kd" || k == "map_Ks" || k == "map_d") {
            cur->maps[k] = t.back();
        } else if (k == "map_bump" || k == "bump" || k == "norm" || k == "map_Bump") {
            cur->maps["bump"] = t.back();
        }
    }
}

// OBJ index token -> 0-based index into an array of n entries (1-based, or negative = relative
// to the end); -1 when the token is not a valid reference (0, past the end, before the start)
int objIndex(const std::string& tok, size_t n) {
    char* end = nullptr;
    const long i = std::strtol(tok.c_str(), &end, 10);
    if (end == tok.c_str()) return -1;
    const long k = i > 0 ? i - 1 : (long)n + i;
    return (i == 0 || k < 0 || k >= (long)n) ? -1 : (int)k;
}

mcrt_material defaultMaterial() {   // RTMaterial constructor defaults (kernel_data.h:89-94)
    mcrt_material m;
    std::memset(&m, 0, sizeof(m));
    m.uber_kd = {0.25f, 0.25f, 0.25f, 0.0f};
    m.uber_ks = {0.25f, 0.25f, 0.25f, 0.0f};
    m.uber_opacity = {1.0f, 1.0f, 1.0f, 0.0f};
    m.uber_roughness = {0.1f, 0.1f};
    m.uber_eta = 1.5f;
    m.uber_normalMapId = m.uber_diffuseTexId = m.uber_glossyTexId = m.uber_specReflectionTexId = -1;
    m.uber_transmissionTexId = m.uber_opacityTexId = m.uber_roughnessTexId = m.uber_iorTexId = -1;
    return m;
}

float f32(double v) { return (float)v; }
// |x|^2 of a 3-vector as the Python loader's numpy computes it (BLAS dot: fma chain)
double dot3(const double* x, const double* y) { return std::fma(x[2], y[2], std::fma(x[1], y[1], x[0] * y[0])); }

struct Corner {
    int v, t, n;
    double fn[3];
    bool operator<(const Corner& o) const {
        if (v != o.v) return v < o.v;
        if (t != o.t) return t < o.t;
        if (n != o.n) return n < o.n;
        for (int a = 0; a < 3; ++a)   // by value, as the Python loader's tuple keys (+0 == -0)
            if (fn[a] != o.fn[a]) return fn[a] < o.fn[a];
        return false;
    }
};

// shape arrays of one (object, material) run; tangent frame and area as mcrt/scenes.py builds them
void addShape(mcrt_obj_scene_s& S, const std::vector<double>& P, const std::vector<double>& N,
              const std::vector<double>& UV, const std::vector<uint32_t>& tris, int material) {
    const uint32_t v0 = (uint32_t)S.positions.size(), i0 = (uint32_t)S.indices.size();
    const size_t n = P.size() / 3;
    for (size_t k = 0; k < n; ++k) {
        const float p[3] = {f32(P[3 * k]), f32(P[3 * k + 1]), f32(P[3 * k + 2])};
        const float nn[3] = {f32(N[3 * k]), f32(N[3 * k + 1]), f32(N[3 * k + 2])};
        S.positions.push_back({p[0], p[1], p[2], 0.0f});
        S.normals.push_back({nn[0], nn[1], nn[2], 0.0f});
        S.uvs.push_back({f32(UV[2 * k]), f32(UV[2 * k + 1])});
        // t = N x (0,1,0), or N x (1,0,0) when that is ~0; normalised; binormal = N x t (float32)
        float t[3] = {nn[1] * 0.0f - nn[2] * 1.0f, nn[2] * 0.0f - nn[0] * 0.0f, nn[0] * 1.0f - nn[1] * 0.0f};
        float l = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
        if (l < 1e-4f) {
            t[0] = nn[1] * 0.0f - nn[2] * 0.0f;
            t[1] = nn[2] * 1.0f - nn[0] * 0.0f;
            t[2] = nn[0] * 0.0f - nn[1] * 1.0f;
            l = std::sqrt(t[0] * t[0] + t[1] * t[1] + t[2] * t[2]);
        }
        l = std::max(l, 1e-20f);
        for (float& c : t) c = c / l;
        S.tangents.push_back({t[0], t[1], t[2], 0.0f});
        S.binormals.push_back({nn[1] * t[2] - nn[2] * t[1], nn[2] * t[0] - nn[0] * t[2], nn[0] * t[1] - nn[1] * t[0], 0.0f});
    }
    S.indices.insert(S.indices.end(), tris.begin(), tris.end());
    mcrt_shape sh;
    std::memset(&sh, 0, sizeof(sh));
    sh.toWorldTransform.m0 = {1, 0, 0, 0};
    sh.toWorldTransform.m1 = {0, 1, 0, 0};
    sh.toWorldTransform.m2 = {0, 0, 1, 0};
    sh.toWorldTransform.m3 = {0, 0, 0, 1};
    sh.toWorldInverseTranspose = sh.toWorldTransform;
    sh.startIdx = i0;
    sh.startVertex = v0;
    sh.numTriangles = (uint32_t)(tris.size() / 3);
    sh.materialId = material;
    sh.lightID = -1;
    double area = 0.0;
    for (size_t f = 0; f < tris.size(); f += 3) {
        const mcrt_float3 &a = S.positions[v0 + tris[f]], &b = S.positions[v0 + tris[f + 1]], &c = S.positions[v0 + tris[f + 2]];
        const float e1[3] = {b.x - a.x, b.y - a.y, b.z - a.z}, e2[3] = {c.x - a.x, c.y - a.y, c.z - a.z};
        const float x = e1[1] * e2[2] - e1[2] * e2[1], y = e1[2] * e2[0] - e1[0] * e2[2], z = e1[0] * e2[1] - e1[1] * e2[0];
        area += 0.5 * (double)std::sqrt(x * x + y * y + z * z);
    }
    sh.area = (float)area;
    S.shapes.push_back(sh);
    for (size_t k = 0; k < n; ++k) {
        const mcrt_float3& p = S.positions[v0 + k];
        const float q[3] = {p.x, p.y, p.z};
        for (int a = 0; a < 3; ++a) {
            if (S.positions.size() == n && k == 0) S.bmin[a] = S.bmax[a] = q[a];
            S.bmin[a] = std::min(S.bmin[a], q[a]);
            S.bmax[a] = std::max(S.bmax[a], q[a]);
        }
    }
}

}  // namespace

MCRT_API mcrt_status mcrt_obj_load(const char* path, uint32_t flags, mcrt_obj_scene* out) {
    if (!path || !out) return MCRT_ERROR_INVALID_ARG;
    *out = nullptr;
    std::ifstream f(path);
    if (!f) return MCRT_ERROR_INVALID_ARG;
    auto* S = new mcrt_obj_scene_s();
    std::string base = path;
    const size_t slash = base.find_last_of('/');
    base = slash == std::string::npos ? std::string(".") : base.substr(0, slash);
    std::vector<double> V, VT, VN;
    struct Run {
        std::string obj, mat;
        std::vector<std::vector<int>> faces;   // (v, vt, vn) triples per corner
    };
    std::vector<Run> runs;
    std::map<std::string, Mtl> mtl;
    std::string curMat, curObj;
    bool haveMat = false, haveObj = false;
    std::string line;
    size_t lineNo = 0;
    while (std::getline(f, line)) {
        ++lineNo;
        const auto t = split(line);
        if (t.empty() || t[0][0] == '#') continue;
        const std::string& k = t[0];
        if (k == "v" && t.size() >= 4) {
            for (int c = 0; c < 3; ++c) V.push_back(std::strtod(t[1 + c].c_str(), nullptr));
        } else if (k == "vt" && t.size() >= 2) {
            VT.push_back(std::strtod(t[1].c_str(), nullptr));
            VT.push_back(t.size() >= 3 ? std::strtod(t[2].c_str(), nullptr) : 0.0);
        } else if (k == "vn" && t.size() >= 4) {
            for (int c = 0; c < 3; ++c) VN.push_back(std::strtod(t[1 + c].c_str(), nullptr));
        } else if (k == "f") {
            std::vector<int> face;
            for (size_t i = 1; i < t.size(); ++i) {
                std::vector<std::string> p;
                std::string cur;
                for (char ch : t[i]) {
                    if (ch == '/') { p.push_back(cur); cur.clear(); }
                    else cur += ch;
                }
                p.push_back(cur);
                const int v = objIndex(p[0], V.size() / 3);
                const int vt = p.size() > 1 && !p[1].empty() ? objIndex(p[1], VT.size() / 2) : -2;
                const int vn = p.size() > 2 && !p[2].empty() ? objIndex(p[2], VN.size() / 3) : -2;
                if (v < 0 || vt == -1 || vn == -1) {   // a reference outside the arrays read so far
                    mcrt::set_last_error(std::string(path) + ":" + std::to_string(lineNo) + ": face index '" + t[i] +
                                         "' out of range (" + std::to_string(V.size() / 3) + " v, " +
                                         std::to_string(VT.size() / 2) + " vt, " + std::to_string(VN.size() / 3) +
                                         " vn so far)");
                    delete S;
                    return MCRT_ERROR_INVALID_ARG;
                }
                face.push_back(v);
                face.push_back(vt < 0 ? -1 : vt);
                face.push_back(vn < 0 ? -1 : vn);
            }
            const std::string obj = haveObj ? curObj : std::string("\x01"), mat = haveMat ? curMat : std::string("\x01");
            if (runs.empty() || runs.back().obj != obj || runs.back().mat != mat) runs.push_back(Run{obj, mat, {}});
            runs.back().faces.push_back(face);
        } else if (k == "usemtl") {
            curMat = joinFrom(t, 1);
            haveMat = true;
        } else if (k == "o" || k == "g") {
            curObj = joinFrom(t, 1);
            haveObj = true;
        } else if (k == "mtllib") {
            for (size_t i = 1; i < t.size(); ++i) {
                const std::string p = base + "/" + t[i];
                if (std::ifstream(p)) parseMtl(p, mtl);
                else S->warnings += "missing MTL library " + p + "\n";
            }
        }
    }
    std::map<std::string, int> texCache, matIds;
    auto texture = [&](std::string fname) -> int {
        auto it = texCache.find(fname);
        if (it != texCache.end()) return it->second;
        std::string p = fname;
        for (char& ch : p)
            if (ch == '\\') ch = '/';
        p = base + "/" + p;
        std::vector<uint8_t> rgba;
        int W = 0, H = 0, tid = -1;
        std::string why;
        if (readPng(p, rgba, W, H, why)) {
            mcrt_texture_desc d;
            std::memset(&d, 0, sizeof(d));
            d.width = (uint16_t)W;
            d.height = (uint16_t)H;
            d.format = 3;
            d.wrap = 0;   // RT_TEX_WRAP_REPEAT (RTScene.cpp:739)
            d.memOffset = (uint32_t)S->texData.size();
            int levels = 1;
            if (flags & MCRT_OBJ_MIPS) appendMips(S->texData, rgba, W, H, levels);
            else S->texData.insert(S->texData.end(), rgba.begin(), rgba.end());
            d.numMipLevels = (uint16_t)levels;
            tid = (int)S->textures.size();
            S->textures.push_back(d);
        } else {
            S->warnings += "texture " + p + " skipped: " + why + "\n";
        }
        texCache[fname] = tid;
        return tid;
    };
    auto material = [&](const std::string& name) -> int {
        auto it = matIds.find(name);
        if (it != matIds.end()) return it->second;
        const auto mi = mtl.find(name);
        const Mtl m = mi != mtl.end() ? mi->second : Mtl();
        mcrt_material M = defaultMaterial();
        const double rough = std::min(std::max(std::sqrt(2.0 / (m.Ns + 2.0)), 0.00001), 1.0);   // RTScene.cpp:840
        M.uber_kd = {f32(m.Kd[0]), f32(m.Kd[1]), f32(m.Kd[2]), 0.0f};
        M.uber_ks = {f32(m.Ks[0]), f32(m.Ks[1]), f32(m.Ks[2]), 0.0f};
        M.uber_kr = {0, 0, 0, 0};
        M.uber_kt = {0, 0, 0, 0};
        M.uber_opacity = {1, 1, 1, 0};
        M.uber_roughness = {f32(rough), f32(rough)};
        M.uber_eta = 1.5f;
        const std::pair<const char*, int32_t*> slots[4] = {{"map_Kd", &M.uber_diffuseTexId}, {"bump", &M.uber_normalMapId},
                                                           {"map_d", &M.uber_opacityTexId}, {"map_Ks", &M.uber_glossyTexId}};
        for (const auto& s : slots) {
            auto mp = m.maps.find(s.first);
            if (mp != m.maps.end()) {
                const int tid = texture(mp->second);
                if (tid >= 0) *s.second = tid;
            }
        }
        const int id = (int)S->materials.size();
        S->materials.push_back(M);
        matIds[name] = id;
        return id;
    };
    for (const Run& r : runs) {
        const int mid = material(r.mat);
        std::map<Corner, uint32_t> cornerId;
        std::vector<double> P, N, UV;
        std::vector<uint32_t> tris;
        for (const auto& face : r.faces) {
            const size_t nc = face.size() / 3;
            bool needFlat = false;
            for (size_t c = 0; c < nc; ++c) needFlat |= face[3 * c + 2] < 0;
            double fn[3] = {0, 0, 0};
            if (needFlat && nc >= 3) {   // GenNormals on the left-handed, flipped polygon
                auto vp = [&](size_t c, int a) { return V[3 * face[3 * c] + a] * (a == 2 ? -1.0 : 1.0); };
                const double a[3] = {vp(0, 0), vp(0, 1), vp(0, 2)}, b[3] = {vp(2, 0), vp(2, 1), vp(2, 2)},
                             c[3] = {vp(1, 0), vp(1, 1), vp(1, 2)};
                const double u[3] = {b[0] - a[0], b[1] - a[1], b[2] - a[2]}, v[3] = {c[0] - a[0], c[1] - a[1], c[2] - a[2]};
                fn[0] = u[1] * v[2] - u[2] * v[1];
                fn[1] = u[2] * v[0] - u[0] * v[2];
                fn[2] = u[0] * v[1] - u[1] * v[0];
                const double ln = std::sqrt(dot3(fn, fn));
                if (ln > 0) for (double& x : fn) x /= ln;
                else { fn[0] = 0; fn[1] = 1; fn[2] = 0; }
            }
            std::vector<uint32_t> ids;
            for (size_t c = 0; c < nc; ++c) {
                Corner key{face[3 * c], face[3 * c + 1], face[3 * c + 2], {0, 0, 0}};
                if (needFlat) std::memcpy(key.fn, fn, sizeof(fn));
                auto it = cornerId.find(key);
                if (it == cornerId.end()) {
                    const uint32_t id = (uint32_t)(P.size() / 3);
                    cornerId[key] = id;
                    for (int a = 0; a < 3; ++a) P.push_back(V[3 * key.v + a] * (a == 2 ? -1.0 : 1.0));
                    for (int a = 0; a < 3; ++a) N.push_back(key.n >= 0 ? VN[3 * key.n + a] * (a == 2 ? -1.0 : 1.0) : fn[a]);
                    UV.push_back(key.t >= 0 ? VT[2 * key.t] : 0.0);
                    UV.push_back(key.t >= 0 ? VT[2 * key.t + 1] : 0.0);
                    ids.push_back(id);
                } else {
                    ids.push_back(it->second);
                }
            }
            for (size_t i = 1; i + 1 < ids.size(); ++i) {   // fan, winding reversed
                tris.push_back(ids[0]);
                tris.push_back(ids[i + 1]);
                tris.push_back(ids[i]);
            }
        }
        if (tris.empty()) continue;
        addShape(*S, P, N, UV, tris, mid);
        const auto mi = mtl.find(r.mat);
        if ((flags & MCRT_OBJ_EMISSIVE_LIGHTS) && mi != mtl.end() && mi->second.hasKe &&
            std::max(mi->second.Ke[0], std::max(mi->second.Ke[1], mi->second.Ke[2])) > 0.0) {
            mcrt_light L;   // triangle-mesh area light on the shape (RTScene.cpp:525-545)
            std::memset(&L, 0, sizeof(L));
            L.intensity = {f32(mi->second.Ke[0]), f32(mi->second.Ke[1]), f32(mi->second.Ke[2]), 0.0f};
            L.type = MCRT_TRIANGLE_MESH_AREA_LIGHT;
            L.shapeId = (int32_t)(S->shapes.size() - 1);
            L.flags = MCRT_LIGHT_FLAG_AREA;
            L.area = S->shapes.back().area;
            S->shapes.back().lightID = (int32_t)S->lights.size();
            S->lights.push_back(L);
        }
    }
    *out = S;
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_obj_add_directional_light(mcrt_obj_scene s, const float dir[3], const float intensity[3]) {
    if (!s || !dir || !intensity) return MCRT_ERROR_INVALID_ARG;
    // RTScene::setLight (RTScene.cpp:482-494): on the scene's bounding sphere, facing along d
    const double dd[3] = {dir[0], dir[1], dir[2]};
    const double dl = std::sqrt(dot3(dd, dd));
    if (!(dl > 0.0)) return MCRT_ERROR_INVALID_ARG;
    const double d[3] = {dir[0] / dl, dir[1] / dl, dir[2] / dl};
    const float e[3] = {s->bmax[0] - s->bmin[0], s->bmax[1] - s->bmin[1], s->bmax[2] - s->bmin[2]};
    const float radius = std::sqrt(std::fma(e[2], e[2], std::fma(e[1], e[1], e[0] * e[0]))) * 0.5f;
    mcrt_light L;
    std::memset(&L, 0, sizeof(L));
    L.type = MCRT_DIRECTIONAL_LIGHT;
    L.shapeId = -1;
    L.intensity = {intensity[0], intensity[1], intensity[2], 0.0f};
    L.d = {f32(d[0]), f32(d[1]), f32(d[2]), 0.0f};
    L.radius = radius;
    float p[3];
    for (int a = 0; a < 3; ++a) p[a] = f32(((double)s->bmin[a] + s->bmax[a]) * 0.5 - d[a] * radius);
    L.p = {p[0], p[1], p[2], 0.0f};
    L.flags = MCRT_LIGHT_FLAG_DELTA_DIRECTION;
    L.area = (float)M_PI * radius * radius;
    s->lights.push_back(L);
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_obj_add_point_light(mcrt_obj_scene s, const float pos[3], const float intensity[3]) {
    if (!s || !pos || !intensity) return MCRT_ERROR_INVALID_ARG;
    mcrt_light L;
    std::memset(&L, 0, sizeof(L));
    L.type = MCRT_POINT_LIGHT;
    L.shapeId = -1;
    L.p = {pos[0], pos[1], pos[2], 0.0f};
    L.intensity = {intensity[0], intensity[1], intensity[2], 0.0f};
    L.flags = MCRT_LIGHT_FLAG_DELTA_POSITION;
    s->lights.push_back(L);
    return MCRT_OK;
}

MCRT_API mcrt_status mcrt_obj_scene_desc(mcrt_obj_scene s, mcrt_scene_desc* d) {
    if (!s || !d) return MCRT_ERROR_INVALID_ARG;
    for (auto& L : s->lights) L.choicePdf = 1.0f / (float)s->lights.size();   // RTScene.cpp:811-819
    std::memset(d, 0, sizeof(*d));
    d->shapes = s->shapes.data();
    d->num_shapes = (uint32_t)s->shapes.size();
    d->indices = s->indices.data();
    d->num_indices = (uint32_t)s->indices.size();
    d->positions = s->positions.data();
    d->num_vertices = (uint32_t)s->positions.size();
    d->uvs = s->uvs.data();
    d->normals = s->normals.data();
    d->tangents = s->tangents.data();
    d->binormals = s->binormals.data();
    d->colors = nullptr;
    d->textures = s->textures.empty() ? nullptr : s->textures.data();
    d->num_textures = (uint32_t)s->textures.size();
    d->tex_data = s->texData.empty() ? nullptr : s->texData.data();
    d->tex_data_bytes = s->texData.size();
    d->lights = s->lights.empty() ? nullptr : s->lights.data();
    d->num_lights = (uint32_t)s->lights.size();
    d->materials = s->materials.empty() ? nullptr : s->materials.data();
    d->num_materials = (uint32_t)s->materials.size();
    return MCRT_OK;
}

MCRT_API const char* mcrt_obj_warnings(mcrt_obj_scene s) { return s ? s->warnings.c_str() : ""; }

MCRT_API void mcrt_obj_free(mcrt_obj_scene s) { delete s; }

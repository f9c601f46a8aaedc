// TEST INFRASTRUCTURE ONLY -- oracle/_ref driver.
//
// Links the reference's OWN C++ sources, compiled in place from /root/reference
// by oracle/refbuild/Makefile (nothing is copied into this repo):
//   third_party/RadeonRays/RadeonRays/src/accelerator/bvh2.cpp  (Bvh2 SAH builder)
//   third_party/RadeonRays/RadeonRays/src/primitive/mesh.cpp    (Mesh::GetFaceBounds)
//   third_party/RadeonRays/RadeonRays/src/accelerator/bvh.cpp   (Bvh, the 2-level builder)
//   third_party/RadeonRays/RadeonRays/src/translator/plain_bvh_translator.cpp (skip links)
//   third_party/RadeonRays/UnitTest/utils.cpp                  (brute-force golden)
//   third_party/RadeonRays/UnitTest/tiny_obj_loader.cpp        (CornellBox orig.objm)
// and exposes them through a tiny C interface for tests/ (ctypes).
#include "accelerator/bvh.h"
#include "accelerator/bvh2.h"
#include "primitive/mesh.h"
#include "translator/plain_bvh_translator.h"
#include "math/mathutils.h"
#include "utils.h"
#include "tiny_obj_loader.h"

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <tuple>
#include <vector>

namespace RadeonRays {
// Bvh2 grants its node array to this friend (bvh2.h:172); only read access here.
class QBvhTranslator {
public:
    static std::size_t count(const Bvh2& b) { return b.m_nodecount; }
    static const void* nodes(const Bvh2& b) { return b.m_nodes; }
};
}  // namespace RadeonRays

using namespace RadeonRays;

namespace {
struct ShapeSet {
    std::vector<std::unique_ptr<Mesh>> meshes;
    std::vector<TestShape> tests;
};

// positions: per shape, vstride bytes between vertices (xyz floats); indices: 3 per face.
// transforms: 16 floats per shape (row major, RR matrix m00..m33) or nullptr.
ShapeSet make_shapes(int nshapes, const float* const* positions, const int* nverts, int vstride,
                     const int* const* indices, const int* nfaces, const float* transforms) {
    ShapeSet s;
    for (int i = 0; i < nshapes; ++i) {
        auto m = std::unique_ptr<Mesh>(new Mesh(positions[i], nverts[i], vstride, indices[i], 0, nullptr, nfaces[i]));
        m->SetId(i);
        if (transforms) {
            const float* t = transforms + 16 * i;
            matrix M(t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], t[8], t[9], t[10], t[11], t[12], t[13], t[14], t[15]);
            m->SetTransform(M, inverse(M));
        }
        // TestShape wants tightly packed xyz
        std::vector<float> p(3 * (size_t)nverts[i]);
        for (int v = 0; v < nverts[i]; ++v) {
            const float* src = (const float*)((const char*)positions[i] + (size_t)v * vstride);
            p[3 * v] = src[0]; p[3 * v + 1] = src[1]; p[3 * v + 2] = src[2];
        }
        s.tests.emplace_back(p.data(), nverts[i], indices[i], 3 * nfaces[i], nullptr, nfaces[i]);
        s.tests.back().shape = m.get();
        s.meshes.push_back(std::move(m));
    }
    return s;
}
}  // namespace

extern "C" {

__attribute__((visibility("default")))
int64_t rr_bvh_build(int nshapes, const float* const* positions, const int* nverts, int vstride,
                     const int* const* indices, const int* nfaces, const float* transforms,
                     float traversal_cost, int num_bins, int use_sah, void* out_nodes, int64_t max_nodes) {
    ShapeSet s = make_shapes(nshapes, positions, nverts, vstride, indices, nfaces, transforms);
    std::vector<const Shape*> shapes;
    for (auto& m : s.meshes) shapes.push_back(m.get());
    Bvh2 bvh(traversal_cost, num_bins, use_sah != 0);
    bvh.Build(shapes.begin(), shapes.end());
    std::size_t n = QBvhTranslator::count(bvh);
    if (out_nodes) std::memcpy(out_nodes, QBvhTranslator::nodes(bvh), 64 * (n < (size_t)max_nodes ? n : (size_t)max_nodes));
    return (int64_t)n;
}

// rays: 48-B RadeonRays rays; out: 32-B Intersection (TestIntersections) / int (1 hit, -1 miss)
__attribute__((visibility("default")))
void rr_test_intersections(int nshapes, const float* const* positions, const int* nverts, int vstride,
                           const int* const* indices, const int* nfaces, const float* transforms,
                           const void* rays, int nrays, void* out_isects) {
    ShapeSet s = make_shapes(nshapes, positions, nverts, vstride, indices, nfaces, transforms);
    auto* isect = reinterpret_cast<Intersection*>(out_isects);
    for (int i = 0; i < nrays; ++i) { isect[i].shapeid = -1; isect[i].primid = -1; }
    TestIntersections(s.tests.data(), (int)s.tests.size(), reinterpret_cast<const ray*>(rays), nrays, isect);
}

__attribute__((visibility("default")))
void rr_test_occlusions(int nshapes, const float* const* positions, const int* nverts, int vstride,
                        const int* const* indices, const int* nfaces, const float* transforms,
                        const void* rays, int nrays, int32_t* out) {
    ShapeSet s = make_shapes(nshapes, positions, nverts, vstride, indices, nfaces, transforms);
    std::vector<char> hits(nrays);
    TestOcclusions(s.tests.data(), (int)s.tests.size(), reinterpret_cast<const ray*>(rays), nrays,
                   reinterpret_cast<bool*>(hits.data()));
    for (int i = 0; i < nrays; ++i) out[i] = hits[i] ? 1 : -1;
}

// tiny_obj_loader (as the RR conformance fixture loads orig.objm, conformance_test_cl.h:118)
struct ObjHandle { std::vector<tinyobj::shape_t> shapes; std::vector<tinyobj::material_t> mats; };
__attribute__((visibility("default")))
void* rr_load_obj(const char* path, const char* mtl_base) {
    auto* h = new ObjHandle();
    std::string err = tinyobj::LoadObj(h->shapes, h->mats, path, mtl_base);
    if (!err.empty() && h->shapes.empty()) { delete h; return nullptr; }
    return h;
}
__attribute__((visibility("default")))
int rr_obj_num_shapes(void* h) { return (int)static_cast<ObjHandle*>(h)->shapes.size(); }
__attribute__((visibility("default")))
void rr_obj_shape(void* h, int i, const float** pos, int* npos_floats, const int** idx, int* nidx) {
    auto& m = static_cast<ObjHandle*>(h)->shapes[i].mesh;
    *pos = m.positions.data(); *npos_floats = (int)m.positions.size();
    *idx = reinterpret_cast<const int*>(m.indices.data()); *nidx = (int)m.indices.size();
}
__attribute__((visibility("default")))
void rr_obj_free(void* h) { delete static_cast<ObjHandle*>(h); }

// ---------------------------------------------------------------------------
// Two-level (instanced) acceleration structure, as IntersectorTwoLevel::Process builds it
// (RR/src/intersector/intersector_2level.cpp:166-470) for the scene RTScene::attachMesh makes
// (APP/raytracing/scene/RTScene.cpp:564-672): the first shape with a given (startIdx,
// startVertex, numTriangles) is a Mesh with its own transform, every later shape with the same
// key an Instance of it (CreateInstance + SetTransform).  The list handling below (world order,
// std::partition, per-mesh Bvh over object-space face bounds, top Bvh over transform_bbox'ed
// bounds, PlainBvhTranslator, Face/ShapeData records) mirrors Process; the Bvh, translator,
// Mesh and transform_bbox code that runs is the reference's own.
// Buffers are exactly the ones intersect_bvh2level_skiplinks.cl reads.
struct Rr2lShapeData {   // IntersectorTwoLevel::ShapeData (intersector_2level.cpp:39-49), 112 B
    int id;
    int bvhidx;
    unsigned int shapeDisabled;
    int padding1;
    matrix minv;
    float lv[4];
    float av[4];
};
struct Rr2lFace {   // IntersectorTwoLevel::Face (intersector_2level.cpp:51-58), 20 B
    int idx[3];
    int shape_id;
    int prim_id;
};
struct Rr2l {
    std::vector<PlainBvhTranslator::Node> nodes;
    std::vector<float> vertices;   // float3 = 4 floats
    std::vector<Rr2lFace> faces;
    std::vector<Rr2lShapeData> shapes;
    int root = -1;
    int nummeshes = 0, numinstances = 0;
};

// shapes: per shape (startIdx, startVertex, numTriangles) + 16-float m (local->world, row
// major) + 16-float minv; indices: per-shape local vertex indices; positions: float4 stride.
__attribute__((visibility("default")))
void* rr2l_build(int nshapes, const uint32_t* keys, const float* m16, const float* minv16, const uint32_t* indices,
                 const float* positions4, float traversal_cost, int num_bins, int use_sah) {
    struct Ent { bool inst; int base; int id; };   // base: index into `ents` of the Mesh
    std::vector<std::unique_ptr<Mesh>> meshOf(nshapes);
    std::vector<Ent> ents;
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, int> first;
    for (int i = 0; i < nshapes; ++i) {
        auto k = std::make_tuple(keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]);
        auto it = first.find(k);
        if (it == first.end()) {
            first[k] = i;
            const uint32_t* idx = indices + keys[3 * i];
            const int nf = (int)keys[3 * i + 2];
            int nv = 0;
            for (int j = 0; j < 3 * nf; ++j) nv = std::max(nv, (int)idx[j] + 1);
            meshOf[i].reset(new Mesh(positions4 + 4 * (size_t)keys[3 * i + 1], nv, 16, (const int*)idx, 0, nullptr, nf));
            ents.push_back({false, i, i});
        } else {
            ents.push_back({true, it->second, i});
        }
    }
    auto M = [&](const float* t) {
        return matrix(t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7], t[8], t[9], t[10], t[11], t[12], t[13], t[14], t[15]);
    };
    // world.shapes_ order = attach order = shape id order; partition meshes before instances
    std::vector<int> shapes(nshapes);
    for (int i = 0; i < nshapes; ++i) shapes[i] = i;
    auto firstinst = std::partition(shapes.begin(), shapes.end(), [&](int s) { return !ents[s].inst; });
    const int nummeshes = (int)(firstinst - shapes.begin());
    const int numinstances = nshapes - nummeshes;
    auto* out = new Rr2l();
    out->nummeshes = nummeshes;
    out->numinstances = numinstances;
    std::vector<std::unique_ptr<Bvh>> bvhs(nummeshes + 1);
    std::vector<Bvh const*> bvhptrs(nummeshes + 1);
    std::vector<int> vstart(nummeshes), fstart(nummeshes);
    int numvertices = 0, numfaces = 0;
    for (int i = 0; i < nummeshes; ++i) {
        bvhs[i].reset(new Bvh(traversal_cost, num_bins, use_sah != 0));
        Mesh const* mesh = meshOf[shapes[i]].get();
        fstart[i] = numfaces;
        vstart[i] = numvertices;
        numfaces += mesh->num_faces();
        numvertices += mesh->num_vertices();
    }
    bvhs[nummeshes].reset(new Bvh(traversal_cost, num_bins, use_sah != 0));
    std::vector<bbox> bounds(numfaces);
    std::vector<bbox> object_bounds(nummeshes + numinstances);
    for (int i = 0; i < nummeshes; ++i) {
        Mesh const* mesh = meshOf[shapes[i]].get();
        for (int j = 0; j < mesh->num_faces(); ++j) mesh->GetFaceBounds(j, true, bounds[fstart[i] + j]);
        bvhs[i]->Build(&bounds[fstart[i]], mesh->num_faces());
        object_bounds[i] = transform_bbox(bvhs[i]->Bounds(), M(m16 + 16 * shapes[i]));
        bvhptrs[i] = bvhs[i].get();
    }
    auto meshSlot = [&](int shapeIdx) {   // position of the instance's base Mesh in `shapes`
        const int base = ents[shapeIdx].base;
        for (int k = 0; k < nummeshes; ++k)
            if (shapes[k] == base) return k;
        return -1;
    };
    for (int i = nummeshes; i < nummeshes + numinstances; ++i)
        object_bounds[i] = transform_bbox(bvhs[meshSlot(shapes[i])]->Bounds(), M(m16 + 16 * shapes[i]));
    bvhs[nummeshes]->Build(&object_bounds[0], nummeshes + numinstances);
    bvhptrs[nummeshes] = bvhs[nummeshes].get();
    PlainBvhTranslator tr;
    tr.Flush();
    tr.Process(&bvhptrs[0], &fstart[0], nummeshes);
    out->nodes = tr.nodes_;
    out->root = tr.root_;
    out->vertices.resize(4 * (size_t)numvertices);
    for (int i = 0; i < nummeshes; ++i) {
        Mesh const* mesh = meshOf[shapes[i]].get();
        float3 const* v = mesh->GetVertexData();
        for (int j = 0; j < mesh->num_vertices(); ++j) {
            float* o = &out->vertices[4 * ((size_t)vstart[i] + j)];
            o[0] = v[j].x; o[1] = v[j].y; o[2] = v[j].z; o[3] = v[j].w;
        }
    }
    out->faces.resize(numfaces);
    for (int i = 0; i < nummeshes; ++i) {
        int const* reordering = bvhs[i]->GetIndices();
        Mesh const* mesh = meshOf[shapes[i]].get();
        Mesh::Face const* f = mesh->GetFaceData();
        for (int j = 0; j < mesh->num_faces(); ++j) {
            Rr2lFace& d = out->faces[fstart[i] + j];
            const int fi = reordering[j];
            d.idx[0] = f[fi].idx[0] + vstart[i];
            d.idx[1] = f[fi].idx[1] + vstart[i];
            d.idx[2] = f[fi].idx[2] + vstart[i];
            d.shape_id = shapes[i];
            d.prim_id = fi;
        }
    }
    int const* topindices = bvhs[nummeshes]->GetIndices();
    out->shapes.resize(nummeshes + numinstances);
    for (int i = 0; i < nummeshes + numinstances; ++i) {
        const int s = shapes[topindices[i]];
        Rr2lShapeData& d = out->shapes[i];
        std::memset(&d, 0, sizeof(d));
        d.id = s;
        d.shapeDisabled = 0;
        d.minv = M(minv16 + 16 * s);
        d.bvhidx = ents[s].inst ? tr.roots_[meshSlot(s)] : tr.roots_[topindices[i]];
    }
    return out;
}
// sizes: nodes (32 B each), vertices (16 B), faces (20 B), shapes (112 B), root, meshes, instances
__attribute__((visibility("default")))
void rr2l_sizes(void* h, int64_t* out7) {
    auto* r = static_cast<Rr2l*>(h);
    out7[0] = (int64_t)r->nodes.size();
    out7[1] = (int64_t)r->vertices.size() / 4;
    out7[2] = (int64_t)r->faces.size();
    out7[3] = (int64_t)r->shapes.size();
    out7[4] = r->root;
    out7[5] = r->nummeshes;
    out7[6] = r->numinstances;
}
__attribute__((visibility("default")))
void rr2l_copy(void* h, void* nodes, void* vertices, void* faces, void* shapes) {
    auto* r = static_cast<Rr2l*>(h);
    if (nodes) std::memcpy(nodes, r->nodes.data(), 32 * r->nodes.size());
    if (vertices) std::memcpy(vertices, r->vertices.data(), 4 * r->vertices.size());
    if (faces) std::memcpy(faces, r->faces.data(), sizeof(Rr2lFace) * r->faces.size());
    if (shapes) std::memcpy(shapes, r->shapes.data(), sizeof(Rr2lShapeData) * r->shapes.size());
}
__attribute__((visibility("default")))
void rr2l_free(void* h) { delete static_cast<Rr2l*>(h); }

}  // extern "C"

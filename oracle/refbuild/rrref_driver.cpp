// TEST INFRASTRUCTURE ONLY -- oracle/_ref driver.
//
// Links the reference's OWN C++ sources, compiled in place from /root/reference
// by oracle/refbuild/Makefile (nothing is copied into this repo):
//   third_party/RadeonRays/RadeonRays/src/accelerator/bvh2.cpp  (Bvh2 SAH builder)
//   third_party/RadeonRays/RadeonRays/src/primitive/mesh.cpp    (Mesh::GetFaceBounds)
//   third_party/RadeonRays/UnitTest/utils.cpp                  (brute-force golden)
//   third_party/RadeonRays/UnitTest/tiny_obj_loader.cpp        (CornellBox orig.objm)
// and exposes them through a tiny C interface for tests/ (ctypes).
#include "accelerator/bvh2.h"
#include "primitive/mesh.h"
#include "utils.h"
#include "tiny_obj_loader.h"

#include <cstdint>
#include <cstring>
#include <memory>
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

}  // extern "C"

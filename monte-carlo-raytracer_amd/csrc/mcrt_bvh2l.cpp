// mcrt_bvh2l.cpp -- host build of the two-level (instanced) acceleration structure.
//
// What RadeonRays does when a mesh is shared (RTScene::attachMesh -> CreateInstance,
// APP/raytracing/scene/RTScene.cpp:572-596; CalcIntersectionDevice::Preprocess switches to
// IntersectorTwoLevel, RR/src/device/calc_intersection_device.cpp:68-105):
//   * one object-space BVH per distinct mesh, over its face bounds (RR Bvh, accelerator/bvh.cpp,
//     1 primitive per leaf, binned SAH over all three axes);
//   * one top-level BVH over the world-space boxes of every shape (meshes first, then
//     instances: std::partition over the world's shape list, intersector_2level.cpp:196-201),
//     each box = transform_bbox(mesh BVH bounds, shape transform) (mathutils.h:142-158);
//   * traversal transforms the ray into object space with the shape's world-to-local matrix
//     at a top-level leaf (intersect_bvh2level_skiplinks.cl:213-246).
// The trees built here are RR Bvh's, node for node (the split arithmetic below restates
// bvh.cpp:73-437 in scalar float, no contraction: this file is compiled -ffp-contract=off;
// pinned by tests/test_bvh2l_cpu.py against the reference's own bvh.cpp compiled into
// oracle/_ref/librrref.so).  The layout is ours: the same 64-B records as the flat BVH
// (mcrt_bvh.cpp) so one traversal loop serves both levels --
//   internal: both child boxes + child indices (int4 (c0, c1, 0, 0), c0/c1 >= 1)
//   triangle: float4 (v0, -1), float4 (v1 - v0, primId bits), float4 (v2 - v0, 0), int4 (-1, ...)
//             (object-space vertices of the mesh, RR's vertex buffer)
//   instance: float4 minv.m0, minv.m1, minv.m2 (world -> object rows), int4 (-2, bottom root,
//             shape id, 0)
// Records: [top tree][mesh 0 tree][mesh 1 tree]...; the top root is record 0.
#include <algorithm>
#include <atomic>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <map>
#include <thread>
#include <tuple>
#include <vector>

#include "mcrt_internal.h"

namespace mcrt {
namespace {

// RR bbox / float3 arithmetic (math/bbox.h, math/float3.h): std::min/std::max per component.
struct Box {
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    float hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    void grow(const float* p) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], p[a]);
            hi[a] = std::max(hi[a], p[a]);
        }
    }
    void grow(const Box& b) {
        for (int a = 0; a < 3; ++a) {
            lo[a] = std::min(lo[a], b.lo[a]);
            hi[a] = std::max(hi[a], b.hi[a]);
        }
    }
    float ext(int a) const { return hi[a] - lo[a]; }
    float center(int a) const { return 0.5f * (hi[a] + lo[a]); }
    float area() const {
        const float x = ext(0), y = ext(1), z = ext(2);
        return 2.f * (x * y + x * z + y * z);
    }
    int maxdim() const {   // bbox.h:191-203
        const float x = ext(0), y = ext(1), z = ext(2);
        if (x >= y && x >= z) return 0;
        if (y >= x && y >= z) return 1;
        if (z >= x && z >= y) return 2;
        return 0;
    }
};

// RR transform_point (mathutils.h:111-118 via matrix * float4, matrix.h:182-193)
inline void xform(const mcrt_mat4& m, const float* p, float* o) {
    const mcrt_float4* r[3] = {&m.m0, &m.m1, &m.m2};
    for (int i = 0; i < 3; ++i) {
        float acc = 0.0f;
        acc += r[i]->x * p[0];
        acc += r[i]->y * p[1];
        acc += r[i]->z * p[2];
        acc += r[i]->w * 0.0f;
        o[i] = acc + r[i]->w;
    }
}

// transform_bbox (mathutils.h:142-158): the 8 corners pmin + (0|ext) of the box
Box transformBox(const Box& b, const mcrt_mat4& m) {
    const float e[3] = {b.ext(0), b.ext(1), b.ext(2)};
    static const int sel[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}, {0, 0, 1}};
    Box out;
    for (int c = 0; c < 8; ++c) {
        float p[3], q[3];
        for (int a = 0; a < 3; ++a) p[a] = b.lo[a] + (sel[c][a] ? e[a] : 0.0f);
        xform(m, p, q);
        if (c == 0) {
            for (int a = 0; a < 3; ++a) out.lo[a] = out.hi[a] = q[a];
        } else {
            out.grow(q);
        }
    }
    return out;
}

// One RR Bvh (bvh.cpp) over `n` primitive boxes.  Output in pre-order (the order both
// Bvh::AllocateNode and PlainBvhTranslator::ProcessNode visit): node p's left child is p + 1,
// its right child p + 2 * nLeft; every leaf holds exactly one primitive (bvh.cpp:33, :90) whose
// packed position equals its request's start index, so subtrees can be built concurrently.
class ObjBvh {
public:
    ObjBvh(const Box* bounds, int n, float cost, int bins, bool sah, int threads)
        : bounds_(bounds), cost_(cost), bins_(bins), sah_(sah), budget_(threads - 1) {
        nodeBox.resize(2 * (size_t)n - 1);
        nodeLeft.resize(2 * (size_t)n - 1);   // internal: prims in left subtree; leaf: -1 - prim
        indices.resize(n);
        cen_.resize(3 * (size_t)n);
        Box root, croot;
        for (int i = 0; i < n; ++i) root.grow(bounds[i]);   // Bvh::Build, bvh.cpp:41-49
        for (int i = 0; i < n; ++i) {
            indices[i] = i;
            for (int a = 0; a < 3; ++a) cen_[3 * i + a] = bounds[i].center(a);
            croot.grow(&cen_[3 * i]);
        }
        rootBox = root;
        build(0, 0, n, root, croot, 0);
    }
    std::vector<Box> nodeBox;
    std::vector<int> nodeLeft;
    std::vector<int> indices;   // Bvh::GetIndices: primitive of each packed leaf slot
    Box rootBox;                // Bvh::Bounds
    std::atomic<int> height{0};

private:
    struct Split {
        int dim = 0;
        float split = NAN;
    };
    const Box* bounds_;
    float cost_;
    int bins_;
    bool sah_;
    std::atomic<int> budget_;
    std::vector<float> cen_;

    float c(int prim, int axis) const { return cen_[3 * prim + axis]; }

    // FindSahSplit (bvh.cpp:253-361)
    Split sahSplit(int start, int num, const Box& box, const Box& cbox) const {
        Split s;
        const float ce[3] = {cbox.ext(0), cbox.ext(1), cbox.ext(2)};
        if (ce[0] * ce[0] + ce[1] * ce[1] + ce[2] * ce[2] == 0.f) return s;
        struct Bin {
            Box b;
            int count = 0;
        };
        std::vector<Bin> bins(bins_);
        std::vector<Box> right(bins_ - 1);
        int splitidx = -1;
        float sah = FLT_MAX;
        const float invarea = 1.f / box.area();
        for (int axis = 0; axis < 3; ++axis) {
            const float rootminc = cbox.lo[axis];
            const float rng = ce[axis];
            const float invrng = 1.f / rng;
            if (rng == 0.f) continue;
            for (auto& b : bins) b = Bin();
            for (int i = start; i < start + num; ++i) {
                const int idx = indices[i];
                const int bi = (int)std::min<float>((float)bins_ * ((c(idx, axis) - rootminc) * invrng), (float)(bins_ - 1));
                ++bins[bi].count;
                bins[bi].b.grow(bounds_[idx]);
            }
            Box rb;
            for (int i = bins_ - 1; i > 0; --i) {
                rb.grow(bins[i].b);
                right[i - 1] = rb;
            }
            Box lb;
            int lc = 0, rc = num;
            for (int i = 0; i < bins_ - 1; ++i) {
                lb.grow(bins[i].b);
                lc += bins[i].count;
                rc -= bins[i].count;
                const float t = cost_ + ((float)lc * lb.area() + (float)rc * right[i].area()) * invarea;
                if (t < sah) {
                    s.dim = axis;
                    splitidx = i;
                    sah = t;
                }
            }
        }
        if (splitidx != -1) s.split = cbox.lo[s.dim] + (float)(splitidx + 1) * (ce[s.dim] / (float)bins_);
        return s;
    }

    // BuildNode (bvh.cpp:73-251) for the request (start, num) at pre-order slot p
    void build(int p, int start, int num, const Box& box, const Box& cbox, int level) {
        int h = height.load(std::memory_order_relaxed);
        while (level > h && !height.compare_exchange_weak(h, level)) {
        }
        nodeBox[p] = box;
        if (num < 2) {
            nodeLeft[p] = -1 - start;
            return;
        }
        int axis = cbox.maxdim();
        float border = cbox.center(axis);
        if (sah_) {
            const Split ss = sahSplit(start, num, box, cbox);
            if (!std::isnan(ss.split)) {
                axis = ss.dim;
                border = ss.split;
            }
        }
        Box lb, rb, lcb, rcb;
        int* P = indices.data();
        int splitidx = start;
        const bool near2far = (num + start) & 0x1;
        if (cbox.ext(axis) > 0.f) {
            // the reference's two-sided partition, including its swap sequence (the order
            // inside a range matters for later median splits)
            int first = start, last = start + num;
            auto goesLeft = [&](int prim) { return near2far ? c(prim, axis) < border : c(prim, axis) >= border; };
            while (true) {
                while (first != last && goesLeft(P[first])) {
                    lb.grow(bounds_[P[first]]);
                    lcb.grow(&cen_[3 * P[first]]);
                    ++first;
                }
                if (first == last--) break;
                rb.grow(bounds_[P[first]]);
                rcb.grow(&cen_[3 * P[first]]);
                while (first != last && !goesLeft(P[last])) {
                    rb.grow(bounds_[P[last]]);
                    rcb.grow(&cen_[3 * P[last]]);
                    --last;
                }
                if (first == last) break;
                lb.grow(bounds_[P[last]]);
                lcb.grow(&cen_[3 * P[last]]);
                std::swap(P[first++], P[last]);
            }
            splitidx = first;
        }
        if (splitidx == start || splitidx == start + num) {
            // median fallback; the boxes grown by the partition above are kept (bvh.cpp:198-212)
            splitidx = start + (num >> 1);
            for (int i = start; i < splitidx; ++i) {
                lb.grow(bounds_[P[i]]);
                lcb.grow(&cen_[3 * P[i]]);
            }
            for (int i = splitidx; i < start + num; ++i) {
                rb.grow(bounds_[P[i]]);
                rcb.grow(&cen_[3 * P[i]]);
            }
        }
        const int nl = splitidx - start;
        nodeLeft[p] = nl;
        const int pl = p + 1, pr = p + 2 * nl;
        if (num >= 65536 && budget_.fetch_sub(1) > 0) {
            std::thread t([&, pl, start, nl, level] { build(pl, start, nl, lb, lcb, level + 1); });
            build(pr, splitidx, num - nl, rb, rcb, level + 1);
            t.join();
            budget_.fetch_add(1);
        } else {
            if (num >= 65536) budget_.fetch_add(1);
            build(pl, start, nl, lb, lcb, level + 1);
            build(pr, splitidx, num - nl, rb, rcb, level + 1);
        }
    }
};

inline void putBox2(float* r, const Box& a, const Box& b) {
    r[0] = a.lo[0]; r[1] = a.hi[0]; r[2] = a.lo[1]; r[3] = a.hi[1];
    r[4] = b.lo[0]; r[5] = b.hi[0]; r[6] = b.lo[1]; r[7] = b.hi[1];
    r[8] = a.lo[2]; r[9] = a.hi[2]; r[10] = b.lo[2]; r[11] = b.hi[2];
}
inline void putInts(float* r, int a, int b, int c, int d) {
    const int32_t v[4] = {a, b, c, d};
    std::memcpy(r + 12, v, 16);
}

// Internal records of tree `t` placed at record offset `base` (children offset too).
void emitInternal(const ObjBvh& t, int base, std::vector<float>& rec) {
    const int nn = (int)t.nodeBox.size();
    for (int p = 0; p < nn; ++p) {
        const int nl = t.nodeLeft[p];
        if (nl < 0) continue;
        const int c0 = p + 1, c1 = p + 2 * nl;
        float* r = &rec[16 * ((size_t)base + p)];
        putBox2(r, t.nodeBox[c0], t.nodeBox[c1]);
        putInts(r, base + c0, base + c1, 0, 0);
    }
}

}  // namespace

bool shapes_are_instanced(const mcrt_shape* shapes, size_t n) {
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, int> seen;
    for (size_t i = 0; i < n; ++i) {
        if (shapes[i].numTriangles == 0) continue;
        if (!seen.emplace(std::make_tuple(shapes[i].startIdx, shapes[i].startVertex, shapes[i].numTriangles), 0).second)
            return true;
    }
    return false;
}

bool build_bvh2l(const mcrt_shape* shapes, size_t nshapes, const uint32_t* indices, const mcrt_float4* positions,
                 const mcrt_mat4* worldToLocal, float cost, int bins, bool sah, int threads, Bvh2lOut& out) {
    // meshes and instances (RTScene::attachMesh: the first shape with a mesh's data owns it)
    struct Ent {
        bool inst;
        int mesh;   // index into `meshes`
    };
    std::vector<int> meshShape;   // shape owning each mesh, in first-attach order
    std::vector<Ent> ent(nshapes, Ent{false, -1});
    std::map<std::tuple<uint32_t, uint32_t, uint32_t>, int> key2mesh;
    std::vector<int> world;   // shapes in the top level, world order (zero-triangle shapes skipped)
    for (size_t i = 0; i < nshapes; ++i) {
        const mcrt_shape& s = shapes[i];
        if (s.numTriangles == 0) continue;
        auto k = std::make_tuple(s.startIdx, s.startVertex, s.numTriangles);
        auto it = key2mesh.find(k);
        if (it == key2mesh.end()) {
            key2mesh[k] = (int)meshShape.size();
            ent[i] = Ent{false, (int)meshShape.size()};
            meshShape.push_back((int)i);
        } else {
            ent[i] = Ent{true, it->second};
        }
        world.push_back((int)i);
    }
    if (world.empty()) return false;
    // std::partition(meshes first) with libstdc++'s bidirectional algorithm, as the reference
    // host code gets it (intersector_2level.cpp:196-201); the top tree's input order follows it
    {
        auto first = world.begin(), last = world.end();
        while (true) {
            while (first != last && !ent[*first].inst) ++first;
            if (first == last) break;
            --last;
            while (first != last && ent[*last].inst) --last;
            if (first == last) break;
            std::iter_swap(first, last);
            ++first;
        }
    }
    const int numShapesTop = (int)world.size();
    const int numMeshes = (int)meshShape.size();
    // per-mesh object-space trees (face bounds: Mesh::GetFaceBounds(objectspace = true) =
    // transform_point with the identity matrix, mesh.cpp:115-143)
    static const mcrt_mat4 I = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    std::vector<ObjBvh*> trees(numMeshes, nullptr);
    {
        std::atomic<int> next{0};
        const int nt = std::max(1, std::min(threads, numMeshes));
        const int inner = std::max(1, threads / nt);
        auto work = [&] {
            for (int m; (m = next.fetch_add(1)) < numMeshes;) {
                const mcrt_shape& s = shapes[meshShape[m]];
                std::vector<Box> fb(s.numTriangles);
                for (uint32_t f = 0; f < s.numTriangles; ++f) {
                    float v[3][3];
                    for (int c = 0; c < 3; ++c) {
                        const mcrt_float4& p = positions[s.startVertex + indices[s.startIdx + 3 * f + c]];
                        const float q[3] = {p.x, p.y, p.z};
                        xform(I, q, v[c]);
                    }
                    Box b;   // bbox(v0, v1) then grow(v2)
                    for (int a = 0; a < 3; ++a) {
                        b.lo[a] = std::min(v[0][a], v[1][a]);
                        b.hi[a] = std::max(v[0][a], v[1][a]);
                    }
                    b.grow(v[2]);
                    fb[f] = b;
                }
                trees[m] = new ObjBvh(fb.data(), (int)s.numTriangles, cost, bins, sah, inner);
            }
        };
        std::vector<std::thread> pool;
        for (int t = 1; t < nt; ++t) pool.emplace_back(work);
        work();
        for (auto& t : pool) t.join();
    }
    // top level over the world-space boxes
    std::vector<Box> ob(numShapesTop);
    for (int i = 0; i < numShapesTop; ++i) {
        const int si = world[i];
        ob[i] = transformBox(trees[ent[si].mesh]->rootBox, shapes[si].toWorldTransform);
    }
    ObjBvh top(ob.data(), numShapesTop, cost, bins, sah, 1);
    // records: [top][mesh 0][mesh 1]...
    const size_t topN = 2 * (size_t)numShapesTop - 1;
    std::vector<size_t> meshBase(numMeshes);
    size_t total = topN;
    int maxBottom = 0;
    for (int m = 0; m < numMeshes; ++m) {
        meshBase[m] = total;
        total += trees[m]->nodeBox.size();
        maxBottom = std::max(maxBottom, trees[m]->height.load());
    }
    if (total > (size_t)0x7fffffff) {
        for (auto* t : trees) delete t;
        return false;
    }
    std::vector<float> rec(16 * total);
    emitInternal(top, 0, rec);
    for (size_t p = 0; p < topN; ++p) {
        const int nl = top.nodeLeft[p];
        if (nl >= 0) continue;
        const int si = world[top.indices[-1 - nl]];
        mcrt_mat4 minv;
        if (worldToLocal) {
            minv = worldToLocal[si];
        } else {   // inverse = transpose(inverse transpose)
            const mcrt_mat4& t = shapes[si].toWorldInverseTranspose;
            minv.m0 = {t.m0.x, t.m1.x, t.m2.x, t.m3.x};
            minv.m1 = {t.m0.y, t.m1.y, t.m2.y, t.m3.y};
            minv.m2 = {t.m0.z, t.m1.z, t.m2.z, t.m3.z};
            minv.m3 = {t.m0.w, t.m1.w, t.m2.w, t.m3.w};
        }
        float* r = &rec[16 * p];
        std::memcpy(r + 0, &minv.m0, 16);
        std::memcpy(r + 4, &minv.m1, 16);
        std::memcpy(r + 8, &minv.m2, 16);
        putInts(r, -2, (int)meshBase[ent[si].mesh], si, 0);
    }
    for (int m = 0; m < numMeshes; ++m) {
        const ObjBvh& t = *trees[m];
        const int base = (int)meshBase[m];
        emitInternal(t, base, rec);
        const mcrt_shape& s = shapes[meshShape[m]];
        for (size_t p = 0; p < t.nodeBox.size(); ++p) {
            const int nl = t.nodeLeft[p];
            if (nl >= 0) continue;
            const int f = t.indices[-1 - nl];
            float v[3][3];
            for (int c = 0; c < 3; ++c) {
                const mcrt_float4& q = positions[s.startVertex + indices[s.startIdx + 3 * f + c]];
                v[c][0] = q.x; v[c][1] = q.y; v[c][2] = q.z;
            }
            float* r = &rec[16 * (base + p)];
            const int32_t negOne = -1;
            r[0] = v[0][0]; r[1] = v[0][1]; r[2] = v[0][2]; std::memcpy(&r[3], &negOne, 4);
            r[4] = v[1][0] - v[0][0]; r[5] = v[1][1] - v[0][1]; r[6] = v[1][2] - v[0][2]; std::memcpy(&r[7], &f, 4);
            r[8] = v[2][0] - v[0][0]; r[9] = v[2][1] - v[0][1]; r[10] = v[2][2] - v[0][2]; r[11] = 0.0f;
            putInts(r, -1, -1, 0, 0);
        }
    }
    out.records = std::move(rec);
    out.numNodes = total;
    out.topNodes = topN;
    out.numMeshes = numMeshes;
    out.numInstances = numShapesTop - numMeshes;
    out.depth = top.height.load() + maxBottom + 1;   // + the return marker
    out.topBox[0] = top.rootBox.lo[0]; out.topBox[1] = top.rootBox.lo[1]; out.topBox[2] = top.rootBox.lo[2];
    out.topBox[3] = top.rootBox.hi[0]; out.topBox[4] = top.rootBox.hi[1]; out.topBox[5] = top.rootBox.hi[2];
    for (auto* t : trees) delete t;
    return true;
}

}  // namespace mcrt

// wide.h -- 4-wide quantized BVH records of the round-3 wide-tree experiment (tools/experiments/wide_tree.patch
// holds the product integration; measured slower than the Bvh2, profiles/r03/ab/README.txt item 1), shared by the
// host build and the traversal model of tools/widesim.
// The RadeonRays Bvh2 (the parity tree, mcrt_bvh.cpp / mcrt_sahbuild.hip) is collapsed into
// 4-wide nodes: each node's up to four children are the largest-area descendants of a Bvh2 node,
// their boxes stored as 8-bit offsets from the node's origin in power-of-two steps, so a node --
// origin, exponents, 4 x 6 quantized planes, 4 child references -- is ONE 64-B record, the size
// of a Bvh2 record, and a step tests four boxes instead of two.  Every quantized plane decodes
// (fma(q, 2^e, origin), exact to evaluate on host and device alike) to a float on the outer side
// of the Bvh2 box it replaces, and the slab test evaluates it with the reference's own formula
// (fma(plane, 1/d, -o/d), intersect_bvh2_lds.cl:54-63), which is monotone in the plane: every box
// test the reference passes, the wide tree passes too.  Triangles are the Bvh2 leaf records (same
// triangle test, same hit arithmetic), so the closest hit can differ only between triangles at
// (nearly) the same t, which the two trees visit in different orders.
//
// Node record (16 x 32-bit words):
//   w0..w2  origin x, y, z (float)
//   w3      byte 0..2: exponents e_x, e_y, e_z + 127 (plane step 2^e, a normal float's bits << 23)
//           byte 3: bits 0-3 child valid, bits 4-7 child is a triangle
//   w4..w9  quantized planes lo.x, hi.x, lo.y, hi.y, lo.z, hi.z: byte c = child c's plane
//   w10..13 child c: node index (internal) or triangle record index (leaf)
//   w14,15  0
// Triangle record (4 x float4): (v0, shapeId bits), (v1, primId bits), (v2, 0), (0, 0, 0, 0) --
//   the world-space vertices the Bvh2 builder saw, so the traversal rebuilds the Bvh2 leaf exactly:
//   its edges v1 - v0, v2 - v0 (the mcrt_bvh.cpp leaf record's, bit for bit) and its box (the
//   per-axis min / max of the vertices, the child box the Bvh2 parent holds).  Testing that exact
//   leaf box before the triangle makes the set of triangles a query tests with the full ray
//   interval the reference's set: any-hit answers are identical to the Bvh2's.
//
// Numbering: level by level (breadth first); a node's internal children take consecutive node
// indices and its triangle children consecutive triangle records, in child order.  The device
// builder (mcrt_widebuild.hip) produces the same arrays as this host restatement.
#pragma once
#include <stdint.h>

#include <cstddef>
#include <string>
#include <vector>

#include <cmath>

#define WIDE_K 4
// the quantization helpers below are shared by the host restatement and the device builder
#ifdef __HIPCC__
#define WIDE_HD __host__ __device__
#else
#define WIDE_HD
#endif
#define WIDE_LEAF_BIT 0x80000000u   // stack entries: triangle record (else node index)

namespace mcrt {
struct WideTree {
    std::vector<uint32_t> nodes;   // 16 words per node; node 0 = root
    std::vector<float> tris;       // 16 floats per triangle record, in numbering order (below)
    uint32_t numNodes = 0, numTris = 0;
    int depth = 0;                 // deepest node path (root = 1)
    bool rootIsLeaf = false;       // a one-triangle scene: the root is triangle record 0
};
// Collapses the Bvh2 records (16 floats per node, mcrt_bvh.cpp layout, node 0 = root) into `out`.
// tri9: the world-space triangles the Bvh2 was built from (9 floats each), triangle of (shape s,
// prim p) = shapeFirst[s] + p.  false (with *err) on malformed input or when a leaf record does
// not match its triangle.
bool build_wide(const float* rec2, std::size_t n2, const float* tri9, const uint32_t* shapeFirst,
                std::size_t numShapes, std::size_t numTris, WideTree& out, std::string* err);
// the surface-area order the collapse opens children in: fp32, compiled without contraction
// (-ffp-contract=off; the device builder spells the same operations with __fmul_rn / __fadd_rn)
WIDE_HD inline float wide_area(const float* lo, const float* hi) {
    const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return (dx * dy + dy * dz) + dz * dx;
}
// The decoded plane of quantized value q (0..255) with exponent byte eb and origin o: the exact
// float both the builder and the traversal evaluate.
WIDE_HD inline float wide_plane(uint32_t q, uint32_t eb, float o) {
    union { uint32_t u; float f; } s;
    s.u = eb << 23;
    return __builtin_fmaf((float)q, s.f, o);
}
// smallest exponent byte eb >= 1 (e >= -126) with wide_plane(255, eb, o) >= hmax; 0 if none
WIDE_HD inline uint32_t wide_axis_exponent(float o, float hmax) {
    if (!(hmax > o)) return 127;   // flat axis: every plane is the origin (q = 0)
    int e;
    frexp(((double)hmax - (double)o) / 255.0, &e);   // 2^(e-1) <= ext/255 < 2^e
    e = (e < -126 ? -126 : e > 127 ? 127 : e);
    while (e > -126 && wide_plane(255, (uint32_t)(e - 1 + 127), o) >= hmax) --e;
    while (e <= 127 && wide_plane(255, (uint32_t)(e + 127), o) < hmax) ++e;
    return e > 127 ? 0u : (uint32_t)(e + 127);
}
// largest q with wide_plane(q) <= v (a lo plane); v >= o
WIDE_HD inline uint32_t wide_quant_lo(float v, uint32_t eb, float o) {
    union { uint32_t u; float f; } s;
    s.u = eb << 23;
    const double g = floor(((double)v - (double)o) / (double)s.f);
    int q = (int)(g < 0.0 ? 0.0 : g > 255.0 ? 255.0 : g);
    while (q > 0 && wide_plane((uint32_t)q, eb, o) > v) --q;
    while (q < 255 && wide_plane((uint32_t)q + 1, eb, o) <= v) ++q;
    return (uint32_t)q;
}
// smallest q with wide_plane(q) >= v (a hi plane); v <= wide_plane(255)
WIDE_HD inline uint32_t wide_quant_hi(float v, uint32_t eb, float o) {
    union { uint32_t u; float f; } s;
    s.u = eb << 23;
    const double g = ceil(((double)v - (double)o) / (double)s.f);
    int q = (int)(g < 0.0 ? 0.0 : g > 255.0 ? 255.0 : g);
    while (q < 255 && wide_plane((uint32_t)q, eb, o) < v) ++q;
    while (q > 0 && wide_plane((uint32_t)q - 1, eb, o) >= v) --q;
    return (uint32_t)q;
}

}  // namespace mcrt

// wide.cpp -- host build of the 4-wide quantized tree (wide.h) of the round-3 experiment: the
// specification the device builder (mcrt_widebuild.hip) is checked against record for record,
// and the builder of the analysis tools.  Compiled with -ffp-contract=off.
//
// Collapse: a wide node starts from the two children of a Bvh2 node and, while it has fewer than
// four, replaces its internal child of largest surface area (wide_area; the first on ties) by
// that child's two children, in place (the first child takes the opened slot, the second follows
// it), which keeps the Bvh2's left-to-right order among siblings.
//
// Quantization, per node and axis: origin o = the smallest child lo; step 2^e with the smallest
// e >= -126 for which wide_plane(255, e, o) >= the largest child hi; per child, lo -> the largest q
// with wide_plane(q) <= lo and hi -> the smallest q with wide_plane(q) >= hi.  Each choice is a
// predicate on the decoded fp32 plane itself, so host and device arrive at the same bytes, and
// every decoded box contains its Bvh2 box.
#include "wide.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

namespace mcrt {
namespace {

struct Box {
    float lo[3], hi[3];
};

// child c (0 / 1) box of Bvh2 internal record r (mcrt_bvh.cpp layout)
inline Box childBox(const float* r, int c) {
    Box b;
    const float* xy = r + 4 * c;
    b.lo[0] = xy[0]; b.hi[0] = xy[1]; b.lo[1] = xy[2]; b.hi[1] = xy[3];
    b.lo[2] = r[8 + 2 * c]; b.hi[2] = r[9 + 2 * c];
    return b;
}

inline int32_t word(const float* r, int k) {
    int32_t v;
    std::memcpy(&v, r + k, 4);
    return v;
}
inline bool isLeaf(const float* r) { return word(r, 12) < 0; }

inline uint32_t fbits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

}  // namespace

bool build_wide(const float* rec2, std::size_t n2, const float* tri9, const uint32_t* shapeFirst,
                std::size_t numShapes, std::size_t numTris, WideTree& out, std::string* err) {
    out = WideTree();
    auto bad = [&](const std::string& m) {
        if (err) *err = m;
        return false;
    };
    if (!rec2 || n2 == 0) return bad("empty Bvh2");
    if (n2 >= (std::size_t)WIDE_LEAF_BIT) return bad("Bvh2 too large for 31-bit references");
    // triangle record of Bvh2 leaf record r: the world vertices, checked against the leaf's
    // v0 and edges (the Bvh2 builder's v1 - v0, v2 - v0)
    auto emitTri = [&](const float* r) -> bool {
        const int32_t shape = word(r, 3), prim = word(r, 7);
        if (shape < 0 || (std::size_t)shape >= numShapes || prim < 0) return false;
        const std::size_t k = (std::size_t)shapeFirst[shape] + (std::size_t)prim;
        if (k >= numTris) return false;
        const float* p = tri9 + 9 * k;
        for (int a = 0; a < 3; ++a)
            if (fbits(p[a]) != fbits(r[a]) || fbits(p[3 + a] - p[a]) != fbits(r[4 + a]) ||
                fbits(p[6 + a] - p[a]) != fbits(r[8 + a]))
                return false;
        float t[16] = {p[0], p[1], p[2], r[3], p[3], p[4], p[5], r[7], p[6], p[7], p[8], 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        out.tris.insert(out.tris.end(), t, t + 16);
        ++out.numTris;
        return true;
    };
    std::size_t leaves = 0;
    for (std::size_t i = 0; i < n2; ++i) leaves += isLeaf(rec2 + 16 * i) ? 1 : 0;
    out.tris.reserve(16 * leaves);
    if (isLeaf(rec2)) {
        out.rootIsLeaf = true;
        out.depth = 1;
        return emitTri(rec2) ? true : bad("leaf record does not match its triangle");
    }
    out.nodes.reserve(16 * (leaves / 2 + 2));
    out.nodes.assign(16, 0u);
    out.numNodes = 1;
    std::vector<int32_t> level{0}, next;   // Bvh2 node of wide node (levelBase + i)
    uint32_t levelBase = 0;
    while (!level.empty()) {
        ++out.depth;
        next.clear();
        for (std::size_t li = 0; li < level.size(); ++li) {
            const uint32_t wi = levelBase + (uint32_t)li;
            const float* r = rec2 + 16 * (std::size_t)level[li];
            int32_t cn[WIDE_K];
            Box cb[WIDE_K];
            int n = 0;
            for (int c = 0; c < 2; ++c) {
                const int32_t k = word(r, 12 + c);
                if (k <= 0 || (std::size_t)k >= n2) return bad("Bvh2 child index out of range");
                cn[n] = k;
                cb[n++] = childBox(r, c);
            }
            while (n < WIDE_K) {
                int best = -1;
                float bestA = 0.0f;
                for (int c = 0; c < n; ++c) {
                    if (isLeaf(rec2 + 16 * (std::size_t)cn[c])) continue;
                    const float a = wide_area(cb[c].lo, cb[c].hi);
                    if (best < 0 || a > bestA) { bestA = a; best = c; }
                }
                if (best < 0) break;
                const float* rb = rec2 + 16 * (std::size_t)cn[best];
                const int32_t k0 = word(rb, 12), k1 = word(rb, 13);
                if (k0 <= 0 || k1 <= 0 || (std::size_t)k0 >= n2 || (std::size_t)k1 >= n2)
                    return bad("Bvh2 child index out of range");
                for (int c = n; c > best + 1; --c) { cn[c] = cn[c - 1]; cb[c] = cb[c - 1]; }
                cn[best] = k0; cb[best] = childBox(rb, 0);
                cn[best + 1] = k1; cb[best + 1] = childBox(rb, 1);
                ++n;
            }
            uint32_t w[16] = {};
            float o[3];
            uint32_t eb[3];
            for (int a = 0; a < 3; ++a) {
                float lo = cb[0].lo[a], hi = cb[0].hi[a];
                for (int c = 1; c < n; ++c) { lo = std::min(lo, cb[c].lo[a]); hi = std::max(hi, cb[c].hi[a]); }
                if (!std::isfinite(lo) || !std::isfinite(hi)) return bad("non-finite box");
                o[a] = lo;
                eb[a] = wide_axis_exponent(lo, hi);
                if (eb[a] == 0) return bad("box extent not representable");
                w[a] = fbits(lo);
            }
            uint32_t valid = 0, leafMask = 0;
            for (int c = 0; c < n; ++c) {
                valid |= 1u << c;
                for (int a = 0; a < 3; ++a) {
                    const uint32_t ql = wide_quant_lo(cb[c].lo[a], eb[a], o[a]);
                    const uint32_t qh = wide_quant_hi(cb[c].hi[a], eb[a], o[a]);
                    if (wide_plane(ql, eb[a], o[a]) > cb[c].lo[a] || wide_plane(qh, eb[a], o[a]) < cb[c].hi[a])
                        return bad("quantized box does not contain the Bvh2 box");
                    w[4 + 2 * a] |= ql << (8 * c);
                    w[5 + 2 * a] |= qh << (8 * c);
                }
                const float* rc = rec2 + 16 * (std::size_t)cn[c];
                if (isLeaf(rc)) {
                    leafMask |= 1u << c;
                    w[10 + c] = out.numTris;
                    if (!emitTri(rc)) return bad("leaf record does not match its triangle");
                } else {
                    w[10 + c] = out.numNodes++;
                    next.push_back(cn[c]);
                }
            }
            w[3] = eb[0] | (eb[1] << 8) | (eb[2] << 16) | ((valid | (leafMask << 4)) << 24);
            std::memcpy(&out.nodes[16 * (std::size_t)wi], w, sizeof(w));
            out.nodes.resize(16 * (std::size_t)out.numNodes, 0u);
        }
        levelBase += (uint32_t)level.size();
        level.swap(next);
    }
    if (out.numTris >= WIDE_LEAF_BIT || out.numNodes >= WIDE_LEAF_BIT) return bad("too many records");
    return true;
}

}  // namespace mcrt

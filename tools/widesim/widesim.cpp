// widesim.cpp -- CPU model of the Bvh2 and the 4-wide quantized traversal (analysis tool).
// Builds the wide tree with the experiment's builder (wide.cpp), replays both traversals over
// the same rays and reports per ray the internal steps, triangle steps and the closest hit, so
// the node-visit reduction and the result agreement can be measured before any GPU run.
// Build: g++ -O2 -std=c++17 -shared -fPIC -pthread tools/widesim/widesim.cpp \
//          tools/widesim/wide.cpp -o /tmp/widesim.so
#include <cmath>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <thread>
#include <vector>

#include "wide.h"

using mcrt::WideTree;

namespace {
struct Ray {
    float o[4], d[4];
    int32_t extra[2];
    int32_t bf, pad;
};
WideTree g_wide;
int g_leafbox = 1;
int g_sort = 1;   // 1: hit children by entry distance; 0: stored order
const float* g_rec2 = nullptr;
size_t g_n2 = 0;

inline float dot3(const float* a, const float* b) { return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0])); }
inline void cross3(const float* a, const float* b, float* c) {
    c[0] = fmaf(a[1], b[2], -(a[2] * b[1]));
    c[1] = fmaf(a[2], b[0], -(a[0] * b[2]));
    c[2] = fmaf(a[0], b[1], -(a[1] * b[0]));
}
// RR common.cl:177-218 on a 16-float triangle record
float triHit(const Ray& r, const float* rec, float tmax) {
    const float e1[3] = {rec[4], rec[5], rec[6]}, e2[3] = {rec[8], rec[9], rec[10]};
    float s1[3];
    cross3(r.d, e2, s1);
    const float den = dot3(s1, e1);
    if (den == 0.f) return tmax;
    const float inv = 1.0f / den;
    const float dd[3] = {r.o[0] - rec[0], r.o[1] - rec[1], r.o[2] - rec[2]};
    const float b1 = dot3(dd, s1) * inv;
    float s2[3];
    cross3(dd, e1, s2);
    const float b2 = dot3(r.d, s2) * inv;
    const float t = dot3(e2, s2) * inv;
    if (b1 < 0.f || b1 > 1.f || b2 < 0.f || b1 + b2 > 1.f || t < 0.f || t > tmax) return tmax;
    return t;
}
inline float sinv(float d) { return 1.0f / (fabsf(d) > 1e-8f ? d : copysignf(1e-8f, d)); }
inline void slab(const float lo[3], const float hi[3], const float* inv, const float* oxi, float t, float& t0,
                 float& t1) {
    float a[3], b[3];
    for (int k = 0; k < 3; ++k) {
        a[k] = fmaf(lo[k], inv[k], oxi[k]);
        b[k] = fmaf(hi[k], inv[k], oxi[k]);
    }
    t0 = fmaxf(fmaxf(fmaxf(fminf(a[0], b[0]), fminf(a[1], b[1])), fminf(a[2], b[2])), 0.0f);
    t1 = fminf(fminf(fminf(fmaxf(a[0], b[0]), fmaxf(a[1], b[1])), fmaxf(a[2], b[2])), t);
}
inline int32_t ci(const float* r, int c) {
    int32_t v;
    memcpy(&v, r + 12 + c, 4);
    return v;
}
inline int32_t asInt(float f) {
    int32_t v;
    memcpy(&v, &f, 4);
    return v;
}

// returns hit record (Bvh2 node index / wide triangle index), counts [internal, leaf]
int trace2(const Ray& r, bool any, float& tOut, int* cnt) {
    float inv[3], oxi[3];
    for (int k = 0; k < 3; ++k) { inv[k] = sinv(r.d[k]); oxi[k] = -r.o[k] * inv[k]; }
    float t = r.o[3];
    int hit = -1;
    std::vector<int32_t> st;
    st.reserve(64);
    int32_t node = 0;
    for (;;) {
        const float* n = g_rec2 + 16 * (size_t)node;
        int32_t next = -2;
        if (ci(n, 0) >= 0) {
            ++cnt[0];
            float blo[3] = {n[0], n[2], n[8]}, bhi[3] = {n[1], n[3], n[9]};
            float clo[3] = {n[4], n[6], n[10]}, chi[3] = {n[5], n[7], n[11]};
            float a0, a1, b0, b1;
            slab(blo, bhi, inv, oxi, t, a0, a1);
            slab(clo, chi, inv, oxi, t, b0, b1);
            const bool h0 = a0 <= a1, h1 = b0 <= b1, c1 = h1 && (a0 > b0);
            if (h0 && h1) st.push_back(c1 ? ci(n, 0) : ci(n, 1));
            if (h0 || h1) next = (c1 || !h0) ? ci(n, 1) : ci(n, 0);
        } else {
            ++cnt[1];
            if (r.extra[0] != asInt(n[3])) {
                const float th = triHit(r, n, t);
                if (th < t) {
                    t = th;
                    hit = node;
                    if (any) break;
                }
            }
        }
        if (next == -2) {
            if (st.empty()) break;
            next = st.back();
            st.pop_back();
        }
        node = next;
    }
    tOut = t;
    return hit;
}

int traceW(const Ray& r, bool any, float& tOut, int* cnt) {
    float inv[3], oxi[3];
    for (int k = 0; k < 3; ++k) { inv[k] = sinv(r.d[k]); oxi[k] = -r.o[k] * inv[k]; }
    float t = r.o[3];
    int hit = -1;
    std::vector<uint32_t> st;
    st.reserve(64);
    uint32_t ref = g_wide.rootIsLeaf ? WIDE_LEAF_BIT : 0u;
    for (;;) {
        bool pop = true;
        if (ref & WIDE_LEAF_BIT) {
            ++cnt[1];
            const uint32_t k = ref & ~WIDE_LEAF_BIT;
            const float* tv = &g_wide.tris[16 * (size_t)k];
            // the Bvh2 leaf: its exact box (vertex min / max) and its edge record
            float lo[3], hi[3], t0, t1;
            for (int a = 0; a < 3; ++a) {
                lo[a] = fminf(fminf(tv[a], tv[4 + a]), tv[8 + a]);
                hi[a] = fmaxf(fmaxf(tv[a], tv[4 + a]), tv[8 + a]);
            }
            slab(lo, hi, inv, oxi, t, t0, t1);
            float tr[16] = {tv[0], tv[1], tv[2], tv[3], tv[4] - tv[0], tv[5] - tv[1], tv[6] - tv[2], tv[7],
                            tv[8] - tv[0], tv[9] - tv[1], tv[10] - tv[2], 0.f};
            if (g_leafbox && !(t0 <= t1)) {
                // the reference's own leaf-box test rejects it
            } else if (r.extra[0] != asInt(tr[3])) {
                const float th = triHit(r, tr, t);
                if (th < t) {
                    t = th;
                    hit = (int)k;
                    if (any) break;
                }
            }
        } else {
            ++cnt[0];
            const uint32_t* w = &g_wide.nodes[16 * (size_t)ref];
            float o[3];
            memcpy(o, w, 12);
            const uint32_t meta = w[3];
            const uint32_t valid = (meta >> 24) & 15u, leaf = (meta >> 28) & 15u;
            float tn[WIDE_K];
            uint32_t cr[WIDE_K];
            int m = 0;
            for (int c = 0; c < WIDE_K; ++c) {
                if (!((valid >> c) & 1u)) continue;
                float lo[3], hi[3];
                for (int a = 0; a < 3; ++a) {
                    const uint32_t eb = (meta >> (8 * a)) & 255u;
                    lo[a] = mcrt::wide_plane((w[4 + 2 * a] >> (8 * c)) & 255u, eb, o[a]);
                    hi[a] = mcrt::wide_plane((w[5 + 2 * a] >> (8 * c)) & 255u, eb, o[a]);
                }
                float t0, t1;
                slab(lo, hi, inv, oxi, t, t0, t1);
                if (t0 <= t1) {
                    // insertion by entry distance (stable)
                    int p = m++;
                    while (g_sort == 1 && p > 0 && tn[p - 1] > t0) { tn[p] = tn[p - 1]; cr[p] = cr[p - 1]; --p; }
                    tn[p] = t0;
                    cr[p] = w[10 + c] | (((leaf >> c) & 1u) ? WIDE_LEAF_BIT : 0u);
                }
            }
            if (m > 0 && g_sort == 2) {   // nearest first, the others in stored order
                // (cr/tn hold the hits in stored order: find the nearest)
                int best = 0;
                for (int p = 1; p < m; ++p) if (tn[p] < tn[best]) best = p;
                for (int p = m - 1; p >= 0; --p) if (p != best) st.push_back(cr[p]);
                ref = cr[best];
                pop = false;
            } else if (m > 0) {
                for (int p = m - 1; p >= 1; --p) st.push_back(cr[p]);
                ref = cr[0];
                pop = false;
            }
        }
        if (pop) {
            if (st.empty()) break;
            ref = st.back();
            st.pop_back();
        }
    }
    tOut = t;
    return hit;
}
}  // namespace

extern "C" {
// returns 0 on success; info = [numNodes, numTris, depth]
void ws_set_leafbox(int on) { g_leafbox = on; }
void ws_set_sort(int on) { g_sort = on; }
int ws_build(const float* rec2, size_t n2, const float* tri9, const uint32_t* shapeFirst, size_t nShapes, size_t nTris,
             int64_t* info) {
    g_rec2 = rec2;
    g_n2 = n2;
    std::string err;
    if (!mcrt::build_wide(rec2, n2, tri9, shapeFirst, nShapes, nTris, g_wide, &err)) {
        fprintf(stderr, "build_wide: %s\n", err.c_str());
        return 1;
    }
    info[0] = g_wide.numNodes;
    info[1] = g_wide.numTris;
    info[2] = g_wide.depth;
    return 0;
}
const float* ws_tris() { return g_wide.tris.data(); }
const uint32_t* ws_nodes() { return g_wide.nodes.data(); }
// mode 0: Bvh2, 1: wide.  stats: 2 ints per ray (internal, leaf steps)
void ws_trace(const void* rays, int n, int any, int mode, int32_t* stats, float* tHit, int32_t* hitRec, int threads) {
    const Ray* R = (const Ray*)rays;
    std::vector<std::thread> th;
    for (int w = 0; w < threads; ++w)
        th.emplace_back([=] {
            for (int i = w; i < n; i += threads) {
                int cnt[2] = {0, 0};
                float t = -1.0f;
                int h = -1;
                if (R[i].extra[1] != 0) h = mode ? traceW(R[i], any != 0, t, cnt) : trace2(R[i], any != 0, t, cnt);
                stats[2 * i] = cnt[0];
                stats[2 * i + 1] = cnt[1];
                tHit[i] = t;
                hitRec[i] = h;
            }
        });
    for (auto& x : th) x.join();
}
}

// ---------------------------------------------------------------------------
// Alternative binary tree for the visit-count experiment: binned SAH over all three axes
// (the reference evaluates only the largest centroid extent), 1 triangle per leaf, records in
// the mcrt_bvh.cpp layout (DFS: left = i + 1), leaf records copied from the given Bvh2.
namespace {
struct BPrim { float lo[3], hi[3], c[3]; int leafRec; };
std::vector<float> g_alt;
int g_bins = 32;
void altBuild(std::vector<BPrim>& P, size_t b, size_t e, const float* rec2, std::vector<float>& out, size_t node) {
    // out[node] is ours to fill; returns via recursion
    auto boxOf = [&](size_t i0, size_t i1, float* lo, float* hi) {
        for (int a = 0; a < 3; ++a) { lo[a] = INFINITY; hi[a] = -INFINITY; }
        for (size_t i = i0; i < i1; ++i)
            for (int a = 0; a < 3; ++a) { lo[a] = fminf(lo[a], P[i].lo[a]); hi[a] = fmaxf(hi[a], P[i].hi[a]); }
    };
    float* o = &out[16 * node];
    if (e - b == 1) {
        memcpy(o, rec2 + 16 * (size_t)P[b].leafRec, 64);
        return;
    }
    float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (size_t i = b; i < e; ++i)
        for (int a = 0; a < 3; ++a) { clo[a] = fminf(clo[a], P[i].c[a]); chi[a] = fmaxf(chi[a], P[i].c[a]); }
    int bestA = -1, bestB = 0;
    double bestC = INFINITY;
    const int NB = g_bins;
    std::vector<float> blo(3 * NB), bhi(3 * NB);
    std::vector<int> cnt(NB);
    for (int a = 0; a < 3; ++a) {
        const float ext = chi[a] - clo[a];
        if (!(ext > 0)) continue;
        std::fill(cnt.begin(), cnt.end(), 0);
        for (int k = 0; k < NB; ++k) for (int x = 0; x < 3; ++x) { blo[3 * k + x] = INFINITY; bhi[3 * k + x] = -INFINITY; }
        for (size_t i = b; i < e; ++i) {
            int k = (int)((P[i].c[a] - clo[a]) / ext * NB);
            k = k < 0 ? 0 : k >= NB ? NB - 1 : k;
            ++cnt[k];
            for (int x = 0; x < 3; ++x) { blo[3 * k + x] = fminf(blo[3 * k + x], P[i].lo[x]); bhi[3 * k + x] = fmaxf(bhi[3 * k + x], P[i].hi[x]); }
        }
        std::vector<double> rightC(NB);
        float rl[3] = {INFINITY, INFINITY, INFINITY}, rh[3] = {-INFINITY, -INFINITY, -INFINITY};
        int rc = 0;
        for (int k = NB - 1; k >= 1; --k) {
            rc += cnt[k];
            for (int x = 0; x < 3; ++x) { rl[x] = fminf(rl[x], blo[3 * k + x]); rh[x] = fmaxf(rh[x], bhi[3 * k + x]); }
            const double dx = rh[0] - rl[0], dy = rh[1] - rl[1], dz = rh[2] - rl[2];
            rightC[k] = rc ? rc * (dx * dy + dy * dz + dz * dx) : 0;
        }
        float ll[3] = {INFINITY, INFINITY, INFINITY}, lh[3] = {-INFINITY, -INFINITY, -INFINITY};
        int lc = 0;
        for (int k = 0; k < NB - 1; ++k) {
            lc += cnt[k];
            for (int x = 0; x < 3; ++x) { ll[x] = fminf(ll[x], blo[3 * k + x]); lh[x] = fmaxf(lh[x], bhi[3 * k + x]); }
            if (lc == 0 || lc == (int)(e - b)) continue;
            const double dx = lh[0] - ll[0], dy = lh[1] - ll[1], dz = lh[2] - ll[2];
            const double c = lc * (dx * dy + dy * dz + dz * dx) + rightC[k + 1];
            if (c < bestC) { bestC = c; bestA = a; bestB = k; }
        }
    }
    size_t mid;
    if (bestA < 0) {
        mid = (b + e) / 2;
    } else {
        const float ext = chi[bestA] - clo[bestA];
        auto it = std::partition(P.begin() + b, P.begin() + e, [&](const BPrim& p) {
            int k = (int)((p.c[bestA] - clo[bestA]) / ext * NB);
            k = k < 0 ? 0 : k >= NB ? NB - 1 : k;
            return k <= bestB;
        });
        mid = it - P.begin();
        if (mid == b || mid == e) mid = (b + e) / 2;
    }
    const size_t l = node + 1, r = node + 2 * (mid - b);
    float L[6], R[6];
    boxOf(b, mid, L, L + 3);
    boxOf(mid, e, R, R + 3);
    o[0] = L[0]; o[1] = L[3]; o[2] = L[1]; o[3] = L[4];
    o[4] = R[0]; o[5] = R[3]; o[6] = R[1]; o[7] = R[4];
    o[8] = L[2]; o[9] = L[5]; o[10] = R[2]; o[11] = R[5];
    int32_t ch[4] = {(int32_t)l, (int32_t)r, 0, 0};
    memcpy(o + 12, ch, 16);
    if (e - b > 50000) {
        std::thread t([&] { altBuild(P, b, mid, rec2, out, l); });
        altBuild(P, mid, e, rec2, out, r);
        t.join();
    } else {
        altBuild(P, b, mid, rec2, out, l);
        altBuild(P, mid, e, rec2, out, r);
    }
}
}  // namespace

extern "C" {
// builds the 3-axis SAH tree over the leaves of rec2 and makes it the tree ws_trace mode 0 walks
void ws_build_alt(const float* rec2, size_t n2, int bins) {
    g_bins = bins;
    std::vector<BPrim> P;
    for (size_t i = 0; i < n2; ++i) {
        const float* r = rec2 + 16 * i;
        if (ci(r, 0) >= 0) continue;
        BPrim p;
        p.leafRec = (int)i;
        for (int a = 0; a < 3; ++a) {
            const float v0 = r[a], v1 = r[a] + r[4 + a], v2 = r[a] + r[8 + a];
            p.lo[a] = fminf(fminf(v0, v1), v2);
            p.hi[a] = fmaxf(fmaxf(v0, v1), v2);
            p.c[a] = 0.5f * (p.lo[a] + p.hi[a]);
        }
        P.push_back(p);
    }
    g_alt.assign(16 * (2 * P.size() - 1), 0.0f);
    altBuild(P, 0, P.size(), rec2, g_alt, 0);
    g_rec2 = g_alt.data();
    g_n2 = 2 * P.size() - 1;
}
void ws_use_tree(const float* rec2, size_t n2) { g_rec2 = rec2; g_n2 = n2; }
}
extern "C" {
const float* ws_alt_ptr() { return g_alt.data(); }
size_t ws_alt_n() { return g_alt.size() / 16; }
}

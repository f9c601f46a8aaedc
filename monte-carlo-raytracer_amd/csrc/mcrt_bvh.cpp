// mcrt_bvh.cpp -- host BVH builder of the product (binned SAH, multithreaded) and the
// conversion into the MI355X traversal layout.
//
// Split policy = RadeonRays Bvh2 (RR/src/accelerator/bvh2.cpp:144-712, options from
// RTScene::commit: SAH, 64 bins, traversal cost 10): split axis = largest centroid extent,
// binned SAH on that axis only (> 8 primitives), median fallback, 1 triangle per leaf,
// (axes3 = the perf tree, mcrt_accel_opts.device_build 4: the binned SAH of all three axes,
// cheapest wins -- same records and traversal, a different tree),
// depth-first numbering (left = i + 1, right = i + 2 * nLeft).  The SSE arithmetic of the
// reference (_mm_rcp_ps / _mm_dp_ps) is kept so the tree -- and with it the node-visit
// counts the roofline is priced on -- matches the reference on the same host.
//
// GPU layout (ours): one 64-B record per node of the RR tree, in its DFS numbering, so every
// traversal step is one uniform 64-B fetch whatever the node type:
//   internal: float4 (c0.lo.x, c0.hi.x, c0.lo.y, c0.hi.y)   (child boxes, x/y slab pairs)
//             float4 (c1.lo.x, c1.hi.x, c1.lo.y, c1.hi.y)
//             float4 (c0.lo.z, c0.hi.z, c1.lo.z, c1.hi.z)
//             int4   (child0, child1, 0, 0)                 (child indices >= 1)
//   leaf:     float4 (v0, shapeId bits), float4 (v1 - v0, primId bits), float4 (v2 - v0, 0),
//             int4   (-1, -1, 0, 0); on the device word 13 becomes the parent record's index
//             (k_leaf_parents after every flat build, for the occluder hints)
#include <immintrin.h>

#include <atomic>
#include <cfloat>
#include <cmath>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "mcrt_internal.h"
#include "mcrt_sah.h"

namespace mcrt {
namespace {

struct Req {
    __m128 bmin, bmax, cmin, cmax;
    size_t start, num;
    uint32_t level, index;
};

inline __m128 sa4(__m128 pmin, __m128 pmax) {   // bvh2.cpp:69-75
    __m128 e = _mm_sub_ps(pmax, pmin);
    __m128 xxy = _mm_shuffle_ps(e, e, _MM_SHUFFLE(3, 1, 0, 0));
    __m128 yzz = _mm_shuffle_ps(e, e, _MM_SHUFFLE(3, 2, 2, 1));
    return _mm_mul_ps(_mm_dp_ps(xxy, yzz, 0xff), _mm_set1_ps(2.f));
}
inline uint32_t maxAxis(__m128 pmin, __m128 pmax) {   // bvh2.cpp:83-92
    __m128 xyz = _mm_sub_ps(pmax, pmin);
    __m128 yzx = _mm_shuffle_ps(xyz, xyz, _MM_SHUFFLE(3, 0, 2, 1));
    __m128 m0 = _mm_max_ps(xyz, yzx);
    __m128 m1 = _mm_shuffle_ps(m0, m0, _MM_SHUFFLE(3, 0, 2, 1));
    __m128 m2 = _mm_max_ps(m0, m1);
    return (uint32_t)__builtin_ctz((unsigned)_mm_movemask_ps(_mm_cmpeq_ps(xyz, m2)));
}
inline float lane(__m128 v, uint32_t i) {
    alignas(16) float t[4];
    _mm_store_ps(t, v);
    return t[i];
}

struct Builder {
    const float* tri;
    std::size_t n;
    std::vector<float> amin, amax, acen;   // 4 per primitive
    std::vector<uint32_t> refs;
    // per RR node: kind (0 leaf, 1 internal), own box, children, leaf ref
    std::vector<uint8_t> isInternal;
    std::vector<float> box;               // 6 per node (own box)
    std::vector<uint32_t> leafRef;
    uint32_t bins;
    float cost;
    bool sah;
    bool axes3 = false;   // perf tree: the binned SAH over all three axes (not the reference's tree)
    std::atomic<int> maxDepth{0};

    float sahSplit(const Req& rq, uint32_t axis, float* costOut = nullptr) {   // bvh2.cpp:331-492
        const uint32_t nb = bins;
        std::vector<uint32_t> cnt(nb, 0);
        std::vector<__m128> bmn(nb, _mm_set1_ps(INFINITY)), bmx(nb, _mm_set1_ps(-INFINITY));
        const float cm = lane(rq.cmin, axis);
        const float ce = lane(_mm_sub_ps(rq.cmax, rq.cmin), axis);
        const __m128 cmin4 = _mm_set1_ps(cm), cext4 = _mm_set1_ps(ce);
        const __m128 cinv4 = _mm_rcp_ps(cext4);
        const float areaInv = lane(_mm_rcp_ps(sa4(rq.bmin, rq.bmax)), 0);
        const size_t full4 = rq.num & ~(size_t)3;
        const __m128 nb4 = _mm_set1_ps((float)nb);
        const uint32_t* R = refs.data();
        for (size_t i = rq.start; i < rq.start + full4; i += 4) {
            uint32_t id[4] = {R[i], R[i + 1], R[i + 2], R[i + 3]};
            __m128 c = _mm_set_ps(acen[4 * id[3] + axis], acen[4 * id[2] + axis], acen[4 * id[1] + axis], acen[4 * id[0] + axis]);
            __m128 bi = _mm_mul_ps(_mm_mul_ps(_mm_sub_ps(c, cmin4), cinv4), nb4);
            uint32_t b[4];
            for (int k = 0; k < 4; ++k) b[k] = std::min((uint32_t)lane(bi, k), nb - 1);
            for (int k = 0; k < 4; ++k) ++cnt[b[k]];
            for (int k = 0; k < 4; ++k) {
                bmn[b[k]] = _mm_min_ps(bmn[b[k]], _mm_loadu_ps(&amin[4 * id[k]]));
                bmx[b[k]] = _mm_max_ps(bmx[b[k]], _mm_loadu_ps(&amax[4 * id[k]]));
            }
        }
        const float cei = lane(cinv4, 0);
        for (size_t i = rq.start + full4; i < rq.start + rq.num; ++i) {
            uint32_t id = R[i];
            uint32_t b = std::min((uint32_t)((float)nb * (acen[4 * id + axis] - cm) * cei), nb - 1);
            ++cnt[b];
            bmn[b] = _mm_min_ps(bmn[b], _mm_loadu_ps(&amin[4 * id]));
            bmx[b] = _mm_max_ps(bmx[b], _mm_loadu_ps(&amax[4 * id]));
        }
        std::vector<__m128> rmn(nb - 1), rmx(nb - 1);
        __m128 tmn = _mm_set1_ps(INFINITY), tmx = _mm_set1_ps(-INFINITY);
        for (uint32_t i = nb - 1; i > 0; --i) {
            tmn = _mm_min_ps(tmn, bmn[i]);
            tmx = _mm_max_ps(tmx, bmx[i]);
            rmn[i - 1] = tmn;
            rmx[i - 1] = tmx;
        }
        tmn = _mm_set1_ps(INFINITY);
        tmx = _mm_set1_ps(-INFINITY);
        uint32_t lc = 0;
        size_t rc = rq.num;
        int split = -1;
        float best = FLT_MAX;
        for (uint32_t i = 0; i < nb - 1; ++i) {
            tmn = _mm_min_ps(tmn, bmn[i]);
            tmx = _mm_max_ps(tmx, bmx[i]);
            lc += cnt[i];
            rc -= cnt[i];
            float s = cost + ((float)lc * lane(sa4(tmn, tmx), 0) + (float)rc * lane(sa4(rmn[i], rmx[i]), 0)) * areaInv;
            if (s < best) { split = (int)i; best = s; }
        }
        if (costOut) *costOut = best;
        return cm + (float)(split + 1) * (ce / (float)nb);
    }

    // bvh2.cpp:494-712; returns true for an internal node
    bool handle(const Req& rq, Req& rl, Req& rr) {
        int d = (int)rq.level;
        int prev = maxDepth.load();
        while (d > prev && !maxDepth.compare_exchange_weak(prev, d)) {}
        if (rq.num <= 1) {
            isInternal[rq.index] = 0;
            leafRef[rq.index] = refs[rq.start];
            return false;
        }
        uint32_t ax = maxAxis(rq.cmin, rq.cmax);
        const float ext = lane(_mm_sub_ps(rq.cmax, rq.cmin), ax);
        float split = lane(_mm_mul_ps(_mm_set1_ps(0.5f), _mm_add_ps(rq.cmax, rq.cmin)), ax);
        size_t splitIdx = rq.start;
        const __m128 pinf = _mm_set1_ps(INFINITY), minf = _mm_set1_ps(-INFINITY);
        __m128 lmn = pinf, lmx = minf, rmn = pinf, rmx = minf, lcmn = pinf, lcmx = minf, rcmn = pinf, rcmx = minf;
        uint32_t* R = refs.data();
        auto addL = [&](uint32_t id) {
            lmn = _mm_min_ps(lmn, _mm_loadu_ps(&amin[4 * id]));
            lmx = _mm_max_ps(lmx, _mm_loadu_ps(&amax[4 * id]));
            __m128 c = _mm_loadu_ps(&acen[4 * id]);
            lcmn = _mm_min_ps(lcmn, c);
            lcmx = _mm_max_ps(lcmx, c);
        };
        auto addR = [&](uint32_t id) {
            rmn = _mm_min_ps(rmn, _mm_loadu_ps(&amin[4 * id]));
            rmx = _mm_max_ps(rmx, _mm_loadu_ps(&amax[4 * id]));
            __m128 c = _mm_loadu_ps(&acen[4 * id]);
            rcmn = _mm_min_ps(rcmn, c);
            rcmx = _mm_max_ps(rcmx, c);
        };
        if (ext > 0.0f) {
            if (sah && rq.num > 8) {
                if (axes3) {   // perf tree: the cheapest of the three axes' binned SAH splits
                    float bestCost = FLT_MAX;
                    for (uint32_t a = 0; a < 3; ++a) {
                        if (!(lane(_mm_sub_ps(rq.cmax, rq.cmin), a) > 0.0f)) continue;
                        float c;
                        const float sp = sahSplit(rq, a, &c);
                        if (c < bestCost) { bestCost = c; ax = a; split = sp; }
                    }
                } else {
                    split = sahSplit(rq, ax);
                }
            }
            size_t first = rq.start, last = rq.start + rq.num;
            for (;;) {
                while (first != last && acen[4 * R[first] + ax] < split) { addL(R[first]); ++first; }
                if (first == last--) break;
                addR(R[first]);
                while (first != last && acen[4 * R[last] + ax] >= split) { addR(R[last]); --last; }
                if (first == last) break;
                addL(R[last]);
                std::swap(R[first++], R[last]);
            }
            splitIdx = first;
        }
        if (splitIdx == rq.start || splitIdx == rq.start + rq.num) {
            splitIdx = rq.start + (rq.num >> 1);
            lmn = pinf; lmx = minf; rmn = pinf; rmx = minf; lcmn = pinf; lcmx = minf; rcmn = pinf; rcmx = minf;
            for (size_t i = rq.start; i < splitIdx; ++i) addL(R[i]);
            for (size_t i = splitIdx; i < rq.start + rq.num; ++i) addR(R[i]);
        }
        rl = Req{lmn, lmx, lcmn, lcmx, rq.start, splitIdx - rq.start, rq.level + 1, rq.index + 1};
        rr = Req{rmn, rmx, rcmn, rcmx, splitIdx, rq.num - (splitIdx - rq.start), rq.level + 1,
                 (uint32_t)(rq.index + (splitIdx - rq.start) * 2)};
        isInternal[rq.index] = 1;
        float* bx = &box[6 * (size_t)rq.index];
        bx[0] = lane(rq.bmin, 0); bx[1] = lane(rq.bmin, 1); bx[2] = lane(rq.bmin, 2);
        bx[3] = lane(rq.bmax, 0); bx[4] = lane(rq.bmax, 1); bx[5] = lane(rq.bmax, 2);
        return true;
    }
};

}  // namespace

// The running host's _mm_rcp_ps, tabulated once per process for the device SAH build
// (mcrt_sahbuild.hip): R(m) for x = 1.m over the leading mantissa bits the instruction reads,
// then the device rule (mcrt_sah.h rcp_ps) and the _mm_dp_ps order (sa4) checked against the
// instructions over every exponent and sign.  ok = false -> the device build is refused.
const HostRcp& host_rcp_table() {
    static HostRcp R;
    static std::once_flag once;
    std::call_once(once, []() {
        std::vector<uint32_t> full(1u << 23);
        for (uint32_t m = 0; m < (1u << 23); m += 4) {
            alignas(16) uint32_t in[4] = {(127u << 23) | m, (127u << 23) | (m + 1), (127u << 23) | (m + 2),
                                          (127u << 23) | (m + 3)};
            const __m128 r = _mm_rcp_ps(_mm_castsi128_ps(_mm_load_si128((const __m128i*)in)));
            _mm_storeu_si128((__m128i*)&full[m], _mm_castps_si128(r));
        }
        int bits = 23;
        for (int k = 8; k < 23; ++k) {
            bool same = true;
            const uint32_t low = (1u << (23 - k)) - 1;
            for (uint32_t m = 0; m < (1u << 23) && same; ++m) same = full[m] == full[m & ~low];
            if (same) {
                bits = k;
                break;
            }
        }
        R.bits = bits;
        R.t.resize((size_t)1 << bits);
        for (uint32_t m = 0; m < (1u << bits); ++m) R.t[m] = full[(size_t)m << (23 - bits)];
        bool ok = true;
        uint32_t x = 0x12345u;
        for (uint32_t e = 0; e < 256 && ok; ++e)
            for (int t = 0; t < 512 && ok; ++t) {
                x = x * 1664525u + 1013904223u;
                const uint32_t b = (x & 0x807fffffu) | (e << 23);
                float f;
                std::memcpy(&f, &b, 4);
                const float want = _mm_cvtss_f32(_mm_rcp_ss(_mm_set_ss(f)));
                const float got = sah::rcp_ps(f, R.t.data(), bits);
                if (std::memcmp(&want, &got, 4) != 0 && !(std::isnan(want) && std::isnan(got))) ok = false;
            }
        for (int t = 0; t < 4096 && ok; ++t) {
            alignas(16) float a[4], c[4];
            for (int k = 0; k < 4; ++k) {
                x = x * 1664525u + 1013904223u;
                a[k] = (float)(x >> 8) * 5.9604645e-8f * 2000.0f - 1000.0f;
                x = x * 1664525u + 1013904223u;
                c[k] = (float)(x >> 8) * 5.9604645e-8f * 2000.0f - 1000.0f;
            }
            const float want = lane(sa4(_mm_load_ps(a), _mm_load_ps(c)), 0);
            const float got = sah::sa4(sah::V4{a[0], a[1], a[2], a[3]}, sah::V4{c[0], c[1], c[2], c[3]});
            if (std::memcmp(&want, &got, 4) != 0) ok = false;
        }
        R.ok = ok;
    });
    return R;
}

bool build_bvh(const float* tri, const int32_t* shapeOf, const int32_t* primOf, std::size_t n, float cost, int bins,
               bool sah, int threads, BvhOut& out, bool axes3) {
    if (n == 0) return false;
    Builder b;
    b.axes3 = axes3;
    b.tri = tri;
    b.n = n;
    b.bins = (uint32_t)bins;
    b.cost = cost;
    b.sah = sah;
    b.amin.resize(4 * n);
    b.amax.resize(4 * n);
    b.acen.resize(4 * n);
    b.refs.resize(n);
    const std::size_t count = 2 * n - 1;
    b.isInternal.assign(count, 0);
    b.box.assign(6 * count, 0.0f);
    b.leafRef.assign(count, 0xffffffffu);
    // face bounds (RR/src/primitive/mesh.cpp:130-141) in parallel chunks, scene bounds serially
    if (threads < 1) threads = 1;
    {
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t)
            th.emplace_back([&, t]() {
                for (std::size_t k = (std::size_t)t; k < n; k += (std::size_t)threads) {
                    const float* p = &tri[9 * k];
                    float mn[4], mx[4];
                    for (int c = 0; c < 3; ++c) {
                        float a = p[c], bb = p[3 + c], cc = p[6 + c];
                        float m0 = (bb < a) ? bb : a, x0 = (a < bb) ? bb : a;
                        mn[c] = (cc < m0) ? cc : m0;
                        mx[c] = (x0 < cc) ? cc : x0;
                    }
                    mn[3] = mx[3] = 0.0f;
                    __m128 pmin = _mm_loadu_ps(mn), pmax = _mm_loadu_ps(mx);
                    __m128 cen = _mm_mul_ps(_mm_add_ps(pmin, pmax), _mm_set1_ps(0.5f));
                    _mm_storeu_ps(&b.amin[4 * k], pmin);
                    _mm_storeu_ps(&b.amax[4 * k], pmax);
                    _mm_storeu_ps(&b.acen[4 * k], cen);
                    b.refs[k] = (uint32_t)k;
                }
            });
        for (auto& x : th) x.join();
    }
    __m128 smin = _mm_set1_ps(INFINITY), smax = _mm_set1_ps(-INFINITY), csmin = smin, csmax = smax;
    for (std::size_t k = 0; k < n; ++k) {
        smin = _mm_min_ps(smin, _mm_loadu_ps(&b.amin[4 * k]));
        smax = _mm_max_ps(smax, _mm_loadu_ps(&b.amax[4 * k]));
        __m128 c = _mm_loadu_ps(&b.acen[4 * k]);
        csmin = _mm_min_ps(csmin, c);
        csmax = _mm_max_ps(csmax, c);
    }
    // parallel top-down build (the RR scheme: requests > 4096 refs are shared)
    {
        std::vector<Req> global;
        std::mutex mu;
        std::condition_variable cv;
        std::atomic<std::size_t> done{0};
        bool shutdown = false;
        global.push_back(Req{smin, smax, csmin, csmax, 0, n, 0u, 0u});
        auto worker = [&]() {
            std::vector<Req> local;
            for (;;) {
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&]() { return !global.empty() || shutdown; });
                    if (shutdown && global.empty()) return;
                    local.push_back(global.back());
                    global.pop_back();
                }
                while (!local.empty()) {
                    Req rq = local.back();
                    local.pop_back();
                    Req rl, rr;
                    if (!b.handle(rq, rl, rr)) {
                        if (done.fetch_add(rq.num) + rq.num == n) {
                            std::lock_guard<std::mutex> lk(mu);
                            shutdown = true;
                            cv.notify_all();
                        }
                        continue;
                    }
                    if (rr.num > 4096) {
                        std::lock_guard<std::mutex> lk(mu);
                        global.push_back(rr);
                        cv.notify_one();
                    } else {
                        local.push_back(rr);
                    }
                    local.push_back(rl);
                }
            }
        };
        std::vector<std::thread> th;
        for (int t = 0; t < threads; ++t) th.emplace_back(worker);
        for (auto& x : th) x.join();
    }
    // convert to the GPU layout: one 64-B record per RR node, same DFS numbering
    // (left child = i + 1, right child = i + 1 + size(left)), leaves hold their triangle.
    out.numNodes = count;
    out.numTris = 0;
    for (std::size_t i = 0; i < count; ++i) out.numTris += b.isInternal[i] ? 0 : 1;
    out.nodes = (float*)std::malloc(sizeof(float) * 16 * out.numNodes);
    out.tris = nullptr;
    out.depth = b.maxDepth.load();
    auto leafBox = [&](uint32_t ref, float* bx) {
        const float* p = &tri[9 * (std::size_t)ref];
        for (int c = 0; c < 3; ++c) {
            float a = p[c], bb = p[3 + c], cc = p[6 + c];
            float mn = (cc < bb) ? cc : bb, mx = (bb < cc) ? cc : bb;
            bx[c] = (mn < a) ? mn : a;
            bx[3 + c] = (a < mx) ? mx : a;
        }
    };
    auto childBox = [&](std::size_t c, float* bx) {
        if (b.isInternal[c]) std::memcpy(bx, &b.box[6 * c], sizeof(float) * 6);
        else leafBox(b.leafRef[c], bx);
    };
    // subtree sizes via a reverse scan (size(i) = 1 for leaves, 1 + size(l) + size(r) otherwise)
    std::vector<uint32_t> sz(count, 1);
    for (std::size_t ii = count; ii-- > 0;) {
        if (!b.isInternal[ii]) continue;
        const std::size_t l = ii + 1;
        const std::size_t r = l + sz[l];
        sz[ii] = 1 + sz[l] + sz[r];
    }
    for (std::size_t i = 0; i < count; ++i) {
        float* o = &out.nodes[16 * i];
        if (!b.isInternal[i]) {
            const uint32_t ref = b.leafRef[i];
            const float* p = &tri[9 * (std::size_t)ref];
            o[0] = p[0]; o[1] = p[1]; o[2] = p[2];
            std::memcpy(&o[3], &shapeOf[ref], 4);
            o[4] = p[3] - p[0]; o[5] = p[4] - p[1]; o[6] = p[5] - p[2];
            std::memcpy(&o[7], &primOf[ref], 4);
            o[8] = p[6] - p[0]; o[9] = p[7] - p[1]; o[10] = p[8] - p[2];
            o[11] = 0.0f;
            const int32_t mark[4] = {-1, -1, 0, 0};
            std::memcpy(&o[12], mark, 16);
            continue;
        }
        const std::size_t l = i + 1, r = i + 1 + sz[i + 1];
        float b0[6], b1[6];
        childBox(l, b0);
        childBox(r, b1);
        o[0] = b0[0]; o[1] = b0[3]; o[2] = b0[1]; o[3] = b0[4];
        o[4] = b1[0]; o[5] = b1[3]; o[6] = b1[1]; o[7] = b1[4];
        o[8] = b0[2]; o[9] = b0[5]; o[10] = b1[2]; o[11] = b1[5];
        const int32_t ch[4] = {(int32_t)l, (int32_t)r, 0, 0};
        std::memcpy(&o[12], ch, 16);
    }
    return true;
}

void free_bvh(BvhOut& out) {
    std::free(out.nodes);
    std::free(out.tris);
    out.nodes = nullptr;
    out.tris = nullptr;
}

}  // namespace mcrt

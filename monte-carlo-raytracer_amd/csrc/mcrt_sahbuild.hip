// mcrt_sahbuild.hip -- on-device SAH BVH build for gfx950 that reproduces RadeonRays' Bvh2
// node for node (mcrt_accel_opts.device_build = 2).
//
// RR builds top-down on the host (RR/src/accelerator/bvh2.cpp:144-712, restated in mcrt_bvh.cpp):
// per request, split axis = largest centroid extent; > 8 references: 64-bin SAH on that axis,
// else the centroid midpoint; references partitioned in place by a two-pointer (Hoare) loop; a
// one-sided partition falls back to the median of the current order; 1 reference per leaf;
// depth-first numbering (left = i + 1, right = i + 2 * size(left)).  Here:
//
//   * the split arithmetic is mcrt_sah.h (the SSE sequence restated; _mm_rcp_ps tabulated on
//     the running host), so every split plane is the reference's;
//   * the Hoare loop is replaced by its closed form: with nL = #{c < split}, the k-th reference
//     that sits left of nL but belongs right swaps with the k-th reference, counted from the
//     end, that sits right of nL but belongs left.  Ranks come from prefix counts, so the
//     partition runs in parallel and leaves the references in exactly the reference's order
//     (which the median fallback and the 4-wide/1-wide bin formulas depend on);
//   * bin and child bounds are min/max reductions (order-free; only the sign of a zero bound
//     can differ from the sequential order, which no slab test distinguishes).
//
// Schedule: requests with more than SMALL references are processed level by level over the
// whole GPU (CHUNK references per workgroup: bin, count, scan, slot, swap passes with global
// atomics per request); each request of <= SMALL references is finished by ONE wave that loads
// its references' boxes into LDS and walks its subtree (smaller child first, so the stack stays
// O(log SMALL)), with wave ballots for the prefix counts and a lane-parallel SAH sweep.
// Output: the mcrt_bvh.cpp record layout, same numbering, so it is byte-identical to the host
// build (tests/test_gpu_build.py compares them).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "mcrt_internal.h"
#include "mcrt_sah.h"

namespace {
using namespace mcrt::sah;

constexpr int MAXB = 64;      // bins supported on the device path
#ifndef SAH_SMALL
#define SAH_SMALL 256
#endif
constexpr int SMALL = SAH_SMALL;   // requests up to this many references finish in one wave (LDS)
constexpr int CHUNK = 4096;   // references per workgroup in the level passes
constexpr int LT = 256;       // threads per level-pass workgroup
constexpr int PER = CHUNK / LT;
constexpr int MAX_LEVELS = 4096;

struct Seg {   // one request (bvh2.cpp SplitRequest)
    V4 bmin, bmax, cmin, cmax;
    uint32_t start, num, index, level;
    uint32_t chunk0, pad[3];   // its first chunk in the level's chunk list (contiguous, in order)
};
struct SegState {
    uint32_t axis, sahNode, mode, nL;   // mode 0: partition at `split`; 1: median of the current order
    float split, cm, cinv, areaInv, ce;
    uint32_t chunk0, nchunks, pad;
    int bins[MAXB * 7];   // count, min xyz, max xyz (ordered ints)
    int child[24];        // lmn, lmx, lcmn, lcmx, rmn, rmx, rcmn, rcmx (xyz, ordered ints)
};
struct Chunk {
    uint32_t seg, begin, end, pad;   // positions relative to the request's start
};
struct Counters {
    uint32_t segs, chunks, small, depth, error, pad[3];
};

__device__ __forceinline__ int oi(float f) {   // monotonic float -> int
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float of(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }
__device__ __forceinline__ float axisOf(const float4& v, uint32_t a) { return a == 0 ? v.x : a == 1 ? v.y : v.z; }
__device__ __forceinline__ V4 v4(float4 f) { return V4{f.x, f.y, f.z, f.w}; }

struct Params {
    const float4* cen;
    const float4* amin;
    const float4* amax;
    const float* tri;
    const int* shapeOf;
    const int* primOf;
    uint32_t* refs;
    uint32_t* slots;
    float4* nodes;
    const uint32_t* rcpTable;
    int rcpBits;
    uint32_t nb;
    float nbf;
    float cost;
    int sahOn;
    Counters* ctr;
};

// leaf record (mcrt_bvh.cpp): v0 | shape, v1 - v0 | prim, v2 - v0 | 0, (-1, -1, 0, 0)
__device__ void writeLeaf(const Params& P, uint32_t node, uint32_t ref) {
    const float* p = &P.tri[9 * (size_t)ref];
    float4* o = &P.nodes[4 * (size_t)node];
    o[0] = make_float4(p[0], p[1], p[2], __int_as_float(P.shapeOf[ref]));
    o[1] = make_float4(p[3] - p[0], p[4] - p[1], p[5] - p[2], __int_as_float(P.primOf[ref]));
    o[2] = make_float4(p[6] - p[0], p[7] - p[1], p[8] - p[2], 0.0f);
    o[3] = make_float4(__int_as_float(-1), __int_as_float(-1), 0.0f, 0.0f);
}
// internal record: child boxes (x/y slab pairs, then z) + child indices
__device__ void writeInternal(const Params& P, uint32_t node, const float* b0, const float* b1, uint32_t l, uint32_t r) {
    float4* o = &P.nodes[4 * (size_t)node];
    o[0] = make_float4(b0[0], b0[3], b0[1], b0[4]);
    o[1] = make_float4(b1[0], b1[3], b1[1], b1[4]);
    o[2] = make_float4(b0[2], b0[5], b1[2], b1[5]);
    o[3] = make_float4(__int_as_float((int)l), __int_as_float((int)r), 0.0f, 0.0f);
}
__device__ void childBox(const Params& P, uint32_t num, uint32_t ref, V4 mn, V4 mx, float* bx) {
    if (num == 1) {
        leafBox(&P.tri[9 * (size_t)ref], bx);
    } else {
        bx[0] = mn.x; bx[1] = mn.y; bx[2] = mn.z;
        bx[3] = mx.x; bx[4] = mx.y; bx[5] = mx.z;
    }
}

// child bounds of one reference into side L (b[0..11]) or R (b[12..23]): box min, box max,
// centroid min, centroid max (xyz each); selects keep the register array statically indexed
__device__ __forceinline__ void addSide(float* b, bool L, float4 mn, float4 mx, float4 c) {
    const float v[12] = {mn.x, mn.y, mn.z, mx.x, mx.y, mx.z, c.x, c.y, c.z, c.x, c.y, c.z};
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const bool isMax = (k / 3) & 1;
        const float l = isMax ? fmaxf(b[k], v[k]) : fminf(b[k], v[k]);
        const float r = isMax ? fmaxf(b[12 + k], v[k]) : fminf(b[12 + k], v[k]);
        b[k] = L ? l : b[k];
        b[12 + k] = L ? b[12 + k] : r;
    }
}

// ---------------------------------------------------------------------------
// whole-scene bounds -> root request
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bounds(int n, const float4* __restrict__ amin, const float4* __restrict__ amax,
                                                const float4* __restrict__ cen, int* __restrict__ out) {
    int v[12];
    for (int a = 0; a < 3; ++a) {
        v[a] = v[6 + a] = 0x7fffffff;
        v[3 + a] = v[9 + a] = (int)0x80000000;
    }
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const float4 mn = amin[i], mx = amax[i], c = cen[i];
        const float m[3] = {mn.x, mn.y, mn.z}, M[3] = {mx.x, mx.y, mx.z}, C[3] = {c.x, c.y, c.z};
        for (int a = 0; a < 3; ++a) {
            v[a] = min(v[a], oi(m[a]));
            v[3 + a] = max(v[3 + a], oi(M[a]));
            v[6 + a] = min(v[6 + a], oi(C[a]));
            v[9 + a] = max(v[9 + a], oi(C[a]));
        }
    }
    __shared__ int red[12];
    if (threadIdx.x < 12) red[threadIdx.x] = ((threadIdx.x % 6) >= 3) ? (int)0x80000000 : 0x7fffffff;
    __syncthreads();
    for (int k = 0; k < 12; ++k) {
        const bool isMax = (k % 6) >= 3;
        for (int off = 32; off > 0; off >>= 1) {
            const int o = __shfl_xor(v[k], off);
            v[k] = isMax ? max(v[k], o) : min(v[k], o);
        }
        if ((threadIdx.x & 63) == 0) {
            if (isMax) atomicMax(&red[k], v[k]);
            else atomicMin(&red[k], v[k]);
        }
    }
    __syncthreads();
    if (threadIdx.x < 12) {
        if ((threadIdx.x % 6) >= 3) atomicMax(&out[threadIdx.x], red[threadIdx.x]);
        else atomicMin(&out[threadIdx.x], red[threadIdx.x]);
    }
}

__global__ void k_root(int n, const int* __restrict__ b, Seg* __restrict__ big, Chunk* __restrict__ chunks,
                       uint4* __restrict__ small, Counters* __restrict__ ctr) {
    Seg s;
    s.bmin = V4{of(b[0]), of(b[1]), of(b[2]), 0.0f};
    s.bmax = V4{of(b[3]), of(b[4]), of(b[5]), 0.0f};
    s.cmin = V4{of(b[6]), of(b[7]), of(b[8]), 0.0f};
    s.cmax = V4{of(b[9]), of(b[10]), of(b[11]), 0.0f};
    s.start = 0;
    s.num = (uint32_t)n;
    s.index = 0;
    s.level = 0;
    s.chunk0 = 0;
    if (n == 1) {   // a single triangle: the root is a leaf (k_single_leaf)
        ctr->segs = ctr->chunks = ctr->small = 0;
    } else if (n > SMALL) {
        big[0] = s;
        const uint32_t nc = ((uint32_t)n + CHUNK - 1) / CHUNK;
        for (uint32_t c = 0; c < nc; ++c) chunks[c] = Chunk{0, c * CHUNK, min((c + 1) * CHUNK, (uint32_t)n), 0};
        ctr->segs = 1;
        ctr->chunks = nc;
        ctr->small = 0;
    } else {
        small[0] = make_uint4(0, (uint32_t)n, 0, 0);
        ctr->segs = 0;
        ctr->chunks = 0;
        ctr->small = 1;
    }
    ctr->depth = 0;
}

__global__ void k_single_leaf(Params P) { writeLeaf(P, 0, 0); }

__global__ __launch_bounds__(256) void k_iota(int n, uint32_t* __restrict__ refs) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) refs[i] = (uint32_t)i;
}

// ---------------------------------------------------------------------------
// level passes over the large requests
// ---------------------------------------------------------------------------
// K0: split axis, midpoint, SAH constants (bvh2.cpp:339-348, 505-520); clear bins and bounds
__global__ __launch_bounds__(64) void k_prepare(Params P, const Seg* __restrict__ segs, SegState* __restrict__ st) {
    const Seg g = segs[blockIdx.x];
    SegState& S = st[blockIdx.x];
    for (uint32_t k = threadIdx.x; k < P.nb; k += 64) {
        S.bins[7 * k] = 0;
        for (int a = 0; a < 3; ++a) {
            S.bins[7 * k + 1 + a] = 0x7fffffff;
            S.bins[7 * k + 4 + a] = (int)0x80000000;
        }
    }
    if (threadIdx.x < 24) S.child[threadIdx.x] = ((threadIdx.x / 3) & 1) ? (int)0x80000000 : 0x7fffffff;
    if (threadIdx.x != 0) return;
    const uint32_t ax = maxAxis(g.cmin, g.cmax);
    const float ext = lane(vsub(g.cmax, g.cmin), ax);
    S.axis = ax;
    S.split = 0.5f * (lane(g.cmax, ax) + lane(g.cmin, ax));
    S.mode = ext > 0.0f ? 0u : 1u;
    S.sahNode = (ext > 0.0f && P.sahOn && g.num > 8) ? 1u : 0u;
    S.cm = lane(g.cmin, ax);
    S.ce = ext;
    S.cinv = rcp_ps(ext, P.rcpTable, P.rcpBits);
    S.areaInv = rcp_ps(sa4(g.bmin, g.bmax), P.rcpTable, P.rcpBits);
    S.nL = 0;
    S.chunk0 = g.chunk0;
    S.nchunks = ((g.num + CHUNK - 1) / CHUNK);
}

// K1: SAH bins (bvh2.cpp:357-394), per-wave LDS bins merged into the request's bins
__global__ __launch_bounds__(LT) void k_bin(Params P, const Seg* __restrict__ segs, SegState* __restrict__ st,
                                            const Chunk* __restrict__ chunks) {
    const Chunk ch = chunks[blockIdx.x];
    SegState& S = st[ch.seg];
    if (!S.sahNode) return;
    const Seg g = segs[ch.seg];
    __shared__ int wb[LT / 64][MAXB * 7];
    const int w = threadIdx.x >> 6;
    for (int k = threadIdx.x & 63; k < MAXB; k += 64) {
        wb[w][7 * k] = 0;
        for (int a = 0; a < 3; ++a) {
            wb[w][7 * k + 1 + a] = 0x7fffffff;
            wb[w][7 * k + 4 + a] = (int)0x80000000;
        }
    }
    __syncthreads();
    const uint32_t full4 = g.num & ~3u;
    const uint32_t ax = S.axis;
    const float cm = S.cm, cinv = S.cinv;
    for (uint32_t j = ch.begin + threadIdx.x; j < ch.end; j += LT) {
        const uint32_t id = P.refs[g.start + j];
        const float c = axisOf(P.cen[id], ax);
        const uint32_t b = j < full4 ? binFull(c, cm, cinv, P.nbf, P.nb) : binTail(c, cm, cinv, P.nbf, P.nb);
        const float4 mn = P.amin[id], mx = P.amax[id];
        int* B = &wb[w][7 * b];
        atomicAdd(&B[0], 1);
        atomicMin(&B[1], oi(mn.x));
        atomicMin(&B[2], oi(mn.y));
        atomicMin(&B[3], oi(mn.z));
        atomicMax(&B[4], oi(mx.x));
        atomicMax(&B[5], oi(mx.y));
        atomicMax(&B[6], oi(mx.z));
    }
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < P.nb; k += LT) {
        int c = 0, v[6];
        for (int a = 0; a < 3; ++a) {
            v[a] = 0x7fffffff;
            v[3 + a] = (int)0x80000000;
        }
        for (int q = 0; q < LT / 64; ++q) {
            c += wb[q][7 * k];
            for (int a = 0; a < 3; ++a) {
                v[a] = min(v[a], wb[q][7 * k + 1 + a]);
                v[3 + a] = max(v[3 + a], wb[q][7 * k + 4 + a]);
            }
        }
        if (c == 0) continue;
        atomicAdd(&S.bins[7 * k], c);
        for (int a = 0; a < 3; ++a) {
            atomicMin(&S.bins[7 * k + 1 + a], v[a]);
            atomicMax(&S.bins[7 * k + 4 + a], v[3 + a]);
        }
    }
}

// bins (ordered ints) -> V4 lanes as the reference holds them (empty bin: +inf / -inf in all
// four lanes; otherwise w = 0, the references' w)
__device__ __forceinline__ void binLanes(const int* B, uint32_t& cnt, V4& mn, V4& mx) {
    cnt = (uint32_t)B[0];
    if (cnt == 0) {
        mn = V4{INFINITY, INFINITY, INFINITY, INFINITY};
        mx = V4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    } else {
        mn = V4{of(B[1]), of(B[2]), of(B[3]), 0.0f};
        mx = V4{of(B[4]), of(B[5]), of(B[6]), 0.0f};
    }
}

// K2: SAH sweep per large request (one thread each)
__global__ __launch_bounds__(64) void k_sweep(Params P, const Seg* __restrict__ segs, SegState* __restrict__ st, uint32_t numSegs) {
    const uint32_t s = blockIdx.x * 64 + threadIdx.x;
    if (s >= numSegs) return;
    SegState& S = st[s];
    if (!S.sahNode) return;
    uint32_t cnt[MAXB];
    V4 bmn[MAXB], bmx[MAXB], rmn[MAXB], rmx[MAXB];
    for (uint32_t k = 0; k < P.nb; ++k) binLanes(&S.bins[7 * k], cnt[k], bmn[k], bmx[k]);
    S.split = sweep(cnt, bmn, bmx, rmn, rmx, P.nb, segs[s].num, P.cost, S.areaInv, S.cm, S.ce);
}

// block-wide exclusive scan of one value per thread (LT threads)
__device__ __forceinline__ uint32_t blockScan(uint32_t v, uint32_t* sh, uint32_t& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t y = __shfl_up(x, off);
        if (lane >= off) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    uint32_t base = 0;
    total = 0;
    for (int q = 0; q < LT / 64; ++q) {
        if (q < w) base += sh[q];
        total += sh[q];
    }
    __syncthreads();
    return base + x - v;
}

// K3: left count per chunk + child bounds by side (bvh2.cpp:522-560 addLeft/addRight)
__global__ __launch_bounds__(LT) void k_count(Params P, const Seg* __restrict__ segs, SegState* __restrict__ st,
                                              const Chunk* __restrict__ chunks, uint32_t* __restrict__ chunkL) {
    const Chunk ch = chunks[blockIdx.x];
    SegState& S = st[ch.seg];
    if (S.mode != 0) return;
    const Seg g = segs[ch.seg];
    const uint32_t ax = S.axis;
    const float split = S.split;
    float b[24];
    for (int k = 0; k < 24; ++k) b[k] = ((k / 3) & 1) ? -INFINITY : INFINITY;
    uint32_t cnt = 0;
    for (uint32_t j = ch.begin + threadIdx.x; j < ch.end; j += LT) {
        const uint32_t id = P.refs[g.start + j];
        const float4 c = P.cen[id], mn = P.amin[id], mx = P.amax[id];
        const bool L = axisOf(c, ax) < split;
        cnt += L ? 1u : 0u;
        addSide(b, L, mn, mx, c);
    }
    __shared__ int red[24];
    __shared__ uint32_t tot;
    if (threadIdx.x < 24) red[threadIdx.x] = ((threadIdx.x / 3) & 1) ? (int)0x80000000 : 0x7fffffff;
    if (threadIdx.x == 0) tot = 0;
    __syncthreads();
    for (int k = 0; k < 24; ++k) {
        int v = oi(b[k]);
        const bool isMax = (k / 3) & 1;
        for (int off = 32; off > 0; off >>= 1) {
            const int o = __shfl_xor(v, off);
            v = isMax ? max(v, o) : min(v, o);
        }
        if ((threadIdx.x & 63) == 0) {
            if (isMax) atomicMax(&red[k], v);
            else atomicMin(&red[k], v);
        }
    }
    atomicAdd(&tot, cnt);
    __syncthreads();
    if (threadIdx.x < 24) {
        if ((threadIdx.x / 3) & 1) atomicMax(&S.child[threadIdx.x], red[threadIdx.x]);
        else atomicMin(&S.child[threadIdx.x], red[threadIdx.x]);
    }
    if (threadIdx.x == 0) chunkL[blockIdx.x] = tot;
}

// K4: per request, exclusive scan of its chunks' left counts; one-sided -> median fallback
__global__ __launch_bounds__(64) void k_scan(const Seg* __restrict__ segs, SegState* __restrict__ st,
                                             const uint32_t* __restrict__ chunkL, uint32_t* __restrict__ chunkLb) {
    SegState& S = st[blockIdx.x];
    const Seg g = segs[blockIdx.x];
    __shared__ uint32_t mode;
    if (threadIdx.x == 0) {
        uint32_t run = 0;
        if (S.mode == 0)
            for (uint32_t c = 0; c < S.nchunks; ++c) {
                chunkLb[S.chunk0 + c] = run;
                run += chunkL[S.chunk0 + c];
            }
        S.nL = run;
        if (S.mode == 0 && (run == 0 || run == g.num)) S.mode = 1;
        mode = S.mode;
    }
    __syncthreads();
    if (mode == 1 && threadIdx.x < 24) S.child[threadIdx.x] = ((threadIdx.x / 3) & 1) ? (int)0x80000000 : 0x7fffffff;
}

// prefix counts of the left flag over a chunk: thread t owns PER consecutive positions
__device__ __forceinline__ void chunkFlags(const Params& P, const Seg& g, const SegState& S, uint32_t begin,
                                           uint32_t end, uint32_t limit, uint32_t& mask, uint32_t& before,
                                           uint32_t* sh) {
    const uint32_t j0 = begin + threadIdx.x * PER;
    mask = 0;
    for (int k = 0; k < PER; ++k) {
        const uint32_t j = j0 + k;
        if (j < end && j < limit) {
            const uint32_t id = P.refs[g.start + j];
            if (axisOf(P.cen[id], S.axis) < S.split) mask |= 1u << k;
        }
    }
    uint32_t total;
    before = blockScan(__popc(mask), sh, total);
}

// K5: slots of the misplaced left references (right of nL), numbered from the end
__global__ __launch_bounds__(LT) void k_slots(Params P, const Seg* __restrict__ segs, const SegState* __restrict__ st,
                                              const Chunk* __restrict__ chunks, const uint32_t* __restrict__ chunkLb) {
    const Chunk ch = chunks[blockIdx.x];
    const SegState& S = st[ch.seg];
    if (S.mode != 0 || ch.end <= S.nL) return;
    const Seg g = segs[ch.seg];
    __shared__ uint32_t sh[LT / 64];
    uint32_t mask, before;
    chunkFlags(P, g, S, ch.begin, ch.end, ch.end, mask, before, sh);
    uint32_t Lb = chunkLb[blockIdx.x] + before;
    const uint32_t j0 = ch.begin + threadIdx.x * PER;
    for (int k = 0; k < PER; ++k) {
        const uint32_t j = j0 + k;
        if (mask >> k & 1u) {
            if (j >= S.nL) P.slots[g.start + (S.nL - Lb - 1)] = j;
            ++Lb;
        }
    }
}

// K6: each misplaced right reference (left of nL) swaps with its slot partner
__global__ __launch_bounds__(LT) void k_swap(Params P, const Seg* __restrict__ segs, const SegState* __restrict__ st,
                                             const Chunk* __restrict__ chunks, const uint32_t* __restrict__ chunkLb) {
    const Chunk ch = chunks[blockIdx.x];
    const SegState& S = st[ch.seg];
    if (S.mode != 0 || ch.begin >= S.nL) return;
    const Seg g = segs[ch.seg];
    __shared__ uint32_t sh[LT / 64];
    uint32_t mask, before;
    // positions >= nL may already hold swapped-in references from other chunks: not read
    chunkFlags(P, g, S, ch.begin, ch.end, S.nL, mask, before, sh);
    uint32_t Lb = chunkLb[blockIdx.x] + before;
    const uint32_t j0 = ch.begin + threadIdx.x * PER;
    uint32_t* R = P.refs + g.start;
    for (int k = 0; k < PER; ++k) {
        const uint32_t j = j0 + k;
        if (j >= ch.end || j >= S.nL) break;
        if (mask >> k & 1u) {
            ++Lb;
        } else {
            const uint32_t q = P.slots[g.start + (j - Lb)];
            const uint32_t a = R[j];
            R[j] = R[q];
            R[q] = a;
        }
    }
}

// K7: median fallback (bvh2.cpp:562-585): child bounds over the two halves of the current order
__global__ __launch_bounds__(LT) void k_median(Params P, const Seg* __restrict__ segs, SegState* __restrict__ st,
                                               const Chunk* __restrict__ chunks) {
    const Chunk ch = chunks[blockIdx.x];
    SegState& S = st[ch.seg];
    if (S.mode != 1) return;
    const Seg g = segs[ch.seg];
    const uint32_t half = g.num >> 1;
    float b[24];
    for (int k = 0; k < 24; ++k) b[k] = ((k / 3) & 1) ? -INFINITY : INFINITY;
    for (uint32_t j = ch.begin + threadIdx.x; j < ch.end; j += LT) {
        const uint32_t id = P.refs[g.start + j];
        const float4 c = P.cen[id], mn = P.amin[id], mx = P.amax[id];
        addSide(b, j < half, mn, mx, c);
    }
    for (int k = 0; k < 24; ++k) {
        int v = oi(b[k]);
        const bool isMax = (k / 3) & 1;
        for (int off = 32; off > 0; off >>= 1) {
            const int o = __shfl_xor(v, off);
            v = isMax ? max(v, o) : min(v, o);
        }
        if ((threadIdx.x & 63) == 0) {
            if (isMax) atomicMax(&S.child[k], v);
            else atomicMin(&S.child[k], v);
        }
    }
}

// K8: the request's record, leaf records of single-reference children, next requests
__global__ __launch_bounds__(64) void k_emit(Params P, const Seg* __restrict__ segs, const SegState* __restrict__ st,
                                             uint32_t numSegs, Seg* __restrict__ next, Chunk* __restrict__ nextChunks,
                                             uint4* __restrict__ small, uint32_t capSegs, uint32_t capChunks,
                                             uint32_t capSmall) {
    const uint32_t s = blockIdx.x * 64 + threadIdx.x;
    if (s >= numSegs) return;
    const Seg g = segs[s];
    const SegState& S = st[s];
    const uint32_t nl = S.mode == 0 ? S.nL : (g.num >> 1);
    const uint32_t nr = g.num - nl;
    const int* c = S.child;
    const V4 lmn{of(c[0]), of(c[1]), of(c[2]), 0.0f}, lmx{of(c[3]), of(c[4]), of(c[5]), 0.0f};
    const V4 lcmn{of(c[6]), of(c[7]), of(c[8]), 0.0f}, lcmx{of(c[9]), of(c[10]), of(c[11]), 0.0f};
    const V4 rmn{of(c[12]), of(c[13]), of(c[14]), 0.0f}, rmx{of(c[15]), of(c[16]), of(c[17]), 0.0f};
    const V4 rcmn{of(c[18]), of(c[19]), of(c[20]), 0.0f}, rcmx{of(c[21]), of(c[22]), of(c[23]), 0.0f};
    const uint32_t li = g.index + 1, ri = g.index + nl * 2;
    const uint32_t lref = P.refs[g.start], rref = P.refs[g.start + nl];
    float b0[6], b1[6];
    childBox(P, nl, lref, lmn, lmx, b0);
    childBox(P, nr, rref, rmn, rmx, b1);
    writeInternal(P, g.index, b0, b1, li, ri);
    atomicMax(&P.ctr->depth, g.level + 1);
    const uint32_t cs[2] = {g.start, g.start + nl}, cn[2] = {nl, nr}, ci[2] = {li, ri}, cr[2] = {lref, rref};
    const V4 cb[2][4] = {{lmn, lmx, lcmn, lcmx}, {rmn, rmx, rcmn, rcmx}};
    for (int k = 0; k < 2; ++k) {
        if (cn[k] == 1) {
            writeLeaf(P, ci[k], cr[k]);
        } else if (cn[k] > (uint32_t)SMALL) {
            const uint32_t slot = atomicAdd(&P.ctr->segs, 1u);
            const uint32_t nc = (cn[k] + CHUNK - 1) / CHUNK;
            const uint32_t c0 = atomicAdd(&P.ctr->chunks, nc);
            if (slot >= capSegs || c0 + nc > capChunks) {
                atomicOr(&P.ctr->error, 1u);
                continue;
            }
            next[slot] = Seg{cb[k][0], cb[k][1], cb[k][2], cb[k][3], cs[k], cn[k], ci[k], g.level + 1, c0, {0, 0, 0}};
            for (uint32_t q = 0; q < nc; ++q)
                nextChunks[c0 + q] = Chunk{slot, q * CHUNK, min((q + 1) * CHUNK, cn[k]), 0};
        } else {
            const uint32_t slot = atomicAdd(&P.ctr->small, 1u);
            if (slot >= capSmall) {
                atomicOr(&P.ctr->error, 2u);
                continue;
            }
            small[slot] = make_uint4(cs[k], cn[k], ci[k], g.level + 1);
        }
    }
}

// ---------------------------------------------------------------------------
// one wave finishes a request of <= SMALL references in LDS
// ---------------------------------------------------------------------------
struct SNode {
    V4 bmin, bmax, cmin, cmax;
    uint32_t s0, num, index, level;
};

__device__ __forceinline__ float wmin(float v) {
    for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off));
    return v;
}
__device__ __forceinline__ float wmax(float v) {
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off));
    return v;
}

// one lane builds a whole subtree of <= LANE_T references (no SAH below 9, bvh2.cpp:509): the
// reference's own two-pointer loop on its slice of perm, serially
constexpr uint32_t LANE_T = 8;
__device__ __forceinline__ void laneSubtree(const Params& P, const SNode& root, float (*C)[SMALL], float (*MN)[SMALL],
                                            float (*MX)[SMALL], const uint32_t* gid, uint16_t* perm,
                                            uint32_t& maxLevel) {
    SNode st[4];
    int sp = 0;
    st[sp++] = root;
    while (sp > 0) {
        const SNode nd = st[--sp];
        const uint32_t ax = maxAxis(nd.cmin, nd.cmax);
        const float ext = lane(vsub(nd.cmax, nd.cmin), ax);
        const float split = 0.5f * (lane(nd.cmax, ax) + lane(nd.cmin, ax));
        const float* CA = C[ax > 2 ? 0 : ax];
        const uint32_t s0 = nd.s0, num = nd.num;
        uint32_t nl = 0;
        bool median = !(ext > 0.0f);
        if (!median) {
            uint32_t first = s0, last = s0 + num;
            for (;;) {
                while (first != last && CA[perm[first]] < split) ++first;
                if (first == last--) break;
                while (first != last && CA[perm[last]] >= split) --last;
                if (first == last) break;
                const uint16_t t = perm[first];
                perm[first] = perm[last];
                perm[last] = t;
                ++first;
            }
            nl = first - s0;
            median = nl == 0 || nl == num;
        }
        if (median) nl = num >> 1;
        const uint32_t nr = num - nl;
        float b[24];
        for (int k = 0; k < 24; ++k) b[k] = ((k / 3) & 1) ? -INFINITY : INFINITY;
        for (uint32_t j = 0; j < num; ++j) {
            const uint32_t e = perm[s0 + j];
            addSide(b, j < nl, make_float4(MN[0][e], MN[1][e], MN[2][e], 0.0f),
                    make_float4(MX[0][e], MX[1][e], MX[2][e], 0.0f), make_float4(C[0][e], C[1][e], C[2][e], 0.0f));
        }
        const V4 lmn{b[0], b[1], b[2], 0.0f}, lmx{b[3], b[4], b[5], 0.0f}, lcmn{b[6], b[7], b[8], 0.0f},
            lcmx{b[9], b[10], b[11], 0.0f};
        const V4 rmn{b[12], b[13], b[14], 0.0f}, rmx{b[15], b[16], b[17], 0.0f}, rcmn{b[18], b[19], b[20], 0.0f},
            rcmx{b[21], b[22], b[23], 0.0f};
        const uint32_t li = nd.index + 1, ri = nd.index + nl * 2;
        const uint32_t lref = gid[perm[s0]], rref = gid[perm[s0 + nl]];
        float b0[6], b1[6];
        childBox(P, nl, lref, lmn, lmx, b0);
        childBox(P, nr, rref, rmn, rmx, b1);
        writeInternal(P, nd.index, b0, b1, li, ri);
        if (nl == 1) writeLeaf(P, li, lref);
        if (nr == 1) writeLeaf(P, ri, rref);
        maxLevel = max(maxLevel, nd.level + 1);
        const SNode L{lmn, lmx, lcmn, lcmx, s0, nl, li, nd.level + 1};
        const SNode R{rmn, rmx, rcmn, rcmx, s0 + nl, nr, ri, nd.level + 1};
        const bool leftFirst = nl >= nr;
        if ((leftFirst ? L : R).num > 1) st[sp++] = leftFirst ? L : R;
        if ((leftFirst ? R : L).num > 1) st[sp++] = leftFirst ? R : L;
    }
}

__global__ __launch_bounds__(64) void k_small(Params P, const uint4* __restrict__ list) {
    __shared__ float C[3][SMALL], MN[3][SMALL], MX[3][SMALL];
    __shared__ uint32_t gid[SMALL];
    __shared__ uint16_t perm[SMALL];
    __shared__ uint8_t flag[SMALL];
    __shared__ uint16_t slot[SMALL / 2];
    __shared__ int bins[MAXB * 7];
    __shared__ SNode stack[24];
    __shared__ SNode laneList[64];
    const int ln = threadIdx.x;
    const uint4 item = list[blockIdx.x];
    const uint32_t start = item.x, num0 = item.y;
    // load the references' boxes; root bounds by reduction
    float r[12];
    for (int k = 0; k < 12; ++k) r[k] = ((k / 3) & 1) ? -INFINITY : INFINITY;
    for (uint32_t e = ln; e < num0; e += 64) {
        const uint32_t id = P.refs[start + e];
        const float4 c = P.cen[id], mn = P.amin[id], mx = P.amax[id];
        gid[e] = id;
        perm[e] = (uint16_t)e;
        C[0][e] = c.x; C[1][e] = c.y; C[2][e] = c.z;
        MN[0][e] = mn.x; MN[1][e] = mn.y; MN[2][e] = mn.z;
        MX[0][e] = mx.x; MX[1][e] = mx.y; MX[2][e] = mx.z;
        const float v[12] = {mn.x, mn.y, mn.z, mx.x, mx.y, mx.z, c.x, c.y, c.z, c.x, c.y, c.z};
        for (int k = 0; k < 12; ++k) r[k] = ((k / 3) & 1) ? fmaxf(r[k], v[k]) : fminf(r[k], v[k]);
    }
    for (int k = 0; k < 12; ++k) r[k] = ((k / 3) & 1) ? wmax(r[k]) : wmin(r[k]);
    // nodes of > LANE_T references: the whole wave, one at a time (stack, wave-uniform sp);
    // subtrees of <= LANE_T: collected in laneList and built one per lane
    int sp = 0, nLane = 0;
    const SNode root{V4{r[0], r[1], r[2], 0.0f}, V4{r[3], r[4], r[5], 0.0f}, V4{r[6], r[7], r[8], 0.0f},
                     V4{r[9], r[10], r[11], 0.0f}, 0u, num0, item.z, item.w};
    if (ln == 0) {
        if (num0 <= LANE_T) laneList[0] = root;
        else stack[0] = root;
    }
    if (num0 <= LANE_T) nLane = 1;
    else sp = 1;
    __syncthreads();
    uint32_t maxLevel = item.w;
    while (sp > 0 || nLane > 0) {
        if (sp == 0 || nLane >= 63) {
            if (ln < nLane) laneSubtree(P, laneList[ln], C, MN, MX, gid, perm, maxLevel);
            nLane = 0;
            __syncthreads();
            continue;
        }
        const SNode nd = stack[--sp];
        __syncthreads();
        const uint32_t s0 = nd.s0, num = nd.num;
        const uint32_t ax = maxAxis(nd.cmin, nd.cmax);
        const float ext = lane(vsub(nd.cmax, nd.cmin), ax);
        float split = 0.5f * (lane(nd.cmax, ax) + lane(nd.cmin, ax));
        const float* CA = C[ax > 2 ? 0 : ax];
        bool median = !(ext > 0.0f);
        uint32_t nL = 0;
        if (!median) {
            if (P.sahOn && num > 8) {
                const float cm = lane(nd.cmin, ax);
                const float cinv = rcp_ps(ext, P.rcpTable, P.rcpBits);
                const float areaInv = rcp_ps(sa4(nd.bmin, nd.bmax), P.rcpTable, P.rcpBits);
                for (uint32_t k = ln; k < P.nb; k += 64) {
                    bins[7 * k] = 0;
                    for (int a = 0; a < 3; ++a) {
                        bins[7 * k + 1 + a] = 0x7fffffff;
                        bins[7 * k + 4 + a] = (int)0x80000000;
                    }
                }
                __syncthreads();
                const uint32_t full4 = num & ~3u;
                for (uint32_t j = ln; j < num; j += 64) {
                    const uint32_t e = perm[s0 + j];
                    const float c = CA[e];
                    const uint32_t b = j < full4 ? binFull(c, cm, cinv, P.nbf, P.nb) : binTail(c, cm, cinv, P.nbf, P.nb);
                    int* B = &bins[7 * b];
                    atomicAdd(&B[0], 1);
                    atomicMin(&B[1], oi(MN[0][e]));
                    atomicMin(&B[2], oi(MN[1][e]));
                    atomicMin(&B[3], oi(MN[2][e]));
                    atomicMax(&B[4], oi(MX[0][e]));
                    atomicMax(&B[5], oi(MX[1][e]));
                    atomicMax(&B[6], oi(MX[2][e]));
                }
                __syncthreads();
                // ln-parallel sweep (bvh2.cpp:396-491): ln i prices the split after bin i; the
                // prefix / suffix min-max scans are exact, the first minimum wins (strict <)
                uint32_t cnt;
                V4 bmn, bmx;
                const uint32_t nb = P.nb;
                if ((uint32_t)ln < nb) binLanes(&bins[7 * ln], cnt, bmn, bmx);
                else { cnt = 0; bmn = V4{INFINITY, INFINITY, INFINITY, INFINITY}; bmx = V4{-INFINITY, -INFINITY, -INFINITY, -INFINITY}; }
                // inclusive prefix over bins 0..i (left side) and inclusive suffix over bins i+1..nb-1
                float pv[8] = {bmn.x, bmn.y, bmn.z, bmn.w, bmx.x, bmx.y, bmx.z, bmx.w};
                uint32_t pc = cnt;
                for (int off = 1; off < 64; off <<= 1) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const float o = __shfl_up(pv[q], off);
                        if (ln >= off) pv[q] = q < 4 ? fmin_ps(o, pv[q]) : fmax_ps(o, pv[q]);
                    }
                    const uint32_t oc = __shfl_up(pc, off);
                    if (ln >= off) pc += oc;
                }
                const V4 pmn{pv[0], pv[1], pv[2], pv[3]}, pmx{pv[4], pv[5], pv[6], pv[7]};
                // suffix: bins i+1.. -> shift by one then scan downwards
                V4 smn = V4{INFINITY, INFINITY, INFINITY, INFINITY}, smx = V4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
                {
                    float sv[8];
                    const float bv[8] = {bmn.x, bmn.y, bmn.z, bmn.w, bmx.x, bmx.y, bmx.z, bmx.w};
                    for (int q = 0; q < 8; ++q) {
                        const float o = __shfl_down(bv[q], 1);
                        sv[q] = (ln + 1 < 64) ? o : (q < 4 ? INFINITY : -INFINITY);
                    }
                    for (int off = 1; off < 64; off <<= 1)
#pragma unroll
                        for (int q = 0; q < 8; ++q) {
                            const float o = __shfl_down(sv[q], off);
                            if (ln + off < 64) sv[q] = q < 4 ? fmin_ps(sv[q], o) : fmax_ps(sv[q], o);
                        }
                    smn = V4{sv[0], sv[1], sv[2], sv[3]};
                    smx = V4{sv[4], sv[5], sv[6], sv[7]};
                }
                float s = INFINITY;
                bool valid = (uint32_t)ln < nb - 1;
                if (valid) {
                    const uint32_t lc = pc;
                    const uint64_t rc = (uint64_t)num - lc;
                    const float a = (float)lc * sa4(pmn, pmx);
                    const float b = (float)rc * sa4(smn, smx);
                    s = P.cost + (a + b) * areaInv;
                }
                // first i with s < running best: best starts at FLT_MAX, NaN never wins
                const bool cand = valid && (s < 3.402823466e+38f);
                // argmin with the lowest index among equal minima (sequential strict <)
                float bs = cand ? s : INFINITY;
                int bi = cand ? ln : 64;
                for (int off = 32; off > 0; off >>= 1) {
                    const float os = __shfl_xor(bs, off);
                    const int ob = __shfl_xor(bi, off);
                    if (os < bs || (os == bs && ob < bi)) {
                        bs = os;
                        bi = ob;
                    }
                }
                const int sidx = bi < 64 ? bi : -1;
                const float step = (float)((double)ext / (double)P.nbf);
                split = cm + (float)(sidx + 1) * step;
            }
            // left flags and count
            for (uint32_t j0 = 0; j0 < num; j0 += 64) {
                const uint32_t j = j0 + ln;
                bool L = false;
                if (j < num) {
                    L = CA[perm[s0 + j]] < split;
                    flag[j] = L ? 1 : 0;
                }
                nL += __popcll(__ballot(L));
            }
            median = (nL == 0 || nL == num);
            __syncthreads();
            if (!median) {
                const uint64_t lt = (ln == 0) ? 0ull : (~0ull >> (64 - ln));
                uint32_t run = 0;
                for (uint32_t j0 = 0; j0 < num; j0 += 64) {   // slots of misplaced lefts
                    const uint32_t j = j0 + ln;
                    const bool L = j < num && flag[j];
                    const uint64_t m = __ballot(L);
                    const uint32_t Lb = run + __popcll(m & lt);
                    if (L && j >= nL) slot[nL - Lb - 1] = (uint16_t)j;
                    run += __popcll(m);
                }
                __syncthreads();
                run = 0;
                for (uint32_t j0 = 0; j0 < nL; j0 += 64) {   // misplaced rights swap
                    const uint32_t j = j0 + ln;
                    const bool in = j < nL;
                    const bool L = in && flag[j];
                    const uint64_t m = __ballot(L);
                    const uint32_t Lb = run + __popcll(m & lt);
                    if (in && !L) {
                        const uint32_t q = slot[j - Lb];
                        const uint16_t a = perm[s0 + j];
                        perm[s0 + j] = perm[s0 + q];
                        perm[s0 + q] = a;
                    }
                    run += __popcll(m);
                }
                __syncthreads();
            }
        }
        const uint32_t nl = median ? (num >> 1) : nL;
        const uint32_t nr = num - nl;
        // child bounds by side
        float b[24];
        for (int k = 0; k < 24; ++k) b[k] = ((k / 3) & 1) ? -INFINITY : INFINITY;
        for (uint32_t j = ln; j < num; j += 64) {
            const uint32_t e = perm[s0 + j];
            addSide(b, j < nl, make_float4(MN[0][e], MN[1][e], MN[2][e], 0.0f),
                    make_float4(MX[0][e], MX[1][e], MX[2][e], 0.0f), make_float4(C[0][e], C[1][e], C[2][e], 0.0f));
        }
        for (int k = 0; k < 24; ++k) b[k] = ((k / 3) & 1) ? wmax(b[k]) : wmin(b[k]);
        const V4 lmn{b[0], b[1], b[2], 0.0f}, lmx{b[3], b[4], b[5], 0.0f}, lcmn{b[6], b[7], b[8], 0.0f},
            lcmx{b[9], b[10], b[11], 0.0f};
        const V4 rmn{b[12], b[13], b[14], 0.0f}, rmx{b[15], b[16], b[17], 0.0f}, rcmn{b[18], b[19], b[20], 0.0f},
            rcmx{b[21], b[22], b[23], 0.0f};
        const uint32_t li = nd.index + 1, ri = nd.index + nl * 2;
        const uint32_t lref = gid[perm[s0]], rref = gid[perm[s0 + nl]];
        if (ln == 0) {
            float b0[6], b1[6];
            childBox(P, nl, lref, lmn, lmx, b0);
            childBox(P, nr, rref, rmn, rmx, b1);
            writeInternal(P, nd.index, b0, b1, li, ri);
            if (nl == 1) writeLeaf(P, li, lref);
            if (nr == 1) writeLeaf(P, ri, rref);
        }
        maxLevel = max(maxLevel, nd.level + 1);
        // larger child first, so the smaller is processed next (stack depth O(log SMALL))
        const SNode L{lmn, lmx, lcmn, lcmx, s0, nl, li, nd.level + 1};
        const SNode R{rmn, rmx, rcmn, rcmx, s0 + nl, nr, ri, nd.level + 1};
        const bool leftFirst = nl >= nr;
        const SNode& A = leftFirst ? L : R;
        const SNode& B2 = leftFirst ? R : L;
        if (sp + 2 > 24) {   // not reached: depth O(log SMALL) with the smaller child first
            if (ln == 0) atomicOr(&P.ctr->error, 4u);
            return;
        }
        for (const SNode* c : {&A, &B2}) {
            if (c->num <= 1) continue;
            if (c->num <= LANE_T) {
                if (ln == 0) laneList[nLane] = *c;
                ++nLane;
            } else {
                if (ln == 0) stack[sp] = *c;
                ++sp;
            }
        }
        __syncthreads();
    }
    for (int off = 32; off > 0; off >>= 1) maxLevel = max(maxLevel, (uint32_t)__shfl_xor((int)maxLevel, off));
    if (ln == 0) atomicMax(&P.ctr->depth, maxLevel);
}

}  // namespace

namespace mcrt {

hipError_t gpu_build_sah(const mcrt_shape* dShapes, const std::vector<uint32_t>& shapeFirst, const uint32_t* dIndices,
                         const float4* dPositions, size_t n, float cost, int bins, bool sah, hipStream_t st,
                         float4** nodesOut, int* depthOut, const char** why) {
    *why = nullptr;
    if (bins < 2 || bins > MAXB) {
        *why = "device SAH build supports 2..64 bins";
        return hipErrorInvalidValue;
    }
    if (n == 0 || n > 0x7fffffffull) {
        *why = "bad triangle count";
        return hipErrorInvalidValue;
    }
    const HostRcp& R = host_rcp_table();
    if (!R.ok) {
        *why = "host _mm_rcp_ps / _mm_dp_ps not reproducible on the device";
        return hipErrorNotSupported;
    }
    const size_t numNodes = 2 * n - 1;
    const uint32_t capSegs = (uint32_t)(2 * (n / SMALL) + 4);
    const uint32_t capChunks = (uint32_t)(n / CHUNK + capSegs + 4);
    const uint32_t capSmall = (uint32_t)(n / 2 + 2);
    // prims (tri, shape/prim ids, boxes, centroids) as the LBVH path computes them
    float* tri = nullptr;
    int *shapeOf = nullptr, *primOf = nullptr, *cb = nullptr;
    float4 *amin = nullptr, *amax = nullptr, *cen = nullptr, *nodes = nullptr;
    uint32_t *refs = nullptr, *slots = nullptr, *chunkL = nullptr, *chunkLb = nullptr, *rtab = nullptr,
             *dShapeFirst = nullptr;
    Seg *segA = nullptr, *segB = nullptr;
    SegState* state = nullptr;
    Chunk *chA = nullptr, *chB = nullptr;
    uint4* small = nullptr;
    Counters* ctr = nullptr;
    hipError_t e = hipSuccess;
    auto A = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, bytes > 0 ? bytes : 4);
    };
    A((void**)&tri, sizeof(float) * 9 * n);
    A((void**)&shapeOf, sizeof(int) * n);
    A((void**)&primOf, sizeof(int) * n);
    A((void**)&amin, sizeof(float4) * n);
    A((void**)&amax, sizeof(float4) * n);
    A((void**)&cen, sizeof(float4) * n);
    A((void**)&cb, sizeof(int) * 16);
    A((void**)&nodes, sizeof(float4) * 4 * numNodes);
    A((void**)&refs, sizeof(uint32_t) * n);
    A((void**)&slots, sizeof(uint32_t) * n);
    A((void**)&chunkL, sizeof(uint32_t) * capChunks);
    A((void**)&chunkLb, sizeof(uint32_t) * capChunks);
    A((void**)&rtab, sizeof(uint32_t) * R.t.size());
    A((void**)&dShapeFirst, sizeof(uint32_t) * shapeFirst.size());
    A((void**)&segA, sizeof(Seg) * capSegs);
    A((void**)&segB, sizeof(Seg) * capSegs);
    A((void**)&state, sizeof(SegState) * capSegs);
    A((void**)&chA, sizeof(Chunk) * capChunks);
    A((void**)&chB, sizeof(Chunk) * capChunks);
    A((void**)&small, sizeof(uint4) * capSmall);
    A((void**)&ctr, sizeof(Counters));
    if (e == hipSuccess) e = hipMemcpyAsync(rtab, R.t.data(), sizeof(uint32_t) * R.t.size(), hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
        e = hipMemcpyAsync(dShapeFirst, shapeFirst.data(), sizeof(uint32_t) * shapeFirst.size(), hipMemcpyHostToDevice, st);
    int depth = 0;
    if (e == hipSuccess) {
        const int g = (int)((n + 255) / 256);
        e = launch_build_prims((int)n, dShapes, dShapeFirst, (int)shapeFirst.size(), dIndices, dPositions, tri, shapeOf,
                               primOf, amin, amax, cen, cb, st);
        const int init[16] = {0x7fffffff, 0x7fffffff, 0x7fffffff, (int)0x80000000, (int)0x80000000, (int)0x80000000,
                              0x7fffffff, 0x7fffffff, 0x7fffffff, (int)0x80000000, (int)0x80000000, (int)0x80000000};
        if (e == hipSuccess) e = hipMemcpyAsync(cb, init, sizeof(init), hipMemcpyHostToDevice, st);
        Params P{cen, amin, amax, tri, shapeOf, primOf, refs, slots, nodes, rtab, R.bits, (uint32_t)bins,
                 (float)bins, cost, sah ? 1 : 0, ctr};
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_bounds, dim3(std::min(g, 2048)), dim3(256), 0, st, (int)n, amin, amax, cen, cb);
            hipLaunchKernelGGL(k_iota, dim3(g), dim3(256), 0, st, (int)n, refs);
            e = hipMemsetAsync(ctr, 0, sizeof(Counters), st);
        }
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_root, dim3(1), dim3(1), 0, st, (int)n, cb, segA, chA, small, ctr);
            e = hipGetLastError();
        }
        Counters hc{};
        if (e == hipSuccess) e = hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        uint32_t numSegs = hc.segs, numChunks = hc.chunks;
        int levels = 0;
        while (e == hipSuccess && numSegs > 0) {
            if (++levels > MAX_LEVELS) {
                *why = "device SAH build: too many levels of large requests";
                e = hipErrorNotSupported;
                break;
            }
            const dim3 S(numSegs), Cg(numChunks), S64((numSegs + 63) / 64);
            hipLaunchKernelGGL(k_prepare, S, dim3(64), 0, st, P, segA, state);
            hipLaunchKernelGGL(k_bin, Cg, dim3(LT), 0, st, P, segA, state, chA);
            hipLaunchKernelGGL(k_sweep, S64, dim3(64), 0, st, P, segA, state, numSegs);
            hipLaunchKernelGGL(k_count, Cg, dim3(LT), 0, st, P, segA, state, chA, chunkL);
            hipLaunchKernelGGL(k_scan, S, dim3(64), 0, st, segA, state, chunkL, chunkLb);
            hipLaunchKernelGGL(k_slots, Cg, dim3(LT), 0, st, P, segA, state, chA, chunkLb);
            hipLaunchKernelGGL(k_swap, Cg, dim3(LT), 0, st, P, segA, state, chA, chunkLb);
            hipLaunchKernelGGL(k_median, Cg, dim3(LT), 0, st, P, segA, state, chA);
            e = hipMemsetAsync(ctr, 0, 2 * sizeof(uint32_t), st);   // next level's segs, chunks
            if (e != hipSuccess) break;
            hipLaunchKernelGGL(k_emit, S64, dim3(64), 0, st, P, segA, state, numSegs, segB, chB, small, capSegs,
                               capChunks, capSmall);
            if ((e = hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, st)) != hipSuccess) break;
            if ((e = hipStreamSynchronize(st)) != hipSuccess) break;
            if (hc.error) {
                *why = "device SAH build: capacity exceeded";
                e = hipErrorNotSupported;
                break;
            }
            numSegs = hc.segs;
            numChunks = hc.chunks;
            std::swap(segA, segB);
            std::swap(chA, chB);
        }
        if (e == hipSuccess && hc.small > 0) {
            hipLaunchKernelGGL(k_small, dim3(hc.small), dim3(64), 0, st, P, small);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpyAsync(&hc, ctr, sizeof(Counters), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e == hipSuccess && hc.error) {
            *why = "device SAH build: stack or capacity exceeded";
            e = hipErrorNotSupported;
        }
        if (e == hipSuccess && n == 1) {   // a single triangle: the root is a leaf
            hipLaunchKernelGGL(k_single_leaf, dim3(1), dim3(1), 0, st, P);
            e = hipStreamSynchronize(st);
        }
        depth = (int)hc.depth;
    }
    for (void* p : {(void*)tri, (void*)shapeOf, (void*)primOf, (void*)amin, (void*)amax, (void*)cen, (void*)cb,
                    (void*)refs, (void*)slots, (void*)chunkL, (void*)chunkLb, (void*)rtab,
                    (void*)dShapeFirst, (void*)segA, (void*)segB, (void*)state, (void*)chA, (void*)chB, (void*)small,
                    (void*)ctr})
        if (p) (void)hipFree(p);
    if (e != hipSuccess) {
        if (nodes) (void)hipFree(nodes);
        if (!*why) *why = hipGetErrorString(e);
        return e;
    }
    *nodesOut = nodes;
    *depthOut = depth;
    return hipSuccess;
}

}  // namespace mcrt

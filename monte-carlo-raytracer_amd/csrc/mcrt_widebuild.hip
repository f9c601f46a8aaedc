// mcrt_widebuild.hip -- on-device build of the 4-wide quantized tree (mcrt_wide.h) from the
// Bvh2 records already on the device, level by level:
//   k_wide_count  one thread per wide node of the level: collapse its Bvh2 node (open the child
//                 of largest area until four children), count internal and triangle children;
//   scan          rocPRIM inclusive scan of the packed (internal << 32 | triangle) counts;
//   k_wide_emit   the same collapse again, quantize (mcrt_wide.h helpers, the host's own
//                 predicates), write the node record, the next level's Bvh2 nodes and the
//                 triangle records (world vertices recomputed with the Bvh2 build's arithmetic
//                 and checked against the leaf record's v0 and edges).
// The numbering equals the host restatement's (mcrt_wide.cpp): nodes breadth first, a node's
// internal children consecutive, triangle records in the order their parents are numbered.
// Compiled with -ffp-contract=off (wide_area must round like the host's).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include <rocprim/device/device_scan.hpp>

#include "mcrt_internal.h"
#include "mcrt_wide.h"

namespace {

struct Kids {
    int n;
    int32_t node[WIDE_K];
    float lo[WIDE_K][3], hi[WIDE_K][3];
};

__device__ __forceinline__ bool recLeaf(const int4* rec, int32_t k) { return rec[4 * (size_t)k + 3].x < 0; }

__device__ __forceinline__ void recChild(const float4* rec, int32_t b, int c, float* lo, float* hi) {
    const float4 q = rec[4 * (size_t)b + c], z = rec[4 * (size_t)b + 2];
    lo[0] = q.x; hi[0] = q.y; lo[1] = q.z; hi[1] = q.w;
    lo[2] = c ? z.z : z.x; hi[2] = c ? z.w : z.y;
}

// mcrt_wide.cpp build_wide: the collapse of Bvh2 node b; false on a malformed record
__device__ bool collapse(const float4* rec, uint32_t n2, int32_t b, Kids& k) {
    const int4* r4 = reinterpret_cast<const int4*>(rec);
    const int4 ch = r4[4 * (size_t)b + 3];
    if (ch.x <= 0 || ch.y <= 0 || (uint32_t)ch.x >= n2 || (uint32_t)ch.y >= n2) return false;
    k.n = 2;
    k.node[0] = ch.x;
    k.node[1] = ch.y;
    recChild(rec, b, 0, k.lo[0], k.hi[0]);
    recChild(rec, b, 1, k.lo[1], k.hi[1]);
    while (k.n < WIDE_K) {
        int best = -1;
        float bestA = 0.0f;
        for (int c = 0; c < k.n; ++c) {
            if (recLeaf(r4, k.node[c])) continue;
            const float a = mcrt::wide_area(k.lo[c], k.hi[c]);
            if (best < 0 || a > bestA) { bestA = a; best = c; }
        }
        if (best < 0) break;
        const int32_t nb = k.node[best];
        const int4 cc = r4[4 * (size_t)nb + 3];
        if (cc.x <= 0 || cc.y <= 0 || (uint32_t)cc.x >= n2 || (uint32_t)cc.y >= n2) return false;
        for (int c = k.n; c > best + 1; --c) {
            k.node[c] = k.node[c - 1];
            for (int a = 0; a < 3; ++a) { k.lo[c][a] = k.lo[c - 1][a]; k.hi[c][a] = k.hi[c - 1][a]; }
        }
        k.node[best] = cc.x;
        k.node[best + 1] = cc.y;
        recChild(rec, nb, 0, k.lo[best], k.hi[best]);
        recChild(rec, nb, 1, k.lo[best + 1], k.hi[best + 1]);
        ++k.n;
    }
    return true;
}

__global__ __launch_bounds__(256) void k_wide_count(const float4* __restrict__ rec, uint32_t n2,
                                                    const int32_t* __restrict__ level, uint32_t count,
                                                    unsigned long long* __restrict__ counts, int* __restrict__ bad) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    Kids k;
    uint32_t ni = 0, nl = 0;
    if (!collapse(rec, n2, level[i], k)) {
        *bad = 1;
    } else {
        const int4* r4 = reinterpret_cast<const int4*>(rec);
        for (int c = 0; c < k.n; ++c) {
            if (recLeaf(r4, k.node[c])) ++nl; else ++ni;
        }
    }
    counts[i] = ((unsigned long long)ni << 32) | nl;
}

// RR transform_point with separately rounded operations (mcrt_gpubuild.hip xrow, mcrt_capi.cpp
// xformPoint): the world vertices the Bvh2 build saw
__device__ __forceinline__ float xrowW(const mcrt_float4& r, float x, float y, float z) {
    float acc = 0.0f;
    acc = __fadd_rn(acc, __fmul_rn(r.x, x));
    acc = __fadd_rn(acc, __fmul_rn(r.y, y));
    acc = __fadd_rn(acc, __fmul_rn(r.z, z));
    acc = __fadd_rn(acc, __fmul_rn(r.w, 0.0f));
    return __fadd_rn(acc, r.w);
}

__global__ __launch_bounds__(256) void k_wide_emit(const float4* __restrict__ rec, uint32_t n2,
                                                   const int32_t* __restrict__ level, uint32_t count,
                                                   uint32_t levelBase, uint32_t triBase,
                                                   const unsigned long long* __restrict__ counts,
                                                   const unsigned long long* __restrict__ incl,
                                                   uint4* __restrict__ nodes, float4* __restrict__ tris,
                                                   int32_t* __restrict__ nextLevel, const mcrt_shape* __restrict__ shapes,
                                                   uint32_t numShapes, const uint32_t* __restrict__ indices,
                                                   const float4* __restrict__ positions, int* __restrict__ bad) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= count) return;
    Kids k;
    if (!collapse(rec, n2, level[i], k)) {
        *bad = 1;
        return;
    }
    const unsigned long long ex = incl[i] - counts[i];
    uint32_t nextInt = (uint32_t)(ex >> 32), nextTri = (uint32_t)(ex & 0xffffffffull);
    const uint32_t nodeBase = levelBase + count;   // first node index of the next level
    const int4* r4 = reinterpret_cast<const int4*>(rec);
    uint32_t w[16];
    for (int q = 0; q < 16; ++q) w[q] = 0u;
    float o[3];
    uint32_t eb[3];
    for (int a = 0; a < 3; ++a) {
        float lo = k.lo[0][a], hi = k.hi[0][a];
        for (int c = 1; c < k.n; ++c) { lo = fminf(lo, k.lo[c][a]); hi = fmaxf(hi, k.hi[c][a]); }
        if (!isfinite(lo) || !isfinite(hi)) { *bad = 2; return; }
        o[a] = lo;
        eb[a] = mcrt::wide_axis_exponent(lo, hi);
        if (eb[a] == 0) { *bad = 2; return; }
        w[a] = __float_as_uint(lo);
    }
    uint32_t valid = 0, leafMask = 0;
    for (int c = 0; c < k.n; ++c) {
        valid |= 1u << c;
        for (int a = 0; a < 3; ++a) {
            const uint32_t ql = mcrt::wide_quant_lo(k.lo[c][a], eb[a], o[a]);
            const uint32_t qh = mcrt::wide_quant_hi(k.hi[c][a], eb[a], o[a]);
            if (mcrt::wide_plane(ql, eb[a], o[a]) > k.lo[c][a] || mcrt::wide_plane(qh, eb[a], o[a]) < k.hi[c][a]) {
                *bad = 3;
                return;
            }
            w[4 + 2 * a] |= ql << (8 * c);
            w[5 + 2 * a] |= qh << (8 * c);
        }
        const int32_t kn = k.node[c];
        if (recLeaf(r4, kn)) {
            leafMask |= 1u << c;
            const uint32_t t = triBase + nextTri++;
            w[10 + c] = t;
            const float4 A = rec[4 * (size_t)kn], E1 = rec[4 * (size_t)kn + 1], E2 = rec[4 * (size_t)kn + 2];
            const int shape = __float_as_int(A.w), prim = __float_as_int(E1.w);
            if (shape < 0 || (uint32_t)shape >= numShapes || prim < 0 || (uint32_t)prim >= shapes[shape].numTriangles) {
                *bad = 4;
                return;
            }
            const mcrt_shape& sh = shapes[shape];
            float p[9];
            for (int v = 0; v < 3; ++v) {
                const float4 x = positions[sh.startVertex + indices[sh.startIdx + 3 * (uint32_t)prim + v]];
                p[3 * v + 0] = xrowW(sh.toWorldTransform.m0, x.x, x.y, x.z);
                p[3 * v + 1] = xrowW(sh.toWorldTransform.m1, x.x, x.y, x.z);
                p[3 * v + 2] = xrowW(sh.toWorldTransform.m2, x.x, x.y, x.z);
            }
            const float r0[3] = {A.x, A.y, A.z}, r1[3] = {E1.x, E1.y, E1.z}, r2[3] = {E2.x, E2.y, E2.z};
            for (int a = 0; a < 3; ++a)
                if (__float_as_uint(p[a]) != __float_as_uint(r0[a]) ||
                    __float_as_uint(__fsub_rn(p[3 + a], p[a])) != __float_as_uint(r1[a]) ||
                    __float_as_uint(__fsub_rn(p[6 + a], p[a])) != __float_as_uint(r2[a])) {
                    *bad = 5;
                    return;
                }
            float4* tr = tris + 4 * (size_t)t;
            tr[0] = make_float4(p[0], p[1], p[2], A.w);
            tr[1] = make_float4(p[3], p[4], p[5], E1.w);
            tr[2] = make_float4(p[6], p[7], p[8], 0.0f);
            tr[3] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        } else {
            w[10 + c] = nodeBase + nextInt;
            nextLevel[nextInt] = kn;
            ++nextInt;
        }
    }
    w[3] = eb[0] | (eb[1] << 8) | (eb[2] << 16) | ((valid | (leafMask << 4)) << 24);
    uint4* dst = nodes + 4 * (size_t)(levelBase + i);
    for (int q = 0; q < 4; ++q) dst[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// a one-triangle scene: the root record is the triangle
__global__ void k_wide_single(const float4* __restrict__ rec, float4* __restrict__ tris,
                              const mcrt_shape* __restrict__ shapes, const uint32_t* __restrict__ indices,
                              const float4* __restrict__ positions, int* __restrict__ bad) {
    const float4 A = rec[0], E1 = rec[1];
    const int shape = __float_as_int(A.w), prim = __float_as_int(E1.w);
    const mcrt_shape& sh = shapes[shape];
    float p[9];
    for (int v = 0; v < 3; ++v) {
        const float4 x = positions[sh.startVertex + indices[sh.startIdx + 3 * (uint32_t)prim + v]];
        p[3 * v + 0] = xrowW(sh.toWorldTransform.m0, x.x, x.y, x.z);
        p[3 * v + 1] = xrowW(sh.toWorldTransform.m1, x.x, x.y, x.z);
        p[3 * v + 2] = xrowW(sh.toWorldTransform.m2, x.x, x.y, x.z);
    }
    if (__float_as_uint(p[0]) != __float_as_uint(A.x) || __float_as_uint(p[1]) != __float_as_uint(A.y) ||
        __float_as_uint(p[2]) != __float_as_uint(A.z))
        *bad = 5;
    tris[0] = make_float4(p[0], p[1], p[2], A.w);
    tris[1] = make_float4(p[3], p[4], p[5], E1.w);
    tris[2] = make_float4(p[6], p[7], p[8], 0.0f);
    tris[3] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
}

}  // namespace

namespace mcrt {

hipError_t gpu_build_wide(const float4* dRec, size_t n2, const mcrt_shape* dShapes, uint32_t numShapes,
                          const uint32_t* dIndices, const float4* dPositions, hipStream_t st, WideDevice& out,
                          const char** why) {
    out = WideDevice();
    *why = nullptr;
    if (n2 == 0 || n2 >= (size_t)WIDE_LEAF_BIT) { *why = "tree size"; return hipErrorInvalidValue; }
    const size_t leaves = (n2 + 1) / 2, internal = n2 - leaves;
    hipError_t e = hipSuccess;
    int* dBad = nullptr;
    auto A = [&](auto** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc((void**)p, bytes);
    };
    A(&dBad, sizeof(int));
    A(&out.tris, 64 * leaves);
    if (e == hipSuccess) e = hipMemsetAsync(dBad, 0, sizeof(int), st);
    int32_t root0;
    if (e == hipSuccess) {
        int4 r3;
        e = hipMemcpy(&r3, reinterpret_cast<const int4*>(dRec) + 3, sizeof(int4), hipMemcpyDeviceToHost);
        root0 = r3.x;
    }
    if (e == hipSuccess && root0 < 0) {   // one triangle
        hipLaunchKernelGGL(k_wide_single, dim3(1), dim3(1), 0, st, dRec, out.tris, dShapes, dIndices, dPositions, dBad);
        int bad = 0;
        e = hipMemcpyAsync(&bad, dBad, sizeof(int), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        hipFree(dBad);
        if (e == hipSuccess && bad) { *why = "leaf record does not match its triangle"; e = hipErrorInvalidValue; }
        if (e != hipSuccess) { hipFree(out.tris); out = WideDevice(); return e; }
        out.numTris = 1;
        out.depth = 1;
        out.rootIsLeaf = true;
        return hipSuccess;
    }
    uint4* nodes = nullptr;
    int32_t *levA = nullptr, *levB = nullptr;
    unsigned long long *counts = nullptr, *incl = nullptr;
    void* tmp = nullptr;
    size_t tmpBytes = 0;
    A(&nodes, 64 * std::max<size_t>(internal, 1));
    A(&levA, 4 * std::max<size_t>(internal, 1));
    A(&levB, 4 * std::max<size_t>(internal, 1));
    A(&counts, 8 * std::max<size_t>(internal, 1));
    A(&incl, 8 * std::max<size_t>(internal, 1));
    if (e == hipSuccess)
        e = rocprim::inclusive_scan(nullptr, tmpBytes, counts, incl, std::max<size_t>(internal, 1),
                                    rocprim::plus<unsigned long long>(), st);
    A(&tmp, std::max<size_t>(tmpBytes, 1));
    const int32_t zero = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(levA, &zero, 4, hipMemcpyHostToDevice, st);
    uint32_t levelBase = 0, count = 1, triBase = 0, numNodes = 1;
    int depth = 0;
    while (e == hipSuccess && count > 0) {
        ++depth;
        const dim3 g((count + 255) / 256), b(256);
        hipLaunchKernelGGL(k_wide_count, g, b, 0, st, dRec, (uint32_t)n2, levA, count, counts, dBad);
        e = rocprim::inclusive_scan(tmp, tmpBytes, counts, incl, (size_t)count, rocprim::plus<unsigned long long>(), st);
        if (e != hipSuccess) break;
        hipLaunchKernelGGL(k_wide_emit, g, b, 0, st, dRec, (uint32_t)n2, levA, count, levelBase, triBase, counts, incl,
                           nodes, out.tris, levB, dShapes, numShapes, dIndices, dPositions, dBad);
        unsigned long long tot = 0;
        int bad = 0;
        e = hipMemcpyAsync(&tot, incl + (count - 1), 8, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipMemcpyAsync(&bad, dBad, sizeof(int), hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) break;
        if (bad) {
            static const char* msg[] = {"", "Bvh2 child index out of range", "box extent not representable",
                                        "quantized box does not contain the Bvh2 box", "bad shape / prim id",
                                        "leaf record does not match its triangle"};
            *why = msg[bad >= 1 && bad <= 5 ? bad : 0];
            e = hipErrorInvalidValue;
            break;
        }
        const uint32_t nInt = (uint32_t)(tot >> 32), nTri = (uint32_t)(tot & 0xffffffffull);
        levelBase += count;
        triBase += nTri;
        numNodes += nInt;
        count = nInt;
        std::swap(levA, levB);
        if (numNodes > internal) { *why = "node count"; e = hipErrorInvalidValue; }
    }
    hipFree(levA);
    hipFree(levB);
    hipFree(counts);
    hipFree(incl);
    hipFree(tmp);
    hipFree(dBad);
    if (e == hipSuccess && triBase != leaves) { *why = "triangle count"; e = hipErrorInvalidValue; }
    if (e == hipSuccess) {   // keep exactly numNodes records
        e = hipMalloc(&out.nodes, 64 * (size_t)numNodes);
        if (e == hipSuccess) e = hipMemcpyAsync(out.nodes, nodes, 64 * (size_t)numNodes, hipMemcpyDeviceToDevice, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
    hipFree(nodes);
    if (e != hipSuccess) {
        if (out.nodes) hipFree(out.nodes);
        if (out.tris) hipFree(out.tris);
        out = WideDevice();
        return e;
    }
    out.numNodes = numNodes;
    out.numTris = triBase;
    out.depth = depth;
    return hipSuccess;
}

}  // namespace mcrt

// mcrt_gpubuild.hip -- on-device BVH build for gfx950 (mcrt_accel_opts.device_build = 1).
//
// The default build (mcrt_bvh.cpp) reproduces RadeonRays' Bvh2::Build node for node on the host
// (bvh2.cpp:144-712), which the bit-exact parity with the reference relies on: equal-t hits
// resolve in RR's visit order.  This builder trades that for build speed (a 10 M-triangle scene
// in tens of milliseconds instead of seconds): a linear BVH (Karras, "Maximizing parallelism in
// the construction of BVHs, octrees and k-d trees", HPG 2012) over 63-bit Morton codes of the
// triangle centroids, sorted with rocPRIM's radix sort.  It writes the SAME 64-B record format
// as the host build (mcrt_bvh.cpp; internal = both child boxes + child indices, leaf = its
// world-space triangle + shape/primitive ids), so traversal and shading are unchanged and the
// triangle data is bit-identical (world transform with RR's transform_point arithmetic,
// RR/include/math/mathutils.h:111-118, no contraction).  Only the tree differs.
//
// Record numbering: internal nodes 0 .. n-2 (0 = root), leaves n-1 .. 2n-2 in Morton order.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "mcrt_internal.h"

namespace {

constexpr int BLOCK = 256;

__device__ __forceinline__ int orderedInt(float f) {   // monotonic float -> int (for atomicMin/Max)
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float orderedFloat(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// RR transform_point (mathutils.h:111-118) for w = 1 input and a zero w column product: the same
// sequence of separately rounded adds as the host build (mcrt_capi.cpp xformPoint).
__device__ __forceinline__ float xrow(const mcrt_float4& r, float x, float y, float z) {
    float acc = 0.0f;
    acc = __fadd_rn(acc, __fmul_rn(r.x, x));
    acc = __fadd_rn(acc, __fmul_rn(r.y, y));
    acc = __fadd_rn(acc, __fmul_rn(r.z, z));
    acc = __fadd_rn(acc, __fmul_rn(r.w, 0.0f));
    return __fadd_rn(acc, r.w);
}

// 1. world-space triangles, their boxes and centroids; block-reduced centroid bounds
__global__ __launch_bounds__(BLOCK) void k_prims(int n, const mcrt_shape* __restrict__ shapes,
                                                 const uint32_t* __restrict__ shapeFirst, int numShapes,
                                                 const uint32_t* __restrict__ indices, const float4* __restrict__ positions,
                                                 float* __restrict__ tri, int* __restrict__ shapeOf, int* __restrict__ primOf,
                                                 float4* __restrict__ bmin, float4* __restrict__ bmax,
                                                 float4* __restrict__ cen, int* __restrict__ cbounds) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    float c[3] = {INFINITY, INFINITY, INFINITY}, C[3] = {-INFINITY, -INFINITY, -INFINITY};
    if (i < n) {
        int lo = 0, hi = numShapes - 1;   // last shape with shapeFirst <= i
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (shapeFirst[mid] <= (uint32_t)i) lo = mid; else hi = mid - 1;
        }
        const mcrt_shape& sh = shapes[lo];
        const uint32_t f = (uint32_t)i - shapeFirst[lo];
        float p[9];
        for (int k = 0; k < 3; ++k) {
            const float4 v = positions[sh.startVertex + indices[sh.startIdx + 3 * f + k]];
            p[3 * k + 0] = xrow(sh.toWorldTransform.m0, v.x, v.y, v.z);
            p[3 * k + 1] = xrow(sh.toWorldTransform.m1, v.x, v.y, v.z);
            p[3 * k + 2] = xrow(sh.toWorldTransform.m2, v.x, v.y, v.z);
        }
        for (int k = 0; k < 9; ++k) tri[9 * (size_t)i + k] = p[k];
        shapeOf[i] = lo;
        primOf[i] = (int)f;
        float mn[3], mx[3];
        for (int a = 0; a < 3; ++a) {   // mesh.cpp:130-141 / mcrt_bvh.cpp face bounds, same selects
            const float x = p[a], y = p[3 + a], z = p[6 + a];
            const float m0 = (y < x) ? y : x, x0 = (x < y) ? y : x;
            mn[a] = (z < m0) ? z : m0;
            mx[a] = (x0 < z) ? z : x0;
        }
        bmin[i] = make_float4(mn[0], mn[1], mn[2], 0.0f);
        bmax[i] = make_float4(mx[0], mx[1], mx[2], 0.0f);
        for (int a = 0; a < 3; ++a) c[a] = C[a] = (mn[a] + mx[a]) * 0.5f;
        cen[i] = make_float4(c[0], c[1], c[2], 0.0f);
    }
    __shared__ float red[6][BLOCK];
    for (int a = 0; a < 3; ++a) { red[a][threadIdx.x] = c[a]; red[3 + a][threadIdx.x] = C[a]; }
    __syncthreads();
    for (int s = BLOCK / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s)
            for (int a = 0; a < 3; ++a) {
                red[a][threadIdx.x] = fminf(red[a][threadIdx.x], red[a][threadIdx.x + s]);
                red[3 + a][threadIdx.x] = fmaxf(red[3 + a][threadIdx.x], red[3 + a][threadIdx.x + s]);
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int a = 0; a < 3; ++a) {
            atomicMin(&cbounds[a], orderedInt(red[a][0]));
            atomicMax(&cbounds[3 + a], orderedInt(red[3 + a][0]));
        }
}

__device__ __forceinline__ uint64_t spread21(uint32_t v) {   // 21 bits -> every third bit
    uint64_t x = v & 0x1fffff;
    x = (x | x << 32) & 0x1f00000000ffffull;
    x = (x | x << 16) & 0x1f0000ff0000ffull;
    x = (x | x << 8) & 0x100f00f00f00f00full;
    x = (x | x << 4) & 0x10c30c30c30c30c3ull;
    x = (x | x << 2) & 0x1249249249249249ull;
    return x;
}

// 2. 63-bit Morton codes of the centroids in the centroid bounds
__global__ __launch_bounds__(BLOCK) void k_morton(int n, const float4* __restrict__ cen, const int* __restrict__ cbounds,
                                                  uint64_t* __restrict__ keys, uint32_t* __restrict__ vals) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const float4 c = cen[i];
    const float cc[3] = {c.x, c.y, c.z};
    uint32_t q[3];
    for (int a = 0; a < 3; ++a) {
        const float lo = orderedFloat(cbounds[a]), hi = orderedFloat(cbounds[3 + a]);
        const float ext = hi - lo;
        float t = ext > 0.0f ? (cc[a] - lo) / ext : 0.5f;
        t = fminf(fmaxf(t, 0.0f), 1.0f);
        q[a] = min((uint32_t)(t * 2097152.0f), 2097151u);
    }
    keys[i] = (spread21(q[0]) << 2) | (spread21(q[1]) << 1) | spread21(q[2]);
    vals[i] = (uint32_t)i;
}

// common-prefix length of sorted keys i and j (index tie-break for equal keys); -1 out of range
__device__ __forceinline__ int delta(const uint64_t* __restrict__ k, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    const uint64_t a = k[i], b = k[j];
    if (a == b) return 64 + __clz((uint32_t)(i ^ j));
    return __clzll((long long)(a ^ b));
}

// 3. Karras hierarchy: one thread per internal node
__global__ __launch_bounds__(BLOCK) void k_hierarchy(int n, const uint64_t* __restrict__ k, int* __restrict__ childL,
                                                     int* __restrict__ childR, int* __restrict__ parent) {
    const int i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n - 1) return;
    const int d = (delta(k, n, i, i + 1) - delta(k, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(k, n, i, i - d);
    int lmax = 2;
    while (delta(k, n, i, i + lmax * d) > dmin) lmax <<= 1;
    int l = 0;
    for (int t = lmax >> 1; t >= 1; t >>= 1)
        if (delta(k, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(k, n, i, j);
    int s = 0;
    for (int div = 2;; div <<= 1) {
        const int t = (l + div - 1) / div;
        if (delta(k, n, i, i + (s + t) * d) > dnode) s += t;
        if (t <= 1) break;
    }
    const int g = i + s * d + min(d, 0);
    const int left = (min(i, j) == g) ? (n - 1) + g : g;
    const int right = (max(i, j) == g + 1) ? (n - 1) + g + 1 : g + 1;
    childL[i] = left;
    childR[i] = right;
    parent[left] = i;
    parent[right] = i;
}

// 4. leaf records + bottom-up boxes, internal records and subtree heights (second arrival
//    at a node merges its children; release/acquire through the arrival counter)
__global__ __launch_bounds__(BLOCK) void k_bottom_up(int n, const uint32_t* __restrict__ vals, const float* __restrict__ tri,
                                                     const int* __restrict__ shapeOf, const int* __restrict__ primOf,
                                                     const float4* __restrict__ pmin, const float4* __restrict__ pmax,
                                                     const int* __restrict__ childL, const int* __restrict__ childR,
                                                     const int* __restrict__ parent, int* __restrict__ arrivals,
                                                     float4* __restrict__ boxMin, float4* __restrict__ boxMax,
                                                     int* __restrict__ height, float4* __restrict__ nodes,
                                                     int* __restrict__ maxHeight) {
    const int j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n) return;
    const uint32_t prim = vals[j];
    const int rec = n == 1 ? 0 : (n - 1) + j;
    const float* p = &tri[9 * (size_t)prim];
    nodes[4 * rec + 0] = make_float4(p[0], p[1], p[2], __int_as_float(shapeOf[prim]));
    nodes[4 * rec + 1] = make_float4(p[3] - p[0], p[4] - p[1], p[5] - p[2], __int_as_float(primOf[prim]));
    nodes[4 * rec + 2] = make_float4(p[6] - p[0], p[7] - p[1], p[8] - p[2], 0.0f);
    *reinterpret_cast<int4*>(&nodes[4 * rec + 3]) = make_int4(-1, -1, 0, 0);
    boxMin[rec] = pmin[prim];
    boxMax[rec] = pmax[prim];
    height[rec] = 0;
    if (n == 1) { atomicMax(maxHeight, 0); return; }
    __threadfence();
    int node = parent[rec];
    while (node >= 0) {
        if (atomicAdd(&arrivals[node], 1) == 0) return;   // the sibling's thread finishes the node
        __threadfence();
        const int l = childL[node], r = childR[node];
        const float4 a0 = boxMin[l], a1 = boxMax[l];
        const float4 b0 = boxMin[r], b1 = boxMax[r];
        // internal record (mcrt_bvh.cpp layout): c0 x/y slabs, c1 x/y slabs, z slabs of both, children
        nodes[4 * node + 0] = make_float4(a0.x, a1.x, a0.y, a1.y);
        nodes[4 * node + 1] = make_float4(b0.x, b1.x, b0.y, b1.y);
        nodes[4 * node + 2] = make_float4(a0.z, a1.z, b0.z, b1.z);
        *reinterpret_cast<int4*>(&nodes[4 * node + 3]) = make_int4(l, r, 0, 0);
        boxMin[node] = make_float4(fminf(a0.x, b0.x), fminf(a0.y, b0.y), fminf(a0.z, b0.z), 0.0f);
        boxMax[node] = make_float4(fmaxf(a1.x, b1.x), fmaxf(a1.y, b1.y), fmaxf(a1.z, b1.z), 0.0f);
        height[node] = 1 + max(height[l], height[r]);
        __threadfence();
        if (node == 0) atomicMax(maxHeight, height[0]);
        node = parent[node];
    }
}

template <class T>
hipError_t dalloc(T** p, size_t count) { return hipMalloc((void**)p, sizeof(T) * (count ? count : 1)); }

}  // namespace

namespace mcrt {

// Builds the BVH of all shapes' triangles on the device into *nodesOut (hipMalloc'ed, 64 B per
// record, 2n-1 records).  shapeFirst: host prefix sum of numTriangles (numShapes entries).
hipError_t gpu_build_bvh(const mcrt_shape* dShapes, const std::vector<uint32_t>& shapeFirst, const uint32_t* dIndices,
                         const float4* dPositions, size_t n, hipStream_t st, float4** nodesOut, int* depthOut) {
    *nodesOut = nullptr;
    const int N = (int)n;
    const int numShapes = (int)shapeFirst.size();
    uint32_t* dFirst = nullptr;
    float* tri = nullptr;
    int *shapeOf = nullptr, *primOf = nullptr, *cb = nullptr, *childL = nullptr, *childR = nullptr, *parent = nullptr,
        *arrivals = nullptr, *height = nullptr, *maxH = nullptr;
    float4 *pmin = nullptr, *pmax = nullptr, *cen = nullptr, *boxMin = nullptr, *boxMax = nullptr, *nodes = nullptr;
    uint64_t *keys = nullptr, *keys2 = nullptr;
    uint32_t *vals = nullptr, *vals2 = nullptr;
    void* tmp = nullptr;
    const size_t R = 2 * n - 1;
    hipError_t e = hipSuccess;
    auto A = [&](auto** p, size_t c) { if (e == hipSuccess) e = dalloc(p, c); };
    A(&dFirst, numShapes);
    A(&tri, 9 * n);
    A(&shapeOf, n);
    A(&primOf, n);
    A(&pmin, n);
    A(&pmax, n);
    A(&cen, n);
    A(&cb, 8);
    A(&keys, n);
    A(&keys2, n);
    A(&vals, n);
    A(&vals2, n);
    A(&childL, n);
    A(&childR, n);
    A(&parent, R);
    A(&arrivals, n);
    A(&boxMin, R);
    A(&boxMax, R);
    A(&height, R);
    A(&maxH, 1);
    A(&nodes, 4 * R);
    size_t tmpBytes = 0;
    if (e == hipSuccess)
        e = rocprim::radix_sort_pairs(nullptr, tmpBytes, keys, keys2, vals, vals2, n, 0, 63, st);
    if (e == hipSuccess) e = hipMalloc(&tmp, tmpBytes ? tmpBytes : 16);
    if (e == hipSuccess) e = hipMemcpyAsync(dFirst, shapeFirst.data(), 4 * numShapes, hipMemcpyHostToDevice, st);
    const int init[8] = {0x7fffffff, 0x7fffffff, 0x7fffffff, (int)0x80000000, (int)0x80000000, (int)0x80000000, 0, 0};
    if (e == hipSuccess) e = hipMemcpyAsync(cb, init, sizeof(init), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = hipMemsetAsync(arrivals, 0, 4 * n, st);
    if (e == hipSuccess) e = hipMemsetAsync(maxH, 0, 4, st);
    if (e == hipSuccess) e = hipMemsetAsync(parent, 0xff, 4 * R, st);   // -1: the root has no parent
    const dim3 g((unsigned)((n + BLOCK - 1) / BLOCK)), b(BLOCK);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_prims, g, b, 0, st, N, dShapes, dFirst, numShapes, dIndices, dPositions, tri, shapeOf, primOf,
                           pmin, pmax, cen, cb);
        hipLaunchKernelGGL(k_morton, g, b, 0, st, N, cen, cb, keys, vals);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = rocprim::radix_sort_pairs(tmp, tmpBytes, keys, keys2, vals, vals2, n, 0, 63, st);
    if (e == hipSuccess) {
        if (N > 1) hipLaunchKernelGGL(k_hierarchy, g, b, 0, st, N, keys2, childL, childR, parent);
        hipLaunchKernelGGL(k_bottom_up, g, b, 0, st, N, vals2, tri, shapeOf, primOf, pmin, pmax, childL, childR, parent,
                           arrivals, boxMin, boxMax, height, nodes, maxH);
        e = hipGetLastError();
    }
    int h = 0;
    if (e == hipSuccess) e = hipMemcpyAsync(&h, maxH, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    void* tmps[] = {dFirst, tri, shapeOf, primOf, pmin, pmax, cen, cb, keys, keys2, vals, vals2, childL, childR,
                    parent, arrivals, boxMin, boxMax, height, maxH, tmp};
    for (void* p : tmps)
        if (p) hipFree(p);
    if (e != hipSuccess) {
        if (nodes) hipFree(nodes);
        return e;
    }
    *nodesOut = nodes;
    *depthOut = h + 1;
    return hipSuccess;
}

// world-space triangles, shape/primitive ids, boxes and centroids (k_prims) for the device SAH
// build (mcrt_sahbuild.hip); cbounds: 16 ints of scratch
hipError_t launch_build_prims(int n, const mcrt_shape* dShapes, const uint32_t* dShapeFirst, int numShapes,
                              const uint32_t* dIndices, const float4* dPositions, float* tri, int* shapeOf, int* primOf,
                              float4* amin, float4* amax, float4* cen, int* cbounds, hipStream_t st) {
    const int init[8] = {0x7fffffff, 0x7fffffff, 0x7fffffff, (int)0x80000000, (int)0x80000000, (int)0x80000000, 0, 0};
    hipError_t e = hipMemcpyAsync(cbounds, init, sizeof(init), hipMemcpyHostToDevice, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_prims, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, n, dShapes, dShapeFirst,
                       numShapes, dIndices, dPositions, tri, shapeOf, primOf, amin, amax, cen, cbounds);
    return hipGetLastError();
}

}  // namespace mcrt

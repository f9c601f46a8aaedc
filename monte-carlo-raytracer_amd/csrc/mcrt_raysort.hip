// mcrt_raysort.hip -- optional global reordering of the extension-ray queue before traversal
// (MCRT_SORT_RAYS=1): key = direction octant | 9-bit-per-axis Morton code of the origin in the
// scene bounds, sorted with rocPRIM's radix sort, then the three queue arrays are gathered into
// the sorted order.  Queue order never changes results (paths are independent).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>

#include "mcrt_internal.h"

namespace {

__device__ __forceinline__ uint32_t spread9(uint32_t v) {   // 9 bits -> every third bit
    uint32_t x = v & 0x1ff;
    x = (x | x << 16) & 0x030000ff;
    x = (x | x << 8) & 0x0300f00f;
    x = (x | x << 4) & 0x030c30c3;
    x = (x | x << 2) & 0x09249249;
    return x;
}

__global__ __launch_bounds__(256) void k_ray_keys(const int* __restrict__ count, const float4* __restrict__ o,
                                                  const float4* __restrict__ d, float4 lo, float4 inv,
                                                  uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                  int octOnly) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= *count) return;
    const float4 p = o[i], v = d[i];
    const uint32_t qx = (uint32_t)fminf(fmaxf((p.x - lo.x) * inv.x, 0.0f), 511.0f);
    const uint32_t qy = (uint32_t)fminf(fmaxf((p.y - lo.y) * inv.y, 0.0f), 511.0f);
    const uint32_t qz = (uint32_t)fminf(fmaxf((p.z - lo.z) * inv.z, 0.0f), 511.0f);
    const uint32_t oct = (v.x < 0.0f ? 1u : 0u) | (v.y < 0.0f ? 2u : 0u) | (v.z < 0.0f ? 4u : 0u);
    keys[i] = octOnly ? oct : (oct << 27) | (spread9(qx) << 2) | (spread9(qy) << 1) | spread9(qz);
    vals[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_gather3(const int* __restrict__ count, const uint32_t* __restrict__ perm,
                                                 const float4* __restrict__ a, const float4* __restrict__ b,
                                                 const float4* __restrict__ c, float4* __restrict__ a2,
                                                 float4* __restrict__ b2, float4* __restrict__ c2) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= *count) return;
    const uint32_t j = perm[i];
    a2[i] = a[j];
    b2[i] = b[j];
    c2[i] = c[j];
}

}  // namespace

namespace mcrt {

size_t ray_sort_temp_bytes(int maxCount) {
    size_t bytes = 0;
    uint32_t* k = nullptr;
    rocprim::radix_sort_pairs(nullptr, bytes, k, k, k, k, (size_t)maxCount, 0, 30, (hipStream_t)0);
    return bytes;
}

// Sorts the queue (o, d, t; device count) into (o2, d2, t2).  scratch: 4 uint32 arrays of
// maxCount + ray_sort_temp_bytes(maxCount) bytes.  The sort always covers maxCount entries
// (the device count is not known on the host); entries past the count are never read.
hipError_t sort_ray_queue(const int* count, const float4* o, const float4* d, const float4* t, float4* o2, float4* d2,
                          float4* t2, int maxCount, float3 sceneLo, float3 sceneHi, void* scratch, size_t tempBytes,
                          hipStream_t st) {
    uint32_t* keys = (uint32_t*)scratch;
    uint32_t* keys2 = keys + maxCount;
    uint32_t* vals = keys2 + maxCount;
    uint32_t* vals2 = vals + maxCount;
    void* tmp = vals2 + maxCount;
    hipMemsetAsync(keys, 0xff, 4 * (size_t)maxCount, st);   // entries past the count sort last
    const float ex = fmaxf(sceneHi.x - sceneLo.x, 1e-20f), ey = fmaxf(sceneHi.y - sceneLo.y, 1e-20f),
                ez = fmaxf(sceneHi.z - sceneLo.z, 1e-20f);
    const float4 lo = make_float4(sceneLo.x, sceneLo.y, sceneLo.z, 0.0f);
    const float4 inv = make_float4(512.0f / ex, 512.0f / ey, 512.0f / ez, 0.0f);
    const dim3 g((unsigned)((maxCount + 255) / 256)), b(256);
    // MCRT_SORT_KEY=octant: the direction octant alone (a stable 3-bit sort keeps the queue's own
    // origin order inside each octant)
    static const int octOnly = [] {
        const char* k = std::getenv("MCRT_SORT_KEY");
        return k && std::strcmp(k, "octant") == 0 ? 1 : 0;
    }();
    hipLaunchKernelGGL(k_ray_keys, g, b, 0, st, count, o, d, lo, inv, keys, vals, octOnly);
    hipError_t e = rocprim::radix_sort_pairs(tmp, tempBytes, keys, keys2, vals, vals2, (size_t)maxCount, 0,
                                             octOnly ? 4 : 30, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gather3, g, b, 0, st, count, vals2, o, d, t, o2, d2, t2);
    return hipGetLastError();
}

}  // namespace mcrt

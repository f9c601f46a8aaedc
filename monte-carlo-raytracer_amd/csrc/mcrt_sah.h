// mcrt_sah.h -- the split arithmetic of RadeonRays' Bvh2 builder (RR/src/accelerator/bvh2.cpp,
// restated on the host in mcrt_bvh.cpp) as plain scalar code that compiles for the host and for
// gfx950, so the on-device SAH builder (mcrt_sahbuild.hip) makes the same decisions bit for bit.
//
// The reference computes with SSE on the host CPU; three of its instructions have no IEEE
// counterpart and are restated exactly here:
//   _mm_rcp_ps  (bvh2.cpp:339-348 centroid-extent and area reciprocals): an implementation-
//               defined ~12-bit approximation.  Its result for x = 1.m * 2^e is R(m) * 2^-e with
//               R tabulated over the mantissa bits the host's instruction reads (measured on the
//               running host at first use, sah_rcp_table in mcrt_sahbuild.hip); zero/denormal
//               inputs give inf, inputs >= 2^125 flush to 0 -- checked on the host as well.
//   _mm_dp_ps   (bvh2.cpp:69-75 surface area): products rounded, then (p0 + p1) + (p2 + p3).
//   min/max_ps  a < b ? a : b / a > b ? a : b (second operand on ties).
// Everything else is single fp32 operations in the reference's order; the file that includes
// this header is compiled with -ffp-contract=off so no product is fused into an add.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SAH_HD __host__ __device__ __forceinline__

namespace mcrt {
namespace sah {

struct V4 {
    float x, y, z, w;
};

SAH_HD float fmin_ps(float a, float b) { return (a < b) ? a : b; }   // MINPS lane semantics
SAH_HD float fmax_ps(float a, float b) { return (a > b) ? a : b; }   // MAXPS lane semantics
SAH_HD V4 vmin(V4 a, V4 b) { return V4{fmin_ps(a.x, b.x), fmin_ps(a.y, b.y), fmin_ps(a.z, b.z), fmin_ps(a.w, b.w)}; }
SAH_HD V4 vmax(V4 a, V4 b) { return V4{fmax_ps(a.x, b.x), fmax_ps(a.y, b.y), fmax_ps(a.z, b.z), fmax_ps(a.w, b.w)}; }
SAH_HD V4 vsub(V4 a, V4 b) { return V4{a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w}; }
SAH_HD float lane(V4 v, uint32_t i) { return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w; }

SAH_HD uint32_t fbits(float f) {
    union { float f; uint32_t u; } c;
    c.f = f;
    return c.u;
}
SAH_HD float bitsf(uint32_t u) {
    union { float f; uint32_t u; } c;
    c.u = u;
    return c.f;
}

// bvh2.cpp:69-75 surface area: dp_ps(e.xxy, e.yzz, 0xff) * 2 with e = pmax - pmin (4 lanes)
SAH_HD float sa4(V4 pmin, V4 pmax) {
    const V4 e = vsub(pmax, pmin);
    const float p0 = e.x * e.y, p1 = e.x * e.z, p2 = e.y * e.z, p3 = e.w * e.w;
    const float s01 = p0 + p1, s23 = p2 + p3;
    return (s01 + s23) * 2.0f;
}

// bvh2.cpp:83-92: index of the largest centroid extent (first lane equal to the max)
SAH_HD uint32_t maxAxis(V4 pmin, V4 pmax) {
    const V4 xyz = vsub(pmax, pmin);
    const V4 yzx = V4{xyz.y, xyz.z, xyz.x, xyz.w};
    const V4 m0 = vmax(xyz, yzx);
    const V4 m1 = V4{m0.y, m0.z, m0.x, m0.w};
    const V4 m2 = vmax(m0, m1);
    if (xyz.x == m2.x) return 0;
    if (xyz.y == m2.y) return 1;
    if (xyz.z == m2.z) return 2;
    if (xyz.w == m2.w) return 3;
    return 32;   // ctz(0): not reached for finite boxes
}

// _mm_rcp_ps on the host that built `table` (R over the top `bits` mantissa bits, exponent 127)
SAH_HD float rcp_ps(float x, const uint32_t* table, int bits) {
    const uint32_t b = fbits(x), s = b & 0x80000000u, e = (b >> 23) & 0xffu;
    if (e == 0) return bitsf(s | 0x7f800000u);                              // 0 / denormal -> inf
    if (e == 255) return (b & 0x7fffffu) ? bitsf(b | 0x400000u) : bitsf(s);   // NaN / inf -> 0
    if (e >= 253) return bitsf(s);                                          // result flushed to 0
    const uint32_t t = table[(b & 0x7fffffu) >> (23 - bits)];
    const uint32_t te = (t >> 23) & 0xffu;
    return bitsf(s | ((te + 127u - e) << 23) | (t & 0x7fffffu));
}

// (uint32_t)float as the host code compiles it on x86-64 (cvttss2si to 64 bits, low half):
// NaN and |x| >= 2^63 give 0
SAH_HD uint32_t f2u32_x86(float t) {
    if (!(t < 9.22337203685477580800e18f) || !(t > -9.22337203685477580800e18f)) return 0u;
    return (uint32_t)(int64_t)t;
}

// bvh2.cpp:372-394: bin of a centroid.  The reference bins the first num & ~3 references of the
// range four at a time ((c - min) * rcp * nb) and the rest one at a time (nb * (c - min) * rcp).
SAH_HD uint32_t binFull(float c, float cm, float cinv, float nbf, uint32_t nb) {
    float t = c - cm;
    t = t * cinv;
    t = t * nbf;
    const uint32_t b = f2u32_x86(t);
    return b < nb - 1 ? b : nb - 1;
}
SAH_HD uint32_t binTail(float c, float cm, float cinv, float nbf, uint32_t nb) {
    float t = c - cm;
    t = nbf * t;
    t = t * cinv;
    const uint32_t b = f2u32_x86(t);
    return b < nb - 1 ? b : nb - 1;
}

// bvh2.cpp:396-491: SAH sweep over the bins -> split plane.  cnt/bmn/bmx: the bins (empty bins
// +inf/-inf in every lane); rmn/rmx: scratch of nb - 1 entries.
SAH_HD float sweep(const uint32_t* cnt, const V4* bmn, const V4* bmx, V4* rmn, V4* rmx, uint32_t nb, uint64_t num,
                   float cost, float areaInv, float cm, float ce) {
    V4 tmn = V4{INFINITY, INFINITY, INFINITY, INFINITY}, tmx = V4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (uint32_t i = nb - 1; i > 0; --i) {
        tmn = vmin(tmn, bmn[i]);
        tmx = vmax(tmx, bmx[i]);
        rmn[i - 1] = tmn;
        rmx[i - 1] = tmx;
    }
    tmn = V4{INFINITY, INFINITY, INFINITY, INFINITY};
    tmx = V4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    uint32_t lc = 0;
    uint64_t rc = num;
    int split = -1;
    float best = 3.402823466e+38f;
    for (uint32_t i = 0; i < nb - 1; ++i) {
        tmn = vmin(tmn, bmn[i]);
        tmx = vmax(tmx, bmx[i]);
        lc += cnt[i];
        rc -= cnt[i];
        const float a = (float)lc * sa4(tmn, tmx);
        const float b = (float)rc * sa4(rmn[i], rmx[i]);
        const float s = cost + (a + b) * areaInv;
        if (s < best) {
            split = (int)i;
            best = s;
        }
    }
    // cm + (split + 1) * (ce / nb): correctly rounded fp32 division (f64 quotient, exact rounding)
    const float step = (float)((double)ce / (double)(float)nb);
    return cm + (float)(split + 1) * step;
}

// face bounds of a leaf record (mcrt_bvh.cpp leafBox): the select order of the host conversion
SAH_HD void leafBox(const float* p, float* bx) {
    for (int c = 0; c < 3; ++c) {
        const float a = p[c], bb = p[3 + c], cc = p[6 + c];
        const float mn = (cc < bb) ? cc : bb, mx = (bb < cc) ? cc : bb;
        bx[c] = (mn < a) ? mn : a;
        bx[3 + c] = (a < mx) ? mx : a;
    }
}

}  // namespace sah
}  // namespace mcrt

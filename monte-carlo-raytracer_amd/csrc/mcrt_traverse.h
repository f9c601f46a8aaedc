// mcrt_traverse.h -- Bvh2 traversal shared by the path-tracing and BDPT kernels.
// (Moved out of mcrt_kernels.hip; see there for the launch structure.)
#pragma once
#include "mcrt_device.h"
#include "mcrt_internal.h"

// ---------------------------------------------------------------------------
// traversal
// ---------------------------------------------------------------------------
#define STACK_LDS 16

// Node-record layouts of the traversal kernels' template parameter LAY (TraceCtx::compact,
// TraceCtx::twoLevel): each layout gets its own kernel instantiation, so a kernel's register
// budget is that of the one loop it runs.
#define LAY_PLAIN 0       // mcrt_bvh.cpp records, traverseOct
#define LAY_COMPACT 1     // descent-compact records, traverseOct2
#define LAY_TWO_LEVEL 3   // mcrt_bvh2l.cpp records, traverse2L
template <typename K>
inline K pickLayout(const TraceCtx& c, K twoLevel, K compact, K plain) {
    return c.twoLevel ? twoLevel : c.compact ? compact : plain;
}

struct TraceRay {
    f3 o, d;
    float tmax;
    int mask;
};

// RR common.cl:220-232
MCRT_DEV f3 safeInvDir(f3 d) {
    const float ooeps = 1e-8f;
    f3 inv;
    inv.x = cl_div(1.0f, (fabsf(d.x) > ooeps ? d.x : copysignf(ooeps, d.x)));
    inv.y = cl_div(1.0f, (fabsf(d.y) > ooeps ? d.y : copysignf(ooeps, d.y)));
    inv.z = cl_div(1.0f, (fabsf(d.z) > ooeps ? d.z : copysignf(ooeps, d.z)));
    return inv;
}

// RR common.cl:177-218; native_recip lowers to v_rcp_f32 on AMD.
MCRT_DEV float triHit(const TraceRay& r, float4 A, float4 E1, float4 E2, float tmax) {
    const f3 e1 = ld3(E1), e2 = ld3(E2);
    const f3 s1 = cl_cross(r.d, e2);
    const float denom = cl_dot(s1, e1);
    if (denom == 0.f) return tmax;
    const float invd = __builtin_amdgcn_rcpf(denom);
    const f3 d = r.o - ld3(A);
    const float b1 = cl_dot(d, s1) * invd;
    const f3 s2 = cl_cross(d, e1);
    const float b2 = cl_dot(r.d, s2) * invd;
    const float temp = cl_dot(e2, s2) * invd;
    if (b1 < 0.f || b1 > 1.f || b2 < 0.f || b1 + b2 > 1.f || temp < 0.f || temp > tmax) return tmax;
    return temp;
}

// Octant-specialised slab tests (1 = on): a wave whose rays all share one direction octant
// runs a loop instantiated for that octant.  With the signs of 1/d known, each axis' entry and
// exit distances are fixed planes of the box -- for a valid box (min <= max) and 1/d > 0,
// fma(min, 1/d, -o/d) <= fma(max, 1/d, -o/d) because fma rounds monotonically -- so the six
// per-axis min/max pairs of fast_intersect_bbox2 (intersect_bvh2_lds.cl:54-63) reduce to picking
// the plane: the same floats, 12 fewer VALU instructions per internal node.  Camera tiles,
// octant-grouped extension queues and directional-light shadow rays are mostly uniform; mixed
// waves take the generic loop.
// Closest (ANY = false) or any (ANY = true) hit over the unified node array (mcrt_bvh.cpp):
// the RadeonRays intersect_bvh2_lds.cl:107-178 loop -- one uniform 64-B fetch per step, an
// internal node tests both child boxes (nearer child first, far child to the stack), a leaf
// tests its triangle.  Returns the hit leaf's node index or -1; tHit = hit distance.
// stk: this lane's LDS stack column ([entry][lane], conflict free); spill: global overflow.
// OCT: the wave's common ray-direction octant (bit k = sign of 1/d along axis k), -1 = mixed.
template <bool ANY, int OCT>
MCRT_DEV int traverseOct(const float4* __restrict__ nodes, const TraceRay& r, f3 inv, uint32_t* stk, uint32_t* spill,
                         int spillCap, int* overflowFlag, float& tHit) {
    // One flat loop with a single exit (node == DONE): stack entry 0 is a DONE sentinel, so a
    // pop is one LDS read and no lane idles at a nested loop boundary waiting for the others.
    constexpr int DONE = -1, POP = -2;
    const f3 oxi = -r.o * inv;   // intersect_bvh2_lds.cl:91
    float t = r.tmax;
    int hit = -1;
    int node = 0;
    stk[0] = (uint32_t)DONE;
    int sp = 1, spillTop = 0;
    while (node != DONE) {
        const float4 n0 = nodes[4 * node + 0];
        const float4 n1 = nodes[4 * node + 1];
        const float4 n2 = nodes[4 * node + 2];
        const int4 n3 = *reinterpret_cast<const int4*>(&nodes[4 * node + 3]);
        // keep the whole 64-B record in one round trip: without this the compiler defers the
        // two words only internal nodes use into a second, dependent load after the branch
        asm volatile("" ::"v"(n1.w), "v"(n2.w));
        int next;
        if (n3.x >= 0) {
            // slab tests of both children (RR intersect_bvh2_lds.cl:54-63, mad -> fma)
            float a0, a1, b0, b1;
            if constexpr (OCT >= 0) {
                constexpr bool SX = (OCT & 1) != 0, SY = (OCT & 2) != 0, SZ = (OCT & 4) != 0;
                const float axn = fmaf(SX ? n0.y : n0.x, inv.x, oxi.x), axf = fmaf(SX ? n0.x : n0.y, inv.x, oxi.x);
                const float ayn = fmaf(SY ? n0.w : n0.z, inv.y, oxi.y), ayf = fmaf(SY ? n0.z : n0.w, inv.y, oxi.y);
                const float azn = fmaf(SZ ? n2.y : n2.x, inv.z, oxi.z), azf = fmaf(SZ ? n2.x : n2.y, inv.z, oxi.z);
                const float bxn = fmaf(SX ? n1.y : n1.x, inv.x, oxi.x), bxf = fmaf(SX ? n1.x : n1.y, inv.x, oxi.x);
                const float byn = fmaf(SY ? n1.w : n1.z, inv.y, oxi.y), byf = fmaf(SY ? n1.z : n1.w, inv.y, oxi.y);
                const float bzn = fmaf(SZ ? n2.w : n2.z, inv.z, oxi.z), bzf = fmaf(SZ ? n2.z : n2.w, inv.z, oxi.z);
                a0 = fmaxf(fmaxf(axn, ayn), fmaxf(azn, 0.0f));
                a1 = fminf(fminf(axf, ayf), fminf(azf, t));
                b0 = fmaxf(fmaxf(bxn, byn), fmaxf(bzn, 0.0f));
                b1 = fminf(fminf(bxf, byf), fminf(bzf, t));
            } else {
                const float ax0 = fmaf(n0.x, inv.x, oxi.x), ax1 = fmaf(n0.y, inv.x, oxi.x);
                const float ay0 = fmaf(n0.z, inv.y, oxi.y), ay1 = fmaf(n0.w, inv.y, oxi.y);
                const float az0 = fmaf(n2.x, inv.z, oxi.z), az1 = fmaf(n2.y, inv.z, oxi.z);
                const float bx0 = fmaf(n1.x, inv.x, oxi.x), bx1 = fmaf(n1.y, inv.x, oxi.x);
                const float by0 = fmaf(n1.z, inv.y, oxi.y), by1 = fmaf(n1.w, inv.y, oxi.y);
                const float bz0 = fmaf(n2.z, inv.z, oxi.z), bz1 = fmaf(n2.w, inv.z, oxi.z);
                a0 = fmaxf(fmaxf(fmaxf(fminf(ax0, ax1), fminf(ay0, ay1)), fminf(az0, az1)), 0.0f);
                a1 = fminf(fminf(fminf(fmaxf(ax0, ax1), fmaxf(ay0, ay1)), fmaxf(az0, az1)), t);
                b0 = fmaxf(fmaxf(fmaxf(fminf(bx0, bx1), fminf(by0, by1)), fminf(bz0, bz1)), 0.0f);
                b1 = fminf(fminf(fminf(fmaxf(bx0, bx1), fmaxf(by0, by1)), fmaxf(bz0, bz1)), t);
            }
            const bool h0 = a0 <= a1, h1 = b0 <= b1;
            const bool c1first = h1 && (a0 > b0);   // intersect_bvh2_lds.cl:128-141
            if (h0 && h1) {   // defer the far child
                if (sp == STACK_LDS) {   // spill entries 1..15 (RR: intersect_bvh2_lds.cl:146-155)
                    if (spillTop + STACK_LDS - 1 <= spillCap) {
                        for (int k = 1; k < STACK_LDS; ++k) spill[(size_t)(spillTop + k - 1) * 64] = stk[k * 64];
                        spillTop += STACK_LDS - 1;
                    } else {
                        *overflowFlag = 1;   // depth beyond capacity: drop (reported by the host)
                    }
                    sp = 1;
                }
                stk[sp * 64] = (uint32_t)(c1first ? n3.x : n3.y);
                ++sp;
            }
            next = (h0 || h1) ? ((c1first || !h0) ? n3.y : n3.x) : POP;
        } else {
            next = POP;
            if (r.mask != __float_as_int(n0.w)) {   // RR_RAY_MASK
                const float th = triHit(r, n0, n1, n2, t);
                if (th < t) {
                    t = th;
                    hit = node;
                    if (ANY) next = DONE;
                }
            }
        }
        if (next == POP) {
            --sp;
            next = (int)stk[sp * 64];
            if (next == DONE && spillTop > 0) {   // refill (intersect_bvh2_lds.cl:182-191)
                spillTop -= STACK_LDS - 1;
                for (int k = 1; k < STACK_LDS; ++k) stk[k * 64] = spill[(size_t)(spillTop + k - 1) * 64];
                sp = STACK_LDS - 1;
                next = (int)stk[sp * 64];
            }
        }
        node = next;
    }
    tHit = t;
    return hit;
}

// ---------------------------------------------------------------------------
// Descent-compact records (mcrt_kernels.hip k_pack_compact), used by the camera-ray launch.
//
// A coherent launch is bound by the vector-memory path, not the ALUs: every step gathers four
// 16-B pieces per lane from a record (measured on k_primary: TA busy 92 % of its cycles, L2 hit
// 94 %).  The records are re-laid out to need fewer loads per step without changing a single box
// value the slab tests see:
//   * a parent's two child boxes are exact float min/max unions (RR bvh2.cpp pulls bounds into
//     parents), so per coordinate slot s (lo.x, hi.x, lo.y, hi.y, lo.z, hi.z) one child holds
//     the node's own value X_s and only the OTHER child's value S_s must be stored, plus a bit
//     saying which child owns X_s;
//   * 80 % of internal steps descend into a child whose box the previous step just tested, so
//     X's slab distances are already in registers (dX_s = fma(X_s, 1/d, -o/d), the same floats).
// Record of internal node i (children A = left, B = right):
//   q0 = (S0, S1, S2, S3), q1 = (S4, S5, wA, wB),      <- a descent reads only these 32 B
//   q2 = (X.lo.x, X.hi.x, X.lo.y, X.hi.y), q3 = (X.lo.z, X.hi.z, 0, 0)   <- + these after a pop
//   child word w = index (bits 0-26) | leaf (bit 27) | owner bits of 3 slots (28-30)
// Leaf record: (v0, shapeId), (v1 - v0, primId), (v2 - v0, 0), (-1, -1, 0, 0) as before: 48 B,
// and the leaf bit in the parent's word says so before the fetch.  A step loads 2, 3 (leaf) or
// 4 (after a pop) pieces instead of 4; the decode reproduces both child boxes exactly (the
// owner's value is X_s bit for bit up to the sign of a zero, which no slab decision can see),
// so the visit order, every box test and every triangle test are those of traverseOct.
// Measured (SM proxy 1080p): k_primary -9 %; the incoherent extension / shadow launches are
// bound by L2 misses instead and ran 2-5 % slower with it, so they keep the plain records.
// ---------------------------------------------------------------------------
#define CW_IDX 0x07FFFFFFu
#define CW_LEAF 0x08000000u
#define CW_NODE 0x0FFFFFFFu   // index | leaf, the part the stack keeps
#define CW_DONE 0x80000000u

template <bool ANY, int OCT>
MCRT_DEV int traverseOct2(const float4* __restrict__ nodes, uint32_t rootWord, const TraceRay& r, f3 inv,
                          uint32_t* stk, uint32_t* spill, int spillCap, int* overflowFlag, float& tHit) {
    const f3 oxi = -r.o * inv;   // intersect_bvh2_lds.cl:91
    float t = r.tmax;
    int hit = -1;
    uint32_t word = rootWord;
    bool popped = true;   // the root's own box comes from its record
    // slab distances of the node's own box per slot (valid after a descent)
    float dx0 = 0.f, dx1 = 0.f, dx2 = 0.f, dx3 = 0.f, dx4 = 0.f, dx5 = 0.f;
    stk[0] = CW_DONE;
    int sp = 1, spillTop = 0;
    while (word != CW_DONE) {
        const uint32_t idx = word & CW_IDX;
        const bool leaf = (word & CW_LEAF) != 0;
        const float4* q = nodes + 4 * (size_t)idx;
        float4 q0, q1, q2 = make_float4(0.f, 0.f, 0.f, 0.f), q3 = q2;
        q0 = q[0];
        q1 = q[1];
        if (leaf || popped) q2 = q[2];
        if (popped && !leaf) q3 = q[3];
        bool pop = true;
        uint32_t next = CW_DONE;
        if (!leaf) {
            if (popped) {
                dx0 = fmaf(q2.x, inv.x, oxi.x); dx1 = fmaf(q2.y, inv.x, oxi.x);
                dx2 = fmaf(q2.z, inv.y, oxi.y); dx3 = fmaf(q2.w, inv.y, oxi.y);
                dx4 = fmaf(q3.x, inv.z, oxi.z); dx5 = fmaf(q3.y, inv.z, oxi.z);
            }
            const uint32_t wA = __float_as_uint(q1.z), wB = __float_as_uint(q1.w);
            const float ds0 = fmaf(q0.x, inv.x, oxi.x), ds1 = fmaf(q0.y, inv.x, oxi.x);
            const float ds2 = fmaf(q0.z, inv.y, oxi.y), ds3 = fmaf(q0.w, inv.y, oxi.y);
            const float ds4 = fmaf(q1.x, inv.z, oxi.z), ds5 = fmaf(q1.y, inv.z, oxi.z);
            // owner masks (all ones: A holds X_s) and the two children's slot distances
            const uint32_t m0 = (uint32_t)__builtin_amdgcn_sbfe((int)wA, 28, 1);
            const uint32_t m1 = (uint32_t)__builtin_amdgcn_sbfe((int)wA, 29, 1);
            const uint32_t m2 = (uint32_t)__builtin_amdgcn_sbfe((int)wA, 30, 1);
            const uint32_t m3 = (uint32_t)__builtin_amdgcn_sbfe((int)wB, 28, 1);
            const uint32_t m4 = (uint32_t)__builtin_amdgcn_sbfe((int)wB, 29, 1);
            const uint32_t m5 = (uint32_t)__builtin_amdgcn_sbfe((int)wB, 30, 1);
#define MCRT_SEL(m, a, b) __uint_as_float(((m) & __float_as_uint(a)) | (~(m) & __float_as_uint(b)))
            const float A0 = MCRT_SEL(m0, dx0, ds0), B0 = MCRT_SEL(m0, ds0, dx0);
            const float A1 = MCRT_SEL(m1, dx1, ds1), B1 = MCRT_SEL(m1, ds1, dx1);
            const float A2 = MCRT_SEL(m2, dx2, ds2), B2 = MCRT_SEL(m2, ds2, dx2);
            const float A3 = MCRT_SEL(m3, dx3, ds3), B3 = MCRT_SEL(m3, ds3, dx3);
            const float A4 = MCRT_SEL(m4, dx4, ds4), B4 = MCRT_SEL(m4, ds4, dx4);
            const float A5 = MCRT_SEL(m5, dx5, ds5), B5 = MCRT_SEL(m5, ds5, dx5);
#undef MCRT_SEL
            float a0, a1, b0, b1;
            if constexpr (OCT >= 0) {
                // per axis the entry plane is lo for 1/d > 0 and hi otherwise (fma is monotone)
                constexpr bool SX = (OCT & 1) != 0, SY = (OCT & 2) != 0, SZ = (OCT & 4) != 0;
                a0 = fmaxf(fmaxf(SX ? A1 : A0, SY ? A3 : A2), fmaxf(SZ ? A5 : A4, 0.0f));
                a1 = fminf(fminf(SX ? A0 : A1, SY ? A2 : A3), fminf(SZ ? A4 : A5, t));
                b0 = fmaxf(fmaxf(SX ? B1 : B0, SY ? B3 : B2), fmaxf(SZ ? B5 : B4, 0.0f));
                b1 = fminf(fminf(SX ? B0 : B1, SY ? B2 : B3), fminf(SZ ? B4 : B5, t));
            } else {   // RR intersect_bvh2_lds.cl:54-63 (fast_intersect_bbox2)
                a0 = fmaxf(fmaxf(fmaxf(fminf(A0, A1), fminf(A2, A3)), fminf(A4, A5)), 0.0f);
                a1 = fminf(fminf(fminf(fmaxf(A0, A1), fmaxf(A2, A3)), fmaxf(A4, A5)), t);
                b0 = fmaxf(fmaxf(fmaxf(fminf(B0, B1), fminf(B2, B3)), fminf(B4, B5)), 0.0f);
                b1 = fminf(fminf(fminf(fmaxf(B0, B1), fmaxf(B2, B3)), fmaxf(B4, B5)), t);
            }
            const bool h0 = a0 <= a1, h1 = b0 <= b1;
            const bool c1first = h1 && (a0 > b0);   // intersect_bvh2_lds.cl:128-141
            if (h0 && h1) {   // defer the far child
                if (sp == STACK_LDS) {   // spill entries 1..15 (RR: intersect_bvh2_lds.cl:146-155)
                    if (spillTop + STACK_LDS - 1 <= spillCap) {
                        for (int k = 1; k < STACK_LDS; ++k) spill[(size_t)(spillTop + k - 1) * 64] = stk[k * 64];
                        spillTop += STACK_LDS - 1;
                    } else {
                        *overflowFlag = 1;   // depth beyond capacity: drop (reported by the host)
                    }
                    sp = 1;
                }
                stk[sp * 64] = (c1first ? wA : wB) & CW_NODE;
                ++sp;
            }
            if (h0 || h1) {
                const bool toB = c1first || !h0;
                next = (toB ? wB : wA) & CW_NODE;
                dx0 = toB ? B0 : A0; dx1 = toB ? B1 : A1; dx2 = toB ? B2 : A2;
                dx3 = toB ? B3 : A3; dx4 = toB ? B4 : A4; dx5 = toB ? B5 : A5;
                pop = false;
            }
        } else if (r.mask != __float_as_int(q0.w)) {   // RR_RAY_MASK
            const float th = triHit(r, q0, q1, q2, t);
            if (th < t) {
                t = th;
                hit = (int)idx;
                if (ANY) pop = false;   // next = DONE
            }
        }
        if (pop) {
            --sp;
            next = stk[sp * 64];
            if (next == CW_DONE && spillTop > 0) {   // refill (intersect_bvh2_lds.cl:182-191)
                spillTop -= STACK_LDS - 1;
                for (int k = 1; k < STACK_LDS; ++k) stk[k * 64] = spill[(size_t)(spillTop + k - 1) * 64];
                sp = STACK_LDS - 1;
                next = stk[sp * 64];
            }
        }
        popped = pop;
        word = next;
    }
    tHit = t;
    return hit;
}

template <bool ANY, int LAY>
MCRT_DEV int traverse(const TraceCtx& c, const TraceRay& r, uint32_t* stk, uint32_t* spill, float& tHit) {
    const f3 inv = safeInvDir(r.d);
#define MCRT_TRAV_CALL(OCT)                                                                                       \
    do {                                                                                                          \
        if constexpr (LAY == LAY_COMPACT)                                                                         \
            return traverseOct2<ANY, OCT>(c.nodes, c.rootWord, r, inv, stk, spill, c.spillCap, c.overflow, tHit); \
        else                                                                                                      \
            return traverseOct<ANY, OCT>(c.nodes, r, inv, stk, spill, c.spillCap, c.overflow, tHit);             \
    } while (0)
    const int oct = (int)(__float_as_uint(inv.x) >> 31) | (int)((__float_as_uint(inv.y) >> 31) << 1) |
                    (int)((__float_as_uint(inv.z) >> 31) << 2);
    const int oct0 = __builtin_amdgcn_readfirstlane(oct);
    if (__all(oct == oct0)) {
        switch (oct0) {
            case 0: MCRT_TRAV_CALL(0);
            case 1: MCRT_TRAV_CALL(1);
            case 2: MCRT_TRAV_CALL(2);
            case 3: MCRT_TRAV_CALL(3);
            case 4: MCRT_TRAV_CALL(4);
            case 5: MCRT_TRAV_CALL(5);
            case 6: MCRT_TRAV_CALL(6);
            case 7: MCRT_TRAV_CALL(7);
            default: break;
        }
    }
    MCRT_TRAV_CALL(-1);
#undef MCRT_TRAV_CALL
}

// RR common.cl:249-277 (triangle_calculate_barycentrics)
MCRT_DEV f2 triBary(f3 p, float4 A, float4 E1, float4 E2) {
    const f3 e1 = ld3(E1), e2 = ld3(E2);
    const f3 e = p - ld3(A);
    const float d00 = cl_dot(e1, e1);
    const float d01 = cl_dot(e1, e2);
    const float d11 = cl_dot(e2, e2);
    const float d20 = cl_dot(e, e1);
    const float d21 = cl_dot(e, e2);
    float denom = (d00 * d11 - d01 * d01);
    if (denom == 0.f) return f2{0.f, 0.f};
    const float invdenom = __builtin_amdgcn_rcpf(denom);
    const float b1 = (d11 * d20 - d01 * d21) * invdenom;
    const float b2 = (d00 * d21 - d01 * d20) * invdenom;
    return f2{b1, b2};
}

// Hit record of the closest-hit kernels: (u, v, shape index bits, primitive index bits), shape
// = -1 on a miss (barycentrics: intersect_bvh2_lds.cl:200-215).  The shading kernels read the
// shape and primitive from here, not from the BVH.
MCRT_DEV float4 closestRecord(const float4* __restrict__ nodes, const TraceRay& r, int tri, float t) {
    if (tri < 0) return make_float4(0.f, 0.f, __int_as_float(-1), __int_as_float(-1));
    const float4 A = nodes[4 * tri], E1 = nodes[4 * tri + 1], E2 = nodes[4 * tri + 2];
    const f3 p = r.o + t * r.d;
    const f2 uv = triBary(p, A, E1, E2);
    return make_float4(uv.x, uv.y, A.w, E1.w);
}

// ---------------------------------------------------------------------------
// Two-level (instanced) traversal over the mcrt_bvh2l.cpp records: RadeonRays'
// IntersectorTwoLevel semantics (intersect_bvh2level_skiplinks.cl:112-318) -- at a top-level
// leaf the ray moves into the shape's object space (world-to-local rows), the shape's own
// BVH is traversed, then the world ray is restored -- on our nearest-first stack traversal
// (the reference walks fixed-order skip links; the closest hit does not depend on the order
// except between triangles at exactly the same t).
// ---------------------------------------------------------------------------
#define BVH_INSTANCE_MARK (-2)

// transform_point / transform_vector (intersect_bvh2level_skiplinks.cl:88-106); ext-vector
// arithmetic contracts exactly like the OpenCL source
MCRT_DEV f3 xfPoint(float4 m0, float4 m1, float4 m2, f3 p) {
    f3 r;
    r.x = m0.x * p.x + m0.y * p.y + m0.z * p.z + m0.w;
    r.y = m1.x * p.x + m1.y * p.y + m1.z * p.z + m1.w;
    r.z = m2.x * p.x + m2.y * p.y + m2.z * p.z + m2.w;
    return r;
}
MCRT_DEV f3 xfVector(float4 m0, float4 m1, float4 m2, f3 p) {
    f3 r;
    r.x = m0.x * p.x + m0.y * p.y + m0.z * p.z;
    r.y = m1.x * p.x + m1.y * p.y + m1.z * p.z;
    r.z = m2.x * p.x + m2.y * p.y + m2.z * p.z;
    return r;
}

// Returns the hit triangle record or -1; hitInst = the instance record it was hit through.
template <bool ANY>
MCRT_DEV int traverse2L(const float4* __restrict__ nodes, const TraceRay& r, uint32_t* stk, uint32_t* spill,
                        int spillCap, int* overflowFlag, float& tHit, int& hitInst) {
    constexpr int DONE = -1, POP = -2, RESTORE = -3;
    const f3 winv = safeInvDir(r.d);
    const f3 woxi = -r.o * winv;
    TraceRay cr = r;   // current-space ray (world at the top level, object below an instance)
    f3 inv = winv, oxi = woxi;
    float t = r.tmax;
    int hit = -1, hinst = -1, inst = -1;
    int node = 0;
    stk[0] = (uint32_t)DONE;
    int sp = 1, spillTop = 0;
    auto push = [&](int v) {
        if (sp == STACK_LDS) {
            if (spillTop + STACK_LDS - 1 <= spillCap) {
                for (int k = 1; k < STACK_LDS; ++k) spill[(size_t)(spillTop + k - 1) * 64] = stk[k * 64];
                spillTop += STACK_LDS - 1;
            } else {
                *overflowFlag = 1;
            }
            sp = 1;
        }
        stk[sp * 64] = (uint32_t)v;
        ++sp;
    };
    auto pop = [&]() -> int {
        --sp;
        int v = (int)stk[sp * 64];
        if (v == DONE && spillTop > 0) {
            spillTop -= STACK_LDS - 1;
            for (int k = 1; k < STACK_LDS; ++k) stk[k * 64] = spill[(size_t)(spillTop + k - 1) * 64];
            sp = STACK_LDS - 1;
            v = (int)stk[sp * 64];
        }
        return v;
    };
    while (node != DONE) {
        const float4 n0 = nodes[4 * node + 0];
        const float4 n1 = nodes[4 * node + 1];
        const float4 n2 = nodes[4 * node + 2];
        const int4 n3 = *reinterpret_cast<const int4*>(&nodes[4 * node + 3]);
        asm volatile("" ::"v"(n1.w), "v"(n2.w));
        int next;
        if (n3.x >= 0) {
            const float ax0 = fmaf(n0.x, inv.x, oxi.x), ax1 = fmaf(n0.y, inv.x, oxi.x);
            const float ay0 = fmaf(n0.z, inv.y, oxi.y), ay1 = fmaf(n0.w, inv.y, oxi.y);
            const float az0 = fmaf(n2.x, inv.z, oxi.z), az1 = fmaf(n2.y, inv.z, oxi.z);
            const float bx0 = fmaf(n1.x, inv.x, oxi.x), bx1 = fmaf(n1.y, inv.x, oxi.x);
            const float by0 = fmaf(n1.z, inv.y, oxi.y), by1 = fmaf(n1.w, inv.y, oxi.y);
            const float bz0 = fmaf(n2.z, inv.z, oxi.z), bz1 = fmaf(n2.w, inv.z, oxi.z);
            const float a0 = fmaxf(fmaxf(fmaxf(fminf(ax0, ax1), fminf(ay0, ay1)), fminf(az0, az1)), 0.0f);
            const float a1 = fminf(fminf(fminf(fmaxf(ax0, ax1), fmaxf(ay0, ay1)), fmaxf(az0, az1)), t);
            const float b0 = fmaxf(fmaxf(fmaxf(fminf(bx0, bx1), fminf(by0, by1)), fminf(bz0, bz1)), 0.0f);
            const float b1 = fminf(fminf(fminf(fmaxf(bx0, bx1), fmaxf(by0, by1)), fmaxf(bz0, bz1)), t);
            const bool h0 = a0 <= a1, h1 = b0 <= b1;
            const bool c1first = h1 && (a0 > b0);
            if (h0 && h1) push(c1first ? n3.x : n3.y);
            next = (h0 || h1) ? ((c1first || !h0) ? n3.y : n3.x) : POP;
        } else if (n3.x == BVH_INSTANCE_MARK) {
            next = POP;
            if (r.mask != n3.z) {   // RR_RAY_MASK at the shape (skiplinks.cl:225-230)
                cr.o = xfPoint(n0, n1, n2, r.o);
                cr.d = xfVector(n0, n1, n2, r.d);
                inv = safeInvDir(cr.d);
                oxi = -cr.o * inv;
                inst = node;
                push(RESTORE);
                next = n3.y;
            }
        } else {
            next = POP;
            const float th = triHit(cr, n0, n1, n2, t);
            if (th < t) {
                t = th;
                hit = node;
                hinst = inst;
                if (ANY) next = DONE;
            }
        }
        if (next == POP) {
            next = pop();
            if (next == RESTORE) {   // back to the top level (skiplinks.cl:287-297)
                cr = r;
                inv = winv;
                oxi = woxi;
                inst = -1;
                next = pop();
            }
        }
        node = next;
    }
    tHit = t;
    hitInst = hinst;
    return hit;
}

// Closest-hit record through an instance: the object-space ray is recomputed from the instance
// rows (same arithmetic as during traversal), barycentrics in object space as the reference.
MCRT_DEV float4 closestRecord2L(const float4* __restrict__ nodes, const TraceRay& r, int tri, int inst, float t) {
    if (tri < 0) return make_float4(0.f, 0.f, __int_as_float(-1), __int_as_float(-1));
    const float4 m0 = nodes[4 * inst], m1 = nodes[4 * inst + 1], m2 = nodes[4 * inst + 2];
    const int shape = reinterpret_cast<const int4*>(&nodes[4 * inst + 3])->z;
    TraceRay cr = r;
    cr.o = xfPoint(m0, m1, m2, r.o);
    cr.d = xfVector(m0, m1, m2, r.d);
    const float4 A = nodes[4 * tri], E1 = nodes[4 * tri + 1], E2 = nodes[4 * tri + 2];
    const f3 p = cr.o + t * cr.d;
    const f2 uv = triBary(p, A, E1, E2);
    return make_float4(uv.x, uv.y, __int_as_float(shape), E1.w);
}

// Closest / any hit over the scene's record layout (LAY; LAY_TWO_LEVEL: RR's IntersectorTwoLevel).
template <int LAY>
MCRT_DEV float4 traceClosest(const TraceCtx& c, const TraceRay& r, uint32_t* stk, uint32_t* spill, float& t) {
    if constexpr (LAY == LAY_TWO_LEVEL) {
        int inst;
        const int tri = traverse2L<false>(c.nodes, r, stk, spill, c.spillCap, c.overflow, t, inst);
        return closestRecord2L(c.nodes, r, tri, inst, t);
    } else {
        const int tri = traverse<false, LAY>(c, r, stk, spill, t);
        return closestRecord(c.nodes, r, tri, t);   // leaf slots are the same in both flat layouts
    }
}
template <int LAY>
MCRT_DEV bool traceAny(const TraceCtx& c, const TraceRay& r, uint32_t* stk, uint32_t* spill) {
    float t;
    if constexpr (LAY == LAY_TWO_LEVEL) {
        int inst;
        return traverse2L<true>(c.nodes, r, stk, spill, c.spillCap, c.overflow, t, inst) >= 0;
    } else {
        return traverse<true, LAY>(c, r, stk, spill, t) >= 0;
    }
}

// XCD-aware workgroup order for the traversal launches.  Workgroups are dealt round-robin to the
// 8 XCDs (block b runs on the XCD of b % 8, MI355X_MICROARCH "Workgroup dispatch"), so in
// launch order every XCD's 4 MB L2 would see rays from the whole image.  xcdRemap turns the
// physical block index `rel` of a section of S blocks into a logical one such that each XCD
// walks contiguous runs of MCRT_XCD_SEG logical blocks (camera tiles / queue slices, which are
// spatially coherent): the rays in flight on one XCD then share BVH nodes.  Runs of SEG blocks
// are dealt to the XCDs in turn (XCD k gets runs k, k+8, ...), which keeps the per-XCD load
// balanced across the image; the tail of < 8*SEG blocks is split in 8 contiguous parts.
// A bijection on [0, S); SEG = 0 is the identity.
#define MCRT_XCD_SEG 128
MCRT_DEV int xcdRemap(int rel, int S) {
    if (MCRT_XCD_SEG <= 0) return rel;
    constexpr int R = 8 * MCRT_XCD_SEG;
    const int round = rel / R, base = round * R;
    const int w = rel - base;
    const int xr = w & 7, pos = w >> 3;
    if (base + R <= S) return base + xr * MCRT_XCD_SEG + pos;
    const int T = S - base, q = T >> 3, rm = T & 7;   // partial round: 8 contiguous parts
    return base + xr * q + min(xr, rm) + pos;
}

// Per-ray spill column: rays are grouped 64 to a wave; lane l of wave w owns entries
// spill[(w * spillCap + k) * 64 + l], k < spillCap (coalesced across the wave).
MCRT_DEV uint32_t* raySpill(const TraceCtx& c, int wave, int lane) {
    return c.spill + (size_t)wave * 64 * c.spillCap + lane;
}


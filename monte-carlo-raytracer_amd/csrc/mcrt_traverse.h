// mcrt_traverse.h -- Bvh2 traversal shared by the path-tracing and BDPT kernels.
// (Moved out of mcrt_kernels.hip; see there for the launch structure.)
#pragma once
#include "mcrt_device.h"
#include "mcrt_internal.h"

// ---------------------------------------------------------------------------
// traversal
// ---------------------------------------------------------------------------
#define STACK_LDS 16

// Node-record layouts of the traversal kernels' template parameter LAY (TraceCtx::twoLevel): each
// layout gets its own kernel instantiation, so a kernel's register budget is that of the one loop
// it runs.
#define LAY_PLAIN 0       // mcrt_bvh.cpp records, traverseOct (and traversePacket)
#define LAY_QUANT 1       // the same tree's compact records (TraceCtx::qnodes), traverseQOct
#define LAY_TWO_LEVEL 3   // mcrt_bvh2l.cpp records, traverse2L
template <typename K>
inline K pickLayout(const TraceCtx& c, K twoLevel, K plain) {
    return c.twoLevel ? twoLevel : plain;
}
template <typename K>
inline K pickLayout(const TraceCtx& c, K twoLevel, K quant, K plain) {
    return c.twoLevel ? twoLevel : c.qnodes ? quant : plain;
}

// Diagnostics (TraceCtx::waveClock): the wave's (start, end) of the constant 100-MHz clock into
// clk[2 * block], one store per wave; the end is taken where the wave has left its traversal loop,
// so it is the wave's, not lane 0's
MCRT_DEV uint32_t waveClockNow() { return (uint32_t)__builtin_amdgcn_s_memrealtime(); }
MCRT_DEV void waveClockStore(uint32_t* clk, uint32_t t0) {
    if (clk && (threadIdx.x & 63) == 0) {
        clk[2 * blockIdx.x] = t0;
        clk[2 * blockIdx.x + 1] = waveClockNow();
    }
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
// Wave-packet traversal (closest hit, plain records) for coherent camera rays.
//
// The 64 lanes of a wave walk ONE node at a time: the node index and the lane mask are wave-
// uniform, so the 64-B record comes through the scalar cache (s_load, no vector-memory address
// work) and every step runs one path (internal or leaf) instead of both.  At an internal node each
// lane in the mask tests both child boxes with its own ray and its own closest t, exactly as
// traverseOct does; the wave descends into a child if any lane hits it, carrying the mask of the
// lanes that do, and defers the other child (with its mask) on a per-wave stack.  When lanes
// hit both children the wave goes first where most of them would (nearer child first per ray).
// So every lane tests exactly the nodes whose box it hit at the parent -- the per-ray traversal's
// rule -- and the closest hit is the same; only the ORDER of a lane's leaves can differ from
// nearer-first, which matters for exactly-equal t (a tie) alone, as for any other visit order.
// ---------------------------------------------------------------------------
// The lane state lives in VGPRs: the current mask is a per-lane flag, stack entry k's node is lane
// k of one VGPR (a pop is one v_readlane with the wave-uniform stack pointer) and its mask bit k of
// a per-lane 64-bit field, so the mask arithmetic runs on the vector units; the scalar unit (ONE
// per CU, shared by its four SIMDs: MI355X_MICROARCH "CU") keeps the node, the stack pointer and
// the wave-level decisions only.  (With 64-bit SGPR masks the camera launch was scalar-bound: SALU
// busy 0.85, profiles/pmc_latest.json round 5; this layout halves the scalar instructions of an
// internal step, profiles/r05/ab/README.txt item 12.)  A level pushes at most 2 entries, so a tree
// of depth D (leaves at level D) needs 2 D entries: the host takes this path for 2 D <= MCRT_PK_STACK
// = 64 (mcrt_capi.cpp finish_accel).
typedef float __attribute__((ext_vector_type(4))) PkV4;
typedef const __attribute__((address_space(4))) PkV4* PkNodes;   // uniform loads -> s_load
static_assert(MCRT_PK_STACK == 64, "the packet stack is one VGPR lane per entry");
MCRT_DEV float4 pkLoad(PkNodes p, int i) {
    const PkV4 v = p[i];
    return make_float4(v.x, v.y, v.z, v.w);
}

// triHit (RR common.cl:177-218) without branches: the same arithmetic, the early outs one final
// select, so a packet's leaf step costs no exec-mask bookkeeping.  SEL (the any-hit packets of the
// bounce-0 shadow rays): each early out a select of tmax kept in a VGPR (the asm barrier stops the
// selects from merging into one OR of lane masks), so no scalar mask arithmetic either
// (k_shadow_extend -4.6 %; the closest-hit camera packets are 2 % faster with the OR-ed lane
// masks: profiles/r05/ab/README.txt item 12).
template <bool SEL = true>
MCRT_DEV float triHitSel(const TraceRay& r, float4 A, float4 E1, float4 E2, float tmax) {
    const f3 e1 = ld3(E1), e2 = ld3(E2);
    const f3 s1 = cl_cross(r.d, e2);
    const float denom = cl_dot(s1, e1);
    const float invd = __builtin_amdgcn_rcpf(denom);
    const f3 d = r.o - ld3(A);
    const float b1 = cl_dot(d, s1) * invd;
    const f3 s2 = cl_cross(d, e1);
    const float b2 = cl_dot(r.d, s2) * invd;
    float temp = cl_dot(e2, s2) * invd;
    __asm__ volatile("" : "+v"(temp));   // computed by every lane: no exec-mask branch around it
    if constexpr (!SEL) {
        const bool miss = denom == 0.f || b1 < 0.f || b1 > 1.f || b2 < 0.f || b1 + b2 > 1.f || temp < 0.f || temp > tmax;
        return miss ? tmax : temp;
    }
    float res = temp;
    auto out = [&](bool miss) {
        res = miss ? tmax : res;
        __asm__ volatile("" : "+v"(res));
    };
    out(denom == 0.f);
    out(b1 < 0.f);
    out(b1 > 1.f);
    out(b2 < 0.f);
    out(b1 + b2 > 1.f);
    out(temp < 0.f);
    out(temp > tmax);
    return res;
}

// min(x, y, z, tc) as v_min_f32 + v_min3_f32: the same value as the fminf chain (the hardware min
// returns the other operand for a quiet NaN, and no operand here is a signalling NaN), without the
// v_max canonicalisation of the loop-carried tc the compiler adds to every node step for fminf.
MCRT_DEV float minFar(float x, float y, float z, float tc) {
    float m, r;
    asm("v_min_f32 %0, %1, %2" : "=v"(m) : "v"(z), "v"(tc));
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(y), "v"(m));
    return r;
}

template <bool ANY, int OCT>
MCRT_DEV int traversePacketOct(const float4* __restrict__ nodes, const TraceRay& r, f3 inv, bool valid,
                                float& tHit) {
    const PkNodes cn = (PkNodes)(const void*)nodes;
    const f3 oxi = -r.o * inv;   // intersect_bvh2_lds.cl:91
    const int lane = (int)__lane_id();
    uint32_t bitsLo = 0, bitsHi = 0;   // stack entry k's mask: bit k
    int stN = 0;                       // stack entry k's node: lane k
    float t = r.tmax;
    int hit = -1;
    uint32_t act = valid ? 1u : 0u;
    uint32_t alive = act;   // any hit: lanes still without a hit
    uint32_t node = 0;
    int sp = 0;
    while (true) {
        if (ANY) act &= alive;
        if (__ballot(act != 0u) != 0) {
            const PkNodes q = (PkNodes)((const char __attribute__((address_space(4)))*)cn + (uint32_t)(node << 6));
            const float4 n0 = pkLoad(q, 0), n1 = pkLoad(q, 1), n2 = pkLoad(q, 2), n3f = pkLoad(q, 3);
            const int c0 = __builtin_amdgcn_readfirstlane(__float_as_int(n3f.x));
            const int c1 = __builtin_amdgcn_readfirstlane(__float_as_int(n3f.y));
            if (c0 >= 0) {
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
                    a1 = minFar(axf, ayf, azf, t);
                    b0 = fmaxf(fmaxf(bxn, byn), fmaxf(bzn, 0.0f));
                    b1 = minFar(bxf, byf, bzf, t);
                } else {   // RR intersect_bvh2_lds.cl:54-63 (fast_intersect_bbox2)
                    const float ax0 = fmaf(n0.x, inv.x, oxi.x), ax1 = fmaf(n0.y, inv.x, oxi.x);
                    const float ay0 = fmaf(n0.z, inv.y, oxi.y), ay1 = fmaf(n0.w, inv.y, oxi.y);
                    const float az0 = fmaf(n2.x, inv.z, oxi.z), az1 = fmaf(n2.y, inv.z, oxi.z);
                    const float bx0 = fmaf(n1.x, inv.x, oxi.x), bx1 = fmaf(n1.y, inv.x, oxi.x);
                    const float by0 = fmaf(n1.z, inv.y, oxi.y), by1 = fmaf(n1.w, inv.y, oxi.y);
                    const float bz0 = fmaf(n2.z, inv.z, oxi.z), bz1 = fmaf(n2.w, inv.z, oxi.z);
                    a0 = fmaxf(fmaxf(fmaxf(fminf(ax0, ax1), fminf(ay0, ay1)), fminf(az0, az1)), 0.0f);
                    a1 = minFar(fmaxf(ax0, ax1), fmaxf(ay0, ay1), fmaxf(az0, az1), t);
                    b0 = fmaxf(fmaxf(fmaxf(fminf(bx0, bx1), fminf(by0, by1)), fminf(bz0, bz1)), 0.0f);
                    b1 = minFar(fmaxf(bx0, bx1), fmaxf(by0, by1), fmaxf(bz0, bz1), t);
                }
                // lanes hitting both children go to the nearer one first: the right one where
                // a0 > b0 (intersect_bvh2_lds.cl:128-141).  The wave takes the majority's first
                // child F with every lane that hits F and prefers it (or hits F only), then the
                // other child S with every lane that hits S, then F AGAIN with the lanes that hit
                // both but preferred S: so each lane visits its two children in its own order, and
                // every lane's sequence of tests -- hence its t at every culling test and the
                // first of equal-t hits it keeps -- is exactly traverseOct's.  (Any hit: the
                // answer does not depend on the order, so no third pass.)
                const uint32_t hL = a0 <= a1 ? act : 0u, hR = b0 <= b1 ? act : 0u;
                const uint32_t hB = hL & hR;
                const uint32_t hP = a0 > b0 ? hB : 0u;   // prefers the right child
                const uint64_t mL = __ballot(hL != 0u), mB = __ballot(hB != 0u), mP = __ballot(hP != 0u);
                const bool goR = (mL == 0) | (2 * __popcll(mP) > __popcll(mB));
                const uint32_t inF = goR ? hR : hL, inS = goR ? hL : hR;
                const uint32_t late = ANY ? 0u : (goR ? hB & ~hP : hP);
                const uint32_t cF = (uint32_t)(goR ? c1 : c0), cS = (uint32_t)(goR ? c0 : c1);
                auto push = [&](uint32_t nodeK, uint32_t in) {
                    const uint32_t m = 1u << (sp & 31), v = in != 0u ? m : 0u;
                    if (sp < 32) bitsLo = (bitsLo & ~m) | v; else bitsHi = (bitsHi & ~m) | v;
                    stN = lane == sp ? (int)nodeK : stN;
                    ++sp;
                };
                if (!ANY && __ballot(late != 0u) != 0) push(cF, late);
                if (__ballot(inS != 0u) != 0) push(cS, inS);
                node = cF;
                act = inF & ~late;
            } else {
                // every lane computes, the active lanes that pass RR_RAY_MASK take the hit
                // t for the lanes outside the mask or whose RR_RAY_MASK matches the leaf's shape
                float th = triHitSel<ANY>(r, n0, n1, n2, t);
                th = act != 0u ? th : t;
                __asm__ volatile("" : "+v"(th));
                th = r.mask != __float_as_int(n0.w) ? th : t;
                const bool take = th < t;
                hit = take ? (int)node : hit;
                t = take ? th : t;
                if (ANY) alive = take ? 0u : alive;   // a lane with a hit is done (next = DONE)
                act = 0u;
            }
        }
        if (ANY && __ballot(alive != 0u) == 0) break;
        if (__ballot(act != 0u) == 0) {
            if (sp == 0) break;
            --sp;
            node = (uint32_t)__builtin_amdgcn_readlane(stN, sp);
            act = ((sp < 32 ? bitsLo : bitsHi) >> (sp & 31)) & 1u;
        }
    }
    tHit = t;
    return hit;
}

// Closest (ANY = false) or any hit of the wave's rays over plain records; lanes with valid = false take
// no part.  Returns the hit leaf's node index or -1 per lane.
template <bool ANY>
MCRT_DEV int traversePacket(const float4* __restrict__ nodes, const TraceRay& r, bool valid, float& tHit) {
    const f3 inv = safeInvDir(r.d);
    const int oct = (int)(__float_as_uint(inv.x) >> 31) | (int)((__float_as_uint(inv.y) >> 31) << 1) |
                    (int)((__float_as_uint(inv.z) >> 31) << 2);
    const uint64_t vm = __ballot(valid);
    const int first = vm ? (int)__builtin_ctzll(vm) : 0;
    const int oct0 = __builtin_amdgcn_readfirstlane(__shfl(oct, first));
    if (__all(!valid || oct == oct0)) {
        switch (oct0) {
            case 0: return traversePacketOct<ANY, 0>(nodes, r, inv, valid, tHit);
            case 1: return traversePacketOct<ANY, 1>(nodes, r, inv, valid, tHit);
            case 2: return traversePacketOct<ANY, 2>(nodes, r, inv, valid, tHit);
            case 3: return traversePacketOct<ANY, 3>(nodes, r, inv, valid, tHit);
            case 4: return traversePacketOct<ANY, 4>(nodes, r, inv, valid, tHit);
            case 5: return traversePacketOct<ANY, 5>(nodes, r, inv, valid, tHit);
            case 6: return traversePacketOct<ANY, 6>(nodes, r, inv, valid, tHit);
            case 7: return traversePacketOct<ANY, 7>(nodes, r, inv, valid, tHit);
            default: break;
        }
    }
    return traversePacketOct<ANY, -1>(nodes, r, inv, valid, tHit);
}

template <bool ANY, int LAY>
MCRT_DEV int traverse(const TraceCtx& c, const TraceRay& r, uint32_t* stk, uint32_t* spill, float& tHit) {
    const f3 inv = safeInvDir(r.d);
#define MCRT_TRAV_CALL(OCT) return traverseOct<ANY, OCT>(c.nodes, r, inv, stk, spill, c.spillCap, c.overflow, tHit)
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

// ---------------------------------------------------------------------------
// Compact records (TraceCtx::qnodes, built by k_qnodes_convert from the 64-B records of a
// depth-first tree): the per-ray walks fetch 32 B per internal node and 48 B per leaf instead of
// 64 B -- two or three 16-B loads instead of four.  The traversal launches are bound by the vector-
// memory pipeline (TA busy 0.94, one cache access per 16-B lane load), not by arithmetic.
//   internal (32 B): (origin.xyz, right child ref) | (x bytes, y bytes, z bytes, meta): for axis a
//     the bytes are (child 0 lo, child 0 hi, child 1 lo, child 1 hi) and a bound decodes as
//     fmaf(q, s_a, origin_a), s_a = qScales(meta) (2^(e_a - 127) times a mantissa, qScales); meta =
//     e_x | e_y << 9 | e_z << 18 | leaf(child 0) << 27.  The left child is the next record
//     (depth-first order, ref + 4); the right child's ref (16-B offset << 1 | leaf bit) is stored.
//   leaf (48 B): (v0 | shape id), (v1 - v0 | prim id), (v2 - v0 | 64-B record index, bit 31 set when
//     the leaf's exact box must come from its parent's 64-B record).
// Why the answers are the 64-B walk's (RR intersect_bvh2_lds.cl:107-178):
//   * every decoded bound is rounded outward (the converter checks each fmaf decode against the
//     exact bound), and fma rounds monotonically, so a decoded box's slab interval contains the
//     exact box's: every internal test the exact walk passes, this walk passes;
//   * at a leaf, for a triangle that would count (its distance within the culling distance), the
//     EXACT box test the 64-B walk runs at the parent (the box is min/max of v0, v0 + e1, v0 + e2,
//     which the converter checked against the box the parent's 64-B record stores, else bit 31
//     sends the lane to that record);
//   * any hit: the culling distance is the ray's tmax throughout, so every box decision is the
//     exact walk's whatever the order, and the answer (hit or not) is the exact walk's;
//   * closest hit: the reference's answer is the nearest hit unless a triangle's box entry and its
//     distance, computed differently, disagree: a triangle X hit at t_X whose leaf box enters at
//     e_X > t_X is culled by the reference if it has already found a hit between t_X and e_X, so
//     its answer depends on its visit order, which the outward boxes change.  A walk is repeated
//     on the exact records (traceClosest<LAY_QUANT>, the reference's order) when its final
//     distance carries a mark:
//       - a near tie: a hit within 2^-18 of the current closest (either side); the culling
//         distance is widened by the same margin once a hit exists, so such a candidate is tested;
//       - an order-dependent pair: a triangle hit nearer than the current closest whose exact box
//         test fails (the walk holds a hit between its t and e) is taken provisionally with the
//         mark; an accepted triangle whose entry e exceeds its t by more than the margin widens the
//         culling distance to e, so any other hit in (t, e] is met and marks a near tie.
//     What stays open is an order-dependent triangle whose whole subtree the compact walk culls
//     above the leaf (its ancestors' entries beyond the culling distance):
//     tests/test_tie_premise_cpu.py enumerates every order-dependent pair of hits beyond the margin
//     -- none on the headline scene at 1080p; on the same scene moved 1000 units from the origin, 1
//     ray in 10^5 (a ray leaving a surface nearly parallel to it, whose slab values carry errors of
//     |o / d| ulp) -- and the GPU tests compare both scenes' frames with the exact walk's bit for
//     bit (test_gpu_quant_nodes.py).
// ---------------------------------------------------------------------------
#define QREF_DONE 0xffffffffu
#define QTIE_HI (1.0f + 0x1.0p-18f)
#define QTIE_LO (1.0f - 0x1.0p-18f)

// The three steps of an internal record from its meta word in one shift each: exponent byte e_k
// at bits 9k..9k+7 with a zero bit above it, so meta << (23 - 9k) puts e_k in the float's exponent
// and a clear sign bit; the fields below land in the mantissa (x: none; y: 1 + e_x / 512, z: 1 +
// e_y / 512 + e_x / 2^18, about 1.24 for exponents near 127), which the converter (k_qnodes_convert)
// quantises with -- and takes one exponent less where that still covers the extent -- so the
// decoded bounds stay outward.
struct QScales { float x, y, z; };
MCRT_DEV QScales qScales(uint32_t meta) {
    return QScales{__uint_as_float(meta << 23), __uint_as_float(meta << 14), __uint_as_float(meta << 5)};
}
MCRT_DEV float qByte(uint32_t w, int k) { return (float)((w >> (8 * k)) & 0xffu); }

// RR common.cl:177-218 without the tmax test: the hit distance or +inf (the caller compares)
MCRT_DEV float triRaw(const TraceRay& r, float4 A, float4 E1, float4 E2) {
    const f3 e1 = ld3(E1), e2 = ld3(E2);
    const f3 s1 = cl_cross(r.d, e2);
    const float denom = cl_dot(s1, e1);
    if (denom == 0.f) return __builtin_inff();
    const float invd = __builtin_amdgcn_rcpf(denom);
    const f3 d = r.o - ld3(A);
    const float b1 = cl_dot(d, s1) * invd;
    const f3 s2 = cl_cross(d, e1);
    const float b2 = cl_dot(r.d, s2) * invd;
    const float temp = cl_dot(e2, s2) * invd;
    if (b1 < 0.f || b1 > 1.f || b2 < 0.f || b1 + b2 > 1.f || temp < 0.f) return __builtin_inff();
    return temp;
}

// fast_intersect_bbox2 (intersect_bvh2_lds.cl:54-63) of one box, entry <= exit; `entry` = the
// clamped entry distance t0 (the compact walk's order-dependence check at a leaf)
template <int OCT>
MCRT_DEV bool slabHit(f3 lo, f3 hi, f3 inv, f3 oxi, float t, float& entry) {
    if constexpr (OCT >= 0) {
        constexpr bool SX = (OCT & 1) != 0, SY = (OCT & 2) != 0, SZ = (OCT & 4) != 0;
        const float xn = fmaf(SX ? hi.x : lo.x, inv.x, oxi.x), xf = fmaf(SX ? lo.x : hi.x, inv.x, oxi.x);
        const float yn = fmaf(SY ? hi.y : lo.y, inv.y, oxi.y), yf = fmaf(SY ? lo.y : hi.y, inv.y, oxi.y);
        const float zn = fmaf(SZ ? hi.z : lo.z, inv.z, oxi.z), zf = fmaf(SZ ? lo.z : hi.z, inv.z, oxi.z);
        entry = fmaxf(fmaxf(xn, yn), fmaxf(zn, 0.0f));
        return entry <= fminf(fminf(xf, yf), fminf(zf, t));
    } else {
        const float x0 = fmaf(lo.x, inv.x, oxi.x), x1 = fmaf(hi.x, inv.x, oxi.x);
        const float y0 = fmaf(lo.y, inv.y, oxi.y), y1 = fmaf(hi.y, inv.y, oxi.y);
        const float z0 = fmaf(lo.z, inv.z, oxi.z), z1 = fmaf(hi.z, inv.z, oxi.z);
        entry = fmaxf(fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1)), 0.0f);
        return entry <= fminf(fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1)), t);
    }
}

// The exact box of 64-B leaf `leaf` as its parent's record stores it (the rare leaves whose box the
// compact record cannot reproduce; the root leaf has no box test, as in the exact walk)
MCRT_DEV bool parentBoxHit(const TraceCtx& c, uint32_t leaf, f3 inv, f3 oxi, float t, float& entry) {
    const int par = reinterpret_cast<const int4*>(&c.nodes[4 * leaf + 3])->y;
    entry = 0.0f;
    if (par < 0) return true;
    const float4 p0 = c.nodes[4 * par], p1 = c.nodes[4 * par + 1], p2 = c.nodes[4 * par + 2];
    const bool right = reinterpret_cast<const int4*>(&c.nodes[4 * par + 3])->y == (int)leaf;
    const f3 lo = right ? f3{p1.x, p1.z, p2.z} : f3{p0.x, p0.z, p2.x};
    const f3 hi = right ? f3{p1.y, p1.w, p2.w} : f3{p0.y, p0.w, p2.y};
    return slabHit<-1>(lo, hi, inv, oxi, t, entry);
}

// The loop state of a compact walk: the next record, the hit so far and the stack (LDS entries
// stk[0..sp), spill entries [0, spillTop) in the ray's spill column).  A walk with a stop rule
// (CAP) leaves the loop with ref != QREF_DONE once its wave has taken at least `cap` steps and at
// most `capLanes` of its lanes are still walking; the state then resumes it exactly
// (mcrt_kernels.hip k_walk_resume), so the visits, hence the answer, are those of one uncut walk.
struct QWalk {
    uint32_t ref;
    float t, tc, tieT;
    int hit, sp, spillTop;
};
MCRT_DEV QWalk qwalkStart(const TraceCtx& c, const TraceRay& r, uint32_t* stk) {
    stk[0] = QREF_DONE;
    return QWalk{c.qroot, r.tmax, r.tmax, -1.0f, -1, 1, 0};
}

template <bool ANY, int OCT, bool CAP = false>
MCRT_DEV void qwalk(const TraceCtx& c, const TraceRay& r, f3 inv, uint32_t* stk, uint32_t* spill, QWalk& w,
                    int cap = 0, int capLanes = 64) {
    const char* __restrict__ base = reinterpret_cast<const char*>(c.qnodes);
    const f3 oxi = -r.o * inv;   // intersect_bvh2_lds.cl:91
    // OCT -2 (lanes of any octants): per axis a byte permutation that puts each child's NEAR bound
    // byte first -- (lo0, hi0, lo1, hi1) as is for a positive inverse direction, (hi0, lo0, hi1, lo1)
    // for a negative one -- so every lane runs the octant-specialised slab test of octant 0 on its
    // own bytes: the same operations, hence the same values, as traverseQOct<OCT> for its octant
    // (one v_perm per axis instead of the generic test's min / max pairs)
    const uint32_t selX = (__float_as_uint(inv.x) >> 31) ? 0x02030001u : 0x03020100u;
    const uint32_t selY = (__float_as_uint(inv.y) >> 31) ? 0x02030001u : 0x03020100u;
    const uint32_t selZ = (__float_as_uint(inv.z) >> 31) ? 0x02030001u : 0x03020100u;
    float t = w.t, tc = w.tc, tieT = w.tieT;
    int hit = w.hit;
    uint32_t ref = w.ref;
    int sp = w.sp, spillTop = w.spillTop;
    constexpr uint32_t POP = QREF_DONE - 1;
    int steps = 0;   // the wave's steps: every active lane takes each one, so the count is uniform
    while (ref != QREF_DONE) {
        if constexpr (CAP) {   // wave-uniform: the step count and the active-lane count
            if (steps >= cap && (int)__popcll(__ballot(1)) <= capLanes) break;
            ++steps;
        }
        const float4* p = reinterpret_cast<const float4*>(base + (size_t)(ref >> 1) * 16);
        const float4 a = p[0];
        const uint4 b = *reinterpret_cast<const uint4*>(p + 1);
        // a leaf's third piece in the same round trip (the leaf bit is in the reference, known
        // before the fetch): without this the compiler issues it after the branch, a second
        // dependent fetch on every leaf visit
        float4 e2;   // only a leaf reads it: no zeroing for the internal nodes
        asm("" : "=v"(e2.x), "=v"(e2.y), "=v"(e2.z), "=v"(e2.w));
        if (ref & 1u) e2 = p[2];
        asm volatile("" ::"v"(e2.w), "v"(b.w));
        uint32_t next;
        if (!(ref & 1u)) {
            const QScales qs = qScales(b.w);
            const float sx = qs.x, sy = qs.y, sz = qs.z;
            uint4 bq = b;
            if constexpr (OCT == -2) {
                bq.x = __builtin_amdgcn_perm(b.x, b.x, selX);
                bq.y = __builtin_amdgcn_perm(b.y, b.y, selY);
                bq.z = __builtin_amdgcn_perm(b.z, b.z, selZ);
            }
            const f3 lo0 = f3{fmaf(qByte(bq.x, 0), sx, a.x), fmaf(qByte(bq.y, 0), sy, a.y), fmaf(qByte(bq.z, 0), sz, a.z)};
            const f3 hi0 = f3{fmaf(qByte(bq.x, 1), sx, a.x), fmaf(qByte(bq.y, 1), sy, a.y), fmaf(qByte(bq.z, 1), sz, a.z)};
            const f3 lo1 = f3{fmaf(qByte(bq.x, 2), sx, a.x), fmaf(qByte(bq.y, 2), sy, a.y), fmaf(qByte(bq.z, 2), sz, a.z)};
            const f3 hi1 = f3{fmaf(qByte(bq.x, 3), sx, a.x), fmaf(qByte(bq.y, 3), sy, a.y), fmaf(qByte(bq.z, 3), sz, a.z)};
            float a0, a1, b0, b1;
            if constexpr (OCT >= 0 || OCT == -2) {   // -2: lo* / hi* are each lane's near / far bounds
                constexpr int O = OCT >= 0 ? OCT : 0;
                constexpr bool SX = (O & 1) != 0, SY = (O & 2) != 0, SZ = (O & 4) != 0;
                const float axn = fmaf(SX ? hi0.x : lo0.x, inv.x, oxi.x), axf = fmaf(SX ? lo0.x : hi0.x, inv.x, oxi.x);
                const float ayn = fmaf(SY ? hi0.y : lo0.y, inv.y, oxi.y), ayf = fmaf(SY ? lo0.y : hi0.y, inv.y, oxi.y);
                const float azn = fmaf(SZ ? hi0.z : lo0.z, inv.z, oxi.z), azf = fmaf(SZ ? lo0.z : hi0.z, inv.z, oxi.z);
                const float bxn = fmaf(SX ? hi1.x : lo1.x, inv.x, oxi.x), bxf = fmaf(SX ? lo1.x : hi1.x, inv.x, oxi.x);
                const float byn = fmaf(SY ? hi1.y : lo1.y, inv.y, oxi.y), byf = fmaf(SY ? lo1.y : hi1.y, inv.y, oxi.y);
                const float bzn = fmaf(SZ ? hi1.z : lo1.z, inv.z, oxi.z), bzf = fmaf(SZ ? lo1.z : hi1.z, inv.z, oxi.z);
                a0 = fmaxf(fmaxf(axn, ayn), fmaxf(azn, 0.0f));
                a1 = minFar(axf, ayf, azf, tc);
                b0 = fmaxf(fmaxf(bxn, byn), fmaxf(bzn, 0.0f));
                b1 = minFar(bxf, byf, bzf, tc);
            } else {
                const float ax0 = fmaf(lo0.x, inv.x, oxi.x), ax1 = fmaf(hi0.x, inv.x, oxi.x);
                const float ay0 = fmaf(lo0.y, inv.y, oxi.y), ay1 = fmaf(hi0.y, inv.y, oxi.y);
                const float az0 = fmaf(lo0.z, inv.z, oxi.z), az1 = fmaf(hi0.z, inv.z, oxi.z);
                const float bx0 = fmaf(lo1.x, inv.x, oxi.x), bx1 = fmaf(hi1.x, inv.x, oxi.x);
                const float by0 = fmaf(lo1.y, inv.y, oxi.y), by1 = fmaf(hi1.y, inv.y, oxi.y);
                const float bz0 = fmaf(lo1.z, inv.z, oxi.z), bz1 = fmaf(hi1.z, inv.z, oxi.z);
                a0 = fmaxf(fmaxf(fmaxf(fminf(ax0, ax1), fminf(ay0, ay1)), fminf(az0, az1)), 0.0f);
                a1 = minFar(fmaxf(ax0, ax1), fmaxf(ay0, ay1), fmaxf(az0, az1), tc);
                b0 = fmaxf(fmaxf(fmaxf(fminf(bx0, bx1), fminf(by0, by1)), fminf(bz0, bz1)), 0.0f);
                b1 = minFar(fmaxf(bx0, bx1), fmaxf(by0, by1), fmaxf(bz0, bz1), tc);
            }
            const uint32_t cl = ref + 4u + ((b.w >> 27) & 1u);   // the next record (+32 B), its leaf bit
            const uint32_t cr = __float_as_uint(a.w);            // the right child's reference
            const bool h0 = a0 <= a1, h1 = b0 <= b1;
            const bool c1first = h1 && (a0 > b0);   // intersect_bvh2_lds.cl:128-141
            if (h0 && h1) {   // defer the far child
                if (sp == STACK_LDS) {   // spill entries 1..15 (RR: intersect_bvh2_lds.cl:146-155)
                    if (spillTop + STACK_LDS - 1 <= c.spillCap) {
                        for (int k = 1; k < STACK_LDS; ++k) spill[(size_t)(spillTop + k - 1) * 64] = stk[k * 64];
                        spillTop += STACK_LDS - 1;
                    } else {
                        *c.overflow = 1;
                    }
                    sp = 1;
                }
                stk[sp * 64] = c1first ? cl : cr;
                ++sp;
            }
            next = (h0 || h1) ? ((c1first || !h0) ? cr : cl) : POP;
        } else {
            next = POP;
            const uint32_t w = __float_as_uint(e2.w);
            const float4 e1 = make_float4(__uint_as_float(b.x), __uint_as_float(b.y), __uint_as_float(b.z), 0.0f);
            // the triangle first: the exact box test (which the 64-B walk runs at the parent) only
            // matters for a triangle that would count, and most leaf visits miss
            const float th = r.mask != __float_as_int(a.w) ? triRaw(r, a, e1, e2) : __builtin_inff();   // RR_RAY_MASK
            if (th <= tc) {
                bool boxHit;
                float ent;
                if (w >> 31) {
                    boxHit = parentBoxHit(c, w & 0x7fffffffu, inv, oxi, tc, ent);
                } else {
                    const f3 v0 = ld3(a), v1 = v0 + ld3(e1), v2 = v0 + ld3(e2);
                    const f3 lo = f3{fminf(fminf(v0.x, v1.x), v2.x), fminf(fminf(v0.y, v1.y), v2.y),
                                     fminf(fminf(v0.z, v1.z), v2.z)};
                    const f3 hi = f3{fmaxf(fmaxf(v0.x, v1.x), v2.x), fmaxf(fmaxf(v0.y, v1.y), v2.y),
                                     fmaxf(fmaxf(v0.z, v1.z), v2.z)};
                    boxHit = slabHit<OCT>(lo, hi, inv, oxi, tc, ent);
                }
                // closest hit: a triangle X whose box entry e lies beyond its distance is ORDER-
                // DEPENDENT in the reference, which culls the leaf at its parent once it holds a hit
                // nearer than e (intersect_bvh2_lds.cl:128-141).  A nearer X whose box test fails
                // here (this walk already holds such a hit) is taken provisionally with the repeat
                // mark; an accepted X with e beyond the tie margin widens the culling distance to
                // e, so any hit in (t_X, e] is met and marks a near tie (tests/test_tie_premise_cpu.py)
                if (th < t && (boxHit || !ANY)) {
                    if (!ANY && (!boxHit || (hit >= 0 && th >= t * QTIE_LO))) tieT = th;
                    t = th;
                    tc = ANY ? th : (boxHit && ent > th * QTIE_HI ? ent : th) * QTIE_HI;
                    hit = (int)(w & 0x7fffffffu);
                    if (ANY) next = QREF_DONE;
                } else if (!ANY && hit >= 0) {   // t <= th <= tc: a near tie
                    tieT = t;
                }
            }
        }
        if (next == POP) {
            --sp;
            next = stk[sp * 64];
            if (next == QREF_DONE && spillTop > 0) {   // refill (intersect_bvh2_lds.cl:182-191)
                spillTop -= STACK_LDS - 1;
                for (int k = 1; k < STACK_LDS; ++k) stk[k * 64] = spill[(size_t)(spillTop + k - 1) * 64];
                sp = STACK_LDS - 1;
                next = stk[sp * 64];
            }
        }
        ref = next;
    }
    w = QWalk{ref, t, tc, tieT, hit, sp, spillTop};
}

// Returns the hit leaf's 64-B record index or -1; tie: a near tie at the final distance (closest hit).
template <bool ANY, int OCT>
MCRT_DEV int traverseQOct(const TraceCtx& c, const TraceRay& r, f3 inv, uint32_t* stk, uint32_t* spill,
                          float& tHit, bool& tie) {
    QWalk w = qwalkStart(c, r, stk);
    qwalk<ANY, OCT>(c, r, inv, stk, spill, w);
    tHit = w.t;
    tie = !ANY && w.hit >= 0 && w.tieT == w.t;
    return w.hit;
}

// The compact walk of one ray: every lane in the byte-permutation form (OCT -2), whatever the octants
// of its wave's rays.  Dispatching octant-uniform waves (41 % of the headline's extension waves) to
// the specialised instantiations and the rest to the generic min / max test cost 2 % more
// (profiles/r05/ab/README.txt item 17).
template <bool ANY>
MCRT_DEV int traverseQ(const TraceCtx& c, const TraceRay& r, uint32_t* stk, uint32_t* spill, float& tHit,
                       bool& tie) {
    return traverseQOct<ANY, -2>(c, r, safeInvDir(r.d), stk, spill, tHit, tie);
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
// Occluder hints for any-hit queries (plain records).  Before walking the tree a shadow ray tests
// ONE leaf named by a hint table -- the occluder the same pixel's bounce-0 shadow ray found in an
// earlier frame, or the last one found from the ray's origin cell -- and is occluded without a walk
// when both tests below pass, with the walk's own arithmetic:
//   * the leaf's triangle (triHit, t < tmax, RR_RAY_MASK);
//   * the leaf's box as its parent record stores it (fast_intersect_bbox2 with t = tmax).
// That answer is the reference's: every box on the root-to-leaf path contains the leaf's box
// (a node's box is the exact min/max union of its subtree's triangle boxes), and for a superset box
// each slab's fma(bound, 1/d, -o/d) interval contains the subset's (fma rounds monotonically), so
// the entry/exit test passes at every ancestor too.  The any-hit walk therefore reaches this leaf
// unless it stops earlier at another hit: occluded either way (intersect_bvh2_lds.cl:229-363 reports
// only hit / no hit).  Any table content is safe: the leaf and its parent link (k_leaf_parents:
// leaf record word 13) are checked against the current tree, a stale or empty entry is a miss.
// ---------------------------------------------------------------------------
MCRT_DEV bool hintOccludes(const TraceCtx& c, const TraceRay& r, uint32_t leaf) {
    if (leaf >= c.numNodes) return false;   // empty (0xffffffff) or stale
    const float4 A = c.nodes[4 * leaf], E1 = c.nodes[4 * leaf + 1], E2 = c.nodes[4 * leaf + 2];
    const int4 n3 = *reinterpret_cast<const int4*>(&c.nodes[4 * leaf + 3]);
    if (n3.x != -1 || r.mask == __float_as_int(A.w)) return false;
    if (!(triHit(r, A, E1, E2, r.tmax) < r.tmax)) return false;
    const int par = n3.y;
    if (par < 0) return leaf == 0;   // the root itself: the walk tests it without a box
    if ((uint32_t)par >= c.numNodes) return false;
    const float4 p0 = c.nodes[4 * par], p1 = c.nodes[4 * par + 1], p2 = c.nodes[4 * par + 2];
    const int4 p3 = *reinterpret_cast<const int4*>(&c.nodes[4 * par + 3]);
    const bool right = p3.y == (int)leaf;
    if (p3.x < 0 || (!right && p3.x != (int)leaf)) return false;
    const f3 inv = safeInvDir(r.d);
    const f3 oxi = -r.o * inv;   // intersect_bvh2_lds.cl:91
    const float x0 = fmaf(right ? p1.x : p0.x, inv.x, oxi.x), x1 = fmaf(right ? p1.y : p0.y, inv.x, oxi.x);
    const float y0 = fmaf(right ? p1.z : p0.z, inv.y, oxi.y), y1 = fmaf(right ? p1.w : p0.w, inv.y, oxi.y);
    const float z0 = fmaf(right ? p2.z : p2.x, inv.z, oxi.z), z1 = fmaf(right ? p2.w : p2.y, inv.z, oxi.z);
    const float b0 = fmaxf(fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1)), 0.0f);
    const float b1 = fminf(fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1)), r.tmax);
    return b0 <= b1;
}

// The hint table slot of a shadow ray: its path's pixel (bounce-0 rays of a TAA-jittered camera
// start on nearly the same surface point every frame) or its origin cell and direction octant
// (rays toward the same directional light from one cell are parallel and close).
MCRT_DEV uint32_t hintCellSlot(const TraceCtx& c, const TraceRay& r) {
    constexpr float G = (float)MCRT_HINT_GRID, g = G - 1.0f;
    const uint32_t cx = (uint32_t)fminf(fmaxf((r.o.x - c.hintLo[0]) * c.hintInvExt[0] * G, 0.0f), g);
    const uint32_t cy = (uint32_t)fminf(fmaxf((r.o.y - c.hintLo[1]) * c.hintInvExt[1] * G, 0.0f), g);
    const uint32_t cz = (uint32_t)fminf(fmaxf((r.o.z - c.hintLo[2]) * c.hintInvExt[2] * G, 0.0f), g);
    const uint32_t oct = (r.d.x < 0.f ? 1u : 0u) | (r.d.y < 0.f ? 2u : 0u) | (r.d.z < 0.f ? 4u : 0u);
    const uint32_t key = ((cz * MCRT_HINT_GRID + cy) * MCRT_HINT_GRID + cx) * 8u + oct;
    return (key * 2654435761u) >> (32 - MCRT_HINT_CELL_BITS) & c.hintMask;
}
MCRT_DEV uint32_t hintSlot(const TraceCtx& c, const TraceRay& r, int path) {
    return c.hintMode == MCRT_HINT_PIXEL ? (uint32_t)path % c.hintPixels : hintCellSlot(c, r);
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
    } else if constexpr (LAY == LAY_QUANT) {
        bool tie;
        int tri = traverseQ<false>(c, r, stk, spill, t, tie);
        if (tie) {   // a near tie at the final distance: the exact walk decides it (reference order)
            if (c.retraces) atomicAdd(c.retraces, 1);
            tri = traverse<false, LAY_PLAIN>(c, r, stk, spill, t);
        }
        return closestRecord(c.nodes, r, tri, t);
    } else {
        const int tri = traverse<false, LAY>(c, r, stk, spill, t);
        return closestRecord(c.nodes, r, tri, t);
    }
}
// The end of a closest-hit compact walk run as QWalk steps (traceClosest<LAY_QUANT>'s tail)
MCRT_DEV float4 qwalkClosest(const TraceCtx& c, const TraceRay& r, uint32_t* stk, uint32_t* spill, const QWalk& w) {
    float t = w.t;
    int tri = w.hit;
    if (w.hit >= 0 && w.tieT == w.t) {
        if (c.retraces) atomicAdd(c.retraces, 1);
        tri = traverse<false, LAY_PLAIN>(c, r, stk, spill, t);
    }
    return closestRecord(c.nodes, r, tri, t);
}
template <int LAY>
MCRT_DEV bool traceAny(const TraceCtx& c, const TraceRay& r, uint32_t* stk, uint32_t* spill) {
    float t;
    if constexpr (LAY == LAY_TWO_LEVEL) {
        int inst;
        return traverse2L<true>(c.nodes, r, stk, spill, c.spillCap, c.overflow, t, inst) >= 0;
    } else if constexpr (LAY == LAY_QUANT) {
        bool tie;
        return traverseQ<true>(c, r, stk, spill, t, tie) >= 0;
    } else {
        return traverse<true, LAY>(c, r, stk, spill, t) >= 0;
    }
}

// One atomic per wave: the lanes whose hint answered (mcrt_framebuffer_hint_counts).
MCRT_DEV void countHintHits(const TraceCtx& c, bool ok) {
    if (!c.hintHits) return;   // counters on only at mcrt_ctx_set_profiling(ctx, 2)
    const uint64_t m = __ballot(ok), act = __ballot(true);
    if (m != 0 && (int)__lane_id() == (int)__builtin_ctzll(act)) atomicAdd(c.hintHits, (int)__popcll(m));
}

// Any hit of one shadow / connection ray: first the occluder hint of its slot (c.hint, plain
// records; mcrt_traverse.h hintOccludes), then the walk, whose occluder becomes the slot's next hint.
template <int LAY>
MCRT_DEV bool shadowOccluded(const TraceCtx& c, const TraceRay& r, int path, uint32_t* stk, uint32_t* spill) {
    if (LAY != LAY_TWO_LEVEL && c.hint) {
        const uint32_t h = hintSlot(c, r, path);
        const bool ok = hintOccludes(c, r, c.hint[h]);
        countHintHits(c, ok);
        if (ok) return true;
        float t;
        bool tie;
        const int leaf = LAY == LAY_QUANT ? traverseQ<true>(c, r, stk, spill, t, tie) : traverse<true, LAY_PLAIN>(c, r, stk, spill, t);
        if (leaf >= 0) c.hint[h] = (uint32_t)leaf;
        return leaf >= 0;
    }
    return traceAny<LAY>(c, r, stk, spill);
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


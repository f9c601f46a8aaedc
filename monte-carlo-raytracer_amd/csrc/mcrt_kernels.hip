// mcrt_kernels.hip -- CDNA4 (gfx950) kernels of the wavefront path tracer.
//
// One frame (= 1 spp, RTPathTracingPass::update semantics, maxDepth D):
//   k_primary            camera ray + closest hit for every pixel of the rank's bands (fused ray gen)
//   for b in 0..D-1:
//     k_shade<b>         surface interaction, emission, 1-light NEE, BSDF sample;
//                        wave64 ballot/popc compaction into the shadow and extension queues
//     k_shadow           any-hit over the shadow queue; radiance += L * V (ShadowPass)
//     k_extend           closest hit over the extension queue (if b + 1 < D)
//   k_accumulate         ReconstructionPass (clamp, weighted running mean)
// Traversal: the RadeonRays Bvh2 as one array of 64-B records (internal nodes hold both child
// boxes, leaves their triangle), one flat loop per ray with a per-lane LDS short stack
// (16 entries, [entry][lane] layout -> conflict free) spilling to a per-ray global column;
// one wave per workgroup, the hardware dispatcher schedules the waves.
#include "mcrt_device.h"
#include "mcrt_internal.h"

// Shading workgroup size (threads; one queue atomic per workgroup and queue).
#ifndef SHADE_BLOCK
#define SHADE_BLOCK 256
#endif
// Occupancy target of the shading kernels (waves per SIMD); 0 = compiler's choice.
#ifndef MCRT_SHADE_WAVES
#define MCRT_SHADE_WAVES 0
#endif
#if MCRT_SHADE_WAVES > 0
#define MCRT_SHADE_ATTR __attribute__((amdgpu_waves_per_eu(MCRT_SHADE_WAVES, MCRT_SHADE_WAVES)))
#else
#define MCRT_SHADE_ATTR
#endif

// ---------------------------------------------------------------------------
// traversal
// ---------------------------------------------------------------------------
#define STACK_LDS 16

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

// Closest (ANY = false) or any (ANY = true) hit over the unified node array (mcrt_bvh.cpp):
// the RadeonRays intersect_bvh2_lds.cl:107-178 loop -- one uniform 64-B fetch per step, an
// internal node tests both child boxes (nearer child first, far child to the stack), a leaf
// tests its triangle.  Returns the hit leaf's node index or -1; tHit = hit distance.
// stk: this lane's LDS stack column ([entry][lane], conflict free); spill: global overflow.
template <bool ANY>
MCRT_DEV int traverse(const float4* __restrict__ nodes, const TraceRay& r, uint32_t* stk, uint32_t* spill, int spillCap,
                      int* overflowFlag, float& tHit) {
    // One flat loop with a single exit (node == DONE): stack entry 0 is a DONE sentinel, so a
    // pop is one LDS read and no lane idles at a nested loop boundary waiting for the others.
    constexpr int DONE = -1, POP = -2;
    const f3 inv = safeInvDir(r.d);
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

// hit record of the closest-hit kernels: (u, v, t, triangle) -- intersect_bvh2_lds.cl:200-215
MCRT_DEV float4 closestRecord(const float4* __restrict__ nodes, const TraceRay& r, int tri, float t) {
    if (tri < 0) return make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
    const float4 A = nodes[4 * tri], E1 = nodes[4 * tri + 1], E2 = nodes[4 * tri + 2];
    const f3 p = r.o + t * r.d;
    const f2 uv = triBary(p, A, E1, E2);
    return make_float4(uv.x, uv.y, t, __int_as_float(tri));
}

// Per-ray spill column: rays are grouped 64 to a wave; lane l of wave w owns entries
// spill[(w * spillCap + k) * 64 + l], k < spillCap (coalesced across the wave).
MCRT_DEV uint32_t* raySpill(const TraceCtx& c, int wave, int lane) {
    return c.spill + (size_t)wave * 64 * c.spillCap + lane;
}

// ---------------------------------------------------------------------------
// RadeonRays-compatible queries on AoS rays (mcrt_trace_closest / mcrt_trace_any).
// One ray per lane, one wave per workgroup (LDS stack 4 KB): the hardware dispatcher keeps
// 8 waves per SIMD resident and refills them as they finish -- measured faster on MI355X
// than a persistent grid pulling work from an atomic queue.
// ---------------------------------------------------------------------------
template <bool ANY>
__global__ __launch_bounds__(64) void k_trace_rays(TraceCtx c, const mcrt_ray* __restrict__ rays, int n,
                                                   mcrt_intersection* __restrict__ hits, int* __restrict__ occl) {
    __shared__ uint32_t lds[STACK_LDS * 64];
    const int lane = threadIdx.x;
    const int i = blockIdx.x * 64 + lane;
    if (i >= n) return;
    const mcrt_ray rr = rays[i];
    if (rr.extra[1] == 0) return;   // inactive: output untouched (intersect_bvh2_lds.cl:88)
    TraceRay r;
    r.o = ld3(rr.o);
    r.d = ld3(rr.d);
    r.tmax = rr.o.w;
    r.mask = rr.extra[0];
    float t;
    const int tri = traverse<ANY>(c.nodes, r, lds + lane, raySpill(c, blockIdx.x, lane), c.spillCap, c.overflow, t);
    if (ANY) {
        occl[i] = tri >= 0 ? 1 : -1;
    } else if (tri >= 0) {
        const float4 h4 = closestRecord(c.nodes, r, tri, t);
        mcrt_intersection h;
        h.shapeid = __float_as_int(c.nodes[4 * tri].w);
        h.primid = __float_as_int(c.nodes[4 * tri + 1].w);
        h.padding[0] = h.padding[1] = 0;
        h.uvwt.x = h4.x; h.uvwt.y = h4.y; h.uvwt.z = 0.0f; h.uvwt.w = t;
        hits[i] = h;
    } else {
        hits[i].shapeid = -1;
        hits[i].primid = -1;
    }
}

// ---------------------------------------------------------------------------
// pixel <-> band tile mapping (8x8 pixel tiles per wave; 8-row blocks dealt to bands)
// ---------------------------------------------------------------------------
MCRT_DEV bool tilePixel(const FrameArgs& f, int tile, int lane, int& x, int& y) {
    const int tb = tile / f.tilesX, tx = tile - tb * f.tilesX;
    const int bpb = f.bandRows >> 3;   // 8-row blocks per band
    const int gb = (tb / bpb) * bpb * f.numBands + f.bandIndex * bpb + (tb % bpb);
    x = tx * 8 + (lane & 7);
    y = gb * 8 + (lane >> 3);
    return x < (int)f.W && y < (int)f.H;
}

MCRT_DEV f3 cameraDir(const mcrt_camera& cam, int x, int y) {   // PathTracing.cl:13-27
    const f2 r = f2{cl_div(1.0f, (float)cam.width), cl_div(1.0f, (float)cam.height)};
    const f2 uv = f2{(float)x * r.x, (float)y * r.y};
    return lerpDirection(ld3(cam.r00), ld3(cam.r10), ld3(cam.r11), ld3(cam.r01), uv.x, uv.y);
}

// Camera ray generation fused with the first closest-hit query (RTPrimaryRaysPass):
// one workgroup = one wave = one 8x8 pixel tile of the rank's bands.
__global__ __launch_bounds__(64) void k_primary(TraceCtx c, FrameArgs f, const mcrt_camera* __restrict__ camp,
                                                float4* __restrict__ hitOut) {
    __shared__ uint32_t lds[STACK_LDS * 64];
    const int lane = threadIdx.x;
    const int tile = blockIdx.x;
    int x, y;
    if (!tilePixel(f, tile, lane, x, y)) return;
    const mcrt_camera& cam = *camp;
    TraceRay r;
    r.o = ld3(cam.pos);
    r.d = cameraDir(cam, x, y);
    r.tmax = 1000.0f;
    r.mask = -1;
    float t;
    const int tri = traverse<false>(c.nodes, r, lds + lane, raySpill(c, tile, lane), c.spillCap, c.overflow, t);
    hitOut[(size_t)y * f.W + x] = closestRecord(c.nodes, r, tri, t);
}

// Closest hit over the extension queue: qO = (o.xyz, pix), qD = (d.xyz, flags); tmax = 1000.
// The grid covers the queue's capacity; workgroups past the device-side count exit at once.
__global__ __launch_bounds__(64) void k_extend(TraceCtx c, const int* __restrict__ count, const float4* __restrict__ qO,
                                               const float4* __restrict__ qD, float4* __restrict__ hitOut) {
    __shared__ uint32_t lds[STACK_LDS * 64];
    const int n = *count;
    if ((int)blockIdx.x * 64 >= n) return;
    const int lane = threadIdx.x;
    const int i = blockIdx.x * 64 + lane;
    if (i >= n) return;
    const float4 o = qO[i], d = qD[i];
    TraceRay r;
    r.o = ld3(o);
    r.d = ld3(d);
    r.tmax = RT_MAX_TRACE_F;
    r.mask = -1;
    float t;
    const int tri = traverse<false>(c.nodes, r, lds + lane, raySpill(c, blockIdx.x, lane), c.spillCap, c.overflow, t);
    hitOut[i] = closestRecord(c.nodes, r, tri, t);
}

// Any hit over the shadow queue + ShadowPass (PathTracing.cl:186-217):
// sO = (o.xyz, tmax), sD = (d.xyz, pix), sL = throughput * L; radiance[pix] += L * V.
__global__ __launch_bounds__(64) void k_shadow(TraceCtx c, const int* __restrict__ count, const float4* __restrict__ sO,
                                               const float4* __restrict__ sD, const float4* __restrict__ sL,
                                               float4* __restrict__ radiance) {
    __shared__ uint32_t lds[STACK_LDS * 64];
    const int n = *count;
    if ((int)blockIdx.x * 64 >= n) return;
    const int lane = threadIdx.x;
    const int i = blockIdx.x * 64 + lane;
    if (i >= n) return;
    const float4 o = sO[i], d = sD[i], L = sL[i];
    TraceRay r;
    r.o = ld3(o);
    r.d = ld3(d);
    r.tmax = o.w;
    r.mask = -1;
    float t;
    const int tri = traverse<true>(c.nodes, r, lds + lane, raySpill(c, blockIdx.x, lane), c.spillCap, c.overflow, t);
    const float V = tri >= 0 ? 0.0f : 1.0f;
    const int pix = __float_as_int(d.w);
    float4 acc = radiance[pix];
    acc.x += L.x * V;
    acc.y += L.y * V;
    acc.z += L.z * V;
    radiance[pix] = acc;
}

// ---------------------------------------------------------------------------
// shading
// ---------------------------------------------------------------------------
// KRN/textures.cl:70-125 (readTexture2Df_linear: bilinear RGBA8, wrap modes)
MCRT_DEV f4 readTex(const SceneArgs& s, int texId, f2 uv) {
    const mcrt_texture_desc tex = s.textures[texId];
    const int w = tex.width, h = tex.height;
    // The reference's compiled kernel folds `-(1/w)` into `-1/w` and so loses the 2.5-ulp
    // metadata: these two reciprocals are correctly rounded there (and here).
    uv.x -= cr_div(1.0f, (float)w) * 0.5f;
    uv.y -= cr_div(1.0f, (float)h) * 0.5f;
    switch (tex.wrap) {
    case 0: uv -= f2{floorf(uv.x), floorf(uv.y)}; break;
    case 1:
        if (uv.x > 1.0f || uv.x < 0.0f) uv.x = 1.0f - (uv.x - floorf(uv.x));
        if (uv.y > 1.0f || uv.y < 0.0f) uv.y = 1.0f - (uv.y - floorf(uv.y));
        break;
    case 2: uv = f2{cl_clamp(uv.x, 0.0f, 1.0f), cl_clamp(uv.y, 0.0f, 1.0f)}; break;
    case 3:
        if (uv.x > 1.0f || uv.x < 0.0f || uv.y > 1.0f || uv.y < 0.0f) return f4{0.0f, 0.0f, 0.0f, 0.0f};
        break;
    }
    int x0 = ((int)floorf(uv.x * w)) % w;
    int y0 = ((int)floorf(uv.y * h)) % h;
    int x1 = (x0 + 1) % w;
    int y1 = (y0 + 1) % h;
    x0 = min(max(x0, 0), w - 1);
    y0 = min(max(y0, 0), h - 1);
    x1 = min(max(x1, 0), w - 1);
    y1 = min(max(y1, 0), h - 1);
    const f2 t = f2{uv.x * w - floorf(uv.x * w), uv.y * h - floorf(uv.y * h)};
    const uchar4* texD = reinterpret_cast<const uchar4*>(s.texData + tex.memOffset);
    const uchar4 c00 = texD[x0 + y0 * w], c10 = texD[x1 + y0 * w], c01 = texD[x0 + y1 * w], c11 = texD[x1 + y1 * w];
    const f4 v00 = f4{(float)c00.x, (float)c00.y, (float)c00.z, (float)c00.w};
    const f4 v10 = f4{(float)c10.x, (float)c10.y, (float)c10.z, (float)c10.w};
    const f4 v01 = f4{(float)c01.x, (float)c01.y, (float)c01.z, (float)c01.w};
    const f4 v11 = f4{(float)c11.x, (float)c11.y, (float)c11.z, (float)c11.w};
    // mix(a, b, t) = fma(b - a, t, a) per component (device-library mix)
    const f4 m0 = f4{fmaf(v10.x - v00.x, t.x, v00.x), fmaf(v10.y - v00.y, t.x, v00.y), fmaf(v10.z - v00.z, t.x, v00.z),
                     fmaf(v10.w - v00.w, t.x, v00.w)};
    const f4 m1 = f4{fmaf(v11.x - v01.x, t.x, v01.x), fmaf(v11.y - v01.y, t.x, v01.y), fmaf(v11.z - v01.z, t.x, v01.z),
                     fmaf(v11.w - v01.w, t.x, v01.w)};
    const f4 m = f4{fmaf(m1.x - m0.x, t.y, m0.x), fmaf(m1.y - m0.y, t.y, m0.y), fmaf(m1.z - m0.z, t.y, m0.z),
                    fmaf(m1.w - m0.w, t.y, m0.w)};
    return m * (1.0f / 255.0f);
}

// KRN/materials.cl:76-91 (getUberMaterialProperties)
MCRT_DEV Uber uberProps(const SceneArgs& s, const mcrt_material& material, f2 uv) {
    Uber u;
    const f4 Kd_opacity = material.uber_diffuseTexId != -1 ? readTex(s, material.uber_diffuseTexId, uv) : f4{1.0f, 1.0f, 1.0f, 1.0f};
    u.Kd = Kd_opacity.xyz * ld3(material.uber_kd);
    u.Ks = (material.uber_glossyTexId != -1 ? readTex(s, material.uber_glossyTexId, uv).xyz : splat3(1.0f)) * ld3(material.uber_ks);
    u.Kr = (material.uber_specReflectionTexId != -1 ? readTex(s, material.uber_specReflectionTexId, uv).xyz : splat3(1.0f)) *
           ld3(material.uber_kr);
    u.Kt.xyz = (material.uber_transmissionTexId != -1 ? readTex(s, material.uber_transmissionTexId, uv).xyz : splat3(1.0f)) *
               ld3(material.uber_kt);
    u.Kt.w = material.uber_kt.w;
    u.opacity = (material.uber_opacityTexId != -1 ? readTex(s, material.uber_opacityTexId, uv).xyz : splat3(1.0f)) *
                ld3(material.uber_opacity) * Kd_opacity.w;
    u.roughness = material.uber_roughnessTexId != -1 ? readTex(s, material.uber_roughnessTexId, uv).xy
                                                      : f2{material.uber_roughness.x, material.uber_roughness.y};
    u.eta = material.uber_iorTexId != -1 ? readTex(s, material.uber_iorTexId, uv).x : material.uber_eta;
    u.roughness = f2{roughnessToAlpha(u.roughness.x), roughnessToAlpha(u.roughness.y)};
    return u;
}

// Wave-aggregated queue append: returns this lane's slot (valid where pred).
// Block-aggregated queue append: ONE global atomic per workgroup instead of one per wave.
// Device-scope atomics on one address serialise across the 8 XCDs (~10+ ns each), which made
// per-wave appends the bottleneck of the shading kernels.  Every thread of the block must call.
template <int NW>
MCRT_DEV int blockAppend(int* counter, bool pred, int* ldsWave /* NW + 1 ints */) {
    const unsigned long long m = __ballot(pred);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (lane == 0) ldsWave[wv] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int sum = 0;
        for (int w = 0; w < NW; ++w) {
            const int c = ldsWave[w];
            ldsWave[w] = sum;
            sum += c;
        }
        ldsWave[NW] = sum ? atomicAdd(counter, sum) : 0;
    }
    __syncthreads();
    const unsigned lo = (unsigned)m, hi = (unsigned)(m >> 32);
    const int prefix = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
    const int slot = ldsWave[NW] + ldsWave[wv] + prefix;
    __syncthreads();   // ldsWave is reused by the next append
    return slot;
}

// May be called under divergent control flow: only active lanes take part.
MCRT_DEV int waveAppend(int* counter, bool pred) {
    const unsigned long long m = __ballot(pred);
    if (m == 0) return 0;
    const int lane = threadIdx.x & 63;
    const int leader = __ffsll((long long)m) - 1;
    int base = 0;
    if (lane == leader) base = atomicAdd(counter, __popcll(m));
    base = __shfl(base, leader);
    const unsigned lo = (unsigned)m, hi = (unsigned)(m >> 32);
    const int prefix = __builtin_amdgcn_mbcnt_hi(hi, __builtin_amdgcn_mbcnt_lo(lo, 0u));
    return base + prefix;
}


// KRN/geometry.cl:9-28
MCRT_DEV void computeTrianglePartialDerivates(f2 uv0, f2 uv1, f2 uv2, f3 p0, f3 p1, f3 p2, f3 normal, f3* dpdu, f3* dpdv) {
    f2 duv02 = uv0 - uv2;
    f2 duv12 = uv1 - uv2;
    f3 dp02 = p0 - p2;
    f3 dp12 = p1 - p2;
    float det = duv02.x * duv12.y - duv02.y * duv12.x;
    if (isNotNearZero(det)) {
        float invdet = cl_div(1.0f, det);
        *dpdu = (duv12.y * dp02 - duv02.y * dp12) * invdet;
        *dpdv = -(-duv12.x * dp02 + duv02.x * dp12) * invdet;
    } else {
        *dpdu = cl_normalize(computeOrthogonalVector(normal));
        *dpdv = cl_normalize(cl_cross(normal, *dpdu));
    }
}

// KRN/samplers.cl:259-269 (sampleDisk); returns the sampled point, *pdf = 1 / area
MCRT_DEV f3 sampleDisk(f3 p, f3 n, float radius, f2 u, float* pdf) {
    f2 p2d = concentricSampleDisc(u);
    f3 t = computeOrthogonalVector(n);
    f3 b = cl_normalize(cl_cross(n, t));
    f3 itp = p + t * p2d.x * radius + b * p2d.y * radius;
    *pdf = cl_div(1.0f, (PI_F * radius * radius));
    return itp;
}

// KRN/samplers.cl:275-285 (sampleTriangle)
MCRT_DEV f3 sampleTriangle(f3 p0, f3 p1, f3 p2, f2 u, f3* gn) {
    const float su0 = cl_sqrt(u.x);
    f2 b = f2{1.0f - su0, u.y * su0};
    f3 itp = b.x * p0 + b.y * p1 + (1 - b.x - b.y) * p2;
    f3 c = cl_cross(p1 - p0, p2 - p0);
    *gn = cl_normalize(c);
    return itp;
}

// computeSurfaceInteraction (geometry.cl:177-215)
MCRT_DEV Frame computeSurfaceInteraction(const SceneArgs& s, int shapeIdx, int primIdx, f2 barycentrics) {
    Frame si;
    const mcrt_shape& shape = s.shapes[shapeIdx];
    const uint32_t i0 = s.indices[shape.startIdx + 3 * primIdx];
    const uint32_t i1 = s.indices[shape.startIdx + 3 * primIdx + 1];
    const uint32_t i2 = s.indices[shape.startIdx + 3 * primIdx + 2];
    const f3 p0 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i0]));
    const f3 p1 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i1]));
    const f3 p2 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i2]));
    const float2 t0 = s.uvs[shape.startVertex + i0], t1 = s.uvs[shape.startVertex + i1], t2 = s.uvs[shape.startVertex + i2];
    const f2 uv0 = f2{t0.x, t0.y}, uv1 = f2{t1.x, t1.y}, uv2 = f2{t2.x, t2.y};
    const f3 n0 = transformVector3(shape.toWorldInverseTranspose, ld3(s.normals[shape.startVertex + i0]));
    const f3 n1 = transformVector3(shape.toWorldInverseTranspose, ld3(s.normals[shape.startVertex + i1]));
    const f3 n2 = transformVector3(shape.toWorldInverseTranspose, ld3(s.normals[shape.startVertex + i2]));
    si.p = p0 * (1.0f - barycentrics.x - barycentrics.y) + p1 * barycentrics.x + p2 * barycentrics.y;
    si.uv = uv0 * (1.0f - barycentrics.x - barycentrics.y) + uv1 * barycentrics.x + uv2 * barycentrics.y;
    si.gn = cl_normalize(cl_cross(p0 - p2, p1 - p2));
    si.sn = cl_normalize(n0 * (1.0f - barycentrics.x - barycentrics.y) + n1 * barycentrics.x + n2 * barycentrics.y);
    f3 dpdu, dpdv;
    computeTrianglePartialDerivates(uv0, uv1, uv2, p0, p1, p2, si.sn, &dpdu, &dpdv);
    si.sdpdu = cl_normalize(dpdu - cl_dot(si.sn, dpdu) * si.sn);
    si.sdpdv = cl_normalize(dpdv - cl_dot(si.sn, dpdv) * si.sn - cl_dot(si.sdpdu, dpdv) * si.sdpdu);
    return si;
}

// applyNormalMapping_internal (materials.cl:11-19)
MCRT_DEV void applyNormalMapping(const SceneArgs& s, int texId, Frame& si) {
    const f3 nm = 2.0f * readTex(s, texId, si.uv).xyz - 1.0f;
    si.sn = cl_normalize(si.sdpdu * nm.x + si.sdpdv * nm.y + si.sn * nm.z);
    si.sdpdu = cl_normalize(cl_cross(si.sn, si.sdpdv));
    si.sdpdv = cl_normalize(cl_cross(si.sdpdu, si.sn));
}

struct LightSample {
    f3 Li, wi;
    float pdf;
    bool shadowSet;   // setRay() was called on the shadow ray
    f3 shadowO;
    float shadowT;
};

// sampleLightLi (lights.cl:45-146)
MCRT_DEV LightSample sampleLightLi(const SceneArgs& s, const mcrt_light& light, const Frame& si, float traceErrorOffset,
                                   f2 u) {
    LightSample r;
    r.Li = splat3(0.0f);
    r.wi = splat3(0.0f);
    r.pdf = 0.0f;
    r.shadowSet = false;
    r.shadowO = splat3(0.0f);
    r.shadowT = 0.0f;
    if (light.type == MCRT_DIRECTIONAL_LIGHT) {
        r.wi = -ld3(light.d);
        r.pdf = 1.0f;
        r.shadowO = si.p + si.gn * traceErrorOffset;
        r.shadowT = 1000.0f;
        r.shadowSet = true;
        r.Li = ld3(light.intensity);
    } else if (light.type == MCRT_POINT_LIGHT) {
        f3 wi = ld3(light.p) - si.p;
        float distSq = cl_dot(wi, wi);
        if (!isNearZero(distSq)) {
            float dist = cl_sqrt(distSq);
            wi = cl_div(wi, dist);
            r.wi = wi;
            r.pdf = 1.0f;
            r.shadowO = si.p + si.gn * traceErrorOffset;
            r.shadowT = dist;
            r.shadowSet = true;
            r.Li = cl_div(ld3(light.intensity), distSq);
        } else {
            r.wi = wi;
        }
    } else if (light.type == MCRT_DISK_AREA_LIGHT || light.type == MCRT_TRIANGLE_MESH_AREA_LIGHT) {
        f3 lp, lgn;
        if (light.type == MCRT_DISK_AREA_LIGHT) {
            lp = sampleDisk(ld3(light.p), ld3(light.d), light.radius, u, &r.pdf);
            lgn = ld3(light.d);
        } else {
            const mcrt_shape shape = s.shapes[light.shapeId];
            int triangleIdx = (int)((uint32_t)((int)floorf(u.x * shape.numTriangles)) % shape.numTriangles);
            u.x = u.x * shape.numTriangles - triangleIdx;
            const uint32_t i0 = s.indices[shape.startIdx + 3 * triangleIdx];
            const uint32_t i1 = s.indices[shape.startIdx + 3 * triangleIdx + 1];
            const uint32_t i2 = s.indices[shape.startIdx + 3 * triangleIdx + 2];
            const f3 p0 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i0]));
            const f3 p1 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i1]));
            const f3 p2 = transformPoint3(shape.toWorldTransform, ld3(s.positions[shape.startVertex + i2]));
            lp = sampleTriangle(p0, p1, p2, u, &lgn);
            r.pdf = cl_div(1.0f, light.area);
        }
        const f3 rayOrigin = si.p + si.gn * traceErrorOffset;
        const f3 rayTarget = lp + lgn * RT_TRACE_OFFSET_F;
        r.wi = light.type == MCRT_DISK_AREA_LIGHT ? cl_normalize(rayTarget - rayOrigin) : cl_normalize(lp - si.p);
        const float distSq = distanceSquared(lp, si.p);
        const float c = absDot(lgn, -r.wi);
        if (isNearZero(c)) {
            r.pdf = 0.0f;
        } else {
            r.pdf *= cl_div(distSq, c);
            r.shadowO = rayOrigin;
            r.shadowT = cl_distance(rayOrigin, rayTarget);
            r.shadowSet = true;
            r.Li = cl_dot(lgn, -r.wi) > 0.0f ? ld3(light.intensity) : splat3(0.0f);
        }
    }
    return r;
}

// PathTracing kernel body (PathTracing.cl:52-184) for one path.
// Returns the radiance term added at this vertex by emission (or by a NaN NEE term
// with no shadow ray).  NEE terms go to the shadow queue.
struct ShadeOut {
    bool pushS, pushE;
    float4 sO, sD, sL;   // shadow ray
    float4 eO, eD, eT;   // extension ray + throughput
};

MCRT_DEV f3 shadePath(const SceneArgs& s, const FrameArgs& f, int bounce, int pix, float4 hit, f3 dir, f3 throughput,
                      int prevFlags, ShadeOut& o) {
    f3 add = splat3(0.0f);
    const int tri = __float_as_int(hit.w);
    if (tri < 0 || s.numLights <= 0) return add;
    const float4 A = s.nodes[4 * tri], E1 = s.nodes[4 * tri + 1];
    const int shapeIdx = __float_as_int(A.w), primIdx = __float_as_int(E1.w);
    const mcrt_shape& shape = s.shapes[shapeIdx];
    Frame si = computeSurfaceInteraction(s, shapeIdx, primIdx, f2{hit.x, hit.y});
    const f3 wo = -dir;
    const bool isBackfacing = cl_dot(si.gn, wo) < 0.0f;
    const float traceErrorOffset = isBackfacing ? -RT_TRACE_OFFSET_F : RT_TRACE_OFFSET_F;
    const int materialId = shape.materialId;
    mcrt_material mat;
    if (materialId != -1) {
        mat = s.materials[materialId];
        if (mat.uber_normalMapId != -1) applyNormalMapping(s, mat.uber_normalMapId, si);
    }
    if (bounce == 0) throughput = splat3(1.0f);
    // emission (PathTracing.cl:82-101)
    if (shape.lightID != -1 && (bounce == 0 || (prevFlags & BSDF_SPECULAR) == BSDF_SPECULAR)) {
        const mcrt_light& L = s.lights[shape.lightID];
        f3 Le = splat3(0.0f);
        if ((L.type == MCRT_DISK_AREA_LIGHT || L.type == MCRT_TRIANGLE_MESH_AREA_LIGHT) && cl_dot(si.gn, wo) > 0.0f)
            Le = ld3(L.intensity);
        return throughput * Le;
    }
    Sampler sampler = makeSampler(f.sampler, (uint32_t)pix, f.frame, bounce, f.W, f.H, s.sobol);
    const bool isUber = materialId != -1 && mat.type == 0;   // materials.cl:130-142: other types evaluate to 0
    Uber um;
    if (isUber) um = uberProps(s, mat, si.uv);
    // next-event estimation, one light (PathTracing.cl:107-136)
    {
        uint32_t lightIdx = (uint32_t)floorf(getSample1D(sampler) * s.numLights);
        lightIdx %= (uint32_t)s.numLights;
        const f2 u = getSample2D(sampler);
        const mcrt_light light = s.lights[lightIdx];
        const LightSample ls = sampleLightLi(s, light, si, traceErrorOffset, u);
        float lightPdf = ls.pdf * light.choicePdf;
        f3 L = splat3(0.0f);
        if (materialId != -1) {
            f3 bsdf = isUber ? evaluateUberBSDF(um, si, wo, ls.wi) : splat3(0.0f);
            bsdf *= absDot(ls.wi, si.sn);
            if (!isNearZero(lightPdf)) L = cl_div(ls.Li * bsdf, lightPdf);
        }
        const f3 term = throughput * L;
        if (term.x != 0.0f || term.y != 0.0f || term.z != 0.0f) {
            if (ls.shadowSet) {
                o.pushS = true;
                o.sO = make_float4(ls.shadowO.x, ls.shadowO.y, ls.shadowO.z, ls.shadowT);
                o.sD = make_float4(ls.wi.x, ls.wi.y, ls.wi.z, __int_as_float(pix));
                o.sL = make_float4(term.x, term.y, term.z, 0.0f);
            } else {
                add = term * 0.0f;   // no shadow ray: V = 0 (a NaN term stays NaN, ShadowPass semantics)
            }
        }
    }
    // extension (PathTracing.cl:138-175)
    if (bounce + 1 < f.maxDepth) {
        const f2 bsdfSample = getSample2D(sampler);
        if (isUber) {
            f3 wi;
            float pdf;
            int sampledType;
            f3 bsdfBounce = sampleUberBSDF(um, si, bsdfSample, wo, &wi, &pdf, &sampledType);
            if (!(isNearZero(pdf) || isBlack(bsdfBounce))) {
                bsdfBounce = cl_div(bsdfBounce, pdf);
                const f3 tp = bsdfBounce * absDot(wi, si.sn);
                const f3 nt = throughput * tp;
                float off = traceErrorOffset;
                if ((sampledType & BSDF_TRANSMISSION) != 0 && cl_dot(si.gn, wi) * cl_sign(off) < 0.0f) off *= -1.0f;
                const f3 no = si.p + si.gn * off;
                bool alive = true;
                f3 tp1 = nt;
                if (f.russianRoulette && bounce + 1 >= f.rrStartDepth) {   // opt-in perf mode
                    const float qr = fmaxf(0.05f, 1.0f - fmaxf(nt.x, fmaxf(nt.y, nt.z)));
                    const float ur = (float)wangHash((uint32_t)pix * 9781u + (uint32_t)f.frame * 6271u + (uint32_t)bounce) * 0x1p-32f;
                    alive = ur >= qr;
                    tp1 = cl_div(nt, (1.0f - qr));
                }
                if (alive) {
                    o.pushE = true;
                    o.eO = make_float4(no.x, no.y, no.z, __int_as_float(pix));
                    o.eD = make_float4(wi.x, wi.y, wi.z, __int_as_float(sampledType));
                    o.eT = make_float4(tp1.x, tp1.y, tp1.z, 0.0f);
                }
            }
        }
    }
    return add;
}

// Bounce 0: every pixel of the band (tile order); writes radiance[pix] (= `=` of ShadowPass).
__global__ __launch_bounds__(SHADE_BLOCK) MCRT_SHADE_ATTR void k_shade0(SceneArgs s, FrameArgs f, const mcrt_camera* __restrict__ camp,
                                                const float4* __restrict__ hits, float4* __restrict__ radiance,
                                                QueueArgs q) {
    const int lane = threadIdx.x & 63;
    const int tile = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int x = 0, y = 0;
    bool valid = tile < f.numTiles && tilePixel(f, tile, lane, x, y);
    __shared__ int ldsWave[SHADE_BLOCK / 64 + 1];
    ShadeOut o;
    o.pushS = o.pushE = false;
    if (valid) {
        const mcrt_camera& cam = *camp;
        const int pix = y * (int)f.W + x;
        const f3 dir = cameraDir(cam, x, y);
        const f3 add = shadePath(s, f, 0, pix, hits[pix], dir, splat3(1.0f), 0, o);
        radiance[pix] = make_float4(add.x, add.y, add.z, 0.0f);
    }
    const int ss = blockAppend<SHADE_BLOCK / 64>(q.shadowCount, o.pushS, ldsWave);
    if (o.pushS) { q.sO[ss] = o.sO; q.sD[ss] = o.sD; q.sL[ss] = o.sL; }
    const int es = blockAppend<SHADE_BLOCK / 64>(q.extCountOut, o.pushE, ldsWave);
    if (o.pushE) { q.eOout[es] = o.eO; q.eDout[es] = o.eD; q.eTout[es] = o.eT; }
}

// Bounce >= 1: the compacted extension queue of the previous bounce.
__global__ __launch_bounds__(SHADE_BLOCK) MCRT_SHADE_ATTR void k_shadeN(SceneArgs s, FrameArgs f, int bounce, const int* __restrict__ countIn,
                                                const float4* __restrict__ qO, const float4* __restrict__ qD,
                                                const float4* __restrict__ qT, const float4* __restrict__ hits,
                                                float4* __restrict__ radiance, QueueArgs q) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = *countIn;
    __shared__ int ldsWave[SHADE_BLOCK / 64 + 1];
    if ((int)blockIdx.x * SHADE_BLOCK >= n) return;   // whole block past the queue: uniform exit
    ShadeOut o;
    o.pushS = o.pushE = false;
    if (i < n) {
        const float4 O = qO[i], D = qD[i], Tp = qT[i];
        const int pix = __float_as_int(O.w);
        const f3 add = shadePath(s, f, bounce, pix, hits[i], ld3(D), ld3(Tp), __float_as_int(D.w), o);
        if (add.x != 0.0f || add.y != 0.0f || add.z != 0.0f || add.x != add.x) {
            float4 r = radiance[pix];
            r.x += add.x; r.y += add.y; r.z += add.z;
            radiance[pix] = r;
        }
    }
    const int ss = blockAppend<SHADE_BLOCK / 64>(q.shadowCount, o.pushS, ldsWave);
    if (o.pushS) { q.sO[ss] = o.sO; q.sD[ss] = o.sD; q.sL[ss] = o.sL; }
    const int es = blockAppend<SHADE_BLOCK / 64>(q.extCountOut, o.pushE, ldsWave);
    if (o.pushE) { q.eOout[es] = o.eO; q.eDout[es] = o.eD; q.eTout[es] = o.eT; }
}

// ---------------------------------------------------------------------------
// ReconstructionPass (KRN/reconstruction.cl:6-60); weight precomputed on the host
// (KRN/filters.cl, uniform per frame).  Band rows only.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_accumulate(FrameArgs f, int frame, float w, const float4* __restrict__ radiance,
                                                    float4* __restrict__ wsum, float* __restrict__ wts,
                                                    float4* __restrict__ image) {
    const int lane = threadIdx.x & 63;
    const int tile = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int x, y;
    if (tile >= f.numTiles || !tilePixel(f, tile, lane, x, y)) return;
    const int pix = y * (int)f.W + x;
    const float4 r4 = radiance[pix];
    const f4 radiance4 = f4{cl_clamp(r4.x, 0.0f, 1000.0f), cl_clamp(r4.y, 0.0f, 1000.0f), cl_clamp(r4.z, 0.0f, 1000.0f),
                            cl_clamp(r4.w, 0.0f, 1000.0f)};
    f4 s;
    float ws;
    if (frame == 0) {
        s = radiance4 * w;
        ws = w;
    } else {
        const float4 o = wsum[pix];
        s = f4{o.x, o.y, o.z, o.w};
        s += radiance4 * w;
        ws = wts[pix] + w;
    }
    wsum[pix] = make_float4(s.x, s.y, s.z, s.w);
    wts[pix] = ws;
    const f4 fin = cl_div(s, ws);
    image[pix] = make_float4(fin.x, fin.y, fin.z, fin.w);
}

// image = sum / weight after a multi-GPU reduce of the accumulators
__global__ __launch_bounds__(256) void k_resolve(int n, const float4* __restrict__ wsum, const float* __restrict__ wts,
                                                 float4* __restrict__ image) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 s = wsum[i];
    const float w = wts[i];
    image[i] = make_float4(cl_div(s.x, w), cl_div(s.y, w), cl_div(s.z, w), cl_div(s.w, w));
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
namespace mcrt {

void launch_trace_rays(bool any, const TraceCtx& c, const mcrt_ray* rays, int n, mcrt_intersection* hits, int* occl,
                       hipStream_t st) {
    const dim3 g((n + 63) / 64), b(64);
    if (any) hipLaunchKernelGGL(k_trace_rays<true>, g, b, 0, st, c, rays, n, hits, occl);
    else hipLaunchKernelGGL(k_trace_rays<false>, g, b, 0, st, c, rays, n, hits, occl);
}
void launch_primary(const TraceCtx& c, const FrameArgs& f, const mcrt_camera* cam, float4* hits, hipStream_t st) {
    hipLaunchKernelGGL(k_primary, dim3(f.numTiles), dim3(64), 0, st, c, f, cam, hits);
}
void launch_extend(const TraceCtx& c, const int* count, const float4* qO, const float4* qD, float4* hits, int maxCount,
                   hipStream_t st) {
    hipLaunchKernelGGL(k_extend, dim3((maxCount + 63) / 64), dim3(64), 0, st, c, count, qO, qD, hits);
}
void launch_shadow(const TraceCtx& c, const int* count, const float4* sO, const float4* sD, const float4* sL,
                   float4* radiance, int maxCount, hipStream_t st) {
    hipLaunchKernelGGL(k_shadow, dim3((maxCount + 63) / 64), dim3(64), 0, st, c, count, sO, sD, sL, radiance);
}
void launch_shade0(const SceneArgs& s, const FrameArgs& f, const mcrt_camera* cam, const float4* hits,
                   float4* radiance, const QueueArgs& q, hipStream_t st) {
    const int blocks = (f.numTiles * 64 + SHADE_BLOCK - 1) / SHADE_BLOCK;
    hipLaunchKernelGGL(k_shade0, dim3(blocks), dim3(SHADE_BLOCK), 0, st, s, f, cam, hits, radiance, q);
}
void launch_shadeN(const SceneArgs& s, const FrameArgs& f, int bounce, const int* countIn, const float4* qO,
                   const float4* qD, const float4* qT, const float4* hits, float4* radiance, const QueueArgs& q,
                   int maxCount, hipStream_t st) {
    const int blocks = (maxCount + SHADE_BLOCK - 1) / SHADE_BLOCK;
    hipLaunchKernelGGL(k_shadeN, dim3(blocks > 0 ? blocks : 1), dim3(SHADE_BLOCK), 0, st, s, f, bounce, countIn, qO, qD,
                       qT, hits, radiance, q);
}
void launch_accumulate(const FrameArgs& f, int frame, float w, const float4* radiance, float4* wsum, float* wts,
                       float4* image, hipStream_t st) {
    const int blocks = (f.numTiles * 64 + 255) / 256;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(256), 0, st, f, frame, w, radiance, wsum, wts, image);
}

void launch_resolve(uint32_t W, uint32_t H, const float4* wsum, const float* wts, float4* image, hipStream_t st) {
    const int n = (int)(W * H);
    hipLaunchKernelGGL(k_resolve, dim3((n + 255) / 256), dim3(256), 0, st, n, wsum, wts, image);
}

}  // namespace mcrt

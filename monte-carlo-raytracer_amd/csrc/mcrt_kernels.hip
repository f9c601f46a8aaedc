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
// Traversal: 64-B two-child nodes (both child boxes in the parent), leaves referenced by
// index into a 48-B triangle array (v0, e1, e2; w = shape id / prim id), per-lane LDS short
// stack (16 entries, [entry][lane] layout -> conflict free) with global spill, persistent
// waves pulling 64-ray chunks from an atomic counter.
#include "mcrt_device.h"
#include "mcrt_internal.h"

// ---------------------------------------------------------------------------
// traversal
// ---------------------------------------------------------------------------
#define STACK_LDS 16
#define TRACE_BLOCK 256

struct TraceRay {
    v3 o, d;
    float tmax;
    int mask;
};

// RR common.cl:220-232
MCRT_DEV v3 safeInvDir(v3 d) {
    const float eps = 1e-8f;
    return mk3(1.0f / (fabsf(d.x) > eps ? d.x : copysignf(eps, d.x)), 1.0f / (fabsf(d.y) > eps ? d.y : copysignf(eps, d.y)),
               1.0f / (fabsf(d.z) > eps ? d.z : copysignf(eps, d.z)));
}

// RR common.cl:177-218; 1/denom as v_rcp_f32 (what native_recip lowers to on AMD).
MCRT_DEV float triHit(const TraceRay& r, float4 A, float4 E1, float4 E2, float tmax) {
    v3 e1 = ld3(E1), e2 = ld3(E2), a = ld3(A);
    v3 s1 = cross(r.d, e2);
    float denom = dot(s1, e1);
    if (denom == 0.f) return tmax;
    float invd = __builtin_amdgcn_rcpf(denom);
    v3 dd = r.o - a;
    float b1 = dot(dd, s1) * invd;
    v3 s2 = cross(dd, e1);
    float b2 = dot(r.d, s2) * invd;
    float t = dot(e2, s2) * invd;
    if (b1 < 0.f || b1 > 1.f || b2 < 0.f || b1 + b2 > 1.f || t < 0.f || t > tmax) return tmax;
    return t;
}

// Closest (ANY = false) or any (ANY = true) hit.  Returns the triangle index or -1 and
// leaves the hit distance in tHit.  stk: this lane's LDS stack column; spill: global.
template <bool ANY>
MCRT_DEV int traverse(const float4* __restrict__ nodes, const float4* __restrict__ tris, const TraceRay& r,
                      uint32_t* stk, uint32_t* spill, int spillCap, int* overflowFlag, float& tHit) {
    const v3 inv = safeInvDir(r.d);
    const v3 oxi = mk3(-r.o.x * inv.x, -r.o.y * inv.y, -r.o.z * inv.z);
    float t = r.tmax;
    int hitTri = -1;
    int node = 0;
    int sp = 0, spillTop = 0;
    for (;;) {
        const float4 n0 = nodes[4 * node + 0];
        const float4 n1 = nodes[4 * node + 1];
        const float4 n2 = nodes[4 * node + 2];
        const int4 n3 = *reinterpret_cast<const int4*>(&nodes[4 * node + 3]);
        // slab tests of both children (RR intersect_bvh2_lds.cl:54-63, mad -> fma)
        float ax0 = fmaf(n0.x, inv.x, oxi.x), ax1 = fmaf(n0.y, inv.x, oxi.x);
        float ay0 = fmaf(n0.z, inv.y, oxi.y), ay1 = fmaf(n0.w, inv.y, oxi.y);
        float az0 = fmaf(n2.x, inv.z, oxi.z), az1 = fmaf(n2.y, inv.z, oxi.z);
        float bx0 = fmaf(n1.x, inv.x, oxi.x), bx1 = fmaf(n1.y, inv.x, oxi.x);
        float by0 = fmaf(n1.z, inv.y, oxi.y), by1 = fmaf(n1.w, inv.y, oxi.y);
        float bz0 = fmaf(n2.z, inv.z, oxi.z), bz1 = fmaf(n2.w, inv.z, oxi.z);
        float a0 = fmaxf(fmaxf(fmaxf(fminf(ax0, ax1), fminf(ay0, ay1)), fminf(az0, az1)), 0.0f);
        float a1 = fminf(fminf(fminf(fmaxf(ax0, ax1), fmaxf(ay0, ay1)), fmaxf(az0, az1)), t);
        float b0 = fmaxf(fmaxf(fmaxf(fminf(bx0, bx1), fminf(by0, by1)), fminf(bz0, bz1)), 0.0f);
        float b1 = fminf(fminf(fminf(fmaxf(bx0, bx1), fmaxf(by0, by1)), fmaxf(bz0, bz1)), t);
        bool h0 = a0 <= a1, h1 = b0 <= b1;
        bool swap = h1 && (a0 > b0);   // nearer child first (intersect_bvh2_lds.cl:128-141)
        int cf = swap ? n3.y : n3.x, cs = swap ? n3.x : n3.y;
        bool hf = swap ? h1 : h0, hs = swap ? h0 : h1;
        // leaf children are intersected immediately, near first
        if (hf && cf < 0) {
            const int ti = ~cf;
            const float4 A = tris[3 * ti], E1 = tris[3 * ti + 1], E2 = tris[3 * ti + 2];
            if (r.mask != __float_as_int(A.w)) {   // RR_RAY_MASK
                float th = triHit(r, A, E1, E2, t);
                if (th < t) {
                    t = th;
                    hitTri = ti;
                    if (ANY) break;
                }
            }
            hf = false;
        }
        if (hs && cs < 0) {
            const int ti = ~cs;
            const float4 A = tris[3 * ti], E1 = tris[3 * ti + 1], E2 = tris[3 * ti + 2];
            if (r.mask != __float_as_int(A.w)) {
                float th = triHit(r, A, E1, E2, t);
                if (th < t) {
                    t = th;
                    hitTri = ti;
                    if (ANY) break;
                }
            }
            hs = false;
        }
        if (hf) {
            if (hs) {   // push the far child
                if (sp == STACK_LDS) {
                    if (spillTop + STACK_LDS <= spillCap) {
                        for (int k = 0; k < STACK_LDS; ++k) spill[(size_t)(spillTop + k) * 64] = stk[k * 64];
                        spillTop += STACK_LDS;
                    } else {
                        *overflowFlag = 1;   // depth beyond capacity: drop (reported by the host)
                    }
                    sp = 0;
                }
                stk[sp * 64] = (uint32_t)cs;
                ++sp;
            }
            node = cf;
        } else if (hs) {
            node = cs;
        } else {
            if (sp == 0) {
                if (spillTop == 0) break;
                spillTop -= STACK_LDS;
                for (int k = 0; k < STACK_LDS; ++k) stk[k * 64] = spill[(size_t)(spillTop + k) * 64];
                sp = STACK_LDS;
            }
            --sp;
            node = (int)stk[sp * 64];
        }
    }
    tHit = t;
    return hitTri;
}

// RR common.cl:249-277
MCRT_DEV void triBary(v3 p, float4 A, float4 E1, float4 E2, float& u, float& v) {
    v3 e1 = ld3(E1), e2 = ld3(E2), e = p - ld3(A);
    float d00 = dot(e1, e1), d01 = dot(e1, e2), d11 = dot(e2, e2), d20 = dot(e, e1), d21 = dot(e, e2);
    float den = d00 * d11 - d01 * d01;
    if (den == 0.f) { u = 0.f; v = 0.f; return; }
    float inv = __builtin_amdgcn_rcpf(den);
    u = (d11 * d20 - d01 * d21) * inv;
    v = (d00 * d21 - d01 * d20) * inv;
}

// Wave-uniform chunk fetch for persistent waves.
MCRT_DEV int nextChunk(int* counter, int lane) {
    int base = 0;
    if (lane == 0) base = atomicAdd(counter, 64);
    return __shfl(base, 0);
}

MCRT_DEV uint32_t* laneSpill(const TraceCtx& c) {
    const int gtid = blockIdx.x * blockDim.x + threadIdx.x;
    const int wave = gtid >> 6, lane = gtid & 63;
    return c.spill + (size_t)wave * 64 * c.spillCap + lane;
}

// ---------------------------------------------------------------------------
// RadeonRays-compatible queries on AoS rays (mcrt_trace_closest / mcrt_trace_any)
// ---------------------------------------------------------------------------
template <bool ANY>
__global__ __launch_bounds__(TRACE_BLOCK) void k_trace_rays(TraceCtx c, const mcrt_ray* __restrict__ rays, int n,
                                                            int* work, mcrt_intersection* __restrict__ hits,
                                                            int* __restrict__ occl) {
    __shared__ uint32_t lds[STACK_LDS * TRACE_BLOCK];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* stk = lds + wv * 64 * STACK_LDS + lane;
    uint32_t* spill = laneSpill(c);
    for (;;) {
        const int base = nextChunk(work, lane);
        if (base >= n) break;
        const int i = base + lane;
        if (i >= n) continue;
        const mcrt_ray rr = rays[i];
        if (rr.extra[1] == 0) continue;   // inactive: output untouched (intersect_bvh2_lds.cl:88)
        TraceRay r;
        r.o = mk3(rr.o.x, rr.o.y, rr.o.z);
        r.d = mk3(rr.d.x, rr.d.y, rr.d.z);
        r.tmax = rr.o.w;
        r.mask = rr.extra[0];
        float t;
        int tri = traverse<ANY>(c.nodes, c.tris, r, stk, spill, c.spillCap, c.overflow, t);
        if (ANY) {
            occl[i] = tri >= 0 ? 1 : -1;
        } else if (tri >= 0) {
            const float4 A = c.tris[3 * tri], E1 = c.tris[3 * tri + 1], E2 = c.tris[3 * tri + 2];
            float u, v;
            triBary(r.o + t * r.d, A, E1, E2, u, v);
            mcrt_intersection h;
            h.shapeid = __float_as_int(A.w);
            h.primid = __float_as_int(E1.w);
            h.padding[0] = h.padding[1] = 0;
            h.uvwt.x = u; h.uvwt.y = v; h.uvwt.z = 0.0f; h.uvwt.w = t;
            hits[i] = h;
        } else {
            hits[i].shapeid = -1;
            hits[i].primid = -1;
        }
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

MCRT_DEV v3 cameraDir(const mcrt_camera& cam, int x, int y) {   // PathTracing.cl:13-35
    const float rx = 1.0f / (float)cam.width, ry = 1.0f / (float)cam.height;
    const float u = (float)x * rx, v = (float)y * ry;
    return normalize(mix(mix(ld3(cam.r00), ld3(cam.r10), u), mix(ld3(cam.r01), ld3(cam.r11), u), v));
}

// Camera ray generation fused with the first closest-hit query (RTPrimaryRaysPass).
__global__ __launch_bounds__(TRACE_BLOCK) void k_primary(TraceCtx c, FrameArgs f, const mcrt_camera* __restrict__ camp,
                                                         int* work, float4* __restrict__ hitOut) {
    __shared__ uint32_t lds[STACK_LDS * TRACE_BLOCK];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* stk = lds + wv * 64 * STACK_LDS + lane;
    uint32_t* spill = laneSpill(c);
    const mcrt_camera cam = *camp;
    const int ntiles = f.numTiles;
    for (;;) {
        int tile = 0;
        if (lane == 0) tile = atomicAdd(work, 1);
        tile = __shfl(tile, 0);
        if (tile >= ntiles) break;
        int x, y;
        if (!tilePixel(f, tile, lane, x, y)) continue;
        TraceRay r;
        r.o = ld3(cam.pos);
        r.d = cameraDir(cam, x, y);
        r.tmax = 1000.0f;
        r.mask = -1;
        float t;
        int tri = traverse<false>(c.nodes, c.tris, r, stk, spill, c.spillCap, c.overflow, t);
        float4 h = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
        if (tri >= 0) {
            const float4 A = c.tris[3 * tri], E1 = c.tris[3 * tri + 1], E2 = c.tris[3 * tri + 2];
            float u, v;
            triBary(r.o + t * r.d, A, E1, E2, u, v);
            h = make_float4(u, v, t, __int_as_float(tri));
        }
        hitOut[(size_t)y * f.W + x] = h;
    }
}

// Closest hit over the extension queue: qO = (o.xyz, pix), qD = (d.xyz, flags); tmax = 1000.
__global__ __launch_bounds__(TRACE_BLOCK) void k_extend(TraceCtx c, const int* __restrict__ count, int* work,
                                                        const float4* __restrict__ qO, const float4* __restrict__ qD,
                                                        float4* __restrict__ hitOut) {
    __shared__ uint32_t lds[STACK_LDS * TRACE_BLOCK];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* stk = lds + wv * 64 * STACK_LDS + lane;
    uint32_t* spill = laneSpill(c);
    const int n = *count;
    for (;;) {
        const int base = nextChunk(work, lane);
        if (base >= n) break;
        const int i = base + lane;
        if (i >= n) continue;
        const float4 o = qO[i], d = qD[i];
        TraceRay r;
        r.o = ld3(o);
        r.d = ld3(d);
        r.tmax = RT_MAX_TRACE_F;
        r.mask = -1;
        float t;
        int tri = traverse<false>(c.nodes, c.tris, r, stk, spill, c.spillCap, c.overflow, t);
        float4 h = make_float4(0.f, 0.f, 0.f, __int_as_float(-1));
        if (tri >= 0) {
            const float4 A = c.tris[3 * tri], E1 = c.tris[3 * tri + 1], E2 = c.tris[3 * tri + 2];
            float u, v;
            triBary(r.o + t * r.d, A, E1, E2, u, v);
            h = make_float4(u, v, t, __int_as_float(tri));
        }
        hitOut[i] = h;
    }
}

// Any hit over the shadow queue + ShadowPass (PathTracing.cl:186-217):
// sO = (o.xyz, tmax), sD = (d.xyz, pix), sL = throughput * L; radiance[pix] += L * V.
__global__ __launch_bounds__(TRACE_BLOCK) void k_shadow(TraceCtx c, const int* __restrict__ count, int* work,
                                                        const float4* __restrict__ sO, const float4* __restrict__ sD,
                                                        const float4* __restrict__ sL, float4* __restrict__ radiance) {
    __shared__ uint32_t lds[STACK_LDS * TRACE_BLOCK];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* stk = lds + wv * 64 * STACK_LDS + lane;
    uint32_t* spill = laneSpill(c);
    const int n = *count;
    for (;;) {
        const int base = nextChunk(work, lane);
        if (base >= n) break;
        const int i = base + lane;
        if (i >= n) continue;
        const float4 o = sO[i], d = sD[i], L = sL[i];
        TraceRay r;
        r.o = ld3(o);
        r.d = ld3(d);
        r.tmax = o.w;
        r.mask = -1;
        float t;
        int tri = traverse<true>(c.nodes, c.tris, r, stk, spill, c.spillCap, c.overflow, t);
        const float V = tri >= 0 ? 0.0f : 1.0f;
        const int pix = __float_as_int(d.w);
        float4 acc = radiance[pix];
        acc.x += L.x * V;
        acc.y += L.y * V;
        acc.z += L.z * V;
        radiance[pix] = acc;
    }
}

// ---------------------------------------------------------------------------
// shading
// ---------------------------------------------------------------------------
// KRN/textures.cl:70-125 (bilinear RGBA8, wrap modes)
MCRT_DEV float4 readTex(const SceneArgs& s, int texId, v2 uv) {
    const mcrt_texture_desc td = s.textures[texId];
    const int w = td.width, h = td.height;
    uv.x -= 1.0f / (float)w * 0.5f;
    uv.y -= 1.0f / (float)h * 0.5f;
    switch (td.wrap) {
    case 0: uv.x -= floorf(uv.x); uv.y -= floorf(uv.y); break;
    case 1:
        if (uv.x > 1.0f || uv.x < 0.0f) uv.x = 1.0f - (uv.x - floorf(uv.x));
        if (uv.y > 1.0f || uv.y < 0.0f) uv.y = 1.0f - (uv.y - floorf(uv.y));
        break;
    case 2: uv.x = clampf(uv.x, 0.0f, 1.0f); uv.y = clampf(uv.y, 0.0f, 1.0f); break;
    case 3:
        if (uv.x > 1.0f || uv.x < 0.0f || uv.y > 1.0f || uv.y < 0.0f) return make_float4(0.f, 0.f, 0.f, 0.f);
        break;
    }
    int x0 = ((int)floorf(uv.x * (float)w)) % w;
    int y0 = ((int)floorf(uv.y * (float)h)) % h;
    int x1 = (x0 + 1) % w, y1 = (y0 + 1) % h;
    x0 = min(max(x0, 0), w - 1); y0 = min(max(y0, 0), h - 1);
    x1 = min(max(x1, 0), w - 1); y1 = min(max(y1, 0), h - 1);
    const float tx = uv.x * (float)w - floorf(uv.x * (float)w);
    const float ty = uv.y * (float)h - floorf(uv.y * (float)h);
    const uchar4* base = reinterpret_cast<const uchar4*>(s.texData + td.memOffset);
    const uchar4 p00 = base[x0 + y0 * w], p10 = base[x1 + y0 * w], p01 = base[x0 + y1 * w], p11 = base[x1 + y1 * w];
    auto lerp = [&](float a, float b, float c, float d) {
        float m0 = a + (b - a) * tx, m1 = c + (d - c) * tx;
        return (m0 + (m1 - m0) * ty) * (1.0f / 255.0f);
    };
    return make_float4(lerp(p00.x, p10.x, p01.x, p11.x), lerp(p00.y, p10.y, p01.y, p11.y),
                       lerp(p00.z, p10.z, p01.z, p11.z), lerp(p00.w, p10.w, p01.w, p11.w));
}

// KRN/materials.cl:76-91
MCRT_DEV Uber uberProps(const SceneArgs& s, const mcrt_material& m, v2 uv) {
    Uber u;
    float4 kdo = make_float4(1.f, 1.f, 1.f, 1.f);
    if (m.uber_diffuseTexId != -1) kdo = readTex(s, m.uber_diffuseTexId, uv);
    u.kd = mk3(kdo.x, kdo.y, kdo.z) * ld3(m.uber_kd);
    v3 t3 = mk3(1, 1, 1);
    if (m.uber_glossyTexId != -1) { float4 t = readTex(s, m.uber_glossyTexId, uv); t3 = mk3(t.x, t.y, t.z); }
    u.ks = t3 * ld3(m.uber_ks);
    t3 = mk3(1, 1, 1);
    if (m.uber_specReflectionTexId != -1) { float4 t = readTex(s, m.uber_specReflectionTexId, uv); t3 = mk3(t.x, t.y, t.z); }
    u.kr = t3 * ld3(m.uber_kr);
    t3 = mk3(1, 1, 1);
    if (m.uber_transmissionTexId != -1) { float4 t = readTex(s, m.uber_transmissionTexId, uv); t3 = mk3(t.x, t.y, t.z); }
    u.kt = t3 * ld3(m.uber_kt);
    u.ktw = m.uber_kt.w;
    t3 = mk3(1, 1, 1);
    if (m.uber_opacityTexId != -1) { float4 t = readTex(s, m.uber_opacityTexId, uv); t3 = mk3(t.x, t.y, t.z); }
    u.op = (t3 * ld3(m.uber_opacity)) * kdo.w;
    v2 r = v2{m.uber_roughness.x, m.uber_roughness.y};
    if (m.uber_roughnessTexId != -1) { float4 t = readTex(s, m.uber_roughnessTexId, uv); r = v2{t.x, t.y}; }
    u.eta = m.uber_eta;
    if (m.uber_iorTexId != -1) u.eta = readTex(s, m.uber_iorTexId, uv).x;
    u.a = v2{roughnessToAlpha(r.x), roughnessToAlpha(r.y)};
    return u;
}

// Wave-aggregated queue append: returns this lane's slot (valid where pred).
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

struct ShadeOut {
    bool pushS, pushE;
    float4 sO, sD, sL;   // shadow ray
    float4 eO, eD, eT;   // extension ray + throughput
};

// PathTracing kernel body (PathTracing.cl:52-184) for one path.
// Returns the radiance term added at this vertex by emission (or by a NaN NEE term
// with no shadow ray).  NEE terms go to the shadow queue.
MCRT_DEV v3 shadePath(const SceneArgs& s, const FrameArgs& f, int bounce, int pix, float4 hit, v3 dir, v3 throughput,
                      int prevFlags, ShadeOut& o) {
    o.pushS = false;
    o.pushE = false;
    v3 add = mk3(0, 0, 0);
    const int tri = __float_as_int(hit.w);
    if (tri < 0 || s.numLights <= 0) return add;
    const float4 A = s.tris[3 * tri], E1 = s.tris[3 * tri + 1];
    const int shapeId = __float_as_int(A.w), primIdx = __float_as_int(E1.w);
    const mcrt_shape& sh = s.shapes[shapeId];
    // computeSurfaceInteraction, geometry.cl:177-215
    const uint32_t ib = sh.startIdx + 3u * (uint32_t)primIdx;
    const uint32_t i0 = s.indices[ib] + sh.startVertex, i1 = s.indices[ib + 1] + sh.startVertex,
                   i2 = s.indices[ib + 2] + sh.startVertex;
    const v3 p0 = xformPt(sh.toWorldTransform, ld3(s.positions[i0]));
    const v3 p1 = xformPt(sh.toWorldTransform, ld3(s.positions[i1]));
    const v3 p2 = xformPt(sh.toWorldTransform, ld3(s.positions[i2]));
    const float2 uv0 = s.uvs[i0], uv1 = s.uvs[i1], uv2 = s.uvs[i2];
    const v3 nn0 = xformVec(sh.toWorldInverseTranspose, ld3(s.normals[i0]));
    const v3 nn1 = xformVec(sh.toWorldInverseTranspose, ld3(s.normals[i1]));
    const v3 nn2 = xformVec(sh.toWorldInverseTranspose, ld3(s.normals[i2]));
    const float bu = hit.x, bv = hit.y, w0 = 1.0f - bu - bv;
    Frame fr;
    fr.p = p0 * w0 + p1 * bu + p2 * bv;
    fr.uv = v2{uv0.x * w0 + uv1.x * bu + uv2.x * bv, uv0.y * w0 + uv1.y * bu + uv2.y * bv};
    fr.gn = normalize(cross(p0 - p2, p1 - p2));
    fr.sn = normalize(nn0 * w0 + nn1 * bu + nn2 * bv);
    v3 dpdu, dpdv;
    {   // geometry.cl:9-28
        const float du02x = uv0.x - uv2.x, du02y = uv0.y - uv2.y, du12x = uv1.x - uv2.x, du12y = uv1.y - uv2.y;
        const v3 dp02 = p0 - p2, dp12 = p1 - p2;
        const float det = du02x * du12y - du02y * du12x;
        if (isNotNearZero(det)) {
            const float invdet = 1.0f / det;
            dpdu = (du12y * dp02 - du02y * dp12) * invdet;
            dpdv = (-((-du12x) * dp02 + du02x * dp12)) * invdet;
        } else {
            dpdu = normalize(orthogonalVector(fr.sn));
            dpdv = normalize(cross(fr.sn, dpdu));
        }
    }
    fr.t = normalize(dpdu - dot(fr.sn, dpdu) * fr.sn);
    fr.b = normalize(dpdv - dot(fr.sn, dpdv) * fr.sn - dot(fr.t, dpdv) * fr.t);
    const v3 wo = -dir;
    float offset = dot(fr.gn, wo) < 0.0f ? -RT_TRACE_OFFSET_F : RT_TRACE_OFFSET_F;
    const int matId = sh.materialId;
    mcrt_material mat;
    if (matId != -1) {
        mat = s.materials[matId];
        if (mat.uber_normalMapId != -1) {   // materials.cl:14-30
            const float4 tn = readTex(s, mat.uber_normalMapId, fr.uv);
            const v3 nm = mk3(2.0f * tn.x - 1.0f, 2.0f * tn.y - 1.0f, 2.0f * tn.z - 1.0f);
            fr.sn = normalize(fr.t * nm.x + fr.b * nm.y + fr.sn * nm.z);
            fr.t = normalize(cross(fr.sn, fr.b));
            fr.b = normalize(cross(fr.t, fr.sn));
        }
    }
    if (bounce == 0) throughput = mk3(1.0f, 1.0f, 1.0f);
    // emission (PathTracing.cl:86-101)
    if (sh.lightID != -1 && (bounce == 0 || (prevFlags & BSDF_SPECULAR) == BSDF_SPECULAR)) {
        const mcrt_light& L = s.lights[sh.lightID];
        v3 Le = mk3(0, 0, 0);
        if ((L.type == MCRT_DISK_AREA_LIGHT || L.type == MCRT_TRIANGLE_MESH_AREA_LIGHT) && dot(fr.gn, wo) > 0.0f)
            Le = ld3(L.intensity);
        return throughput * Le;
    }
    Sampler smp = makeSampler(f.sampler, (uint32_t)pix, f.frame, bounce, f.W, f.H, s.sobol);
    // next-event estimation: one light (PathTracing.cl:107-136, lights.cl:45-146)
    {
        uint32_t li = (uint32_t)floorf(sample1D(smp) * (float)s.numLights);
        li %= (uint32_t)s.numLights;
        const v2 u = sample2D(smp);
        const mcrt_light L = s.lights[li];
        v3 wi = mk3(0, 0, 0), Li = mk3(0, 0, 0);
        float pdf = 0.0f;
        bool shadowSet = false;
        v3 so = mk3(0, 0, 0);
        float stmax = 0.0f;
        const v3 ro = fr.p + fr.gn * offset;
        if (L.type == MCRT_DIRECTIONAL_LIGHT) {
            wi = -ld3(L.d);
            pdf = 1.0f;
            so = ro; stmax = 1000.0f; shadowSet = true;
            Li = ld3(L.intensity);
        } else if (L.type == MCRT_POINT_LIGHT) {
            v3 w = ld3(L.p) - fr.p;
            const float d2 = dot(w, w);
            if (!isNearZero(d2)) {
                const float dist = sqrtf(d2);
                wi = w / dist;
                pdf = 1.0f;
                so = ro; stmax = dist; shadowSet = true;
                Li = ld3(L.intensity) / d2;
            }
        } else if (L.type == MCRT_DISK_AREA_LIGHT || L.type == MCRT_TRIANGLE_MESH_AREA_LIGHT) {
            v3 lp, lg;
            if (L.type == MCRT_DISK_AREA_LIGHT) {   // samplers.cl:259-269
                const v2 d2 = concentricDisc(u);
                const v3 n = ld3(L.d);
                const v3 t = orthogonalVector(n);
                const v3 b = normalize(cross(n, t));
                lp = ld3(L.p) + t * d2.x * L.radius + b * d2.y * L.radius;
                lg = n;
                pdf = 1.0f / (PI_F * L.radius * L.radius);
            } else {   // lights.cl:102-141, samplers.cl:227-231,275-285
                const mcrt_shape& ls = s.shapes[L.shapeId];
                const int nt = (int)ls.numTriangles;
                const int k = (int)((uint32_t)((int)floorf(u.x * (float)ls.numTriangles)) % ls.numTriangles);
                v2 uu = v2{u.x * (float)nt - (float)k, u.y};
                const uint32_t lb = ls.startIdx + 3u * (uint32_t)k;
                const v3 q0 = xformPt(ls.toWorldTransform, ld3(s.positions[ls.startVertex + s.indices[lb]]));
                const v3 q1 = xformPt(ls.toWorldTransform, ld3(s.positions[ls.startVertex + s.indices[lb + 1]]));
                const v3 q2 = xformPt(ls.toWorldTransform, ld3(s.positions[ls.startVertex + s.indices[lb + 2]]));
                const float su0 = sqrtf(uu.x);
                const float bx = 1.0f - su0, by = uu.y * su0;
                lp = bx * q0 + by * q1 + (1.0f - bx - by) * q2;
                lg = normalize(cross(q1 - q0, q2 - q0));
                pdf = 1.0f / L.area;
            }
            const v3 rt = lp + lg * RT_TRACE_OFFSET_F;
            wi = (L.type == MCRT_DISK_AREA_LIGHT) ? normalize(rt - ro) : normalize(lp - fr.p);
            const v3 dd = lp - fr.p;
            const float dist2 = dot(dd, dd);
            const float cth = absDot(lg, -wi);
            if (isNearZero(cth)) {
                pdf = 0.0f;
            } else {
                pdf *= dist2 / cth;
                so = ro;
                stmax = length(ro - rt);
                shadowSet = true;
                Li = dot(lg, -wi) > 0.0f ? ld3(L.intensity) : mk3(0, 0, 0);
            }
        }
        pdf *= L.choicePdf;
        v3 Lo = mk3(0, 0, 0);
        Uber um;
        if (matId != -1) {
            um = uberProps(s, mat, fr.uv);
            v3 bsdf = uberEval(um, fr, wo, wi);
            bsdf = bsdf * absDot(wi, fr.sn);
            if (!isNearZero(pdf)) Lo = (Li * bsdf) / pdf;
        }
        const v3 term = throughput * Lo;
        if (term.x != 0.0f || term.y != 0.0f || term.z != 0.0f) {
            if (shadowSet) {
                o.pushS = true;
                o.sO = make_float4(so.x, so.y, so.z, stmax);
                o.sD = make_float4(wi.x, wi.y, wi.z, __int_as_float(pix));
                o.sL = make_float4(term.x, term.y, term.z, 0.0f);
            } else {
                add = term * 0.0f;   // V = 0 (NaN stays NaN, ShadowPass semantics)
            }
        }
        // extension (PathTracing.cl:138-175)
        if (bounce + 1 < f.maxDepth) {
            const v2 bs = sample2D(smp);
            if (matId != -1) {
                v3 wn;
                float bpdf;
                int st;
                const v3 fb = uberSample(um, fr, bs, wo, wn, bpdf, st);
                if (!(isNearZero(bpdf) || isBlack(fb))) {
                    const v3 tp = (fb / bpdf) * absDot(wn, fr.sn);
                    const v3 nt = throughput * tp;
                    float off = offset;
                    if ((st & BSDF_TRANSMISSION) != 0 && dot(fr.gn, wn) * signf(off) < 0.0f) off *= -1.0f;
                    const v3 no = fr.p + fr.gn * off;
                    bool alive = true;
                    if (f.russianRoulette && bounce + 1 >= f.rrStartDepth) {   // perf mode only
                        const float q = fmaxf(0.05f, 1.0f - fmaxf(nt.x, fmaxf(nt.y, nt.z)));
                        const float ur = (float)wangHash((uint32_t)pix * 9781u + (uint32_t)f.frame * 6271u + (uint32_t)bounce) * 0x1p-32f;
                        alive = ur >= q;
                        o.eT = make_float4(nt.x / (1.0f - q), nt.y / (1.0f - q), nt.z / (1.0f - q), 0.0f);
                    } else {
                        o.eT = make_float4(nt.x, nt.y, nt.z, 0.0f);
                    }
                    if (alive) {
                        o.pushE = true;
                        o.eO = make_float4(no.x, no.y, no.z, __int_as_float(pix));
                        o.eD = make_float4(wn.x, wn.y, wn.z, __int_as_float(st));
                    }
                }
            }
        }
    }
    return add;
}

// Bounce 0: every pixel of the band (tile order); writes radiance[pix] (= `=` of ShadowPass).
__global__ __launch_bounds__(256) void k_shade0(SceneArgs s, FrameArgs f, const mcrt_camera* __restrict__ camp,
                                                const float4* __restrict__ hits, float4* __restrict__ radiance,
                                                QueueArgs q) {
    const int lane = threadIdx.x & 63;
    const int tile = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int x = 0, y = 0;
    bool valid = tile < f.numTiles && tilePixel(f, tile, lane, x, y);
    ShadeOut o;
    o.pushS = o.pushE = false;
    if (valid) {
        const mcrt_camera& cam = *camp;
        const int pix = y * (int)f.W + x;
        const v3 dir = cameraDir(cam, x, y);
        const v3 add = shadePath(s, f, 0, pix, hits[pix], dir, mk3(1, 1, 1), 0, o);
        radiance[pix] = make_float4(add.x, add.y, add.z, 0.0f);
    }
    const int ss = waveAppend(q.shadowCount, o.pushS);
    if (o.pushS) { q.sO[ss] = o.sO; q.sD[ss] = o.sD; q.sL[ss] = o.sL; }
    const int es = waveAppend(q.extCountOut, o.pushE);
    if (o.pushE) { q.eOout[es] = o.eO; q.eDout[es] = o.eD; q.eTout[es] = o.eT; }
}

// Bounce >= 1: the compacted extension queue of the previous bounce.
__global__ __launch_bounds__(256) void k_shadeN(SceneArgs s, FrameArgs f, int bounce, const int* __restrict__ countIn,
                                                const float4* __restrict__ qO, const float4* __restrict__ qD,
                                                const float4* __restrict__ qT, const float4* __restrict__ hits,
                                                float4* __restrict__ radiance, QueueArgs q) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = *countIn;
    ShadeOut o;
    o.pushS = o.pushE = false;
    if (i < n) {
        const float4 O = qO[i], D = qD[i], Tp = qT[i];
        const int pix = __float_as_int(O.w);
        const v3 add = shadePath(s, f, bounce, pix, hits[i], ld3(D), ld3(Tp), __float_as_int(D.w), o);
        if (add.x != 0.0f || add.y != 0.0f || add.z != 0.0f || add.x != add.x) {
            float4 r = radiance[pix];
            r.x += add.x; r.y += add.y; r.z += add.z;
            radiance[pix] = r;
        }
    }
    const int ss = waveAppend(q.shadowCount, o.pushS);
    if (o.pushS) { q.sO[ss] = o.sO; q.sD[ss] = o.sD; q.sL[ss] = o.sL; }
    const int es = waveAppend(q.extCountOut, o.pushE);
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
    const float4 r = radiance[pix];
    const float4 c = make_float4(clampf(r.x, 0.0f, 1000.0f), clampf(r.y, 0.0f, 1000.0f), clampf(r.z, 0.0f, 1000.0f),
                                 clampf(r.w, 0.0f, 1000.0f));
    float4 s;
    float ws;
    if (frame == 0) {
        s = make_float4(c.x * w, c.y * w, c.z * w, c.w * w);
        ws = w;
    } else {
        s = wsum[pix];
        s.x += c.x * w; s.y += c.y * w; s.z += c.z * w; s.w += c.w * w;
        ws = wts[pix] + w;
    }
    wsum[pix] = s;
    wts[pix] = ws;
    image[pix] = make_float4(s.x / ws, s.y / ws, s.z / ws, s.w / ws);
}

// image = sum / weight after a multi-GPU reduce of the accumulators
__global__ __launch_bounds__(256) void k_resolve(int n, const float4* __restrict__ wsum, const float* __restrict__ wts,
                                                 float4* __restrict__ image) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 s = wsum[i];
    const float w = wts[i];
    image[i] = make_float4(s.x / w, s.y / w, s.z / w, s.w / w);
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
namespace mcrt {

void launch_trace_rays(bool any, const TraceCtx& c, const mcrt_ray* rays, int n, int* work, mcrt_intersection* hits,
                       int* occl, int grid, hipStream_t st) {
    if (any)
        hipLaunchKernelGGL(k_trace_rays<true>, dim3(grid), dim3(TRACE_BLOCK), 0, st, c, rays, n, work, hits, occl);
    else
        hipLaunchKernelGGL(k_trace_rays<false>, dim3(grid), dim3(TRACE_BLOCK), 0, st, c, rays, n, work, hits, occl);
}
void launch_primary(const TraceCtx& c, const FrameArgs& f, const mcrt_camera* cam, int* work, float4* hits, int grid,
                    hipStream_t st) {
    hipLaunchKernelGGL(k_primary, dim3(grid), dim3(TRACE_BLOCK), 0, st, c, f, cam, work, hits);
}
void launch_extend(const TraceCtx& c, const int* count, int* work, const float4* qO, const float4* qD, float4* hits,
                   int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_extend, dim3(grid), dim3(TRACE_BLOCK), 0, st, c, count, work, qO, qD, hits);
}
void launch_shadow(const TraceCtx& c, const int* count, int* work, const float4* sO, const float4* sD,
                   const float4* sL, float4* radiance, int grid, hipStream_t st) {
    hipLaunchKernelGGL(k_shadow, dim3(grid), dim3(TRACE_BLOCK), 0, st, c, count, work, sO, sD, sL, radiance);
}
void launch_shade0(const SceneArgs& s, const FrameArgs& f, const mcrt_camera* cam, const float4* hits,
                   float4* radiance, const QueueArgs& q, hipStream_t st) {
    const int blocks = (f.numTiles * 64 + 255) / 256;
    hipLaunchKernelGGL(k_shade0, dim3(blocks), dim3(256), 0, st, s, f, cam, hits, radiance, q);
}
void launch_shadeN(const SceneArgs& s, const FrameArgs& f, int bounce, const int* countIn, const float4* qO,
                   const float4* qD, const float4* qT, const float4* hits, float4* radiance, const QueueArgs& q,
                   int maxCount, hipStream_t st) {
    const int blocks = (maxCount + 255) / 256;
    hipLaunchKernelGGL(k_shadeN, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, s, f, bounce, countIn, qO, qD, qT,
                       hits, radiance, q);
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

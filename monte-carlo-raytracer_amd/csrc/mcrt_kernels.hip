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
#include <algorithm>

#include <rocprim/device/device_scan.hpp>

#include "mcrt_device.h"
#include "mcrt_internal.h"
#include "mcrt_traverse.h"
#include "mcrt_shading.h"

// Shading workgroup sizes (threads; one queue atomic per workgroup and queue).  The extension rays
// a workgroup appends are grouped by direction inside its queue slice, so a larger first-shading
// workgroup hands the incoherent launch longer single-group runs (512 / 256 measured best,
// profiles/r03/ab item 17; the sweep's knobs: tools/experiments/r3_knobs.patch).
#ifndef SHADE0_BLOCK
#define SHADE0_BLOCK 512
#endif
#define SHADEN_BLOCK 256
// (register caps for more resident waves spill and lose: k_shade0 at 5 waves +7 %, the last-bounce
// k_shadeN at 6 waves +33 %; profiles/r04/ab/README.txt items 14-15)
// direction groups of the first shading's extension rays: octant x dominant axis, appended with
// one LDS atomic per record (profiles/r03/ab items 18-19)
#define MCRT_EXT_GROUPS 24

// ---------------------------------------------------------------------------
// RadeonRays-compatible queries on AoS rays (mcrt_trace_closest / mcrt_trace_any).
// One ray per lane, one wave per workgroup (LDS stack 4 KB): the hardware dispatcher keeps
// 8 waves per SIMD resident and refills them as they finish -- measured faster on MI355X
// than a persistent grid pulling work from an atomic queue.
// ---------------------------------------------------------------------------
template <bool ANY, int LAY>
__global__ __launch_bounds__(64) void k_trace_rays(TraceCtx c, const mcrt_ray* __restrict__ rays, int n,
                                                   const int* __restrict__ countDev,
                                                   mcrt_intersection* __restrict__ hits, int* __restrict__ occl) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[STACK_LDS * 64];
    if (countDev) n = min(n, *countDev);   // RR's numrays in remote memory (radeon_rays.h:272-277)
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
    if (ANY) {
        occl[i] = traceAny<LAY>(c, r, lds + lane, raySpill(c, blockIdx.x, lane)) ? 1 : -1;
        return;
    }
    float t;
    const float4 h4 = traceClosest<LAY>(c, r, lds + lane, raySpill(c, blockIdx.x, lane), t);
    if (__float_as_int(h4.z) >= 0) {
        mcrt_intersection h;
        h.shapeid = __float_as_int(h4.z);
        h.primid = __float_as_int(h4.w);
        h.padding[0] = h.padding[1] = 0;
        h.uvwt.x = h4.x; h.uvwt.y = h4.y; h.uvwt.z = 0.0f; h.uvwt.w = t;
        hits[i] = h;
    } else {
        hits[i].shapeid = -1;
        hits[i].primid = -1;
    }
}

// Surface records (SceneArgs::surf): record r of mesh m (meshBase[m] <= r < meshBase[m+1]) is
// triangle p = r - meshBase[m] of the (startIdx, startVertex) range, packed as
// (p0 p1.x | p1.yz p2.xy | p2.z uv0 uv1.x | uv1.y uv2 n0.x | n0.yz n1.xy | n1.z n2) + 2 pad float4.
__global__ void k_surface_records(const uint32_t* __restrict__ meshStartIdx, const uint32_t* __restrict__ meshStartVertex,
                                  const uint32_t* __restrict__ meshBase, int numMeshes, uint32_t numRecords,
                                  const uint32_t* __restrict__ indices, const float4* __restrict__ positions,
                                  const float2* __restrict__ uvs, const float4* __restrict__ normals,
                                  float4* __restrict__ surf) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= numRecords) return;
    int lo = 0, hi = numMeshes - 1;   // last mesh with meshBase <= r
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (meshBase[mid] <= r) lo = mid; else hi = mid - 1;
    }
    const uint32_t p = r - meshBase[lo];
    const uint32_t* ix = indices + meshStartIdx[lo] + 3 * p;
    const uint32_t sv = meshStartVertex[lo];
    const float4 a = positions[sv + ix[0]], b = positions[sv + ix[1]], c = positions[sv + ix[2]];
    const float2 ta = uvs[sv + ix[0]], tb = uvs[sv + ix[1]], tc = uvs[sv + ix[2]];
    const float4 na = normals[sv + ix[0]], nb = normals[sv + ix[1]], nc = normals[sv + ix[2]];
    float4* R = surf + 8 * (size_t)r;
    R[0] = make_float4(a.x, a.y, a.z, b.x);
    R[1] = make_float4(b.y, b.z, c.x, c.y);
    R[2] = make_float4(c.z, ta.x, ta.y, tb.x);
    R[3] = make_float4(tb.y, tc.x, tc.y, na.x);
    R[4] = make_float4(na.y, na.z, nb.x, nb.y);
    R[5] = make_float4(nb.z, nc.x, nc.y, nc.z);
    R[6] = make_float4(0.f, 0.f, 0.f, 0.f);
    R[7] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Packed waves of a batch of n frames: the n waves of tile t (tileAll = t*n .. t*n + n-1) hold the
// tile's 64 x n paths (pixel pi, frame k) in pixel-major order, q = 64 * (tileAll - t*n) + lane =
// pi * n + k.  Each (pi, k) is covered once for any n; for n | 64 a wave is 64/n whole pixels.
MCRT_DEV void packedPath(const FrameArgs& f, int tileAll, int lane, int& k, int& tile, int& pi) {
    tile = tileAll / f.batch;
    const int q = (tileAll - tile * f.batch) * 64 + lane;
    pi = q / f.batch;
    k = q - pi * f.batch;
}

// Slot of a camera-ray hit record (k_primary* write it, k_shade0 / k_aov read it).  Packed waves:
// (tile, pixel-in-tile, frame) with the frames fastest, the packed launches' own order, so a wave's
// 64 records are one contiguous 1-KB run for its writes and reads (frame-plane order,
// k * W*H + pixel, put each lane of a packed wave in another plane).  Else the frame plane's pixel.
MCRT_DEV size_t hitSlot(const FrameArgs& f, int tile, int pi, int k, int x, int y) {
    if (f.primaryPack && f.batch > 1) return ((size_t)tile * 64 + (size_t)pi) * (size_t)f.batch + (size_t)k;
    return (size_t)k * f.W * f.H + (size_t)y * f.W + x;
}

// Camera ray generation fused with the first closest-hit query (RTPrimaryRaysPass):
// one workgroup = one wave = one 8x8 pixel tile of the rank's bands.
template <int LAY>
__global__ __launch_bounds__(64) void k_primary(TraceCtx c, FrameArgs f, const mcrt_camera* __restrict__ camp,
                                                float4* __restrict__ hitOut) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[STACK_LDS * 64];
    const int lane = threadIdx.x;
    const int tileAll = xcdRemap(blockIdx.x, gridDim.x);
    int k, tile, pi = lane;
    if (f.primaryPack && f.batch > 1) {
        // a wave = 64 consecutive (pixel, frame) paths of one tile, frames fastest: the same
        // pixel's TAA-jittered rays walk nearly the same nodes, so the lanes' loads coalesce
        packedPath(f, tileAll, lane, k, tile, pi);
    } else {
        splitTileFrame(f, tileAll, k, tile);
    }
    int x, y;
    if (tile >= f.numTiles || k >= f.batch || !tilePixel(f, tile, pi, x, y)) return;
    const mcrt_camera& cam = camp[k];
    TraceRay r;
    r.o = ld3(cam.pos);
    r.d = cameraDir(cam, x, y);
    r.tmax = 1000.0f;
    r.mask = -1;
    float t;
    hitOut[hitSlot(f, tile, pi, k, x, y)] = traceClosest<LAY>(c, r, lds + lane, raySpill(c, tileAll, lane), t);
}

// The camera-ray launch with wave-packet traversal (traversePacket, plain records): the same rays
// and hit records as k_primary.
__global__ __launch_bounds__(64) void k_primary_pk(TraceCtx c, FrameArgs f, const mcrt_camera* __restrict__ camp,
                                                   float4* __restrict__ hitOut) {
    const int lane = threadIdx.x;
    const int tileAll = orderedTileAll(f, xcdRemap(blockIdx.x, gridDim.x));
    int k, tile, pi = lane;
    if (f.primaryPack && f.batch > 1) {
        packedPath(f, tileAll, lane, k, tile, pi);
    } else {
        splitTileFrame(f, tileAll, k, tile);
    }
    int x = 0, y = 0;
    const bool valid = tile < f.numTiles && k < f.batch && tilePixel(f, tile, pi, x, y);
    TraceRay r;
    r.o = splat3(0.0f);
    r.d = f3{0.0f, 0.0f, 1.0f};
    if (valid) {
        const mcrt_camera& cam = camp[k];
        r.o = ld3(cam.pos);
        r.d = cameraDir(cam, x, y);
    }
    r.tmax = 1000.0f;
    r.mask = -1;
    float t;
    const uint32_t clk0 = (c.waveClock || f.tileCost) ? waveClockNow() : 0u;
    const int tri = traversePacket<false>(c.nodes, r, valid, t);
    if (valid) hitOut[hitSlot(f, tile, pi, k, x, y)] = closestRecord(c.nodes, r, tri, t);
    waveClockStore(c.waveClock, clk0);
    // the wave's time into its tile's cost (the next call's longest-first order): one atomic per wave
    if (f.tileCost && lane == 0 && tile < f.numTiles) atomicAdd(&f.tileCost[tile], waveClockNow() - clk0);
}

// A stopped extension walk (TraceCtx::walkCap) of queue slot i, whose lane owns spill column `col`
// (wave col / 64, lane col % 64), appended to the suspend list for k_walk_resume: MCRT_SUSPEND_F4
// float4 = (slot, next record, t, culling t), (tie t, hit, sp, spillTop), the 16 LDS stack entries
// with entry 0 (the QREF_DONE sentinel) replaced by the column.  Divergent call: suspended lanes only.
MCRT_DEV void suspendWalk(const TraceCtx& c, int i, int col, const QWalk& w, const uint32_t* stk) {
    const int slot = waveAppend(c.suspendCount, true);
    float4* sv = c.suspend + (size_t)slot * MCRT_SUSPEND_F4;
    sv[0] = make_float4(__int_as_float(i), __uint_as_float(w.ref), w.t, w.tc);
    sv[1] = make_float4(w.tieT, __int_as_float(w.hit), __int_as_float(w.sp), __int_as_float(w.spillTop));
    for (int k = 0; k < STACK_LDS / 4; ++k)
        sv[2 + k] = make_float4(__uint_as_float(k == 0 ? (uint32_t)col : stk[(4 * k) * 64]), __uint_as_float(stk[(4 * k + 1) * 64]),
                                __uint_as_float(stk[(4 * k + 2) * 64]), __uint_as_float(stk[(4 * k + 3) * 64]));
}

// Closest hit of queue slot i by a lane owning spill column `col`; over the compact records with a
// stop rule (TraceCtx::walkCap) a walk still running when its wave stops is suspended instead
// (k_walk_resume writes hitOut[i] then).
template <int LAY>
MCRT_DEV void closestOrSuspend(const TraceCtx& c, const TraceRay& r, uint32_t* stk, int col, int i,
                               float4* __restrict__ hitOut) {
    uint32_t* spill = raySpill(c, col >> 6, col & 63);
    if constexpr (LAY == LAY_QUANT) {
        if (c.walkCap > 0) {
            QWalk w = qwalkStart(c, r, stk);
            qwalk<false, -2, true>(c, r, safeInvDir(r.d), stk, spill, w, c.walkCap, c.walkLanes);
            if (w.ref != QREF_DONE)
                suspendWalk(c, i, col, w, stk);
            else
                hitOut[i] = qwalkClosest(c, r, stk, spill, w);
            return;
        }
    }
    float t;
    hitOut[i] = traceClosest<LAY>(c, r, stk, spill, t);
}

// Closest hit over the extension queue: qO = (o.xyz, pix), qD = (d.xyz, flags); tmax = 1000.
// The grid covers the queue's capacity; workgroups past the device-side count exit at once.
template <int LAY>
// perm (optional): the queue walked in this order (BDPT's bounce rays sorted by direction octant and
// origin cell, mcrt::bdpt_light_sort over k_bdpt_vertex's keys); hit records go back to their slots.
__global__ __launch_bounds__(64) void k_extend(TraceCtx c, const int* __restrict__ count, const float4* __restrict__ qO,
                                               const float4* __restrict__ qD, float4* __restrict__ hitOut,
                                               const uint32_t* __restrict__ perm) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[STACK_LDS * 64];
    const int n = *count;
    if ((int)blockIdx.x * 64 >= n) return;
    const int lane = threadIdx.x;
    const int blk = xcdRemap(blockIdx.x, (n + 63) >> 6);
    const int j = blk * 64 + lane;
    if (j >= n) return;
    const int i = perm ? (int)perm[j] : j;
    const float4 o = qO[i], d = qD[i];
    TraceRay r;
    r.o = ld3(o);
    r.d = ld3(d);
    r.tmax = RT_MAX_TRACE_F;
    r.mask = -1;
    closestOrSuspend<LAY>(c, r, lds + lane, j, i, hitOut);
}

// Any hit over the shadow queue + ShadowPass (PathTracing.cl:186-217):
// sO = (o.xyz, tmax), sD = (d.xyz, pix), sL = throughput * L; radiance[pix] += L * V.
template <int LAY>
__global__ __launch_bounds__(64) void k_shadow(TraceCtx c, const int* __restrict__ count, const float4* __restrict__ sO,
                                               const float4* __restrict__ sD, const float4* __restrict__ sL,
                                               float4* __restrict__ radiance) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[STACK_LDS * 64];
    const int n = *count;
    if ((int)blockIdx.x * 64 >= n) return;
    const int lane = threadIdx.x;
    const int blk = xcdRemap(blockIdx.x, (n + 63) >> 6);
    const int i = blk * 64 + lane;
    if (i >= n) return;
    const float4 o = sO[i], d = sD[i], L = sL[i];
    TraceRay r;
    r.o = ld3(o);
    r.d = ld3(d);
    r.tmax = o.w;
    r.mask = -1;
    const int pix = __float_as_int(d.w);
    const uint32_t clk0 = c.waveClock ? waveClockNow() : 0u;
    const float V = shadowOccluded<LAY>(c, r, pix, lds + lane, raySpill(c, blk, lane)) ? 0.0f : 1.0f;
    float4 acc = radiance[pix];
    acc.x += L.x * V;
    acc.y += L.y * V;
    acc.z += L.z * V;
    radiance[pix] = acc;
    waveClockStore(c.waveClock, clk0);
}

// Shadow rays of bounce b and extension rays of bounce b+1 in ONE launch: both only depend on
// the shading of bounce b.  Extension workgroups come first (their rays are the longer ones),
// shadow workgroups fill the extension launch's divergent tail instead of waiting for it.
template <int LAY>
__global__ __launch_bounds__(64) void k_shadow_extend(TraceCtx c, const int* __restrict__ extCount,
                                                      const float4* __restrict__ qO, const float4* __restrict__ qD,
                                                      float4* __restrict__ hitOut, const int* __restrict__ shadowCount,
                                                      const float4* __restrict__ sO, const float4* __restrict__ sD,
                                                      const float4* __restrict__ sL, float4* __restrict__ radiance) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[STACK_LDS * 64];
    const int ne = *extCount;
    const int eb = (ne + 63) >> 6;
    const int lane = threadIdx.x;
    if ((int)blockIdx.x < eb) {
        const int blk = xcdRemap(blockIdx.x, eb);
        const int i = blk * 64 + lane;
        if (i >= ne) return;
        const float4 o = qO[i], d = qD[i];
        TraceRay r;
        r.o = ld3(o);
        r.d = ld3(d);
        r.tmax = RT_MAX_TRACE_F;
        r.mask = -1;
        const uint32_t clk0 = c.waveClock ? waveClockNow() : 0u;
        // with a stop rule the wave stops once it has taken walkCap steps and at most walkLanes
        // lanes are still walking: those are suspended and finished by k_walk_resume in dense
        // waves, so a few long walks no longer hold a mostly idle wave
        closestOrSuspend<LAY>(c, r, lds + lane, i, i, hitOut);
        waveClockStore(c.waveClock, clk0);
    } else {
        const int ns = *shadowCount;
        const int sb = (ns + 63) >> 6;
        if ((int)blockIdx.x - eb >= sb) return;
        const int i = xcdRemap((int)blockIdx.x - eb, sb) * 64 + lane;
        if (LAY != LAY_TWO_LEVEL && c.packet) {
            // bounce-0 shadow rays: a wave's rays leave a few pixels for one light (packed waves), so
            // they walk the tree as one packet (any hit: the answers do not depend on the order)
            const bool valid = i < ns;
            TraceRay r;
            r.o = splat3(0.0f);
            r.d = f3{0.0f, 0.0f, 1.0f};
            r.tmax = 0.0f;
            float4 d = make_float4(0.f, 0.f, 1.f, 0.f);
            if (valid) {
                const float4 o = sO[i];
                d = sD[i];
                r.o = ld3(o);
                r.d = ld3(d);
                r.tmax = o.w;
            }
            r.mask = -1;
            // lanes whose occluder hint holds leave the packet before it starts
            const int pix = __float_as_int(d.w);
            uint32_t h = 0, h2 = 0;
            bool occ = false;
            if (valid && c.hint) {
                h = hintSlot(c, r, pix);
                // the origin cell's occluder as a second candidate (profiles/r04/ab/README.txt item 12)
                h2 = hintCellSlot(c, r);
                const uint32_t l1 = c.hint[h], l2 = c.hintCell[h2];
                const bool o1 = hintOccludes(c, r, l1), o2 = l2 != l1 && hintOccludes(c, r, l2);
                occ = o1 || o2;
            }
            countHintHits(c, occ);
            float tt;
            const int leaf = traversePacket<true>(c.nodes, r, valid && !occ, tt);
            if (leaf >= 0) {
                occ = true;
                if (c.hint) {   // the next hint of the pixel and of the origin cell
                    c.hint[h] = (uint32_t)leaf;
                    c.hintCell[h2] = (uint32_t)leaf;
                }
            }
            if (valid) {
                const float V = occ ? 0.0f : 1.0f;
                const float4 L = sL[i];
                float4 acc = radiance[pix];
                acc.x += L.x * V;
                acc.y += L.y * V;
                acc.z += L.z * V;
                radiance[pix] = acc;
            }
            return;
        }
        if (i >= ns) return;
        const float4 o = sO[i], d = sD[i], L = sL[i];
        TraceRay r;
        r.o = ld3(o);
        r.d = ld3(d);
        r.tmax = o.w;
        r.mask = -1;
        const int pix = __float_as_int(d.w);
        const float V = shadowOccluded<LAY>(c, r, pix, lds + lane, raySpill(c, blockIdx.x, lane)) ? 0.0f : 1.0f;
        float4 acc = radiance[pix];
        acc.x += L.x * V;
        acc.y += L.y * V;
        acc.z += L.z * V;
        radiance[pix] = acc;
    }
}

// The extension walks k_shadow_extend suspended (TraceCtx::walkCap): each lane restores one walk's
// state -- next record, hit so far, LDS stack; its spill entries stay in the spill column the
// suspending lane owned -- and finishes it, then writes its queue slot's hit record.  The same
// steps as one uncut walk, so the same record bit for bit.
__global__ __launch_bounds__(64) void k_walk_resume(TraceCtx c, const float4* __restrict__ qO,
                                                    const float4* __restrict__ qD, float4* __restrict__ hitOut) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[STACK_LDS * 64];
    const int n = *c.suspendCount;
    if ((int)blockIdx.x * 64 >= n) return;
    const int lane = threadIdx.x;
    const int j = blockIdx.x * 64 + lane;
    if (j >= n) return;
    const float4* sv = c.suspend + (size_t)j * MCRT_SUSPEND_F4;
    const float4 s0 = sv[0], s1 = sv[1];
    const int i = __float_as_int(s0.x);
    uint32_t* stk = lds + lane;
    uint32_t col = 0;
    for (int k = 0; k < STACK_LDS / 4; ++k) {
        const float4 e = sv[2 + k];
        if (k == 0) col = __float_as_uint(e.x);   // entry 0 is the QREF_DONE sentinel: saved as the column
        stk[(4 * k) * 64] = k == 0 ? QREF_DONE : __float_as_uint(e.x);
        stk[(4 * k + 1) * 64] = __float_as_uint(e.y);
        stk[(4 * k + 2) * 64] = __float_as_uint(e.z);
        stk[(4 * k + 3) * 64] = __float_as_uint(e.w);
    }
    QWalk w{__float_as_uint(s0.y), s0.z, s0.w, s1.x, __float_as_int(s1.y), __float_as_int(s1.z), __float_as_int(s1.w)};
    const float4 o = qO[i], d = qD[i];
    TraceRay r;
    r.o = ld3(o);
    r.d = ld3(d);
    r.tmax = RT_MAX_TRACE_F;
    r.mask = -1;
    uint32_t* spill = raySpill(c, (int)(col >> 6), (int)(col & 63));
    qwalk<false, -2>(c, r, safeInvDir(r.d), stk, spill, w);
    hitOut[i] = qwalkClosest(c, r, stk, spill, w);
}

// Closest hit over two queues in ONE launch: BDPT's first camera rays (coherent: wave packets when
// cc.packet) and first light rays (per ray, c).  The camera
// workgroups come first; the light workgroups fill their tail (as k_shadow_extend).
// perm1 (optional): queue 1 walked in this order (BDPT's light rays sorted by origin / direction
// cell, mcrt::bdpt_light_sort): the j-th ray traced is slot perm1[j], its hit record goes back to
// that slot.  (As wave packets, the sorted parallel rays of a directional light ran 16 % slower
// than per ray: profiles/r04/ab/README.txt.)
template <int LAY0, int LAY1>
__global__ __launch_bounds__(64) void k_extend_pair(TraceCtx cc, TraceCtx c, const int* __restrict__ count0,
                                                    const float4* __restrict__ qO0, const float4* __restrict__ qD0,
                                                    float4* __restrict__ hit0, const int* __restrict__ count1,
                                                    const float4* __restrict__ qO1, const float4* __restrict__ qD1,
                                                    float4* __restrict__ hit1, const uint32_t* __restrict__ perm1) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[STACK_LDS * 64];
    const int n0 = *count0;
    const int b0 = (n0 + 63) >> 6;
    const int lane = threadIdx.x;
    TraceRay r;
    r.tmax = RT_MAX_TRACE_F;
    r.mask = -1;
    float t;
    if ((int)blockIdx.x < b0) {
        const int blk = xcdRemap(blockIdx.x, b0);
        const int i = blk * 64 + lane;
        if (LAY0 == LAY_PLAIN && cc.packet) {   // camera rays of 8x8 tiles: wave packets
            const bool valid = i < n0;
            r.o = valid ? ld3(qO0[i]) : splat3(0.0f);
            r.d = valid ? ld3(qD0[i]) : f3{0.0f, 0.0f, 1.0f};
            const int tri = traversePacket<false>(cc.nodes, r, valid, t);
            if (valid) hit0[i] = closestRecord(cc.nodes, r, tri, t);
            return;
        }
        if (i >= n0) return;
        r.o = ld3(qO0[i]);
        r.d = ld3(qD0[i]);
        hit0[i] = traceClosest<LAY0>(cc, r, lds + lane, raySpill(cc, blk, lane), t);
    } else {
        const int n1 = *count1;
        const int b1 = (n1 + 63) >> 6;
        if ((int)blockIdx.x - b0 >= b1) return;
        const int j = xcdRemap((int)blockIdx.x - b0, b1) * 64 + lane;
        if (perm1 == nullptr) {
            if (j >= n1) return;
            r.o = ld3(qO1[j]);
            r.d = ld3(qD1[j]);
            closestOrSuspend<LAY1>(c, r, lds + lane, (int)blockIdx.x * 64 + lane, j, hit1);
            return;
        }
        if (j >= n1) return;
        const int i = (int)perm1[j];
        r.o = ld3(qO1[i]);
        r.d = ld3(qD1[i]);
        closestOrSuspend<LAY1>(c, r, lds + lane, (int)blockIdx.x * 64 + lane, i, hit1);
    }
}

// PathTracing kernel body (PathTracing.cl:52-184) for one path.
// Returns the radiance term added at this vertex by emission (or by a NaN NEE term
// with no shadow ray).  NEE terms go to the shadow queue.
struct ShadeOut {
    bool pushS, pushE;
    float4 sO, sD, sL;   // shadow ray
    float4 eO, eD, eT;   // extension ray + throughput
};

// LOD (k_shade0 with mcrt_frame_params.texture_lod): textures at this camera-ray hit are read
// mip-mapped over the pixel footprint given by the ray differentials (ro, dxDir, dyDir).
// EXT = false: the last bounce's instantiation (no extension ray; its sampling code and registers
// are left out, so the launch keeps more waves resident).  RR: the opt-in Russian roulette has its
// own instantiation, so the default one carries none of its registers (k_shade0: 95 VGPRs, 5 waves
// per SIMD, instead of 97 and 4).
template <bool LOD = false, bool EXT = true, bool RR = false>
MCRT_DEV f3 shadePath(const SceneArgs& s, const FrameArgs& f, int bounce, int pix, float4 hit, f3 dir, f3 throughput,
                      int prevFlags, ShadeOut& o, f3 ro = f3{0, 0, 0}, f3 dxDir = f3{0, 0, 0}, f3 dyDir = f3{0, 0, 0}) {
    f3 add = splat3(0.0f);
    const int shapeIdx = __float_as_int(hit.z), primIdx = __float_as_int(hit.w);
    if (shapeIdx < 0 || s.numLights <= 0) return add;
    const mcrt_shape shape = tableEntry(s.shapes, shapeIdx);
    f3 dpdu, dpdv;
    Frame si = computeSurfaceInteraction(s, shape, shapeIdx, primIdx, f2{hit.x, hit.y}, LOD ? &dpdu : nullptr,
                                         LOD ? &dpdv : nullptr);
    TexLod lod{{0.0f, 0.0f}, {0.0f, 0.0f}, false};
    if (LOD) lod = surfaceUVDifferentials(si, dpdu, dpdv, ro, dxDir, dyDir);
    const f3 wo = -dir;
    const bool isBackfacing = cl_dot(si.gn, wo) < 0.0f;
    const float traceErrorOffset = isBackfacing ? -RT_TRACE_OFFSET_F : RT_TRACE_OFFSET_F;
    const int materialId = shape.materialId;
    mcrt_material mat;
    if (materialId != -1) {
        mat = tableEntry(s.materials, materialId);
        if (mat.uber_normalMapId != -1) applyNormalMapping(s, mat.uber_normalMapId, si, lod);
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
    int px = pix, frame = f.frame;
    if (f.batch > 1) {   // batched launch: path id -> (frame k, pixel)
        const int k = (int)((uint32_t)pix / (f.W * f.H));
        px = pix - k * (int)(f.W * f.H);
        frame += k;
    }
    Sampler sampler = makeSampler(f.sampler, (uint32_t)px, frame, bounce, f.W, f.H, s.sobol);
    const bool isUber = materialId != -1 && mat.type == 0;   // materials.cl:130-142: other types evaluate to 0
    Uber um;
    if (isUber) um = uberProps(s, mat, si.uv, lod);
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
    if (EXT && bounce + 1 < f.maxDepth) {
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
                if (RR && bounce + 1 >= f.rrStartDepth) {   // opt-in perf mode
                    const float qr = fmaxf(0.05f, 1.0f - fmaxf(nt.x, fmaxf(nt.y, nt.z)));
                    const float ur = (float)wangHash((uint32_t)px * 9781u + (uint32_t)frame * 6271u + (uint32_t)bounce) * 0x1p-32f;
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
template <bool LOD, bool RR>
__global__ __launch_bounds__(SHADE0_BLOCK) void k_shade0(SceneArgs s, FrameArgs f, const mcrt_camera* __restrict__ camp,
                                                const float4* __restrict__ hits, float4* __restrict__ radiance,
                                                QueueArgs q) {
    const int lane = threadIdx.x & 63;
    // XCD-aware block order: an XCD shades contiguous runs of tiles (their hits share surface
    // records, materials and textures in its L2): k_shade0 -4 %
    const int tileAll = orderedTileAll(f, xcdRemap(blockIdx.x, gridDim.x) * (SHADE0_BLOCK / 64) + (int)(threadIdx.x >> 6));
    int k, tile, pi = lane;   // batch frame k
    if (f.shadePack && f.batch > 1) {
        // as k_primary's packed waves; the bounce-0 shadow rays of a wave (one light direction,
        // nearly one origin) and its extension rays stay together
        packedPath(f, tileAll, lane, k, tile, pi);
    } else {
        splitTileFrame(f, tileAll, k, tile);
    }
    int x = 0, y = 0;
    bool valid = k < f.batch && tile < f.numTiles && tilePixel(f, tile, pi, x, y);
    __shared__ int ldsWave[SHADE0_BLOCK / 64 + 1];
    __shared__ int ldsGroup[MCRT_EXT_GROUPS + 1];
    ShadeOut o;
    o.pushS = o.pushE = false;
    o.eD = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (valid) {
        const mcrt_camera& cam = camp[k];
        const int pix = k * (int)(f.W * f.H) + y * (int)f.W + x;
        const f3 dir = cameraDir(cam, x, y);
        f3 dx = splat3(0.0f), dy = splat3(0.0f);
        if (LOD) cameraDiffDirs(cam, x, y, dx, dy);
        const f3 add = shadePath<LOD, true, RR>(s, f, 0, pix, hits[hitSlot(f, tile, pi, k, x, y)], dir, splat3(1.0f), 0,
                                                o, ld3(cam.pos), dx, dy);
        radiance[pix] = make_float4(add.x, add.y, add.z, 0.0f);
    }
    const int ss = blockAppend<SHADE0_BLOCK / 64>(q.shadowCount, o.pushS, ldsWave);
    if (o.pushS) { q.sO[ss] = o.sO; q.sD[ss] = o.sD; q.sL[ss] = o.sL; }
    // extension rays grouped by direction octant x dominant axis inside the block's queue slice
    int oct = (o.eD.x < 0.0f ? 1 : 0) | (o.eD.y < 0.0f ? 2 : 0) | (o.eD.z < 0.0f ? 4 : 0);
    {
        const float ax = fabsf(o.eD.x), ay = fabsf(o.eD.y), az = fabsf(o.eD.z);
        oct = oct * 3 + (ax >= ay && ax >= az ? 0 : ay >= az ? 1 : 2);
    }
    const int es = blockAppendGroupedLds<MCRT_EXT_GROUPS>(q.extCountOut, o.pushE, oct, ldsGroup);
    if (o.pushE) { q.eOout[es] = o.eO; q.eDout[es] = o.eD; q.eTout[es] = o.eT; }
}

// Bounce >= 1: the compacted extension queue of the previous bounce.  LAST: bounce maxDepth - 1.
template <bool LAST, bool RR>
__global__ __launch_bounds__(SHADEN_BLOCK) void k_shadeN(SceneArgs s, FrameArgs f, int bounce, const int* __restrict__ countIn,
                                                const float4* __restrict__ qO, const float4* __restrict__ qD,
                                                const float4* __restrict__ qT, const float4* __restrict__ hits,
                                                float4* __restrict__ radiance, QueueArgs q) {
    const int n = *countIn;
    __shared__ int ldsWave[SHADEN_BLOCK / 64 + 1];
    __shared__ int ldsGroup[(SHADEN_BLOCK / 64) * 8 + 1];
    if ((int)blockIdx.x * SHADEN_BLOCK >= n) return;   // whole block past the queue: uniform exit
    // XCD-aware block order (xcdRemap): each XCD shades contiguous runs of the queue, whose paths
    // share triangles, materials and textures in that XCD's L2
    const int i = xcdRemap(blockIdx.x, (n + SHADEN_BLOCK - 1) / SHADEN_BLOCK) * SHADEN_BLOCK + threadIdx.x;
    ShadeOut o;
    o.pushS = o.pushE = false;
    o.eD = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (i < n) {
        const float4 O = qO[i], D = qD[i], Tp = qT[i];
        const int pix = __float_as_int(O.w);
        const f3 add = shadePath<false, !LAST, RR>(s, f, bounce, pix, hits[i], ld3(D), ld3(Tp), __float_as_int(D.w), o);
        if (add.x != 0.0f || add.y != 0.0f || add.z != 0.0f || add.x != add.x) {
            float4 r = radiance[pix];
            r.x += add.x; r.y += add.y; r.z += add.z;
            radiance[pix] = r;
        }
    }
    const int ss = blockAppend<SHADEN_BLOCK / 64>(q.shadowCount, o.pushS, ldsWave);
    if (o.pushS) { q.sO[ss] = o.sO; q.sD[ss] = o.sD; q.sL[ss] = o.sL; }
    if (LAST) return;
    // extension rays grouped by direction octant inside the block's queue slice
    const int oct = (o.eD.x < 0.0f ? 1 : 0) | (o.eD.y < 0.0f ? 2 : 0) | (o.eD.z < 0.0f ? 4 : 0);
    const int es = blockAppendGrouped<SHADEN_BLOCK / 64, 8>(q.extCountOut, o.pushE, oct, ldsGroup);
    if (o.pushE) { q.eOout[es] = o.eO; q.eDout[es] = o.eD; q.eTout[es] = o.eT; }
}

// ---------------------------------------------------------------------------
// Per-pixel outputs of the camera-ray hits (mcrt_render_aov), tile order as k_shade0.
//   MCRT_AOV_ALBEDO:     1 float4 = (uber Kd incl. texture, opacity.x); LOD per f.textureLod
//   MCRT_AOV_TEXTURE_LOD: 3 float4 = (duvdx, duvdy), (diffuse-texture LOD, shape, uv),
//                         the diffuse texture read mip-mapped (zeros where untextured)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_aov(SceneArgs s, FrameArgs f, const mcrt_camera* __restrict__ camp,
                                             const float4* __restrict__ hits, int which, float4* __restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int tile = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int x, y;
    if (tile >= f.numTiles || !tilePixel(f, tile, lane, x, y)) return;
    const int pix = y * (int)f.W + x;
    const int stride = which == MCRT_AOV_TEXTURE_LOD ? 3 : 1;
    float4* o = out + (size_t)pix * stride;
    for (int k = 0; k < stride; ++k) o[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const float4 hit = hits[hitSlot(f, tile, lane, 0, x, y)];
    const int shapeIdx = __float_as_int(hit.z), primIdx = __float_as_int(hit.w);
    if (shapeIdx < 0) return;
    const mcrt_camera& cam = *camp;
    f3 dpdu, dpdv, dx, dy;
    const Frame si = computeSurfaceInteraction(s, shapeIdx, primIdx, f2{hit.x, hit.y}, &dpdu, &dpdv);
    cameraDiffDirs(cam, x, y, dx, dy);
    TexLod L = surfaceUVDifferentials(si, dpdu, dpdv, ld3(cam.pos), dx, dy);
    const int materialId = s.shapes[shapeIdx].materialId;
    if (which == MCRT_AOV_TEXTURE_LOD) {
        float lod = 0.0f;
        f4 c = f4{0.0f, 0.0f, 0.0f, 0.0f};
        if (materialId != -1 && s.materials[materialId].uber_diffuseTexId != -1) {
            const int t = s.materials[materialId].uber_diffuseTexId;
            const mcrt_texture_desc tex = s.textures[t];
            lod = mipLod(tex, L.duvdx, L.duvdy);
            c = readTexLodDesc(s, tex, si.uv, lod);
        }
        o[0] = make_float4(L.duvdx.x, L.duvdx.y, L.duvdy.x, L.duvdy.y);
        o[1] = make_float4(lod, __int_as_float(shapeIdx), si.uv.x, si.uv.y);
        o[2] = make_float4(c.x, c.y, c.z, c.w);
    } else {
        L.on = f.textureLod != 0;
        if (materialId != -1 && s.materials[materialId].type == 0) {
            const Uber u = uberProps(s, s.materials[materialId], si.uv, L);
            o[0] = make_float4(u.Kd.x, u.Kd.y, u.Kd.z, u.opacity.x);
        }
    }
}

// ---------------------------------------------------------------------------
// ReconstructionPass (KRN/reconstruction.cl:6-60) with the filters of KRN/filters.cl:12-69,
// evaluated on the device as the reference does (same expression shapes, so clang contracts the
// same products into fma; `/` is the OpenCL-default 2.5-ulp division, cl_div; exp and sin are the
// device library's, like OpenCL's).  The weight is uniform per frame (one pixelOffset per frame,
// RTReconstructionPass.cpp:71-123); pinned against the reference's filters.cl run live
// (oracle/refbuild/clprobe_filters.cl, tests/test_gpu_accumulate.py).  Band rows only.
// ---------------------------------------------------------------------------
MCRT_DEV float filterTriangle(f2 p, f2 radius) {   // filters.cl:17-20
    return fmaxf(0.0f, radius.x - fabsf(p.x)) * fmaxf(0.0f, radius.y - fabsf(p.y));
}
MCRT_DEV float filterGaussian1D(float d, float alpha, float expv) {   // filters.cl:22-25
    return fmaxf(0.0f, expf(-alpha * d * d) - expv);
}
MCRT_DEV float filterMitchell1D(float x, float B, float C) {   // filters.cl:32-39
    x = fabsf(2.0f * x);
    if (x > 1.0f)
        return ((-B - 6*C) * x*x*x + (6*B + 30*C) * x*x + (-12*B - 48*C) * x + (8*B + 24*C)) * (1.f/6.f);
    else
        return ((12 - 9*B - 6*C) * x*x*x + (-18 + 12*B + 6*C) * x*x + (6 - 2*B)) * (1.f/6.f);
}
MCRT_DEV float filterSinc(float x) {   // filters.cl:47-54 (1e-5 is a float literal: no cl_khr_fp64 pragma)
    x = fabsf(x);
    if (x < 1e-5f) return 1.0f;
    return cl_div(sinf(PI_F * x), (PI_F * x));
}
MCRT_DEV float filterWindowedSinc(float x, float radius, float tau) {   // filters.cl:56-64
    x = fabsf(x);
    if (x > radius) return 0.0f;
    const float lanczos = filterSinc(cl_div(x, tau));
    return filterSinc(x) * lanczos;
}
// the switch of reconstruction.cl:23-42
MCRT_DEV float filterWeight(const mcrt_filter& fp) {
    const f2 p = f2{fp.pixelOffset.x, fp.pixelOffset.y}, radius = f2{fp.radius.x, fp.radius.y};
    switch (fp.filterType) {
    case MCRT_TRIANGLE_FILTER: return filterTriangle(p, radius);
    case MCRT_GAUSSIAN_FILTER:
        return filterGaussian1D(p.x, fp.gaussianAlpha, fp.gaussianExpX) * filterGaussian1D(p.y, fp.gaussianAlpha, fp.gaussianExpY);
    case MCRT_MITCHELL_FILTER:
        return filterMitchell1D(cl_div(p.x, radius.x), fp.mitchellB, fp.mitchellC) *
               filterMitchell1D(cl_div(p.y, radius.y), fp.mitchellB, fp.mitchellC);
    case MCRT_LANCZOS_SINC_FILTER:
        return filterWindowedSinc(p.x, radius.x, fp.lanczosSincTau) * filterWindowedSinc(p.y, radius.y, fp.lanczosSincTau);
    default: return 1.0f;   // RT_BOX_FILTER
    }
}

// A batch of f.batch frames (mcrt_render_frames) is accumulated in frame order, frame + k with
// filter filters[k * fstride]: per pixel the same operations as f.batch single-frame launches.
__global__ __launch_bounds__(256) void k_accumulate(FrameArgs f, int frame, const mcrt_filter* __restrict__ filters, int fstride,
                                                    const float4* __restrict__ radiance, float4* __restrict__ wsum,
                                                    float* __restrict__ wts, float4* __restrict__ image) {
    const int lane = threadIdx.x & 63;
    const int tile = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    int x, y;
    if (tile >= f.numTiles || !tilePixel(f, tile, lane, x, y)) return;
    const int pix = y * (int)f.W + x;
    f4 s;
    float ws;
    if (frame != 0) {
        const float4 o = wsum[pix];
        s = f4{o.x, o.y, o.z, o.w};
        ws = wts[pix];
    }
    for (int k = 0; k < f.batch; ++k) {
        const float4 r4 = radiance[(size_t)k * f.W * f.H + pix];
        const f4 radiance4 = f4{cl_clamp(r4.x, 0.0f, 1000.0f), cl_clamp(r4.y, 0.0f, 1000.0f),
                                cl_clamp(r4.z, 0.0f, 1000.0f), cl_clamp(r4.w, 0.0f, 1000.0f)};
        const float w = filterWeight(filters[k * fstride]);
        if (frame + k == 0) {
            s = radiance4 * w;
            ws = w;
        } else {
            s += radiance4 * w;   // contracted to fma, as reconstruction.cl:50
            ws = ws + w;
        }
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

// Tile split, end of job: a rank's own rows of the accumulators in its band order (local 8-row
// block tb at rows 8 tb .. 8 tb + 7, tilePixel's numbering; mcrt.dist.band_rows_of), one packed row
// = W x (sum w*L as 4 floats) then W x sum w, straight from the frame buffer: no full-frame copy
// before the gather.  bpb = band_rows / 8.
__device__ __forceinline__ void bandOwner(int y, int bpb, int numBands, int& r, int& row) {
    const int gb = y >> 3;
    r = (gb / bpb) % numBands;
    row = ((gb / (bpb * numBands)) * bpb + gb % bpb) * 8 + (y & 7);
}

__global__ __launch_bounds__(256) void k_band_pack(int W, int H, int bpb, int numBands, int band,
                                                   const float4* __restrict__ wsum, const float* __restrict__ wts,
                                                   float* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W * H) return;
    const int y = i / W, x = i - y * W;
    int r, row;
    bandOwner(y, bpb, numBands, r, row);
    if (r != band) return;
    float* o = out + (size_t)row * 5 * W;
    const float4 v = wsum[i];
    o[4 * x] = v.x;
    o[4 * x + 1] = v.y;
    o[4 * x + 2] = v.z;
    o[4 * x + 3] = v.w;
    o[4 * W + x] = wts[i];
}

// Rank dst after the gather: every other rank's rows (recv = numBands x maxRows packed rows) into
// the accumulators in place, then the image (k_resolve's division) in the same pass.
__global__ __launch_bounds__(256) void k_band_unpack(int W, int H, int bpb, int numBands, int band, int maxRows,
                                                     const float* __restrict__ recv, float4* __restrict__ wsum,
                                                     float* __restrict__ wts, float4* __restrict__ image) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= W * H) return;
    const int y = i / W, x = i - y * W;
    int r, row;
    bandOwner(y, bpb, numBands, r, row);
    float4 s;
    float w;
    if (r == band) {
        s = wsum[i];
        w = wts[i];
    } else {
        const float* p = recv + ((size_t)r * maxRows + row) * 5 * W;
        s = make_float4(p[4 * x], p[4 * x + 1], p[4 * x + 2], p[4 * x + 3]);
        w = p[4 * W + x];
        wsum[i] = s;
        wts[i] = w;
    }
    image[i] = make_float4(cl_div(s.x, w), cl_div(s.y, w), cl_div(s.z, w), cl_div(s.w, w));
}

// ---------------------------------------------------------------------------
// Post-process (the reference's RTDenoisePass + RTToneMappingPass after reconstruction)
// ---------------------------------------------------------------------------
#define DENOISE_TILE 16
#define DENOISE_RMAX 16
// BilateralDenoise (KRN/Denoise.cl:6-47): a 16x16 tile plus its clamped apron staged in LDS
// once (the reference re-reads the (2r+1)^2 window through the image unit per pixel); the
// window is walked in the reference's order (x outer, y inner) so the sums round identically.
__global__ __launch_bounds__(DENOISE_TILE * DENOISE_TILE) void k_denoise(int W, int H, int r, float ss, float sr,
                                                                         const float4* __restrict__ in,
                                                                         float4* __restrict__ out) {
    __shared__ float4 tile[(DENOISE_TILE + 2 * DENOISE_RMAX) * (DENOISE_TILE + 2 * DENOISE_RMAX)];
    const int TW = DENOISE_TILE + 2 * r;
    const int x0 = blockIdx.x * DENOISE_TILE - r, y0 = blockIdx.y * DENOISE_TILE - r;
    const int tid = threadIdx.y * DENOISE_TILE + threadIdx.x;
    for (int i = tid; i < TW * TW; i += DENOISE_TILE * DENOISE_TILE) {
        const int gx = min(max(x0 + i % TW, 0), W - 1), gy = min(max(y0 + i / TW, 0), H - 1);
        tile[i] = in[(size_t)gy * W + gx];
    }
    __syncthreads();
    const int gx = blockIdx.x * DENOISE_TILE + threadIdx.x, gy = blockIdx.y * DENOISE_TILE + threadIdx.y;
    if (gx >= W || gy >= H) return;
    const float sdSq = ss * ss, srSq = sr * sr;
    const float4 oc = tile[(gy - y0) * TW + (gx - x0)];
    const f4 o = f4{oc.x, oc.y, oc.z, oc.w};
    f4 fc = f4{0.0f, 0.0f, 0.0f, 0.0f};
    float weightSum = 0.0f;
    for (int rx = -r; rx <= r; ++rx) {
        const int x = min(max(rx + gx, 0), W - 1);
        for (int ry = -r; ry <= r; ++ry) {
            const int y = min(max(ry + gy, 0), H - 1);
            const float4 kc = tile[(y - y0) * TW + (x - x0)];
            const f4 k = f4{kc.x, kc.y, kc.z, kc.w};
            const f4 cd = o - k;
            const float d2 = fmaf(cd.w, cd.w, fmaf(cd.z, cd.z, fmaf(cd.y, cd.y, cd.x * cd.x)));   // dot(float4)
            const int sp = (gx - x) * (gx - x) + (gy - y) * (gy - y);
            const float w = expf(cl_div((float)(-sp), (2.0f * sdSq)) - cl_div(d2, (2.0f * srSq)));
            weightSum += w;
            fc += w * k;
        }
    }
    fc = cl_div(fc, weightSum);
    out[(size_t)gy * W + gx] = make_float4(fc.x, fc.y, fc.z, fc.w);
}

// ReinhardToneMapping (KRN/ToneMapping.cl:42-63), luminance of KRN/colors.cl:19-22
__global__ __launch_bounds__(256) void k_tonemap(int n, float Lwhite, const float4* __restrict__ in,
                                                 float4* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 p = in[i];
    const float L = 0.212671f * p.x + 0.715160f * p.y + 0.072169f * p.z;
    const float tL = cl_div(L * (1.0f + cl_div(L, (Lwhite * Lwhite))), (1.0f + L));
    const float s = cl_div(tL, L);
    out[i] = make_float4(p.x * s, p.y * s, p.z * s, p.w);
}

// Dependent-gather ceiling probe (mcrt_ctx_gather_chase): every lane follows a chain of 64-B
// records whose links are read from the record just fetched, fetched as four 16-B pieces -- the
// traversal's access pattern with none of its arithmetic.  The array size decides where the
// records come from (L2, Infinity Cache, HBM), so the traversal's node-visit rate can be set
// against the ceiling of its own access pattern (tools/probe/chase_probe.hip has more variants).
__global__ void k_chase_init(int4* rec, uint32_t n, uint32_t seed) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    const uint32_t nxt = h % n;
    for (int q = 0; q < 4; ++q) rec[4 * i + q] = make_int4((int)nxt, (int)(nxt ^ 1u), (int)(nxt ^ 2u), (int)nxt);
}
__global__ __launch_bounds__(64) void k_chase(const int4* __restrict__ rec, uint32_t n, int steps, uint32_t* sink) {
    const uint32_t chain = blockIdx.x * 64 + threadIdx.x;
    uint32_t h = chain * 0x9E3779B9u + 12345u;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13;
    uint32_t idx = h % n, acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4 a = rec[4 * (size_t)idx], b = rec[4 * (size_t)idx + 1];
        const int4 c = rec[4 * (size_t)idx + 2], d = rec[4 * (size_t)idx + 3];
        asm volatile("" ::"v"(a.y), "v"(b.y), "v"(c.y));
        acc += (uint32_t)(a.z ^ b.z ^ c.z);
        idx = (uint32_t)d.w;
    }
    if (acc == 0xdeadbeefu) sink[0] = idx;   // never true: keeps the loads live
}

// The chase over the compact records' layout: record i is 2 (internal, 32 B) or 3 (leaf, 48 B)
// 16-B units, packed back to back at off[i] (exclusive scan of chase_units); its link is the next
// record's reference (unit offset << 1 | leaf bit), so a leaf's third unit is fetched in the same
// round trip as in mcrt_traverse.h qwalk.
MCRT_DEV uint32_t chaseHash(uint32_t i, uint32_t seed) {
    uint32_t h = i * 2654435761u ^ seed;
    h ^= h >> 15; h *= 2246822519u; h ^= h >> 13; h *= 3266489917u; h ^= h >> 16;
    return h;
}
__global__ void k_chase_units(uint32_t* units, uint32_t n, uint32_t leaf16) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) units[i] = 2u + ((chaseHash((uint32_t)i, 99u) & 0xffffu) < leaf16 ? 1u : 0u);
}
__global__ void k_chase_init_compact(int4* rec, const uint32_t* off, const uint32_t* units, uint32_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t nxt = chaseHash((uint32_t)i, 777u) % n;
    const int ref = (int)((off[nxt] << 1) | (units[nxt] == 3u ? 1u : 0u));
    for (uint32_t q = 0; q < units[i]; ++q) rec[off[i] + q] = make_int4((int)nxt, (int)(nxt ^ 1u), (int)(nxt ^ 2u), ref);
}
__global__ __launch_bounds__(64) void k_chase_compact(const int4* __restrict__ rec, const uint32_t* __restrict__ off,
                                                      const uint32_t* __restrict__ units, uint32_t n, int steps,
                                                      uint32_t* sink) {
    const uint32_t chain = blockIdx.x * 64 + threadIdx.x;
    uint32_t h = chain * 0x9E3779B9u + 12345u;
    h ^= h >> 16; h *= 0x85EBCA6Bu; h ^= h >> 13;
    const uint32_t i0 = h % n;
    uint32_t ref = (off[i0] << 1) | (units[i0] == 3u ? 1u : 0u), acc = 0;
    for (int s = 0; s < steps; ++s) {
        const int4* p = rec + (ref >> 1);
        const int4 a = p[0], b = p[1];
        int4 c;
        asm("" : "=v"(c.x), "=v"(c.y), "=v"(c.z), "=v"(c.w));
        if (ref & 1u) c = p[2];
        asm volatile("" ::"v"(a.y), "v"(b.y), "v"(c.y));
        acc += (uint32_t)(a.z ^ b.z ^ c.z);
        ref = (uint32_t)a.w;
    }
    if (acc == 0xdeadbeefu) sink[0] = ref;   // never true: keeps the loads live
}

// Parent links of the flat tree's leaves (the occluder hints' box test, mcrt_traverse.h
// hintOccludes): every internal record writes its index into word 13 of each child that is a
// triangle leaf (mcrt_bvh.cpp leaves carry -1 there; the traversal never reads it for a leaf).
__global__ __launch_bounds__(256) void k_leaf_parents(float4* __restrict__ nodes, uint32_t n) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int4 w = *reinterpret_cast<const int4*>(&nodes[4 * (size_t)i + 3]);
    if (w.x < 0) return;
    const int ch[2] = {w.x, w.y};
    for (int k = 0; k < 2; ++k) {
        if ((uint32_t)ch[k] >= n) continue;
        int* cw = reinterpret_cast<int*>(&nodes[4 * (size_t)ch[k] + 3]);
        if (cw[0] == -1) cw[1] = (int)i;
    }
}

// Compact records (mcrt_traverse.h traverseQOct has the format and the exactness argument).
// Sizes in 16-B units per 64-B record (internal 2, leaf 3); notDfs: a left child that is not the
// next record (the LBVH's numbering) -- the compact walk takes the left child as the next record.
__global__ __launch_bounds__(256) void k_qnodes_sizes(const float4* __restrict__ nodes, uint32_t n,
                                                      uint32_t* __restrict__ units, int* __restrict__ notDfs) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const int4 w = *reinterpret_cast<const int4*>(&nodes[4 * (size_t)i + 3]);
    units[i] = w.x >= 0 ? 2u : 3u;
    if (w.x >= 0 && w.x != (int)i + 1) atomicOr(notDfs, 1);
}

// One axis of an internal record: its origin (the smaller lo) and the exponent byte e of its step,
// 2^(e - 127) >= extent / 250.  False for non-finite boxes.
MCRT_DEV bool quantExp(float lo0, float hi0, float lo1, float hi1, float& o, uint32_t& e) {
    o = fminf(lo0, lo1);
    const float ext = fmaxf(hi0, hi1) - o;
    if (!(ext >= 0.0f) || ext == __builtin_inff()) return false;
    int k = -126;
    if (ext > 0.0f) frexpf(ext * (1.0f / 250.0f), &k);   // ext / 250 <= 2^k
    e = (uint32_t)min(max(k + 127, 1), 254);
    return true;
}
// The two children's (lo, hi) on that axis as bytes q with fmaf(q, s, o) <= lo and >= hi exactly as
// the traversal decodes them; s = the walk's step (qScales: 2^(e - 127) times a mantissa the meta
// word's lower fields supply: 1 for x, about 1.24 for y and z), so 255 s covers the extent.
// False if no byte reaches.
MCRT_DEV bool quantBytes(float lo0, float hi0, float lo1, float hi1, float o, float sc, uint32_t& bytes) {
    const float b[4] = {lo0, hi0, lo1, hi1};
    bytes = 0;
    for (int j = 0; j < 4; ++j) {
        const bool up = (j & 1) != 0;   // hi bounds round up, lo bounds down
        int q = (int)(up ? ceilf((b[j] - o) / sc) : floorf((b[j] - o) / sc));
        q = min(max(q, 0), 255);
        if (up) {
            while (q < 255 && fmaf((float)q, sc, o) < b[j]) ++q;
            if (fmaf((float)q, sc, o) < b[j]) return false;
        } else {
            while (q > 0 && fmaf((float)q, sc, o) > b[j]) --q;
            if (fmaf((float)q, sc, o) > b[j]) return false;
        }
        bytes |= (uint32_t)q << (8 * j);
    }
    return true;
}

__global__ __launch_bounds__(256) void k_qnodes_convert(const float4* __restrict__ nodes, uint32_t n,
                                                        const uint32_t* __restrict__ off, float4* __restrict__ q,
                                                        int* __restrict__ fail) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const float4 n0 = nodes[4 * (size_t)i], n1 = nodes[4 * (size_t)i + 1], n2 = nodes[4 * (size_t)i + 2];
    const int4 w = *reinterpret_cast<const int4*>(&nodes[4 * (size_t)i + 3]);
    float4* dst = q + off[i];
    if (w.x >= 0) {   // child 0 box (n0.x, n0.z, n2.x)-(n0.y, n0.w, n2.y), child 1 (n1.x, n1.z, n2.z)-(n1.y, n1.w, n2.w)
        float ox, oy, oz;
        uint32_t bx = 0, by = 0, bz = 0, ex = 0, ey = 0, ez = 0;
        bool ok = quantExp(n0.x, n0.y, n1.x, n1.y, ox, ex) && quantExp(n0.z, n0.w, n1.z, n1.w, oy, ey) &&
                  quantExp(n2.x, n2.y, n2.z, n2.w, oz, ez) && (uint32_t)w.y < n;
        const uint32_t leaf0 = ok && reinterpret_cast<const int4*>(&nodes[4 * (size_t)w.x + 3])->x < 0 ? 1u : 0u;
        const uint32_t leaf1 = ok && reinterpret_cast<const int4*>(&nodes[4 * (size_t)w.y + 3])->x < 0 ? 1u : 0u;
        // the y and z steps carry a mantissa from the fields below their exponent (qScales: 1 + e_x / 512
        // for y, 1 + e_y / 512 + e_x / 2^18 for z, about 1.24): one exponent less then often still covers
        // the extent, which gives those axes the x axis's step sizes (1.44 x the ideal step on average
        // instead of 1.79); quantBytes decides, y first (z's mantissa depends on e_y)
        uint32_t meta = ex | (ey << 9) | (ez << 18) | (leaf0 << 27);
        if (ok && ey > 1 && quantBytes(n0.z, n0.w, n1.z, n1.w, oy, qScales(meta - (1u << 9)).y, by)) meta -= 1u << 9;
        if (ok && ez > 1 && quantBytes(n2.x, n2.y, n2.z, n2.w, oz, qScales(meta - (1u << 18)).z, bz)) meta -= 1u << 18;
        const QScales sc = qScales(meta);
        ok = ok && quantBytes(n0.x, n0.y, n1.x, n1.y, ox, sc.x, bx) && quantBytes(n0.z, n0.w, n1.z, n1.w, oy, sc.y, by) &&
             quantBytes(n2.x, n2.y, n2.z, n2.w, oz, sc.z, bz);
        if (!ok) {
            atomicOr(fail, 1);
            return;
        }
        dst[0] = make_float4(ox, oy, oz, __uint_as_float((off[w.y] << 1) | leaf1));
        dst[1] = make_float4(__uint_as_float(bx), __uint_as_float(by), __uint_as_float(bz), __uint_as_float(meta));
        return;
    }
// leaf: its exact box (as the parent's record stores it) must be min / max of v0, v0 + e1, v0 + e2
    // for the compact walk to test it from the triangle; else bit 31 sends the walk to the parent
    bool slow = true;
    const int par = w.y;   // k_leaf_parents
    if (par >= 0 && (uint32_t)par < n) {
        const float4 p0 = nodes[4 * (size_t)par], p1 = nodes[4 * (size_t)par + 1], p2 = nodes[4 * (size_t)par + 2];
        const bool right = reinterpret_cast<const int4*>(&nodes[4 * (size_t)par + 3])->y == (int)i;
        const f3 lo = right ? f3{p1.x, p1.z, p2.z} : f3{p0.x, p0.z, p2.x};
        const f3 hi = right ? f3{p1.y, p1.w, p2.w} : f3{p0.y, p0.w, p2.y};
        const f3 v0 = ld3(n0), v1 = v0 + ld3(n1), v2 = v0 + ld3(n2);
        const f3 l = f3{fminf(fminf(v0.x, v1.x), v2.x), fminf(fminf(v0.y, v1.y), v2.y), fminf(fminf(v0.z, v1.z), v2.z)};
        const f3 h = f3{fmaxf(fmaxf(v0.x, v1.x), v2.x), fmaxf(fmaxf(v0.y, v1.y), v2.y), fmaxf(fmaxf(v0.z, v1.z), v2.z)};
        slow = __float_as_uint(l.x) != __float_as_uint(lo.x) || __float_as_uint(l.y) != __float_as_uint(lo.y) ||
               __float_as_uint(l.z) != __float_as_uint(lo.z) || __float_as_uint(h.x) != __float_as_uint(hi.x) ||
               __float_as_uint(h.y) != __float_as_uint(hi.y) || __float_as_uint(h.z) != __float_as_uint(hi.z);
    }
    dst[0] = n0;
    dst[1] = n1;
    dst[2] = make_float4(n2.x, n2.y, n2.z, __uint_as_float(i | (slow ? 0x80000000u : 0u)));
}

// Longest-first order of the camera / first-shading tiles from the previous call's camera-wave
// times (FrameArgs::tileCost): tiles bucketed by log2 cost in 1/8 steps, buckets in descending
// order (one workgroup; a tile's place inside its bucket is arbitrary -- any order gives the same
// image).  The long waves then start first and the launch ends on short ones: at N = 8 a rank's
// camera launch spent its last 90 us (12 %) on the 1 % longest waves (tools/wave_tail.py).
__global__ __launch_bounds__(1024) void k_tile_order(const uint32_t* __restrict__ cost, int n,
                                                     uint32_t* __restrict__ order) {
    __shared__ uint32_t hist[256];
    for (int b = threadIdx.x; b < 256; b += 1024) hist[b] = 0;
    __syncthreads();
    auto bucket = [](uint32_t c) { return c == 0 ? 0 : min(255, (int)(__log2f((float)c) * 8.0f)); };
    for (int t = threadIdx.x; t < n; t += 1024) atomicAdd(&hist[bucket(cost[t])], 1u);
    __syncthreads();
    if (threadIdx.x == 0) {   // exclusive offsets, heaviest bucket first
        uint32_t acc = 0;
        for (int b = 255; b >= 0; --b) {
            const uint32_t h = hist[b];
            hist[b] = acc;
            acc += h;
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < n; t += 1024) order[atomicAdd(&hist[bucket(cost[t])], 1u)] = (uint32_t)t;
}

// Attainable-bandwidth probe (mcrt_ctx_stream_copy): a persistent grid (8 workgroups per CU)
// strides over the array; each lane keeps 4 independent 16-B nontemporal loads in flight.
__global__ __launch_bounds__(256) void k_stream_copy(const f4* __restrict__ src, f4* __restrict__ dst, size_t n) {
    const size_t step = (size_t)gridDim.x * 1024;
    for (size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x; base < n; base += step) {
        f4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (base + 256 * k < n) v[k] = __builtin_nontemporal_load(src + base + 256 * k);
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (base + 256 * k < n) __builtin_nontemporal_store(v[k], dst + base + 256 * k);
    }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------

namespace mcrt {

void launch_trace_rays(bool any, const TraceCtx& c, const mcrt_ray* rays, int n, const int* countDev,
                       mcrt_intersection* hits, int* occl, hipStream_t st) {
    const dim3 g((n + 63) / 64), b(64);
    {
        if (any)
            hipLaunchKernelGGL(pickLayout(c, k_trace_rays<true, LAY_TWO_LEVEL>, k_trace_rays<true, LAY_QUANT>,
                                          k_trace_rays<true, LAY_PLAIN>),
                               g, b, 0, st, c, rays, n, countDev, hits, occl);
        else
            hipLaunchKernelGGL(pickLayout(c, k_trace_rays<false, LAY_TWO_LEVEL>, k_trace_rays<false, LAY_QUANT>,
                                          k_trace_rays<false, LAY_PLAIN>),
                               g, b, 0, st, c, rays, n, countDev, hits, occl);
    }
}
void launch_surface_records(const uint32_t* meshStartIdx, const uint32_t* meshStartVertex, const uint32_t* meshBase,
                            int numMeshes, uint32_t numRecords, const uint32_t* indices, const float4* positions,
                            const float2* uvs, const float4* normals, float4* surf, hipStream_t st) {
    if (numRecords == 0) return;
    k_surface_records<<<(numRecords + 255) / 256, 256, 0, st>>>(meshStartIdx, meshStartVertex, meshBase, numMeshes,
                                                                numRecords, indices, positions, uvs, normals, surf);
}

void launch_primary(const TraceCtx& c, const FrameArgs& f, const mcrt_camera* cam, float4* hits, hipStream_t st) {
    if (c.packet && !c.twoLevel) {
        hipLaunchKernelGGL(k_primary_pk, dim3(f.numTiles * f.batch), dim3(64), 0, st, c, f, cam, hits);
        return;
    }
    hipLaunchKernelGGL(pickLayout(c, k_primary<LAY_TWO_LEVEL>, k_primary<LAY_PLAIN>), dim3(f.numTiles * f.batch), dim3(64), 0, st, c, f, cam,
                       hits);
}
void launch_extend(const TraceCtx& c, const int* count, const float4* qO, const float4* qD, float4* hits, int maxCount,
                   hipStream_t st, const uint32_t* perm) {
    hipLaunchKernelGGL(pickLayout(c, k_extend<LAY_TWO_LEVEL>, k_extend<LAY_QUANT>, k_extend<LAY_PLAIN>),
                       dim3((maxCount + 63) / 64), dim3(64), 0, st, c,
                       count, qO, qD, hits, perm);
}
void launch_extend_pair(const TraceCtx& cc, const TraceCtx& c, const int* count0, const float4* qO0, const float4* qD0,
                        float4* hit0, const int* count1, const float4* qO1, const float4* qD1, float4* hit1,
                        int maxCount0, int maxCount1, hipStream_t st, const uint32_t* perm1) {
    auto k = c.twoLevel ? k_extend_pair<LAY_TWO_LEVEL, LAY_TWO_LEVEL>
             : c.qnodes ? (cc.packet ? k_extend_pair<LAY_PLAIN, LAY_QUANT> : k_extend_pair<LAY_QUANT, LAY_QUANT>)
                        : k_extend_pair<LAY_PLAIN, LAY_PLAIN>;
    const int blocks = (maxCount0 + 63) / 64 + (maxCount1 + 63) / 64;
    hipLaunchKernelGGL(k, dim3(blocks > 0 ? blocks : 1), dim3(64), 0, st, cc, c, count0, qO0, qD0, hit0, count1, qO1,
                       qD1, hit1, perm1);
}
void launch_shadow(const TraceCtx& c, const int* count, const float4* sO, const float4* sD, const float4* sL,
                   float4* radiance, int maxCount, hipStream_t st) {
    hipLaunchKernelGGL(pickLayout(c, k_shadow<LAY_TWO_LEVEL>, k_shadow<LAY_QUANT>, k_shadow<LAY_PLAIN>),
                       dim3((maxCount + 63) / 64), dim3(64), 0, st, c,
                       count, sO, sD, sL, radiance);
}
void launch_shadow_extend(const TraceCtx& c, const int* extCount, const float4* qO, const float4* qD, float4* hits,
                          const int* shadowCount, const float4* sO, const float4* sD, const float4* sL,
                          float4* radiance, int maxExt, int maxShadow, hipStream_t st) {
    const int blocks = (maxExt + 63) / 64 + (maxShadow + 63) / 64;
    hipLaunchKernelGGL(pickLayout(c, k_shadow_extend<LAY_TWO_LEVEL>, k_shadow_extend<LAY_QUANT>, k_shadow_extend<LAY_PLAIN>),
                       dim3(blocks > 0 ? blocks : 1), dim3(64), 0, st, c, extCount, qO, qD, hits, shadowCount, sO, sD,
                       sL, radiance);
}
void launch_walk_resume(const TraceCtx& c, const float4* qO, const float4* qD, float4* hits, int maxExt,
                        hipStream_t st) {
    // a stopping wave suspends at most walkLanes of its lanes, so the list holds at most walkLanes per
    // 64 queue slots: the grid covers that bound, not the queue's capacity (workgroups past the
    // device-side count exit at once, but each still costs a dispatch: ~0.2 ns, tools/probe/empty_blocks.hip)
    const int64_t waves = (maxExt + 63) / 64;
    const int64_t bound = (waves * std::max(1, std::min(64, c.walkLanes)) + 63) / 64;
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(waves, bound));
    hipLaunchKernelGGL(k_walk_resume, dim3(blocks), dim3(64), 0, st, c, qO, qD, hits);
}
void launch_shade0(const SceneArgs& s, const FrameArgs& f, const mcrt_camera* cam, const float4* hits,
                   float4* radiance, const QueueArgs& q, hipStream_t st) {
    const int blocks = (f.numTiles * f.batch * 64 + SHADE0_BLOCK - 1) / SHADE0_BLOCK;
    auto k = f.russianRoulette ? (f.textureLod ? k_shade0<true, true> : k_shade0<false, true>)
                               : (f.textureLod ? k_shade0<true, false> : k_shade0<false, false>);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(SHADE0_BLOCK), 0, st, s, f, cam, hits, radiance, q);
}
void launch_shadeN(const SceneArgs& s, const FrameArgs& f, int bounce, const int* countIn, const float4* qO,
                   const float4* qD, const float4* qT, const float4* hits, float4* radiance, const QueueArgs& q,
                   int maxCount, hipStream_t st) {
    const int blocks = (maxCount + SHADEN_BLOCK - 1) / SHADEN_BLOCK;
    const bool last = bounce + 1 >= f.maxDepth;
    auto k = f.russianRoulette ? (last ? k_shadeN<true, true> : k_shadeN<false, true>)
                               : (last ? k_shadeN<true, false> : k_shadeN<false, false>);
    hipLaunchKernelGGL(k, dim3(blocks > 0 ? blocks : 1), dim3(SHADEN_BLOCK), 0, st, s, f, bounce, countIn, qO, qD, qT,
                       hits, radiance, q);
}
void launch_aov(const SceneArgs& s, const FrameArgs& f, const mcrt_camera* cam, const float4* hits, int which,
                float4* out, hipStream_t st) {
    const int blocks = (f.numTiles * 64 + 255) / 256;
    hipLaunchKernelGGL(k_aov, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, st, s, f, cam, hits, which, out);
}
void launch_accumulate(const FrameArgs& f, int frame, const mcrt_filter* filters, int filterStride, const float4* radiance,
                       float4* wsum, float* wts, float4* image, hipStream_t st) {
    const int blocks = (f.numTiles * 64 + 255) / 256;
    hipLaunchKernelGGL(k_accumulate, dim3(blocks), dim3(256), 0, st, f, frame, filters, filterStride, radiance, wsum,
                       wts, image);
}

void launch_denoise(int W, int H, int r, float ss, float sr, const float4* in, float4* out, hipStream_t st) {
    hipLaunchKernelGGL(k_denoise, dim3((W + DENOISE_TILE - 1) / DENOISE_TILE, (H + DENOISE_TILE - 1) / DENOISE_TILE),
                       dim3(DENOISE_TILE, DENOISE_TILE), 0, st, W, H, r, ss, sr, in, out);
}
void launch_tonemap(int n, float Lwhite, const float4* in, float4* out, hipStream_t st) {
    hipLaunchKernelGGL(k_tonemap, dim3((n + 255) / 256), dim3(256), 0, st, n, Lwhite, in, out);
}
void launch_chase_init(void* rec, uint32_t n, hipStream_t st) {
    hipLaunchKernelGGL(k_chase_init, dim3((n + 255) / 256), dim3(256), 0, st, reinterpret_cast<int4*>(rec), n, 777u);
}
void launch_chase(const void* rec, uint32_t n, int steps, int waves, uint32_t* sink, hipStream_t st) {
    hipLaunchKernelGGL(k_chase, dim3(waves), dim3(64), 0, st, reinterpret_cast<const int4*>(rec), n, steps, sink);
}

hipError_t chase_compact(uint32_t n, double leafFrac, int steps, int waves, int iters, hipStream_t st, float* bestMs) {
    uint32_t *units = nullptr, *off = nullptr, *sink = nullptr, last[2] = {0, 0};
    int4* rec = nullptr;
    void* tmp = nullptr;
    size_t tmpBytes = 0;
    const uint32_t leaf16 = (uint32_t)std::min(65536.0, std::max(0.0, leafFrac * 65536.0));
    hipError_t e = hipMalloc(&units, 4 * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&off, 4 * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&sink, 4);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_chase_units, dim3((n + 255) / 256), dim3(256), 0, st, units, n, leaf16);
        e = rocprim::exclusive_scan(nullptr, tmpBytes, units, off, 0u, (size_t)n, rocprim::plus<uint32_t>(), st);
    }
    if (e == hipSuccess) e = hipMalloc(&tmp, tmpBytes);
    if (e == hipSuccess) e = rocprim::exclusive_scan(tmp, tmpBytes, units, off, 0u, (size_t)n, rocprim::plus<uint32_t>(), st);
    if (e == hipSuccess) e = hipMemcpyAsync(&last[0], off + n - 1, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&last[1], units + n - 1, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) e = hipMalloc(&rec, 16 * ((size_t)last[0] + last[1]));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_chase_init_compact, dim3((n + 255) / 256), dim3(256), 0, st, rec, off, units, n);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        float best = 1e30f;
        for (int i = 0; i < iters + 1; ++i) {   // launch 0 warms caches and translations
            hipEventRecord(e0, st);
            hipLaunchKernelGGL(k_chase_compact, dim3(waves), dim3(64), 0, st, rec, off, units, n,
                               i == 0 ? std::max(1, steps / 4) : steps, sink);
            hipEventRecord(e1, st);
            hipEventSynchronize(e1);
            float ms = 0.0f;
            hipEventElapsedTime(&ms, e0, e1);
            if (i > 0 && ms < best) best = ms;
        }
        hipEventDestroy(e0);
        hipEventDestroy(e1);
        *bestMs = best;
        e = hipGetLastError();
    }
    (void)hipFree(rec);
    (void)hipFree(tmp);
    (void)hipFree(sink);
    (void)hipFree(off);
    (void)hipFree(units);
    return e;
}

void launch_leaf_parents(float4* nodes, uint32_t n, hipStream_t st) {
    if (n == 0) return;
    hipLaunchKernelGGL(k_leaf_parents, dim3((n + 255) / 256), dim3(256), 0, st, nodes, n);
}

hipError_t build_qnodes(const float4* nodes, uint32_t n, float4** qOut, size_t* unitsOut, hipStream_t st) {
    *qOut = nullptr;
    *unitsOut = 0;
    if (n == 0 || n >= (1u << 31)) return hipErrorNotSupported;
    uint32_t *units = nullptr, *off = nullptr;
    int* flags = nullptr;
    void* tmp = nullptr;
    size_t tmpBytes = 0;
    float4* q = nullptr;
    int h[2] = {0, 0};
    uint32_t lastOff = 0, lastUnits = 0;
    hipError_t e = hipMalloc(&units, 4 * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&off, 4 * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&flags, 2 * sizeof(int));
    if (e == hipSuccess) e = hipMemsetAsync(flags, 0, 2 * sizeof(int), st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_qnodes_sizes, dim3((n + 255) / 256), dim3(256), 0, st, nodes, n, units, flags);
        e = rocprim::exclusive_scan(nullptr, tmpBytes, units, off, 0u, (size_t)n, rocprim::plus<uint32_t>(), st);
    }
    if (e == hipSuccess) e = hipMalloc(&tmp, tmpBytes);
    if (e == hipSuccess) e = rocprim::exclusive_scan(tmp, tmpBytes, units, off, 0u, (size_t)n, rocprim::plus<uint32_t>(), st);
    if (e == hipSuccess) e = hipMemcpyAsync(h, flags, 2 * sizeof(int), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&lastOff, off + n - 1, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipMemcpyAsync(&lastUnits, units + n - 1, 4, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    const size_t total = (size_t)lastOff + lastUnits;
    if (e == hipSuccess && h[0] != 0) e = hipErrorNotSupported;   // not depth-first
    if (e == hipSuccess) e = hipMalloc(&q, 16 * total);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_qnodes_convert, dim3((n + 255) / 256), dim3(256), 0, st, nodes, n, off, q, flags + 1);
        e = hipMemcpyAsync(h + 1, flags + 1, sizeof(int), hipMemcpyDeviceToHost, st);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess && h[1] != 0) e = hipErrorNotSupported;   // a box the bytes cannot bound
    (void)hipFree(tmp);
    (void)hipFree(flags);
    (void)hipFree(off);
    (void)hipFree(units);
    if (e != hipSuccess) {
        if (q) (void)hipFree(q);
        return e;
    }
    *qOut = q;
    *unitsOut = total;
    return hipSuccess;
}

void launch_tile_order(const uint32_t* cost, int n, uint32_t* order, hipStream_t st) {
    hipLaunchKernelGGL(k_tile_order, dim3(1), dim3(1024), 0, st, cost, n, order);
}

void launch_stream_copy(const float4* src, float4* dst, size_t n4, int numCUs, hipStream_t st) {
    const size_t need = (n4 + 1023) / 1024;
    const size_t blocks = std::min(need, (size_t)std::max(numCUs, 1) * 8);
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)blocks), dim3(256), 0, st, reinterpret_cast<const f4*>(src),
                       reinterpret_cast<f4*>(dst), n4);
}


void launch_band_pack(const FrameArgs& f, const float4* wsum, const float* wts, float* out, hipStream_t st) {
    const int n = (int)(f.W * f.H);
    hipLaunchKernelGGL(k_band_pack, dim3((n + 255) / 256), dim3(256), 0, st, (int)f.W, (int)f.H, f.bandRows >> 3,
                       f.numBands, f.bandIndex, wsum, wts, out);
}
void launch_band_unpack(const FrameArgs& f, int maxRows, const float* recv, float4* wsum, float* wts, float4* image,
                        hipStream_t st) {
    const int n = (int)(f.W * f.H);
    hipLaunchKernelGGL(k_band_unpack, dim3((n + 255) / 256), dim3(256), 0, st, (int)f.W, (int)f.H, f.bandRows >> 3,
                       f.numBands, f.bandIndex, maxRows, recv, wsum, wts, image);
}
void launch_resolve(uint32_t W, uint32_t H, const float4* wsum, const float* wts, float4* image, hipStream_t st) {
    const int n = (int)(W * H);
    hipLaunchKernelGGL(k_resolve, dim3((n + 255) / 256), dim3(256), 0, st, n, wsum, wts, image);
}

}  // namespace mcrt

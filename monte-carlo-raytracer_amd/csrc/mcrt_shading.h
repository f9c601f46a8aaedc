// mcrt_shading.h -- surface interaction, textures, materials, light sampling and queue
// helpers shared by the path-tracing (mcrt_kernels.hip) and BDPT (mcrt_bdpt.hip) kernels.
#pragma once
#include "mcrt_device.h"
#include "mcrt_internal.h"

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

// Longest-first order (FrameArgs::tileOrder): the launch's tile slot j runs tile tileOrder[j], the
// batch frames of a tile staying adjacent.  Any order gives the same paths (keyed by pixel, frame).
MCRT_DEV int orderedTileAll(const FrameArgs& f, int tileAll) {
    if (!f.tileOrder) return tileAll;
    const int slot = tileAll / f.batch, part = tileAll - slot * f.batch;
    return slot < f.numTiles ? (int)f.tileOrder[slot] * f.batch + part : tileAll;
}

// Launch index of the batched camera / first-bounce launches -> (batch frame k, 8x8 tile).
MCRT_DEV void splitTileFrame(const FrameArgs& f, int tileAll, int& k, int& tile) {
    if (f.tileMajor) {
        tile = tileAll / f.batch;
        k = tileAll - tile * f.batch;
    } else {
        k = tileAll / f.numTiles;
        tile = tileAll - k * f.numTiles;
    }
}

MCRT_DEV f3 cameraDir(const mcrt_camera& cam, int x, int y) {   // PathTracing.cl:13-27
    const f2 r = f2{cl_div(1.0f, (float)cam.width), cl_div(1.0f, (float)cam.height)};
    const f2 uv = f2{(float)x * r.x, (float)y * r.y};
    return lerpDirection(ld3(cam.r00), ld3(cam.r10), ld3(cam.r11), ld3(cam.r01), uv.x, uv.y);
}

// Entry idx of a small scene table (shapes, materials, texture descriptors).  When the active lanes
// of the wave share idx -- the camera hits of a packed wave, neighbouring pixels on one surface --
// the entry is read with scalar loads through the constant address space (one fetch per wave, off
// the vector-memory pipeline the shading launches are bound by); otherwise per lane.
template <typename T>
MCRT_DEV T tableEntry(const T* tab, int idx) {
    static_assert(sizeof(T) % 4 == 0, "table entries are whole dwords");
    const int u = __builtin_amdgcn_readfirstlane(idx);
    if (__ballot(idx != u) == 0) {
        typedef __attribute__((address_space(4))) const uint32_t ConstWord;
        ConstWord* p = (ConstWord*)(tab + u);
        T r;
        uint32_t* d = reinterpret_cast<uint32_t*>(&r);
#pragma unroll
        for (int w = 0; w < (int)(sizeof(T) / 4); ++w) d[w] = p[w];
        return r;
    }
    return tab[idx];
}


// ---------------------------------------------------------------------------
// shading
// ---------------------------------------------------------------------------
// KRN/textures.cl:70-125 (readTexture2Df_linear: bilinear RGBA8, wrap modes)
MCRT_DEV f4 readTexDesc(const SceneArgs& s, const mcrt_texture_desc& tex, f2 uv) {
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
MCRT_DEV f4 readTex(const SceneArgs& s, int texId, f2 uv) { return readTexDesc(s, tableEntry(s.textures, texId), uv); }

// ---------------------------------------------------------------------------
// Mip-mapped texture reads at camera-ray hits (opt-in, mcrt_frame_params.texture_lod).  The
// reference carries this path but leaves it off (textures.cl:204-209 keeps the bilinear level-0
// read); these restate its pieces: ray differentials (PathTracing.cl:29-33), the pixel's uv
// footprint (computeSurfaceInteractionWithDifferentials, geometry.cl:126-168), the LOD
// (computeMipmapLOD, textures.cl:198-202) and the trilinear read (readTexture2Df_lod,
// textures.cl:148-196).  Pinned against those reference functions compiled into a probe kernel
// (oracle/refbuild/clprobe_lod.cl, tests/test_gpu_texture_lod.py).
// ---------------------------------------------------------------------------
struct TexLod {
    f2 duvdx, duvdy;
    bool on;
};

// computeMipmapLOD (textures.cl:198-202)
MCRT_DEV float mipLod(const mcrt_texture_desc& t, f2 dx, f2 dy) {
    const float w = fmaxf(fmaxf(fabsf(dx.x), fabsf(dx.y)), fmaxf(fabsf(dy.x), fabsf(dy.y)));
    return (float)t.numMipLevels - 1.0f + log2f(fmaxf(w, 1e-8f));
}

// readTexture2Df_lod (textures.cl:148-196); texel stride 4 (computeTexelStride, textures.cl:24-27)
MCRT_DEV f4 readTexLodDesc(const SceneArgs& s, const mcrt_texture_desc& tex, f2 uv, float lod) {
    if (lod < 1e-8f || tex.numMipLevels < 2) return readTexDesc(s, tex, uv);
    if (lod >= (float)(tex.numMipLevels - 1)) {   // the reference reads the last level as 1 x 1
        mcrt_texture_desc top = tex;
        uint16_t w = tex.width, h = tex.height;
        int off = 0;
        for (int i = 0; i < tex.numMipLevels - 1; ++i) {
            off += w * h * 4;
            w = (uint16_t)max(w / 2, 1);
            h = (uint16_t)max(h / 2, 1);
        }
        top.width = 1;
        top.height = 1;
        top.memOffset += off;
        return readTexDesc(s, top, uv);
    }
    const int lower = (int)floorf(lod);
    uint16_t w = tex.width, h = tex.height;
    int off = 0;
    for (int i = 0; i < lower; ++i) {
        off += w * h * 4;
        w = (uint16_t)max(w / 2, 1);
        h = (uint16_t)max(h / 2, 1);
    }
    mcrt_texture_desc lo = tex, hi = tex;
    lo.width = w;
    lo.height = h;
    lo.memOffset += off;
    const int offHi = off + w * h * 4;
    hi.width = (uint16_t)max(w / 2, 1);
    hi.height = (uint16_t)max(h / 2, 1);
    hi.memOffset += offHi;
    const f4 v0 = readTexDesc(s, lo, uv), v1 = readTexDesc(s, hi, uv);
    const float t = lod - (float)lower;
    return f4{fmaf(v1.x - v0.x, t, v0.x), fmaf(v1.y - v0.y, t, v0.y), fmaf(v1.z - v0.z, t, v0.z),
              fmaf(v1.w - v0.w, t, v0.w)};
}

// readTexture2Df with the LOD path switched on (textures.cl:204-209 with line 207 active)
MCRT_DEV f4 readTexL(const SceneArgs& s, int texId, f2 uv, const TexLod& L) {
    if (!L.on) return readTex(s, texId, uv);
    const mcrt_texture_desc tex = tableEntry(s.textures, texId);
    return readTexLodDesc(s, tex, uv, mipLod(tex, L.duvdx, L.duvdy));
}

// solveLinearSystem2x2 (matrix.cl:72-83) with A = makeMat2(a00, a01, a10, a11)
MCRT_DEV bool solve2x2(float a00, float a01, float a10, float a11, f2 B, f2* x) {
    const float det = a00 * a11 - a10 * a01;
    if (fabsf(det) < 1e-8f) return false;
    *x = f2{cl_div(a11 * B.x - a01 * B.y, det), cl_div(a00 * B.y - a10 * B.x, det)};
    return true;
}

// Ray differentials of the camera ray through pixel (x, y) (GeneratePerspectiveRays,
// PathTracing.cl:22-33): both offset rays start at the camera position.
MCRT_DEV void cameraDiffDirs(const mcrt_camera& cam, int x, int y, f3& dx, f3& dy) {
    const f2 r = f2{cl_div(1.0f, (float)cam.width), cl_div(1.0f, (float)cam.height)};
    const f2 uv = f2{(float)x * r.x, (float)y * r.y};
    dx = lerpDirection(ld3(cam.r00), ld3(cam.r10), ld3(cam.r11), ld3(cam.r01), uv.x + r.x, uv.y);
    dy = lerpDirection(ld3(cam.r00), ld3(cam.r10), ld3(cam.r11), ld3(cam.r01), uv.x, uv.y + r.y);
}

// KRN/materials.cl:76-91 (getUberMaterialProperties)
// nonDelta (BDPT): hasMaterialNonDeltaComponents (materials.cl:163-183) of the same material at the
// same uv, from these texture reads instead of a second set
MCRT_DEV Uber uberProps(const SceneArgs& s, const mcrt_material& material, f2 uv, const TexLod& L = TexLod{{0, 0}, {0, 0}, false},
                        bool* nonDelta = nullptr) {
    Uber u;
    const f4 Kd_opacity = material.uber_diffuseTexId != -1 ? readTexL(s, material.uber_diffuseTexId, uv, L) : f4{1.0f, 1.0f, 1.0f, 1.0f};
    u.Kd = Kd_opacity.xyz * ld3(material.uber_kd);
    const f3 glossy = material.uber_glossyTexId != -1 ? readTexL(s, material.uber_glossyTexId, uv, L).xyz : splat3(1.0f);
    u.Ks = glossy * ld3(material.uber_ks);
    u.Kr = (material.uber_specReflectionTexId != -1 ? readTexL(s, material.uber_specReflectionTexId, uv, L).xyz : splat3(1.0f)) *
           ld3(material.uber_kr);
    u.Kt.xyz = (material.uber_transmissionTexId != -1 ? readTexL(s, material.uber_transmissionTexId, uv, L).xyz : splat3(1.0f)) *
               ld3(material.uber_kt);
    u.Kt.w = material.uber_kt.w;
    const f3 opTex = material.uber_opacityTexId != -1 ? readTexL(s, material.uber_opacityTexId, uv, L).xyz : splat3(1.0f);
    u.opacity = opTex * ld3(material.uber_opacity) * Kd_opacity.w;
    if (nonDelta) {
        const f3 Kd = material.uber_diffuseTexId != -1 ? Kd_opacity.xyz : ld3(material.uber_kd);
        const f3 Ks = material.uber_glossyTexId != -1 ? glossy : ld3(material.uber_ks);
        const f3 op = material.uber_opacityTexId != -1 ? opTex : ld3(material.uber_opacity);
        const f3 kd = Kd * op, ks = Ks * op;
        *nonDelta = !isBlack(kd) || !isBlack(ks);
    }
    u.roughness = material.uber_roughnessTexId != -1 ? readTexL(s, material.uber_roughnessTexId, uv, L).xy
                                                      : f2{material.uber_roughness.x, material.uber_roughness.y};
    u.eta = material.uber_iorTexId != -1 ? readTexL(s, material.uber_iorTexId, uv, L).x : material.uber_eta;
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

// Block-aggregated append grouped by a small key (G groups): within the block's slice of the
// queue the records are ordered by group (then wave, then lane), so the traversal waves that
// read the queue see rays of one group (e.g. the direction octant) together.  One global
// atomic per block; every thread of the block must call.  lds: NW * G + 1 ints.
template <int NW, int G>
MCRT_DEV int blockAppendGrouped(int* counter, bool pred, int group, int* lds) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    unsigned long long mine = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const unsigned long long m = __ballot(pred && group == g);
        if (g == group) mine = m;
        if (lane == 0) lds[g * NW + wv] = __popcll(m);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int sum = 0;
        for (int i = 0; i < G * NW; ++i) {   // (group, wave) order
            const int c = lds[i];
            lds[i] = sum;
            sum += c;
        }
        lds[G * NW] = sum ? atomicAdd(counter, sum) : 0;
    }
    __syncthreads();
    const int prefix = __builtin_amdgcn_mbcnt_hi((unsigned)(mine >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)mine, 0u));
    const int slot = lds[G * NW] + (pred ? lds[group * NW + wv] : 0) + prefix;
    __syncthreads();
    return slot;
}

// The same grouping with one LDS atomic per record instead of G ballots per wave (for many
// groups): records of a group are contiguous in the block's slice, their order inside the group
// is the LDS atomics' order (queue order never changes a result: every record carries its path).
// Every thread of the block must call.  lds: G + 1 ints.
template <int G>
MCRT_DEV int blockAppendGroupedLds(int* counter, bool pred, int group, int* lds) {
    for (int g = threadIdx.x; g < G; g += blockDim.x) lds[g] = 0;
    __syncthreads();
    const int local = pred ? atomicAdd(&lds[group], 1) : 0;
    __syncthreads();
    if (threadIdx.x == 0) {
        int sum = 0;
        for (int g = 0; g < G; ++g) {
            const int c = lds[g];
            lds[g] = sum;
            sum += c;
        }
        lds[G] = sum ? atomicAdd(counter, sum) : 0;
    }
    __syncthreads();
    const int slot = lds[G] + (pred ? lds[group] : 0) + local;
    __syncthreads();
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
MCRT_DEV Frame computeSurfaceInteraction(const SceneArgs& s, const mcrt_shape& shape, int shapeIdx, int primIdx,
                                         f2 barycentrics, f3* dpduOut = nullptr, f3* dpdvOut = nullptr) {
    Frame si;
    // the triangle's surface record (SceneArgs::surf): the same floats the index path gathers
    const float4* R = s.surf + 8 * ((size_t)tableEntry(s.surfBase, shapeIdx) + (uint32_t)primIdx);
    const float4 r0 = R[0], r1 = R[1], r2 = R[2], r3 = R[3], r4 = R[4], r5 = R[5];
    const f3 p0 = transformPoint3(shape.toWorldTransform, mk3(r0.x, r0.y, r0.z));
    const f3 p1 = transformPoint3(shape.toWorldTransform, mk3(r0.w, r1.x, r1.y));
    const f3 p2 = transformPoint3(shape.toWorldTransform, mk3(r1.z, r1.w, r2.x));
    const f2 uv0 = f2{r2.y, r2.z}, uv1 = f2{r2.w, r3.x}, uv2 = f2{r3.y, r3.z};
    const f3 n0 = transformVector3(shape.toWorldInverseTranspose, mk3(r3.w, r4.x, r4.y));
    const f3 n1 = transformVector3(shape.toWorldInverseTranspose, mk3(r4.z, r4.w, r5.x));
    const f3 n2 = transformVector3(shape.toWorldInverseTranspose, mk3(r5.y, r5.z, r5.w));
    si.p = p0 * (1.0f - barycentrics.x - barycentrics.y) + p1 * barycentrics.x + p2 * barycentrics.y;
    si.uv = uv0 * (1.0f - barycentrics.x - barycentrics.y) + uv1 * barycentrics.x + uv2 * barycentrics.y;
    si.gn = cl_normalize(cl_cross(p0 - p2, p1 - p2));
    si.sn = cl_normalize(n0 * (1.0f - barycentrics.x - barycentrics.y) + n1 * barycentrics.x + n2 * barycentrics.y);
    f3 dpdu, dpdv;
    computeTrianglePartialDerivates(uv0, uv1, uv2, p0, p1, p2, si.sn, &dpdu, &dpdv);
    si.sdpdu = cl_normalize(dpdu - cl_dot(si.sn, dpdu) * si.sn);
    si.sdpdv = cl_normalize(dpdv - cl_dot(si.sn, dpdv) * si.sn - cl_dot(si.sdpdu, dpdv) * si.sdpdu);
    if (dpduOut) *dpduOut = dpdu;
    if (dpdvOut) *dpdvOut = dpdv;
    return si;
}
MCRT_DEV Frame computeSurfaceInteraction(const SceneArgs& s, int shapeIdx, int primIdx, f2 barycentrics,
                                         f3* dpduOut = nullptr, f3* dpdvOut = nullptr) {
    return computeSurfaceInteraction(s, tableEntry(s.shapes, shapeIdx), shapeIdx, primIdx, barycentrics, dpduOut, dpdvOut);
}

// The pixel's uv footprint at a camera-ray hit (computeSurfaceInteractionWithDifferentials,
// geometry.cl:126-168): intersect the two offset rays with the tangent plane, express the
// offsets in (dpdu, dpdv) on the two axes the geometric normal is least aligned with.
// dpdu, dpdv: computeTrianglePartialDerivates' (unnormalised) output.
MCRT_DEV TexLod surfaceUVDifferentials(const Frame& si, f3 dpdu, f3 dpdv, f3 o, f3 dxDir, f3 dyDir) {
    TexLod L;
    L.on = true;
    const float d = cl_dot(si.gn, si.p);
    const float tx = cl_div(-(cl_dot(si.gn, o) - d), cl_dot(si.gn, dxDir));
    const f3 px = o + tx * dxDir;
    const float ty = cl_div(-(cl_dot(si.gn, o) - d), cl_dot(si.gn, dyDir));
    const f3 py = o + ty * dyDir;
    float a00, a01, a10, a11;
    f2 Bx, By;
    if (fabsf(si.gn.x) > fabsf(si.gn.y) && fabsf(si.gn.x) > fabsf(si.gn.z)) {
        a00 = dpdu.y; a01 = dpdv.y; a10 = dpdu.z; a11 = dpdv.z;
        Bx = f2{px.y, px.z} - f2{si.p.y, si.p.z};
        By = f2{py.y, py.z} - f2{si.p.y, si.p.z};
    } else if (fabsf(si.gn.y) > fabsf(si.gn.z)) {
        a00 = dpdu.x; a01 = dpdv.x; a10 = dpdu.z; a11 = dpdv.z;
        Bx = f2{px.x, px.z} - f2{si.p.x, si.p.z};
        By = f2{py.x, py.z} - f2{si.p.x, si.p.z};
    } else {
        a00 = dpdu.x; a01 = dpdv.x; a10 = dpdu.y; a11 = dpdv.y;
        Bx = f2{px.x, px.y} - f2{si.p.x, si.p.y};
        By = f2{py.x, py.y} - f2{si.p.x, si.p.y};
    }
    if (!solve2x2(a00, a01, a10, a11, Bx, &L.duvdx)) L.duvdx = f2{0.0f, 0.0f};
    if (!solve2x2(a00, a01, a10, a11, By, &L.duvdy)) L.duvdy = f2{0.0f, 0.0f};
    return L;
}

// applyNormalMapping_internal (materials.cl:11-19)
MCRT_DEV void applyNormalMapping(const SceneArgs& s, int texId, Frame& si, const TexLod& L = TexLod{{0, 0}, {0, 0}, false}) {
    const f3 nm = 2.0f * readTexL(s, texId, si.uv, L).xyz - 1.0f;
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
    f3 lightPos, lightNormal;   // *lightPosition, *lightNormal (BDPT s = 1 strategy)
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
    r.lightPos = splat3(0.0f);
    r.lightNormal = splat3(0.0f);
    if (light.type == MCRT_DIRECTIONAL_LIGHT) {
        r.wi = -ld3(light.d);
        r.lightPos = si.p + r.wi * light.radius * 2.0f;
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
            r.lightPos = ld3(light.p);
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
        r.lightPos = lp;
        r.lightNormal = lgn;
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


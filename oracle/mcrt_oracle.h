/*
 * mcrt_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path (compix/Monte-Carlo-Raytracer):
 * the OpenCL path tracer (assets/kernels/ sources) and the RadeonRays Bvh2 +
 * LDS traversal it calls (third_party/RadeonRays/RadeonRays/src/...).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / CPU baseline -- the product
 * (monte-carlo-raytracer_amd/) never links it.
 *
 * Parity pinning (DESIGN.md "Oracle"):
 *   - Bvh2 build: bit-compared against the reference's own bvh2.cpp compiled
 *     from /root/reference by oracle/refbuild (oracle/_ref/librrref.so).
 *   - traversal: RadeonRays conformance protocol against the reference's own
 *     brute force (UnitTest/utils.cpp, also in librrref.so).
 *   - integrator: against the reference OpenCL kernels compiled for gfx950
 *     and run through the ROCm OpenCL runtime on the GPU box
 *     (oracle/refbuild/clref_runner.cpp), fixtures in tests/golden/.
 */
#ifndef MCRT_ORACLE_H
#define MCRT_ORACLE_H

#include "../include/mcrt_capi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* rng.cl / samplers.cl */
uint32_t orc_wang_hash(uint32_t seed);
uint32_t orc_xorshift(uint32_t* state);
float    orc_rand_float(uint32_t* state);
float    orc_sobol_sample(uint32_t idx, uint32_t dim, uint32_t scramble, const uint32_t* mats);
/* Fills n (u1, u2x, u2y, ub.x, ub.y) sampler draws for pixel/frame/bounce like MAKE_SAMPLER. */
void     orc_sampler_draws(int sampler, uint32_t pix, int frame, int bounce, int W, int H,
                           const uint32_t* sobol, float out[5]);

/* Scene handle: keeps pointers to the caller's arrays (not copied). */
typedef struct orc_scene orc_scene;
orc_scene* orc_scene_create(const mcrt_scene_desc* desc);
void       orc_scene_destroy(orc_scene* s);

/* Bvh2 build (RR bvh2.h/bvh2.cpp). Returns node count (>0) or -1. */
int64_t orc_bvh_build(orc_scene* s, float traversal_cost, int num_bins, int use_sah);
/* Copies the 64-B RR nodes out (64 * count bytes). */
int64_t orc_bvh_nodes(orc_scene* s, void* out, int64_t max_nodes);

/* intersect_main / occluded_main (RR intersect_bvh2_lds.cl). visits may be NULL;
 * if not, visits[i] receives the node fetch count of ray i. */
void orc_trace_closest(orc_scene* s, const mcrt_ray* rays, int n, mcrt_intersection* hits, int32_t* visits, int threads);
void orc_trace_any(orc_scene* s, const mcrt_ray* rays, int n, int32_t* hits, int32_t* visits, int threads);

/* Premise of the compact walk's near-tie repeat: 6 floats per ray (layout at orc_tie_premise in
 * mcrt_oracle.c; tests/test_tie_premise_cpu.py). */
void orc_tie_premise(orc_scene* s, const mcrt_ray* rays, int n, float alpha, float* out, int threads);
/* RR UnitTest/utils.cpp brute force (world-space triangles of all shapes). */
void orc_brute_closest(orc_scene* s, const mcrt_ray* rays, int n, mcrt_intersection* hits);
void orc_brute_any(orc_scene* s, const mcrt_ray* rays, int n, int32_t* hits);

/* One PT frame for rows [y0, y1) (GeneratePerspectiveRays + maxDepth x (PathTracing,
 * occluded, ShadowPass, intersect)).  radiance: W*H float4, rows outside untouched.
 * stats (may be NULL, 8 x int64): [0] primary closest queries, [1] their node visits,
 * [2] extension closest queries, [3] their visits, [4] any-hit queries, [5] their visits,
 * [6] leaf visits among [3], [7] leaf visits among [5]
 * (visits = RR Bvh2 node fetches of intersect_bvh2_lds.cl, the V of SURVEY.md §8d). */
void orc_render_frame(orc_scene* s, const mcrt_camera* cam, int frame, int max_depth, int sampler,
                      int y0, int y1, int threads, float* radiance, int64_t* stats);
/* Same, but only every `stride`-th row starting at y0 (bounded CPU-baseline samples). */
/* BDPT (KRN/BDPT.cl, RTBDPTPass order): persistent per-frame-buffer state (the sampled light
 * vertices the s = 1 strategy reads from the previous frame) + one frame over rows (NULL = all) */
typedef struct orc_bdpt orc_bdpt;
orc_bdpt* orc_bdpt_create(int W, int H, int D);
void orc_bdpt_destroy(orc_bdpt* b);
void orc_bdpt_render(orc_scene* s, orc_bdpt* b, const mcrt_camera* cam, int frame, int sampler, const int32_t* rows,
                     int nrows, int threads, float* radiance, int32_t* camCounts, int32_t* lightCounts, int64_t* stats);
/* per-node touched marks of later renders: NULL or 4 x num_nodes bytes (bench.py roofline) */
void orc_set_touched(orc_scene* s, uint8_t* touched);
/* per-pixel path log of later PT renders (divergence diagnostics, tools/oracle_divergence.py):
 * NULL (off) or W*H*depth records of ORC_PATHLOG_FLOATS floats, one per bounce b:
 *   [0] shapeid (int32 bits; -2 = no ray this bounce) [1] primid [2] u [3] v [4] t   (hit of bounce b)
 *   [5] sampled BxDF type (int32; -1 = none) [6] light index (int32; -1 = none)
 *   [7] occlusion result (int32; -2 = no shadow query) [8..10] shadow o [11..13] shadow d [14] tmax
 *   [15..17] next ray o [18..20] next ray d [21] next ray active (1/0) [22..23] BSDF sample u
 *   [24..26] o [27..29] d [30] tmax of the ray traced for bounce b's hit [31] unused */
#define ORC_PATHLOG_FLOATS 32
void orc_set_pathlog(orc_scene* s, float* log, int depth);
void orc_render_rows(orc_scene* s, const mcrt_camera* cam, int frame, int max_depth, int sampler,
                     const int32_t* rows, int nrows, int threads, float* radiance, int64_t* stats);

/* ReconstructionPass (reconstruction.cl:6-60). */
/* one frame of ReconstructionPass with an explicit filter weight */
void orc_accumulate_w(int W, int H, int frame, float w, const float* radiance, float* wsum, float* wts, float* image);
void orc_accumulate(int W, int H, int frame, const mcrt_filter* f, const float* radiance,
                    float* wsum, float* wts, float* image);

/* Unit-level entry points for per-stage golden tests. */
/* sampleUberBSDF in shading space with an identity frame (n=y, t=x, b=z). out: f[3], wi[3], pdf, type */
void orc_sample_uber(const float kd[3], const float ks[3], const float kr[3], const float kt[4],
                     const float rough_alpha[2], const float opacity[3], float eta,
                     const float wo[3], const float u[2], float out[8]);
void orc_eval_uber(const float kd[3], const float ks[3], const float kt[4], const float rough_alpha[2],
                   const float opacity[3], float eta, const float wo[3], const float wi[3], float out[3]);
float orc_pdf_uber(const float kd[3], const float ks[3], const float kr[3], const float kt[4],
                   const float rough_alpha[2], const float opacity[3], float eta,
                   const float wo[3], const float wi[3]);
float orc_roughness_to_alpha(float r);

/* Post-process passes (test restatements): BilateralDenoise (KRN/Denoise.cl:6-47) and
 * ReinhardToneMapping (KRN/ToneMapping.cl:42-63) on RGBA32F images (W*H float4). */
void orc_denoise(int W, int H, int radius, float sigma_spatial, float sigma_range, const float* in, float* out);
void orc_tonemap(int W, int H, float Lwhite, const float* in, float* out);

#ifdef __cplusplus
}
#endif
#endif

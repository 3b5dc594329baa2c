/*
 * pt_oracle.h — CPU ORACLE for the pathTrace hot path.  TEST INFRASTRUCTURE ONLY.
 *
 * This is a scalar C restatement of the reference kernel `pathTrace`
 * (`RTrace/raytrace.metal:11-111`) and its helpers in `RTrace/sampling.metal`,
 * under the arithmetic contract written down in DESIGN.md §3.  It is the parity
 * checker for the HIP kernel and the CPU baseline reported by bench.py.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it;
 * the product (gpuraytracer_amd/, librtpt.so) never links or calls it.
 *
 * Pinning: the reference is Swift + Metal and cannot be built or run here
 * (no swift/xcrun/metal), and it holds no golden vectors or
 * tests.  Its only artefacts are two tonemapped PNGs of an earlier revision.
 * PARITY UNPINNED against a Metal run: the oracle is pinned by analytic
 * known-answer tests, by an independent numpy restatement (oracle/pt_oracle_np.py)
 * and by the geometry of Sources/gpuRaytracer/example.png (light footprint).
 */
#ifndef PT_ORACLE_H
#define PT_ORACLE_H

#include <stdint.h>
#include <stddef.h>
#include "../include/rt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

/* sampling.metal:107-122 */
float pto_halton(uint32_t i, uint32_t d);
/* DESIGN.md §3 portable sincos (stands in for MSL sincos, sampling.metal:43) */
void pto_sincos(float x, float* s, float* c);

/* Ray/primitive tests of the contract.  Return 1 on hit, t in *t. */
int pto_ray_triangle(const float o[3], const float d[3], const float v0[3], const float v1[3],
                     const float v2[3], float tmin, float tmax, float* t);
int pto_ray_sphere(const float o[3], const float d[3], const float c[3], float radius,
                   float tmin, float tmax, float* t);

/* generateCameraRay (sampling.metal:125-157): direction for pixel (x,y), jitter (jx,jy). */
void pto_camera_ray(const CameraGPU* cam, int32_t x, int32_t y, float jx, float jy, float dir[3]);

/* sampleAreaLight (sampling.metal:198-236) */
void pto_sample_area_light(const SquareLightGPU* light, float ux, float uy, const float p[3],
                           float ldir[3], float* ldist, float color[3]);

/* sampleCosineWeightedHemisphere + alignHemisphereWithNormal (sampling.metal:39-66) */
void pto_cosine_direction(float ux, float uy, const float n[3], float d[3]);

/* One sample of pathTrace for pixel (x,y), sample index n: the per-sample
 * `accumulatedColor` of raytrace.metal:44-102. */
void pto_trace_sample(const CameraGPU* cam, const MaterialGPU* mats, const SquareLightGPU* light,
                      const rt_float3* verts, uint32_t n_tri, const SphereGPU* spheres,
                      uint32_t n_sph, uint32_t seed, int32_t x, int32_t y, uint32_t n,
                      uint32_t bounces, float acc[3]);

/* Full render (raytrace.metal:11-111) of rows y = row_start + j*row_step,
 * j < row_count, samples [sample_base, sample_base+spp).
 * sum_in  (optional, row_count*W*4 floats): running sums to continue from;
 *          then S = sample_base + spp else S = spp.
 * sum_out (optional): running sums after this call.
 * out     (optional): (sum/S, 1) rgba32F, row_count*W*4 floats.
 * nthreads: worker threads over rows (<=0: 1). Returns 0 on success. */
int pto_render(const CameraGPU* cam, const MaterialGPU* mats, const SquareLightGPU* light,
               const rt_float3* verts, uint32_t n_tri, const SphereGPU* spheres, uint32_t n_sph,
               const uint32_t* seeds, uint32_t spp, uint32_t bounces, uint32_t sample_base,
               uint32_t row_start, uint32_t row_step, uint32_t row_count, const float* sum_in,
               float* sum_out, float* out, int nthreads);

/* Independent restatement of the scene builders (RTrace/scene.swift:14-240). */
int pto_cornell_box(int32_t width, int32_t height, CameraGPU* cam, MaterialGPU* mats,
                    rt_float3* verts, SquareLightGPU* light, uint32_t* n_tri);
int pto_random_spheres(int32_t width, int32_t height, uint32_t n_spheres, uint64_t seed,
                       CameraGPU* cam, MaterialGPU* mats, rt_float3* verts,
                       SquareLightGPU* light, uint32_t* n_tri, SphereGPU* spheres);
void pto_seed_splitmix(uint64_t key, uint32_t* seeds, size_t n);

/* MIS integrator (Sources/gpuRaytracer/shaders.metal:635-707): rows as in
 * pto_render; out (optional) = (sum over camera rays, camera_rays) float4,
 * out8 (optional) = the tonemapped RGBA8 of :688-706. */
int pto_render_mis(const CameraGPU* cam, const MaterialGPU* mats, const SquareLightGPU* light,
                   const rt_float3* verts, uint32_t n_tri, uint32_t camera_rays,
                   uint32_t mis_samples, uint32_t row_start, uint32_t row_step,
                   uint32_t row_count, float* out, uint8_t* out8, int nthreads);
/* Sources/gpuRaytracer/main.swift:21-67 scene (1.5 x 1.5 light) */
int pto_cornell_box_mis(int32_t width, int32_t height, CameraGPU* cam, MaterialGPU* mats,
                        rt_float3* verts, SquareLightGPU* light, uint32_t* n_tri);
/* pow(x, y), x in [0, 1], of the DESIGN.md §3.11 contract */
float pto_pow(float x, float y);

/* image.swift:35-65 epilogue */
void pto_tonemap_rgba8(const float* rgba32f, size_t n_pixels, uint8_t* rgba8);

/* Closest-hit primitive id of every pixel's camera ray through the pixel
 * centre (-1: miss), H*W int32 (geometry check against example.png). */
int pto_primary_ids(const CameraGPU* cam, const MaterialGPU* mats, const SquareLightGPU* light,
                    const rt_float3* verts, uint32_t n_tri, int32_t* ids);

/* Count of ray/primitive tests issued by one render (for the VALU roofline). */
uint64_t pto_last_tests(void);

#ifdef __cplusplus
}
#endif
#endif

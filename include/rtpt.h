/*
 * rtpt.h — C-ABI of the MI355X path-tracing hot path (librtpt.so).
 *
 * Drop-in boundary for the reference's Metal dispatch of `kernel pathTrace`
 * (`RTrace/raytrace.metal:11-111`).  The reference host (`RTrace/renderer.swift`)
 * builds the scene arrays, copies them into MTLBuffers/textures in
 * `Renderer.init()` (`renderer.swift:29-115`), then `Renderer.draw()`
 * (`renderer.swift:117-146`) binds them to the argument table and dispatches a
 * W×H grid.  Here the same arrays (same `shaderTypes.h` layout, see
 * rt_types.h) cross a plain C boundary instead:
 *
 *   Renderer.init()   -> rt_create()     + rt_set_seeds() / rt_fill_seeds()
 *   Renderer.draw()   -> rt_render()     (synchronous, like waitUntilCompleted)
 *   deinit (ARC)      -> rt_destroy()
 *
 * No torch / HIP types appear in any signature; the optional stream is an
 * opaque pointer (a hipStream_t).  All calls return an rt_status; the message
 * of the last failure on a context is in rt_last_error().
 *
 * Semantics of the rendered value per pixel are SURVEY.md Appendix A with the
 * arithmetic contract of DESIGN.md §3 (identical on the CPU oracle).
 */
#ifndef RTPT_H
#define RTPT_H

#include "rt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

#define RTPT_ABI_VERSION 3

/* Maximum bounce count: Halton dimensions 2+5b..5+5b must stay inside the
 * 24-entry `primes[]` table (`RTrace/sampling.metal:97-104`); b <= 3. */
#define RT_MAX_BOUNCES 4

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = 1,   /* null pointer, bad size, bad partition        */
    RT_ERR_NO_DEVICE = 2,     /* no HIP device / bad ordinal                  */
    RT_ERR_OUT_OF_MEMORY = 3, /* hipMalloc failed                             */
    RT_ERR_LAUNCH = 4,        /* kernel launch or execution error             */
    RT_ERR_STATE = 5,         /* e.g. render before seeds, accumulate mismatch */
    RT_ERR_COMM = 6           /* collective (gather) failure                  */
} rt_status;

typedef struct rt_ctx rt_ctx;

/* Scene input: the Metal argument table of pathTrace (raytrace.metal:11-19),
 * minus the acceleration structure (geometry is the arrays themselves).
 * All arrays are COPIED by rt_create; the caller keeps ownership
 * (renderer.swift:61-72 copies with makeBuffer(bytes:) as well). */
typedef struct rt_scene_desc {
    const CameraGPU* camera;             /* buffer(0): cameras[0] is used           */
    const MaterialGPU* materials;        /* buffer(1): one per triangle             */
    const SquareLightGPU* square_lights; /* buffer(2): squareLights[0] is used      */
    uint32_t n_square_lights;            /* >= 1                                    */
    const rt_float3* vertices;           /* buffer(3): 3 per triangle, 16-B stride  */
    uint32_t n_triangles;                /* triangle primitive ids 0..n_triangles-1 */
    const SphereGPU* spheres;            /* optional sphere primitives (config 4),  */
    uint32_t n_spheres;                  /*   primitive ids follow the triangles    */
    int32_t device;                      /* HIP device ordinal                      */
} rt_scene_desc;

/* Output flags */
#define RT_OUT_DEVICE 0x1u  /* `out` is a device pointer (else host memory)          */
#define RT_OUT_FP16   0x2u  /* store rgba16F (the reference texture format,
                               renderer.swift:74-82) instead of rgba32F             */
#define RT_OUT_NONE   0x4u  /* no image output (use with RT_KEEP_SUM)                 */
#define RT_KEEP_SUM   0x8u  /* also write the running per-pixel sum into the context,
                               so that a following call may set accumulate=1
                               (progressive rendering)               */

typedef struct rt_render_params {
    uint32_t spp;          /* samples this call (reference: 400, raytrace.metal:24) */
    uint32_t bounces;      /* 0..RT_MAX_BOUNCES (reference: 3, raytrace.metal:25)   */
    uint32_t sample_base;  /* global index n of the first sample (Halton i=seed+n) */
    uint32_t row_start;    /* rows rendered: y = row_start + j*row_step,           */
    uint32_t row_step;     /*   j = 0..row_count-1 (multi-GPU interleaved tiles)    */
    uint32_t row_count;    /*   0 => all rows                                      */
    uint32_t accumulate;   /* 1: continue the context's running per-pixel sum,
                              which must then hold exactly samples
                              [0, sample_base) of the same rows (written by a
                              previous call with RT_KEEP_SUM)                       */
    uint32_t flags;        /* RT_OUT_* */
} rt_render_params;

/* Renderer.init(): validate and copy the scene to the device, precompute the
 * per-primitive records (edges, normals, shading frames). */
int rt_create(const rt_scene_desc* scene, rt_ctx** out_ctx);

/* Seed texture (renderer.swift:84-110): W*H uint32 row-major, values are the
 * per-pixel Halton offsets (reference range [0, 2^20)).  W,H must equal the
 * camera resolution. */
int rt_set_seeds(rt_ctx* ctx, const uint32_t* seeds, int32_t width, int32_t height);

/* Deterministic replacement for the unseeded arc4random() seeds
 * (renderer.swift:99-101): seed[p] = splitmix64(key + p) mod 2^20, generated on
 * the device.  rt_seed_splitmix() below is the host form of the same function. */
int rt_fill_seeds(rt_ctx* ctx, uint64_t key);

/* Renderer.draw(): render and block until done (commit+waitUntilCompleted).
 * out: row_count*W pixels, rgba32F (16 B) or rgba16F (8 B) by flags; value
 * (sum/S, 1) where S = samples in the sum. */
int rt_render(rt_ctx* ctx, const rt_render_params* params, void* out);

/* Asynchronous variant: enqueue on `hip_stream` (a hipStream_t, may be NULL
 * for the null stream); `out` must be a device pointer.  No host sync. */
int rt_render_async(rt_ctx* ctx, const rt_render_params* params, void* out_device,
                    void* hip_stream);

/* Device time of the most recent render kernel (hipEvents on its stream), ms.
 * Synchronizes on that event. */
int rt_last_kernel_ms(rt_ctx* ctx, float* ms);

int rt_destroy(rt_ctx* ctx);

/* Diagnostic counters of a -DRT_STATS build of the kernel (reads and clears
 * up to 16 uint64 counters; RT_ERR_STATE in normal builds). */
int rt_debug_stats(rt_ctx* ctx, uint64_t* out, int n);

/* Message of the last failure on ctx (or of the last failed rt_create when
 * ctx is NULL).  Never NULL. */
const char* rt_last_error(const rt_ctx* ctx);
const char* rt_status_string(int status);
int rt_abi_version(void);

/* ---- host-side helpers (no device needed) ---------------------------- */

/* seeds[p] = splitmix64(key + p) mod 2^20 for p in [0, n). */
void rt_seed_splitmix(uint64_t key, uint32_t* seeds, size_t n);

/* initCornellBox() (RTrace/scene.swift:14-62): 36 triangles in reference
 * primitive order; camera resolution overridden to width×height.
 * Arrays: materials[36], vertices[108], one light. */
#define RT_CORNELL_TRIANGLES 36
int rt_scene_cornell_box(int32_t width, int32_t height, CameraGPU* camera,
                         MaterialGPU* materials, rt_float3* vertices,
                         SquareLightGPU* light, uint32_t* n_triangles);

/* Config-4 scene: Cornell walls + light (primIds 0-9, 34-35 -> 12 triangles)
 * plus n_spheres spheres from PCG32(seed).
 * materials[12], vertices[36], spheres[n_spheres]. */
#define RT_SPHERE_SCENE_TRIANGLES 12
int rt_scene_random_spheres(int32_t width, int32_t height, uint32_t n_spheres,
                            uint64_t seed, CameraGPU* camera, MaterialGPU* materials,
                            rt_float3* vertices, SquareLightGPU* light,
                            uint32_t* n_triangles, SphereGPU* spheres);

/* ---- MIS integrator ----------------------------------------------------
 * The SwiftPM build's kernel `drawTriangle` (Sources/gpuRaytracer/shaders.metal:
 * 635-707, bound at Sources/gpuRaytracer/computeShader.swift:99-189): per pixel
 * `camera_rays` hash-jittered camera rays; a camera ray that hits the light
 * adds light.emittedRadiance, a surface hit adds the one-bounce three-strategy
 * MIS estimate of recursiveMultiImportanceSampling (:543-625) with
 * samplesPerStrategy = mis_samples / 3.  Triangle scenes only. */
typedef struct rt_mis_params {
    uint32_t camera_rays;   /* cameraRaysPerPixel (:644), reference 6 */
    uint32_t mis_samples;   /* misSamples (:648), reference 300 */
    uint32_t row_start, row_step, row_count;  /* as rt_render_params */
    uint32_t flags;         /* RT_OUT_DEVICE: both outputs are device pointers */
} rt_mis_params;

/* out_rgba32f (optional): (sum of the camera-ray radiances, camera_rays) per
 *   pixel, row_count*W float4 -- the reference's textBuffer (:627-633,705)
 *   plus the divisor.
 * out_rgba8 (optional): the reference's pixels (:248-257,688-706): exposure
 *   1/(1.2*2^ev100), Reinhard, clamp, gamma 1/2.2, uchar(c*255), alpha 255.
 * At least one output must be non-null.  Synchronous. */
int rt_render_mis(rt_ctx* ctx, const rt_mis_params* params, float* out_rgba32f,
                  uint8_t* out_rgba8);

/* The SwiftPM scene (Sources/gpuRaytracer/main.swift:21-67, :96-173): the
 * RTrace room with a 1.5 x 1.5 light.  Arrays as rt_scene_cornell_box. */
int rt_scene_cornell_box_mis(int32_t width, int32_t height, CameraGPU* camera,
                             MaterialGPU* materials, rt_float3* vertices,
                             SquareLightGPU* light, uint32_t* n_triangles);

/* How rt_create would lay a scene out on the device (host-only, no device). */
typedef struct rt_scene_info {
    uint32_t n_triangles;
    uint32_t n_triangle_pairs;   /* >0: every (2k,2k+1) shares v0 and an edge -> pair records */
    uint32_t n_spheres;
    uint32_t lds_bytes;          /* intersection records staged per workgroup (0: read from global) */
    uint32_t n_sphere_nodes;     /* sphere BVH nodes per layout (32 B each, 8 layouts, global) */
    uint32_t n_triangle_bvh_nodes; /* GPU-built triangle BVH nodes per layout (0: LDS layouts) */
    uint32_t n_box_clusters;     /* pair runs on the faces of one oriented box (slab-tested first) */
    uint32_t pair_free_mask;     /* pairs in no box cluster (bit k = pair k) */
    uint32_t sphere_bvh_lds_bytes; /* compact sphere BVH staged in LDS (0: read from global) */
} rt_scene_info;
int rt_scene_describe(const rt_scene_desc* scene, rt_scene_info* info);

/* The reference's image epilogue (RTrace/image.swift:35-65): fp16 round trip,
 * ×2 exposure, Reinhard, gamma 1/2.2, clamp, truncating UInt8, alpha 255.
 * in: n_pixels rgba32F (host), out: n_pixels*4 bytes. */
void rt_tonemap_rgba8(const float* rgba32f, size_t n_pixels, uint8_t* rgba8);

#ifdef __cplusplus
}
#endif

#endif /* RTPT_H */

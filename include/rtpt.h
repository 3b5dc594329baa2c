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

#define RTPT_ABI_VERSION 7

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
#define RT_OUT_RGBA8  0x10u /* store the reference's 8-bit image instead (4 B/px):
                               the epilogue of RTrace/image.swift:35-65 fused into
                               the kernel's store -- rgba16F round trip
                               (renderer.swift:74-82), x2 exposure, Reinhard,
                               pow(v, 1/2.2), clamp, truncating UInt8, alpha 255.
                               Exclusive with RT_OUT_FP16.                         */

typedef struct rt_render_params {
    uint32_t spp;          /* samples this call (reference: 400, raytrace.metal:24) */
    uint32_t bounces;      /* 0..RT_MAX_BOUNCES (reference: 3, raytrace.metal:25)   */
    uint32_t sample_base;  /* global index n of the first sample (Halton i=seed+n) */
    uint32_t row_start;    /* rows rendered: y = row_start + j*row_step,           */
    uint32_t row_step;     /*   j = 0..row_count-1 (multi-GPU interleaved tiles)    */
    uint32_t row_count;    /*   0 => all rows                                      */
    uint32_t accumulate;   /* 1: continue the context's running per-pixel sum,
                              which must then hold the samples [first,
                              sample_base) of the same rows, written by previous
                              calls with RT_KEEP_SUM (the first of them started
                              at sample index `first`); the image is the sum
                              divided by the samples it holds                      */
    uint32_t flags;        /* RT_OUT_* */
} rt_render_params;

/* Renderer.init(): validate and copy the scene to the device, precompute the
 * per-primitive records (edges, normals, shading frames).  Default options. */
int rt_create(const rt_scene_desc* scene, rt_ctx** out_ctx);

/* ---- creation options ----------------------------------------------------
 * Speed-only choices of one context: which record layout / kernel serves the
 * scene, how the acceleration structures are built, lanes per pixel.  None of
 * them changes a rendered value (every layout and build is bit-exact against
 * the oracle).  They are per context and the library reads no environment
 * variable: a caller (Swift, C, Python) sets them here or gets the defaults,
 * which are the measured-best choices.  Zero-initialised fields mean
 * "default", so `rt_create_options o = {0};` is valid. */
typedef enum rt_scene_layout {
    RT_LAYOUT_AUTO = 0,        /* measured best for the scene (box clusters, sphere
                                  kernel, triangle BVH above 384 triangles)        */
    RT_LAYOUT_PAIRS = 1,       /* shared-edge pair records in LDS, no box clusters   */
    RT_LAYOUT_SINGLE = 2,      /* one record per triangle in LDS                     */
    RT_LAYOUT_GLOBAL = 3,      /* one record per triangle, read from global memory   */
    RT_LAYOUT_PAIRS_SMEM = 4,  /* pair records by scalar loads, no LDS               */
    RT_LAYOUT_SORTED = 5,      /* pair records + octant sort of the paths per bounce */
    RT_LAYOUT_BVH = 6          /* triangle BVH at any triangle count                 */
} rt_scene_layout;

typedef enum rt_tri_bvh_build {
    RT_TRI_BVH_DEFAULT = 0,    /* = RT_TRI_BVH_GPU_SAH                               */
    RT_TRI_BVH_HOST_SAH = 1,   /* host binned SAH (32 bins), uploaded                */
    RT_TRI_BVH_GPU_LBVH = 2,   /* GPU Morton LBVH (Karras hierarchy + refit)         */
    RT_TRI_BVH_GPU_SAH = 3     /* GPU binned SAH, the host build's rules             */
} rt_tri_bvh_build;

typedef enum rt_walk_scheduler {
    RT_WALK_AUTO = 0,          /* measured best per scene                            */
    RT_WALK_LOCKSTEP = 1,      /* a wave's lanes run each bounce's queries together  */
    RT_WALK_FREE = 2,          /* every lane runs its own path state; lanes whose
                                  walk ended park until half the wave has, then
                                  shade and start their next query together        */
    RT_WALK_SORTED = 3         /* between bounces the paths of a workgroup are
                                  counting-sorted by direction octant (ballots),
                                  finished paths dropped: a wave walks one BVH
                                  layout                                           */
} rt_walk_scheduler;

typedef struct rt_create_options {
    uint32_t scene_layout;     /* rt_scene_layout                                    */
    uint32_t lanes_per_pixel;  /* 0 = auto, else 1, 4 or 16                          */
    uint32_t tri_bvh_build;    /* rt_tri_bvh_build                                   */
    uint32_t tri_leaf_max;     /* triangles per BVH leaf at most, 0 = 1; 1..128      */
    float tri_leaf_cost;       /* SAH leaf rule: box step cost in triangle tests,
                                  0 = 1.0                                            */
    uint32_t sphere_leaf_max;  /* spheres per BVH leaf at most, 0 = 1; 1..255        */
    uint32_t sphere_median;    /* 1: median splits instead of the exact SAH sweep    */
    uint32_t walk_scheduler;   /* rt_walk_scheduler (BVH scenes)                     */
    uint32_t walk_leaf_den;    /* RT_WALK_FREE: parked leaves are tested once they
                                  are >= 1/den of the walking lanes, 0 = default;
                                  1..64 (1: only when every walker is parked, so
                                  leaves stay parked into the service phase)       */
    uint32_t reserved[7];      /* must be 0                                          */
} rt_create_options;

/* The defaults (all zero). */
void rt_create_options_default(rt_create_options* opt);

/* rt_create with options (NULL = defaults).  RT_ERR_INVALID_ARG for a value
 * outside its range. */
int rt_create_ex(const rt_scene_desc* scene, const rt_create_options* opt, rt_ctx** out_ctx);

/* Seed texture (renderer.swift:84-110): W*H uint32 row-major, values are the
 * per-pixel Halton offsets (reference range [0, 2^20)).  W,H must equal the
 * camera resolution. */
int rt_set_seeds(rt_ctx* ctx, const uint32_t* seeds, int32_t width, int32_t height);

/* Deterministic replacement for the unseeded arc4random() seeds
 * (renderer.swift:99-101): seed[p] = splitmix64(key + p) mod 2^20, generated on
 * the device.  rt_seed_splitmix() below is the host form of the same function. */
int rt_fill_seeds(rt_ctx* ctx, uint64_t key);

/* Renderer.draw(): render and block until done (commit+waitUntilCompleted).
 * out: row_count*W pixels, rgba32F (16 B), rgba16F (8 B) or RGBA8 (4 B) by
 * flags; value (sum/S, 1) where S = samples in the sum. */
int rt_render(rt_ctx* ctx, const rt_render_params* params, void* out);

/* Asynchronous variant: enqueue on `hip_stream` (a hipStream_t, may be NULL
 * for the null stream); `out` must be a device pointer.  No host sync. */
int rt_render_async(rt_ctx* ctx, const rt_render_params* params, void* out_device,
                    void* hip_stream);

/* Device time of the most recent render kernel (hipEvents on its stream), ms.
 * Synchronizes on that event. */
int rt_last_kernel_ms(rt_ctx* ctx, float* ms);

int rt_destroy(rt_ctx* ctx);

/* ---- multi-GPU: row-interleaved tiles + one RCCL gather ----
 * north_star: "the image is row-tile-partitioned across the 8 GPUs of one node
 * with a single RCCL gather of tiles over xGMI at the end of each spp batch".
 * One process (or thread) per GPU, one context per GPU.  Rank k of N renders
 * the rows y = k, k+N, k+2N, ... with the global y (so the frame is
 * bit-identical to a single-GPU render) and the tiles are gathered to rank 0
 * by one ncclGather over xGMI, then placed at their rows by one kernel on rank
 * 0 (rt_place_tiles).  The reference's draw (renderer.swift:117-146) has no multi-GPU
 * path; this extends it. */
#define RT_COMM_ID_BYTES 128   /* ncclUniqueId */

/* Rank 0 makes the communicator id and hands it to every rank out of band
 * (MPI, a TCP store, a file).  RT_ERR_COMM on failure. */
int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]);

/* Join the N-rank communicator (collective: every rank calls it with the same
 * id).  RT_ERR_INVALID_ARG for a bad rank/world, RT_ERR_COMM for RCCL errors,
 * RT_ERR_STATE if the context already has a communicator. */
int rt_comm_init(rt_ctx* ctx, int32_t rank, int32_t world, const uint8_t id[RT_COMM_ID_BYTES]);

/* Renderer.draw() across the communicator (collective): render this rank's
 * rows with params (which name the whole frame: row_start 0, row_step 0 or 1,
 * row_count 0; the partition is y = rank (mod world)), then gather every tile into `frame` on rank 0 --
 * H*W pixels in the format of params->flags (rgba32F / rgba16F / RGBA8), host
 * memory (the call then blocks) or device memory with RT_OUT_DEVICE (enqueued
 * on `hip_stream`, a hipStream_t; NULL is the HIP null stream, as for
 * rt_render_async; no host sync).  `frame` is
 * ignored on other ranks.  With RT_OUT_NONE (progressive batches into the
 * running sums) nothing is gathered.  RT_ERR_STATE without rt_comm_init,
 * RT_ERR_COMM when the gather fails. */
int rt_render_gather(rt_ctx* ctx, const rt_render_params* params, void* frame, void* hip_stream);

/* The communicator as RCCL sees it (ncclCommCount / ncclCommUserRank): lets a
 * caller prove that N ranks joined.  RT_ERR_STATE without rt_comm_init. */
int rt_comm_info(const rt_ctx* ctx, int32_t* count, int32_t* rank);

/* Row layout of rt_render_gather (host-only, no device): rank `rank` of
 * `world` owns rows y = rank + j*world, j < rows; every rank sends a tile
 * padded to rows_max rows (tile_bytes = rows_max * row_bytes, the ncclGather
 * count), so rank 0 receives world tiles back to back.  rows is 0 for a rank
 * past the last row (world > height).  Pixel bytes by flags (16 / 8 / 4). */
typedef struct rt_tile_layout_info {
    uint32_t rows;
    uint32_t rows_max;
    uint64_t row_bytes;
    uint64_t tile_bytes;
} rt_tile_layout_info;
int rt_tile_layout(int32_t width, int32_t height, int32_t world, int32_t rank, uint32_t flags,
                   rt_tile_layout_info* out);

/* Rank 0's placement step of rt_render_gather on its own: `gathered_device`
 * holds `world` tiles of rt_tile_layout's tile_bytes back to back (device
 * memory); tile row j of rank k lands at frame row k + j*world.  `frame` is
 * H*W pixels in the format of flags, device memory with RT_OUT_DEVICE
 * (enqueued on hip_stream; NULL is the HIP null stream) or host memory (the
 * call blocks).  The same code rt_render_gather runs after its ncclGather. */
int rt_place_tiles(rt_ctx* ctx, const void* gathered_device, int32_t world, uint32_t flags,
                   void* frame, void* hip_stream);

/* The same placement on host memory (no device). */
int rt_place_tiles_host(const void* gathered, int32_t width, int32_t height, int32_t world,
                        uint32_t flags, void* frame);

/* Which kernel instantiation the most recent rt_render/rt_render_async
 * launched, with its launch shape: lets a caller (bench, tests) state which
 * configuration it timed or checked.  `kernel` is the demangled name rocprofv3
 * reports, e.g. "rt::path_trace_kernel<3, 6, false, true, 4>". */
typedef struct rt_launch_info {
    char kernel[96];
    uint32_t lanes_per_pixel;   /* 1, 4 or 16 lanes trace one pixel's samples     */
    uint32_t halton_tables;     /* 1: LDS low-digit Halton tables filled (§3.3)   */
    uint32_t small_index;       /* 1: fixed-digit Halton (max index < 3^13)       */
    uint32_t block_threads;
    uint32_t grid_x, grid_y;
    uint32_t lds_bytes;         /* dynamic LDS per workgroup                      */
} rt_launch_info;
int rt_last_launch(const rt_ctx* ctx, rt_launch_info* info);

/* How rt_create built the scene: which triangle-BVH build ran (rt_tri_bvh_build,
 * 0 = no triangle BVH), its nodes per octant layout, the wall times of the
 * build (device sync / upload included) and of the host scene compile, and the
 * peak temporary device memory of the GPU SAH build (KiB; 0 for the others). */
typedef struct rt_build_stats {
    uint32_t tri_bvh_build;
    uint32_t tri_bvh_nodes;
    float tri_bvh_build_ms;
    float scene_compile_ms;
    uint32_t tri_bvh_temp_kib;
} rt_build_stats;
int rt_build_info(const rt_ctx* ctx, rt_build_stats* info);

/* Self-check of the kernels' short correctly rounded sqrt and reciprocal
 *  against the IEEE expansions on every one of the 2^32 float
 * bit patterns, on the current device: mismatches[0] sqrt, [1] reciprocal
 * (both 0 for a library whose results equal the oracle's). */
int rt_math_selfcheck(uint64_t* mismatches);

/* Hash of the sources this library was built from (gpuraytracer_amd/srchash.py:
 * csrc/ + include/): a loader can refuse a stale binary. */
const char* rt_build_sha(void);

/* Diagnostic counters of a -DRT_STATS build of the kernel (reads and clears
 * up to 32 uint64 counters, slots in rt_trace.hpp; RT_ERR_STATE in normal
 * builds). */
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
 * At least one output must be non-null.  Synchronous.  When camera_rays is
 * above the kernel's lanes per pixel (2) the frame runs as one workgroup per
 * round of camera rays and an ordered per-pixel sum: the context then keeps a
 * device buffer of 16 B per camera ray and pixel (46 MB at 800x600 x 6; frames
 * that would need more than 1 GB run without the split). */
int rt_render_mis(rt_ctx* ctx, const rt_mis_params* params, float* out_rgba32f,
                  uint8_t* out_rgba8);

/* The SwiftPM scene (Sources/gpuRaytracer/main.swift:21-67, :96-173): the
 * RTrace room with a 1.5 x 1.5 light.  Arrays as rt_scene_cornell_box. */
int rt_scene_cornell_box_mis(int32_t width, int32_t height, CameraGPU* camera,
                             MaterialGPU* materials, rt_float3* vertices,
                             SquareLightGPU* light, uint32_t* n_triangles);

/* How rt_create would lay a scene out on the device (host-only, no device),
 * with default options; rt_scene_describe_ex with `opt` (NULL = defaults).
 * It describes the lockstep kernels: with walk_scheduler FREE or SORTED a BVH
 * scene runs another kernel, whose name and LDS bytes rt_last_launch reports. */
typedef struct rt_scene_info {
    uint32_t n_triangles;
    uint32_t n_triangle_pairs;   /* >0: every (2k,2k+1) shares v0 and an edge -> pair records */
    uint32_t n_spheres;
    uint32_t lds_bytes;          /* intersection records staged per workgroup (0: read from global) */
    uint32_t n_sphere_nodes;     /* sphere BVH nodes per layout (32 B each, 8 layouts, global) */
    uint32_t n_triangle_bvh_nodes; /* triangle BVH nodes per layout (0: LDS layouts); 2n - 1 with
                                      one triangle per leaf (tri_leaf_max <= 1), an upper bound
                                      with larger leaves */
    uint32_t n_box_clusters;     /* pair runs on the faces of one oriented box (slab-tested first) */
    uint32_t pair_free_mask;     /* pairs in no box cluster (bit k = pair k) */
    uint32_t sphere_kernel_lds_bytes; /* dynamic LDS of the sphere kernel (its pair records; 0: sphere kernel not taken) */
    uint32_t kernel_layout;      /* the kernel layout a render (bounces >= 1) takes with these
                                    options (rt_kernel.hpp KernelLayout: 0 triangles in LDS,
                                    1 pairs, 2 global, 3 sorted pairs, 4 pairs by scalar loads,
                                    5 triangle BVH, 6 pairs + box clusters, 7 sphere kernel,
                                    8/9 free-running, 10/11 sorted BVH walks) */
    uint32_t kernel_lds_bytes;   /* that kernel's dynamic LDS per workgroup: exactly what its
                                    staging loops write (rt_last_launch reports the same) */
} rt_scene_info;
int rt_scene_describe(const rt_scene_desc* scene, rt_scene_info* info);
int rt_scene_describe_ex(const rt_scene_desc* scene, const rt_create_options* opt, rt_scene_info* info);

/* The reference's image epilogue (RTrace/image.swift:35-65): fp16 round trip,
 * ×2 exposure, Reinhard, gamma 1/2.2, clamp, truncating UInt8, alpha 255.
 * in: n_pixels rgba32F (host), out: n_pixels*4 bytes. */
void rt_tonemap_rgba8(const float* rgba32f, size_t n_pixels, uint8_t* rgba8);

#ifdef __cplusplus
}
#endif

#endif /* RTPT_H */

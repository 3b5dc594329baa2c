// rt_api.cpp — the C-ABI of librtpt.so (include/rtpt.h).
//
// Replaces the Metal host boundary of the reference:
//   Renderer.init()  (RTrace/renderer.swift:29-115)  -> rt_create / rt_set_seeds
//   Renderer.draw()  (RTrace/renderer.swift:117-146) -> rt_render
// Inputs are copied at create time (makeBuffer(bytes:) semantics), the context
// owns every device buffer, and every failure is returned as an rt_status with
// a message (the reference fatalError()s / force-unwraps instead).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <new>
#include <string>
#include <vector>

#include "../../include/rtpt.h"
#include "rt_kernel.hpp"
#include "rt_scene.hpp"

// RT_TRI_BVH_DEFAULT resolves to this build: the GPU binned SAH builds the host
// build's tree (same rules, same render rate) in a tenth of the time or less --
// the measured build times and rates are in DESIGN.md §5 and profiles/
constexpr uint32_t kDefaultTriBuild = RT_TRI_BVH_GPU_SAH;

struct rt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    rt::CompiledScene scene;
    float4* d_tri_isect = nullptr;
    float4* d_tri_shade = nullptr;
    float4* d_pair_isect = nullptr;
    float4* d_clusters = nullptr;
    float4* d_clu_oct = nullptr;     // rt_scene.hpp clu_oct
    uint32_t* d_sph_lds = nullptr;
    uint16_t* d_sph_lds_id = nullptr;
    uint4* d_sph_box = nullptr;      // the leaf-box layout of the sphere BVH (rt_scene.hpp sph_box)
    float4* d_sph_isect = nullptr;
    float4* d_sph_shade = nullptr;
    float4* d_sph_nodes = nullptr;
    uint32_t* d_sph_perm = nullptr;
    uint4* d_tri_nodes = nullptr;    // triangle BVH: 8 compact layouts (build_tri_sah / rt_lbvh.hip)
    uint32_t tri_build = kDefaultTriBuild;  // rt_create_options.tri_bvh_build (resolved)
    float4* d_tri_sorted = nullptr;
    uint32_t* d_tri_perm = nullptr;
    uint32_t tri_bvh_nodes = 0;      // per layout
    uint32_t tri_bvh_build_used = 0; // rt_tri_bvh_build of the built tree (0: none)
    float tri_bvh_build_ms = 0.0f;   // wall time of the triangle-BVH build
    size_t tri_bvh_temp_bytes = 0;   // peak temporaries of the GPU SAH build
    float scene_compile_ms = 0.0f;   // host scene compile (rt_scene.cpp compile_scene)
    float4* d_mis_shade = nullptr;
    float4* d_mis_tab = nullptr;   // Halton table of the MIS integrator
    uint32_t mis_tab_S = 0;        // samples per strategy it was built for
    void* d_out8 = nullptr;        // staging for host RGBA8 outputs
    size_t out8_cap = 0;
    void* d_mis_part = nullptr;    // per-ray MIS results of a split launch (rt_mis.hip)
    size_t mis_part_cap = 0;
    uint32_t* d_seeds = nullptr;
    bool seeds_ready = false;
    uint32_t seed_max = 0xFFFFFFFFu;  // max seed value (bounds the Halton index)
    float4* d_sum = nullptr;
    size_t sum_cap = 0;  // pixels
    bool sum_valid = false;
    uint32_t sum_row_start = 0, sum_row_step = 0, sum_row_count = 0;
    uint32_t sum_first = 0, sum_samples = 0;  // the sum holds samples [first, first + samples)
    void* d_out = nullptr;  // staging for host outputs
    size_t out_cap = 0;     // bytes
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed = false;
    rt::LaunchInfo launch{};  // what the last rt_render launched (rt_last_launch)
    bool launched = false;
    ncclComm_t comm = nullptr;  // rt_comm_init: row-tile gather over RCCL
    int rank = 0, world = 1;
    void* d_tile = nullptr;     // this rank's rows before the gather
    size_t tile_cap = 0;
    void* d_gather = nullptr;   // rank 0: world x rows_max x W pixels
    size_t gather_cap = 0;
    hipEvent_t ev_tiles = nullptr;  // end of the last gather's reads of d_tile / d_gather
    bool tiles_pending = false;
    uint32_t lanes = 0;  // rt_create_options.lanes_per_pixel (0 = auto)
    rt::SceneMem scene_mem = rt::SceneMem::kAuto;  // rt_create_options.scene_layout
    uint32_t walk = 0;   // rt_create_options.walk_scheduler
    uint32_t walk_leaf_den = 0;  // rt_create_options.walk_leaf_den
    std::string err;
};

namespace {

thread_local std::string g_create_err = "no error";

int fail(rt_ctx* ctx, int status, const std::string& msg) {
    if (ctx)
        ctx->err = msg;
    else
        g_create_err = msg;
    return status;
}

int hip_fail(rt_ctx* ctx, int status, const char* what, hipError_t e) {
    return fail(ctx, status, std::string(what) + ": " + hipGetErrorString(e));
}

// Makes ctx->device current for the duration of an API call, restores after.
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

template <typename T>
hipError_t upload(T** dptr, const void* src, size_t bytes, hipStream_t s) {
    *dptr = nullptr;
    if (bytes == 0) return hipSuccess;
    hipError_t e = hipMalloc((void**)dptr, bytes);
    if (e != hipSuccess) return e;
    e = hipMemcpyAsync(*dptr, src, bytes, hipMemcpyHostToDevice, s);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(s);
}

void release(rt_ctx* c) {
    if (!c) return;
    DeviceGuard g(c->device);
    if (c->tiles_pending) (void)hipEventSynchronize(c->ev_tiles);  // a gather may still read d_tile
    (void)hipFree(c->d_tri_isect);
    (void)hipFree(c->d_tri_shade);
    (void)hipFree(c->d_pair_isect);
    (void)hipFree(c->d_clusters);
    (void)hipFree(c->d_clu_oct);
    (void)hipFree(c->d_sph_lds);
    (void)hipFree(c->d_sph_lds_id);
    (void)hipFree(c->d_sph_box);
    (void)hipFree(c->d_sph_isect);
    (void)hipFree(c->d_sph_shade);
    (void)hipFree(c->d_sph_nodes);
    (void)hipFree(c->d_sph_perm);
    (void)hipFree(c->d_tri_nodes);
    (void)hipFree(c->d_tri_sorted);
    (void)hipFree(c->d_tri_perm);
    (void)hipFree(c->d_mis_shade);
    (void)hipFree(c->d_mis_tab);
    (void)hipFree(c->d_out8);
    (void)hipFree(c->d_mis_part);
    (void)hipFree(c->d_seeds);
    (void)hipFree(c->d_sum);
    (void)hipFree(c->d_out);
    if (c->comm) (void)ncclCommDestroy(c->comm);
    (void)hipFree(c->d_tile);
    (void)hipFree(c->d_gather);
    if (c->ev_tiles) (void)hipEventDestroy(c->ev_tiles);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
}

// Resolves row partition defaults and validates it against the frame height.
bool resolve_rows(const rt_ctx* c, const rt_render_params* p, uint32_t* start, uint32_t* step,
                  uint32_t* count) {
    const uint32_t H = (uint32_t)c->scene.cam.H;
    *start = p->row_start;
    *step = p->row_step ? p->row_step : 1u;
    if (*start >= H) return false;
    const uint32_t avail = (H - 1u - *start) / *step + 1u;
    *count = p->row_count ? p->row_count : avail;
    return *count <= avail;
}

int render_impl(rt_ctx* c, const rt_render_params* p, void* out, bool out_is_device,
                hipStream_t stream, bool sync) {
    if (!p) return fail(c, RT_ERR_INVALID_ARG, "params is null");
    if (p->bounces > RT_MAX_BOUNCES)
        return fail(c, RT_ERR_INVALID_ARG,
                    "bounces > 4: Halton dimensions would leave primes[24] (sampling.metal:97)");
    if (!c->seeds_ready) return fail(c, RT_ERR_STATE, "seeds not set (rt_set_seeds/rt_fill_seeds)");
    uint32_t start, step, count;
    if (!resolve_rows(c, p, &start, &step, &count))
        return fail(c, RT_ERR_INVALID_ARG, "row partition outside the frame");
    const bool want_out = !(p->flags & RT_OUT_NONE);
    const bool keep_sum = (p->flags & RT_KEEP_SUM) != 0;
    if (want_out && !out) return fail(c, RT_ERR_INVALID_ARG, "out is null");
    if (p->accumulate) {
        if (!c->sum_valid || c->sum_row_start != start || c->sum_row_step != step ||
            c->sum_row_count != count ||
            (uint64_t)c->sum_first + c->sum_samples != (uint64_t)p->sample_base)
            return fail(c, RT_ERR_STATE,
                        "accumulate: context sum does not end at sample_base for these rows "
                        "(render with RT_KEEP_SUM first)");
    }
    const uint64_t total = (uint64_t)(p->accumulate ? c->sum_samples : 0u) + p->spp;
    if (total == 0 || total > 0xFFFFFFFFull)
        return fail(c, RT_ERR_INVALID_ARG, "samples in the sum must be in [1, 2^32)");

    const size_t W = (size_t)c->scene.cam.W;
    const size_t pixels = (size_t)count * W;
    if ((p->flags & RT_OUT_FP16) && (p->flags & RT_OUT_RGBA8))
        return fail(c, RT_ERR_INVALID_ARG, "RT_OUT_FP16 and RT_OUT_RGBA8 are exclusive");
    const size_t px_bytes = (p->flags & RT_OUT_RGBA8) ? 4u : (p->flags & RT_OUT_FP16) ? 8u : 16u;
    hipError_t e;
    if (keep_sum || p->accumulate) {
        if (c->sum_cap < pixels) {
            (void)hipFree(c->d_sum);
            c->d_sum = nullptr;
            c->sum_cap = 0;
            c->sum_valid = false;
            if ((e = hipMalloc((void**)&c->d_sum, pixels * sizeof(float4))) != hipSuccess)
                return hip_fail(c, RT_ERR_OUT_OF_MEMORY, "hipMalloc(sum)", e);
            c->sum_cap = pixels;
        }
    }
    void* kout = nullptr;
    if (want_out) {
        if (out_is_device) {
            kout = out;
        } else {
            if (c->out_cap < pixels * px_bytes) {
                (void)hipFree(c->d_out);
                c->d_out = nullptr;
                c->out_cap = 0;
                if ((e = hipMalloc(&c->d_out, pixels * px_bytes)) != hipSuccess)
                    return hip_fail(c, RT_ERR_OUT_OF_MEMORY, "hipMalloc(out staging)", e);
                c->out_cap = pixels * px_bytes;
            }
            kout = c->d_out;
        }
    }

    rt::KParams K;
    memset(&K, 0, sizeof(K));
    K.tri_isect = c->d_tri_isect;
    K.tri_shade = c->d_tri_shade;
    K.pair_isect = c->d_pair_isect;
    K.clusters = c->d_clusters;
    K.clu_oct = c->d_clu_oct;
    K.nC = (uint32_t)(c->scene.clusters.size() / (4 * rt::kCluF4));
    K.pair_free = c->scene.pair_free_mask;
    K.sph_isect = c->d_sph_isect;
    K.sph_lds = c->scene.sph_lds.empty() ? nullptr : c->d_sph_lds;
    K.sph_lds_id = c->d_sph_lds_id;
    K.sph_box = c->scene.sph_box.empty() ? nullptr : c->d_sph_box;
    K.sph_shade = c->d_sph_shade;
    K.sph_nodes = c->d_sph_nodes;
    K.sph_perm = c->d_sph_perm;
    K.tri_nodes = c->d_tri_nodes;
    K.tri_sorted = c->d_tri_sorted;
    K.tri_perm = c->d_tri_perm;
    K.nTN = c->tri_bvh_nodes;
    K.seeds = c->d_seeds;
    K.sum = (keep_sum || p->accumulate) ? c->d_sum : nullptr;
    K.out = kout;
    K.nT = (uint32_t)c->scene.tri_isect.size();
    K.nS = (uint32_t)c->scene.sph_isect.size();
    K.nP = (uint32_t)c->scene.pair_isect.size();
    K.nN = c->scene.sph_layout_nodes;
    K.nE = c->scene.sph_lds_entries;
    const rt::CamConst& cam = c->scene.cam;
    memcpy(K.cam_pos, cam.pos, sizeof(K.cam_pos));
    memcpy(K.cam_u, cam.u, sizeof(K.cam_u));
    memcpy(K.cam_v, cam.v, sizeof(K.cam_v));
    memcpy(K.cam_w, cam.w, sizeof(K.cam_w));
    K.halfW = cam.halfW;
    K.halfH = cam.halfH;
    K.W = cam.W;
    K.H = cam.H;
    memcpy(K.light_center, c->scene.light.center, sizeof(K.light_center));
    {  // rt_kernel.hip shade(): the sample point's zero terms drop out exactly unless -0 is involved
        uint32_t by, bz;
        memcpy(&by, &K.light_center[1], 4);
        memcpy(&bz, &K.light_center[2], 4);
        K.light_plain = (by != 0x80000000u && bz != 0x80000000u) ? 1u : 0u;
    }
    memcpy(K.light_color, c->scene.light.color, sizeof(K.light_color));
    K.spp = p->spp;
    K.sample_base = p->sample_base;
    K.row_start = start;
    K.row_step = step;
    K.row_count = count;
    K.accumulate = p->accumulate ? 1u : 0u;
    K.samples_total = (uint32_t)total;
    K.flags = ((p->flags & RT_OUT_FP16) ? rt::kOutFp16 : 0u) | ((p->flags & RT_OUT_RGBA8) ? rt::kOutRgba8 : 0u);
    K.lanes = c->lanes;
    K.walk = c->walk;
    K.walk_leaf_den = c->walk_leaf_den;
    {
        const uint64_t imax = (uint64_t)c->seed_max + p->sample_base + (p->spp ? p->spp - 1u : 0u);
        K.max_index = imax > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)imax;
    }

    if (keep_sum && !p->accumulate) c->sum_valid = false;  // being overwritten
    (void)hipEventRecord(c->ev0, stream);
    e = rt::launch_path_trace(K, p->bounces, c->scene_mem, stream, &c->launch);
    if (e != hipSuccess) return hip_fail(c, RT_ERR_LAUNCH, "path_trace launch", e);
    c->launched = true;
    (void)hipEventRecord(c->ev1, stream);
    c->timed = true;
    if (keep_sum || p->accumulate) {  // the kernel (re)wrote the running sums
        c->sum_valid = true;
        c->sum_row_start = start;
        c->sum_row_step = step;
        c->sum_row_count = count;
        if (!p->accumulate) c->sum_first = p->sample_base;
        c->sum_samples = (uint32_t)total;
    }
    if (want_out && !out_is_device) {
        if ((e = hipMemcpyAsync(out, kout, pixels * px_bytes, hipMemcpyDeviceToHost, stream)) !=
            hipSuccess)
            return hip_fail(c, RT_ERR_LAUNCH, "hipMemcpyAsync(out)", e);
    }
    if (sync) {
        if ((e = hipStreamSynchronize(stream)) != hipSuccess)
            return hip_fail(c, RT_ERR_LAUNCH, "path_trace execution", e);
        uint32_t short_end = 0;  // RT_LDS_CHECK builds (rt_kernel.hip)
        if (rt::lds_check_result(&short_end) == hipSuccess && short_end)
            return fail(c, RT_ERR_LAUNCH, "LDS overflow: staged records end at byte " + std::to_string(short_end) +
                                              ", past the dispatch's dynamic LDS");
    }
    return RT_OK;
}

int ensure_staging(rt_ctx* c, void** buf, size_t* cap, size_t bytes, const char* what);

int nccl_fail(rt_ctx* ctx, const char* what, ncclResult_t r) {
    return fail(ctx, RT_ERR_COMM, std::string(what) + ": " + ncclGetErrorString(r));
}

size_t pixel_bytes(uint32_t flags) {
    return (flags & RT_OUT_RGBA8) ? 4u : (flags & RT_OUT_FP16) ? 8u : 16u;
}

// Row layout of the gather (rt_tile_layout): rank k of N owns the frame rows
// y = k + j*N, j < rows; every rank sends a tile padded to rows_max rows, so
// the gathered buffer holds N tiles of tile_bytes back to back.  A rank past
// the last row (N > H) owns no row and sends its padded tile all the same.
struct TileLayout {
    uint32_t rows, rows_max;
    size_t row_bytes, tile_bytes;
};

TileLayout tile_layout(uint32_t W, uint32_t H, uint32_t N, uint32_t rank, uint32_t flags) {
    TileLayout L;
    L.rows = rank < H ? (H - 1u - rank) / N + 1u : 0u;
    L.rows_max = (H + N - 1u) / N;
    L.row_bytes = (size_t)W * pixel_bytes(flags);
    L.tile_bytes = (size_t)L.rows_max * L.row_bytes;
    return L;
}

bool tile_args_ok(int32_t W, int32_t H, int32_t N) { return W > 0 && H > 0 && N > 0; }

// Rank 0's placement after the gather: tile row j of rank k -> frame row
// k + j*N (rt_kernel.hip place_tiles_kernel, one launch on `stream`).  A host
// frame is assembled in the context's staging buffer, then copied down once
// the kernel has finished.
int place_tiles_impl(rt_ctx* c, const void* gathered, uint32_t N, uint32_t flags, void* frame,
                     hipStream_t stream) {
    const uint32_t W = (uint32_t)c->scene.cam.W, H = (uint32_t)c->scene.cam.H;
    const TileLayout L = tile_layout(W, H, N, 0, flags);
    const bool dev = (flags & RT_OUT_DEVICE) != 0;
    const size_t frame_bytes = (size_t)H * L.row_bytes;
    void* dst = frame;
    int st;
    if (!dev) {
        if ((st = ensure_staging(c, &c->d_out, &c->out_cap, frame_bytes, "hipMalloc(frame staging)")) != RT_OK)
            return st;
        dst = c->d_out;
    }
    hipError_t e = rt::launch_place_tiles(gathered, dst, L.row_bytes, L.tile_bytes, H, N, stream);
    if (e != hipSuccess) return hip_fail(c, RT_ERR_LAUNCH, "place_tiles launch", e);
    if (!dev) {
        if ((e = hipStreamSynchronize(stream)) != hipSuccess ||
            (e = hipMemcpyAsync(frame, dst, frame_bytes, hipMemcpyDeviceToHost, stream)) != hipSuccess ||
            (e = hipStreamSynchronize(stream)) != hipSuccess)
            return hip_fail(c, RT_ERR_LAUNCH, "frame copy to host", e);
    }
    return RT_OK;
}

// rt_render_gather: this rank's interleaved rows into d_tile, one ncclGather of
// the (padded, equal-sized) tiles to rank 0, then place_tiles_dev.
int render_gather_impl(rt_ctx* c, const rt_render_params* p, void* frame, hipStream_t stream) {
    if (!p) return fail(c, RT_ERR_INVALID_ARG, "params is null");
    if (!c->comm) return fail(c, RT_ERR_STATE, "no communicator (rt_comm_init)");
    if (p->row_start || p->row_step > 1 || p->row_count)
        return fail(c, RT_ERR_INVALID_ARG, "rt_render_gather partitions the rows itself: "
                                           "params must name the whole frame (row_start 0, "
                                           "row_step 0 or 1, row_count 0)");
    if ((p->flags & RT_OUT_FP16) && (p->flags & RT_OUT_RGBA8))
        return fail(c, RT_ERR_INVALID_ARG, "RT_OUT_FP16 and RT_OUT_RGBA8 are exclusive");
    const bool want_out = !(p->flags & RT_OUT_NONE);
    const bool dev = (p->flags & RT_OUT_DEVICE) != 0;
    if (want_out && c->rank == 0 && !frame) return fail(c, RT_ERR_INVALID_ARG, "frame is null on rank 0");
    const uint32_t H = (uint32_t)c->scene.cam.H, W = (uint32_t)c->scene.cam.W, N = (uint32_t)c->world;
    const TileLayout L = tile_layout(W, H, N, (uint32_t)c->rank, p->flags);
    hipError_t e;
    // d_tile / d_gather are reused: a previous call on another stream may still
    // be gathering from them (RT_OUT_DEVICE returns without a host sync)
    if (c->tiles_pending && (e = hipStreamWaitEvent(stream, c->ev_tiles, 0)) != hipSuccess)
        return hip_fail(c, RT_ERR_LAUNCH, "hipStreamWaitEvent(previous gather)", e);
    int st;
    if (want_out && (st = ensure_staging(c, &c->d_tile, &c->tile_cap, L.tile_bytes, "hipMalloc(tile)")) != RT_OK)
        return st;
    if (L.rows > 0) {  // a rank past the last row renders nothing but still joins the gather
        rt_render_params q = *p;
        q.row_start = (uint32_t)c->rank;
        q.row_step = N;
        q.row_count = L.rows;
        q.flags = p->flags | RT_OUT_DEVICE;
        if ((st = render_impl(c, &q, c->d_tile, true, stream, false)) != RT_OK) return st;
    }
    if (!want_out) return RT_OK;
    if (c->rank == 0 && (st = ensure_staging(c, &c->d_gather, &c->gather_cap, L.tile_bytes * N,
                                             "hipMalloc(gather)")) != RT_OK)
        return st;
    ncclResult_t r = ncclGather(c->d_tile, c->rank == 0 ? c->d_gather : nullptr, L.tile_bytes, ncclUint8,
                                0, c->comm, stream);
    if (r != ncclSuccess) return nccl_fail(c, "ncclGather", r);
    if (c->rank == 0 && (st = place_tiles_impl(c, c->d_gather, N, p->flags, frame, stream)) != RT_OK)
        return st;
    if ((e = hipEventRecord(c->ev_tiles, stream)) != hipSuccess)
        return hip_fail(c, RT_ERR_LAUNCH, "hipEventRecord(gather)", e);
    c->tiles_pending = true;
    if (!dev) {
        e = hipStreamSynchronize(stream);
        if (e != hipSuccess) return hip_fail(c, RT_ERR_COMM, "render+gather execution", e);
    }
    return RT_OK;
}

// halton(i, d) of the SwiftPM kernel (Sources/gpuRaytracer/shaders.metal:32-47),
// the same loop as RTrace/sampling.metal:107-122.
float halton_host(uint32_t i, uint32_t d) {
    static const uint32_t primes[24] = RT_PRIMES_INIT;
    const uint32_t b = primes[d];
    float f = 1.0f;
    const float invB = 1.0f / (float)b;
    float r = 0.0f;
    while (i > 0) {
        f = f * invB;
        r = r + f * (float)(i % b);
        i = i / b;
    }
    return r;
}

// MIS sample table: the u of every strategy depends only on the sample index
// (haltonRandom(i, d), shaders.metal:556,564,584,595,617), not on the pixel.
int mis_table(rt_ctx* c, uint32_t S) {
    if (c->d_mis_tab && c->mis_tab_S == S) return RT_OK;
    std::vector<float> t((size_t)S * 12u);
    for (uint32_t i = 0; i < S; ++i) {
        float* q = &t[(size_t)i * 12u];
        q[0] = halton_host(i, 0);            // light sampling :556
        q[1] = halton_host(i, 1);
        q[2] = 0.0f;
        q[3] = 0.0f;
        q[4] = halton_host(i + S, 2);        // cosine :564
        q[5] = halton_host(i + S, 3);
        q[6] = halton_host(i, 6);            // its secondary NEE :584
        q[7] = halton_host(i, 7);
        q[8] = halton_host(i + 2 * S, 4);    // VNDF :595
        q[9] = halton_host(i + 2 * S, 5);
        q[10] = halton_host(i + S, 6);       // its secondary NEE :617
        q[11] = halton_host(i + S, 7);
    }
    (void)hipFree(c->d_mis_tab);
    c->d_mis_tab = nullptr;
    c->mis_tab_S = 0;
    hipError_t e = upload(&c->d_mis_tab, t.data(), t.size() * sizeof(float), c->stream);
    if (e != hipSuccess) return hip_fail(c, RT_ERR_OUT_OF_MEMORY, "MIS table upload", e);
    c->mis_tab_S = S;
    return RT_OK;
}

int ensure_staging(rt_ctx* c, void** buf, size_t* cap, size_t bytes, const char* what) {
    if (*cap >= bytes) return RT_OK;
    (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(buf, bytes);
    if (e != hipSuccess) return hip_fail(c, RT_ERR_OUT_OF_MEMORY, what, e);
    *cap = bytes;
    return RT_OK;
}

int render_mis_impl(rt_ctx* c, const rt_mis_params* p, float* out, uint8_t* out8) {
    if (!p) return fail(c, RT_ERR_INVALID_ARG, "params is null");
    if (!out && !out8) return fail(c, RT_ERR_INVALID_ARG, "both outputs are null");
    if (!c->scene.sph_isect.empty())
        return fail(c, RT_ERR_INVALID_ARG,
                    "the MIS integrator traces triangle scenes only (shaders.metal:459-509)");
    if (c->scene.tri_isect.empty()) return fail(c, RT_ERR_INVALID_ARG, "scene has no triangles");
    if (p->camera_rays == 0) return fail(c, RT_ERR_INVALID_ARG, "camera_rays must be >= 1");
    if (p->mis_samples < 3 || p->mis_samples / 3u > (1u << 20))
        return fail(c, RT_ERR_INVALID_ARG, "mis_samples must be in [3, 3 * 2^20]");
    rt_render_params rp;
    memset(&rp, 0, sizeof(rp));
    rp.row_start = p->row_start;
    rp.row_step = p->row_step;
    rp.row_count = p->row_count;
    uint32_t start, step, count;
    if (!resolve_rows(c, &rp, &start, &step, &count))
        return fail(c, RT_ERR_INVALID_ARG, "row partition outside the frame");
    const uint32_t S = p->mis_samples / 3u;  // samplesPerStrategy (:546)
    int st = mis_table(c, S);
    if (st != RT_OK) return st;
    const bool dev = (p->flags & RT_OUT_DEVICE) != 0;
    const size_t pixels = (size_t)count * (size_t)c->scene.cam.W;
    float4* kout = nullptr;
    uchar4* kout8 = nullptr;
    if (out) {
        if (!dev && (st = ensure_staging(c, &c->d_out, &c->out_cap, pixels * 16u, "hipMalloc(out staging)")) != RT_OK)
            return st;
        kout = dev ? reinterpret_cast<float4*>(out) : reinterpret_cast<float4*>(c->d_out);
    }
    if (out8) {
        if (!dev && (st = ensure_staging(c, &c->d_out8, &c->out8_cap, pixels * 4u, "hipMalloc(out8 staging)")) != RT_OK)
            return st;
        kout8 = dev ? reinterpret_cast<uchar4*>(out8) : reinterpret_cast<uchar4*>(c->d_out8);
    }

    rt::MisParams K;
    memset(&K, 0, sizeof(K));
    K.tri_isect = c->d_tri_isect;
    K.clusters = c->d_clusters;
    K.nC = (uint32_t)(c->scene.clusters.size() / (4 * rt::kCluF4));
    K.pair_free = c->scene.pair_free_mask;
    K.pair_isect = c->d_pair_isect;
    K.mis_shade = c->d_mis_shade;
    K.u_tab = c->d_mis_tab;
    K.tri_nodes = c->d_tri_nodes;
    K.tri_sorted = c->d_tri_sorted;
    K.tri_perm = c->d_tri_perm;
    K.nTN = c->tri_bvh_nodes;
    K.out = kout;
    K.out8 = kout8;
    K.nT = (uint32_t)c->scene.tri_isect.size();
    K.nP = (uint32_t)c->scene.pair_isect.size();
    const rt::CamConst& cam = c->scene.cam;
    memcpy(K.cam_pos, cam.pos, sizeof(K.cam_pos));
    memcpy(K.cam_u, cam.u, sizeof(K.cam_u));
    memcpy(K.cam_v, cam.v, sizeof(K.cam_v));
    memcpy(K.cam_w, cam.w, sizeof(K.cam_w));
    K.halfW = cam.halfW;
    K.halfH = cam.halfH;
    K.W = cam.W;
    K.H = cam.H;
    const rt::MisLightConst& ml = c->scene.mis_light;
    memcpy(K.l_center, ml.center, sizeof(K.l_center));
    memcpy(K.l_tangent, ml.tangent, sizeof(K.l_tangent));
    memcpy(K.l_bitangent, ml.bitangent, sizeof(K.l_bitangent));
    memcpy(K.l_radiance, ml.radiance, sizeof(K.l_radiance));
    K.l_width = ml.width;
    K.l_depth = ml.depth;
    K.l_area = ml.area;
    K.exposure = ml.exposure;
    K.camera_rays = p->camera_rays;
    K.S = S;
    K.row_start = start;
    K.row_step = step;
    K.row_count = count;
    const size_t pb = rt::mis_part_bytes(K.camera_rays, pixels);
    if (c->mis_part_cap > 2 * pb) {  // a much smaller (or unsplit) frame: give the memory back
        const hipError_t e0 = hipStreamSynchronize(c->stream);  // the last launch may still read it
        if (e0 != hipSuccess) return hip_fail(c, RT_ERR_LAUNCH, "hipStreamSynchronize(mis)", e0);
        (void)hipFree(c->d_mis_part);
        c->d_mis_part = nullptr;
        c->mis_part_cap = 0;
    }
    if (pb) {
        if ((st = ensure_staging(c, &c->d_mis_part, &c->mis_part_cap, pb, "hipMalloc(mis records)")) != RT_OK)
            return st;
        K.part = reinterpret_cast<float4*>(c->d_mis_part);
    }

    hipError_t e;
    (void)hipEventRecord(c->ev0, c->stream);
    e = rt::launch_mis(K, c->scene_mem, c->stream);
    if (e != hipSuccess) return hip_fail(c, RT_ERR_LAUNCH, "mis launch", e);
    (void)hipEventRecord(c->ev1, c->stream);
    c->timed = true;
    if (out && !dev &&
        (e = hipMemcpyAsync(out, kout, pixels * 16u, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
        return hip_fail(c, RT_ERR_LAUNCH, "hipMemcpyAsync(out)", e);
    if (out8 && !dev &&
        (e = hipMemcpyAsync(out8, kout8, pixels * 4u, hipMemcpyDeviceToHost, c->stream)) != hipSuccess)
        return hip_fail(c, RT_ERR_LAUNCH, "hipMemcpyAsync(out8)", e);
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess)
        return hip_fail(c, RT_ERR_LAUNCH, "mis execution", e);
    return RT_OK;
}

// rt_create_options (include/rtpt.h) -> the context's choices and the host
// builds' options.  False (with *why) for a value outside its range.
struct Resolved {
    uint32_t lanes = 0, tri_build = RT_TRI_BVH_HOST_SAH, walk = RT_WALK_AUTO, walk_leaf_den = 0;
    rt::SceneMem mem = rt::SceneMem::kAuto;
    uint32_t tri_leaf_max = rt::kTriLeafMax;
    double tri_leaf_cost = 1.0;
    rt::BuildOptions build;
};

bool resolve_options(const rt_create_options* o, Resolved* r, const char** why) {
    *r = Resolved();
    if (!o) return true;
    for (uint32_t v : o->reserved)
        if (v != 0) { *why = "rt_create_options.reserved must be zero"; return false; }
    switch (o->scene_layout) {
        case RT_LAYOUT_AUTO: r->mem = rt::SceneMem::kAuto; break;
        case RT_LAYOUT_PAIRS: r->mem = rt::SceneMem::kPairLds; break;
        case RT_LAYOUT_SINGLE: r->mem = rt::SceneMem::kLdsSingle; break;
        case RT_LAYOUT_GLOBAL: r->mem = rt::SceneMem::kSmem; break;
        case RT_LAYOUT_PAIRS_SMEM: r->mem = rt::SceneMem::kPairSmem; break;
        case RT_LAYOUT_SORTED: r->mem = rt::SceneMem::kPairSorted; break;
        case RT_LAYOUT_BVH: r->mem = rt::SceneMem::kTriBvh; break;
        default: *why = "rt_create_options.scene_layout out of range"; return false;
    }
    if (o->lanes_per_pixel != 0 && o->lanes_per_pixel != 1 && o->lanes_per_pixel != 4 &&
        o->lanes_per_pixel != 16) {
        *why = "rt_create_options.lanes_per_pixel must be 0, 1, 4 or 16";
        return false;
    }
    r->lanes = o->lanes_per_pixel;
    switch (o->tri_bvh_build) {
        case RT_TRI_BVH_DEFAULT: r->tri_build = kDefaultTriBuild; break;
        case RT_TRI_BVH_HOST_SAH: case RT_TRI_BVH_GPU_LBVH: case RT_TRI_BVH_GPU_SAH:
            r->tri_build = o->tri_bvh_build; break;
        default: *why = "rt_create_options.tri_bvh_build out of range"; return false;
    }
    if (o->tri_leaf_max > 128) { *why = "rt_create_options.tri_leaf_max must be <= 128"; return false; }
    if (o->tri_leaf_max) r->tri_leaf_max = o->tri_leaf_max;
    if (!(o->tri_leaf_cost >= 0.0f) || o->tri_leaf_cost > 1e6f) {
        *why = "rt_create_options.tri_leaf_cost must be in [0, 1e6]";
        return false;
    }
    if (o->tri_leaf_cost > 0.0f) r->tri_leaf_cost = o->tri_leaf_cost;
    if (o->sphere_leaf_max > 255) { *why = "rt_create_options.sphere_leaf_max must be <= 255"; return false; }
    if (o->sphere_leaf_max) r->build.sphere_leaf_max = o->sphere_leaf_max;
    if (o->sphere_median > 1) { *why = "rt_create_options.sphere_median must be 0 or 1"; return false; }
    r->build.sphere_sah = o->sphere_median == 0;
    if (o->walk_scheduler > RT_WALK_SORTED) { *why = "rt_create_options.walk_scheduler out of range"; return false; }
    r->walk = o->walk_scheduler;
    if (o->walk_leaf_den > 64) { *why = "rt_create_options.walk_leaf_den must be <= 64"; return false; }
    r->walk_leaf_den = o->walk_leaf_den;
    return true;
}

}  // namespace

extern "C" {

void rt_create_options_default(rt_create_options* opt) {
    if (opt) memset(opt, 0, sizeof(*opt));
}

int rt_abi_version(void) { return RTPT_ABI_VERSION; }

const char* rt_status_string(int s) {
    switch (s) {
        case RT_OK: return "RT_OK";
        case RT_ERR_INVALID_ARG: return "RT_ERR_INVALID_ARG";
        case RT_ERR_NO_DEVICE: return "RT_ERR_NO_DEVICE";
        case RT_ERR_OUT_OF_MEMORY: return "RT_ERR_OUT_OF_MEMORY";
        case RT_ERR_LAUNCH: return "RT_ERR_LAUNCH";
        case RT_ERR_STATE: return "RT_ERR_STATE";
        case RT_ERR_COMM: return "RT_ERR_COMM";
        default: return "RT_ERR_UNKNOWN";
    }
}

const char* rt_last_error(const rt_ctx* ctx) {
    return ctx ? ctx->err.c_str() : g_create_err.c_str();
}

int rt_create(const rt_scene_desc* d, rt_ctx** out_ctx) { return rt_create_ex(d, nullptr, out_ctx); }

int rt_create_ex(const rt_scene_desc* d, const rt_create_options* opt, rt_ctx** out_ctx) {
    if (!out_ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "out_ctx is null");
    *out_ctx = nullptr;
    if (!d) return fail(nullptr, RT_ERR_INVALID_ARG, "scene desc is null");
    if (!d->camera) return fail(nullptr, RT_ERR_INVALID_ARG, "camera is null");
    if (!d->square_lights || d->n_square_lights < 1)
        return fail(nullptr, RT_ERR_INVALID_ARG, "square_lights[0] is required (raytrace.metal:22)");
    Resolved ro;
    const char* why = nullptr;
    if (!resolve_options(opt, &ro, &why)) return fail(nullptr, RT_ERR_INVALID_ARG, why);
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0)
        return fail(nullptr, RT_ERR_NO_DEVICE,
                    std::string("no HIP device: ") + (e != hipSuccess ? hipGetErrorString(e) : "count 0"));
    if (d->device < 0 || d->device >= count)
        return fail(nullptr, RT_ERR_NO_DEVICE, "device ordinal out of range");

    rt_ctx* c = new (std::nothrow) rt_ctx();
    if (!c) return fail(nullptr, RT_ERR_OUT_OF_MEMORY, "host allocation");
    c->device = d->device;
    c->lanes = ro.lanes;
    c->tri_build = ro.tri_build;
    c->scene_mem = ro.mem;
    c->walk = ro.walk;
    c->walk_leaf_den = ro.walk_leaf_den;
    DeviceGuard g(c->device);
    const char* err = nullptr;
    using clk = std::chrono::steady_clock;
    const auto t_compile = clk::now();
    if (!rt::compile_scene(*d->camera, d->materials, d->vertices, d->n_triangles,
                           d->square_lights[0], d->spheres, d->n_spheres, &c->scene, &err, ro.build)) {
        delete c;
        return fail(nullptr, RT_ERR_INVALID_ARG, err);
    }
    c->scene_compile_ms = std::chrono::duration<float, std::milli>(clk::now() - t_compile).count();
    int status = RT_OK;
    std::string msg;
    do {
        if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess) {
            status = RT_ERR_NO_DEVICE; msg = std::string("hipStreamCreate: ") + hipGetErrorString(e); break;
        }
        if ((e = hipEventCreate(&c->ev0)) != hipSuccess || (e = hipEventCreate(&c->ev1)) != hipSuccess ||
            (e = hipEventCreateWithFlags(&c->ev_tiles, hipEventDisableTiming)) != hipSuccess) {
            status = RT_ERR_NO_DEVICE; msg = std::string("hipEventCreate: ") + hipGetErrorString(e); break;
        }
        const rt::CompiledScene& s = c->scene;
        if ((e = upload(&c->d_tri_isect, s.tri_isect.data(), s.tri_isect.size() * sizeof(rt::TriIsect), c->stream)) != hipSuccess ||
            (e = upload(&c->d_tri_shade, s.tri_shade.data(), s.tri_shade.size() * sizeof(rt::TriShade), c->stream)) != hipSuccess ||
            (e = upload(&c->d_pair_isect, s.pair_isect.data(), s.pair_isect.size() * sizeof(rt::PairIsect), c->stream)) != hipSuccess ||
            (e = upload(&c->d_clusters, s.clusters.data(), s.clusters.size() * sizeof(float), c->stream)) != hipSuccess ||
            (e = upload(&c->d_clu_oct, s.clu_oct.data(), s.clu_oct.size() * sizeof(float), c->stream)) != hipSuccess ||
            (e = upload(&c->d_sph_lds, s.sph_lds.data(), s.sph_lds.size() * sizeof(uint32_t), c->stream)) != hipSuccess ||
            (e = upload(&c->d_sph_lds_id, s.sph_lds_id.data(), s.sph_lds_id.size() * sizeof(uint16_t), c->stream)) != hipSuccess ||
            (e = upload(&c->d_sph_box, s.sph_box.data(), s.sph_box.size() * sizeof(uint32_t), c->stream)) != hipSuccess ||
            (e = upload(&c->d_sph_isect, s.sph_isect.data(), s.sph_isect.size() * sizeof(rt::SphIsect), c->stream)) != hipSuccess ||
            (e = upload(&c->d_sph_shade, s.sph_shade.data(), s.sph_shade.size() * sizeof(rt::SphShade), c->stream)) != hipSuccess ||
            (e = upload(&c->d_sph_nodes, s.sph_nodes.data(), s.sph_nodes.size() * sizeof(rt::BvhNode), c->stream)) != hipSuccess ||
            (e = upload(&c->d_sph_perm, s.sph_perm.data(), s.sph_perm.size() * sizeof(uint32_t), c->stream)) != hipSuccess ||
            (e = upload(&c->d_mis_shade, s.mis_shade.data(), s.mis_shade.size() * sizeof(rt::MisShade), c->stream)) != hipSuccess) {
            status = RT_ERR_OUT_OF_MEMORY; msg = std::string("scene upload: ") + hipGetErrorString(e); break;
        }
        // Triangle BVH, built on the device (replaces setupAccelerationStructures,
        // computeShader.swift:45-97): above kTriBvhMinTriangles or when the records
        // do not fit the LDS layouts, or when forced (RTPT_SCENE_MEM=bvh).
        const uint32_t nT = (uint32_t)s.tri_isect.size();
        const size_t lds_pairs = rt::kernel_lds_bytes(nT, (uint32_t)s.pair_isect.size(), 0, 0);
        const size_t lds_single = rt::kernel_lds_bytes(nT, 0, 0, 0);
        const bool need_bvh = nT > 0 && (c->scene_mem == rt::SceneMem::kTriBvh ||
                                         (c->scene_mem == rt::SceneMem::kAuto &&
                                          (nT > rt::kTriBvhMinTriangles ||
                                           std::min(lds_pairs, lds_single) > rt::kMaxLdsBytes)));
        if (need_bvh) {
            const size_t nn = 2 * (size_t)nT - 1;
            const auto t_build = clk::now();
            if (c->tri_build == RT_TRI_BVH_GPU_SAH) {  // GPU binned SAH (rt_gsah.hip)
                if ((e = hipMalloc((void**)&c->d_tri_nodes, rt::kTriCompactLayouts * nn * sizeof(uint4))) != hipSuccess ||
                    (e = hipMalloc((void**)&c->d_tri_sorted, 3 * (size_t)nT * sizeof(float4))) != hipSuccess ||
                    (e = hipMalloc((void**)&c->d_tri_perm, (size_t)nT * sizeof(uint32_t))) != hipSuccess) {
                    status = RT_ERR_OUT_OF_MEMORY; msg = std::string("hipMalloc(triangle BVH): ") + hipGetErrorString(e); break;
                }
                uint32_t total = 0;
                size_t temp = 0;
                if ((e = rt::build_tri_gsah(c->d_tri_isect, nT, s.margin, ro.tri_leaf_max, ro.tri_leaf_cost,
                                            c->d_tri_nodes, c->d_tri_sorted, c->d_tri_perm, &total, &temp,
                                            c->stream)) != hipSuccess) {
                    status = (e == hipErrorInvalidValue) ? RT_ERR_INVALID_ARG
                             : (e == hipErrorOutOfMemory) ? RT_ERR_OUT_OF_MEMORY : RT_ERR_LAUNCH;
                    msg = std::string("triangle BVH build: ") + hipGetErrorString(e); break;
                }
                c->tri_bvh_nodes = total;
                c->tri_bvh_temp_bytes = temp;
            } else if (c->tri_build == RT_TRI_BVH_GPU_LBVH) {  // GPU Morton build (rt_lbvh.hip)
                if ((e = hipMalloc((void**)&c->d_tri_nodes, rt::kTriCompactLayouts * nn * sizeof(uint4))) != hipSuccess ||
                    (e = hipMalloc((void**)&c->d_tri_sorted, 3 * (size_t)nT * sizeof(float4))) != hipSuccess ||
                    (e = hipMalloc((void**)&c->d_tri_perm, (size_t)nT * sizeof(uint32_t))) != hipSuccess) {
                    status = RT_ERR_OUT_OF_MEMORY; msg = std::string("hipMalloc(triangle BVH): ") + hipGetErrorString(e); break;
                }
                if ((e = rt::build_tri_lbvh(c->d_tri_isect, nT, s.tri_lo, s.tri_hi, s.margin, c->d_tri_nodes,
                                            c->d_tri_sorted, c->d_tri_perm, c->stream)) != hipSuccess) {
                    status = (e == hipErrorInvalidValue) ? RT_ERR_INVALID_ARG : RT_ERR_LAUNCH;
                    msg = std::string("triangle BVH build: ") + hipGetErrorString(e); break;
                }
            } else {  // host binned SAH (rt_scene.cpp build_tri_sah), uploaded
                std::vector<uint32_t> nodes, perm;
                std::vector<rt::TriIsect> sorted;
                if (!rt::build_tri_sah(s.tri_isect, s.margin, &nodes, &sorted, &perm, ro.tri_leaf_max,
                                       ro.tri_leaf_cost)) {
                    status = RT_ERR_INVALID_ARG; msg = "triangle BVH build: too many triangles (2^24)"; break;
                }
                if ((e = upload(&c->d_tri_nodes, nodes.data(), nodes.size() * sizeof(uint32_t), c->stream)) != hipSuccess ||
                    (e = upload(&c->d_tri_sorted, sorted.data(), sorted.size() * sizeof(rt::TriIsect), c->stream)) != hipSuccess ||
                    (e = upload(&c->d_tri_perm, perm.data(), perm.size() * sizeof(uint32_t), c->stream)) != hipSuccess) {
                    status = RT_ERR_OUT_OF_MEMORY; msg = std::string("triangle BVH upload: ") + hipGetErrorString(e); break;
                }
                c->tri_bvh_nodes = (uint32_t)(nodes.size() / (4 * rt::kTriCompactLayouts));
            }
            if (c->tri_build == RT_TRI_BVH_GPU_LBVH) c->tri_bvh_nodes = (uint32_t)nn;
            c->tri_bvh_build_used = c->tri_build;
            c->tri_bvh_build_ms = std::chrono::duration<float, std::milli>(clk::now() - t_build).count();
        }
        const size_t npx = (size_t)s.cam.W * (size_t)s.cam.H;
        if ((e = hipMalloc((void**)&c->d_seeds, npx * sizeof(uint32_t))) != hipSuccess) {
            status = RT_ERR_OUT_OF_MEMORY; msg = std::string("hipMalloc(seeds): ") + hipGetErrorString(e); break;
        }
    } while (0);
    if (status != RT_OK) {
        release(c);
        delete c;
        return fail(nullptr, status, msg);
    }
    *out_ctx = c;
    return RT_OK;
}

int rt_set_seeds(rt_ctx* c, const uint32_t* seeds, int32_t width, int32_t height) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "ctx is null");
    if (!seeds) return fail(c, RT_ERR_INVALID_ARG, "seeds is null");
    if (width != c->scene.cam.W || height != c->scene.cam.H)
        return fail(c, RT_ERR_INVALID_ARG, "seed texture size must equal the camera resolution");
    DeviceGuard g(c->device);
    const size_t bytes = (size_t)width * (size_t)height * sizeof(uint32_t);
    hipError_t e = hipMemcpyAsync(c->d_seeds, seeds, bytes, hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, RT_ERR_LAUNCH, "seed upload", e);
    uint32_t mx = 0;
    for (size_t k = 0, n = (size_t)width * (size_t)height; k < n; ++k) mx = seeds[k] > mx ? seeds[k] : mx;
    c->seed_max = mx;
    c->seeds_ready = true;
    return RT_OK;
}

int rt_fill_seeds(rt_ctx* c, uint64_t key) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "ctx is null");
    DeviceGuard g(c->device);
    const uint64_t n = (uint64_t)c->scene.cam.W * (uint64_t)c->scene.cam.H;
    hipError_t e = rt::launch_fill_seeds(c->d_seeds, key, n, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return hip_fail(c, RT_ERR_LAUNCH, "fill_seeds", e);
    c->seed_max = 0xFFFFFu;  // splitmix64(.) mod 2^20
    c->seeds_ready = true;
    return RT_OK;
}

int rt_render(rt_ctx* c, const rt_render_params* p, void* out) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "ctx is null");
    DeviceGuard g(c->device);
    const bool dev = p && (p->flags & RT_OUT_DEVICE);
    return render_impl(c, p, out, dev, c->stream, true);
}

int rt_render_async(rt_ctx* c, const rt_render_params* p, void* out_device, void* hip_stream) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "ctx is null");
    DeviceGuard g(c->device);
    return render_impl(c, p, out_device, true, (hipStream_t)hip_stream, false);
}

int rt_last_kernel_ms(rt_ctx* c, float* ms) {
    if (!c || !ms) return fail(c, RT_ERR_INVALID_ARG, "null argument");
    if (!c->timed) return fail(c, RT_ERR_STATE, "no render yet");
    DeviceGuard g(c->device);
    hipError_t e = hipEventSynchronize(c->ev1);
    if (e == hipSuccess) e = hipEventElapsedTime(ms, c->ev0, c->ev1);
    if (e != hipSuccess) return hip_fail(c, RT_ERR_LAUNCH, "hipEventElapsedTime", e);
    return RT_OK;
}

int rt_comm_unique_id(uint8_t id[RT_COMM_ID_BYTES]) {
    if (!id) return fail(nullptr, RT_ERR_INVALID_ARG, "id is null");
    static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    const ncclResult_t r = ncclGetUniqueId(&u);
    if (r != ncclSuccess) return nccl_fail(nullptr, "ncclGetUniqueId", r);
    memcpy(id, &u, sizeof(u));
    return RT_OK;
}

int rt_comm_init(rt_ctx* c, int32_t rank, int32_t world, const uint8_t id[RT_COMM_ID_BYTES]) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "ctx is null");
    if (!id) return fail(c, RT_ERR_INVALID_ARG, "id is null");
    if (world < 1 || rank < 0 || rank >= world)
        return fail(c, RT_ERR_INVALID_ARG, "need 0 <= rank < world");
    if (c->comm) return fail(c, RT_ERR_STATE, "context already has a communicator");
    DeviceGuard g(c->device);
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, world, u, rank);
    if (r != ncclSuccess) return nccl_fail(c, "ncclCommInitRank", r);
    c->comm = comm;
    c->rank = rank;
    c->world = world;
    return RT_OK;
}

int rt_render_gather(rt_ctx* c, const rt_render_params* p, void* frame, void* hip_stream) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "ctx is null");
    DeviceGuard g(c->device);
    // NULL is the HIP null stream (rt_render_async's convention): a caller on
    // the default stream (torch's current stream is handle 0) gets its work
    // ordered after everything it enqueued there
    hipStream_t s = (hipStream_t)hip_stream;
    return render_gather_impl(c, p, frame, s);
}

int rt_comm_info(const rt_ctx* c, int32_t* count, int32_t* rank) {
    if (!c || !count || !rank) return fail(nullptr, RT_ERR_INVALID_ARG, "null argument");
    rt_ctx* m = const_cast<rt_ctx*>(c);  // the error message slot only
    if (!c->comm) return fail(m, RT_ERR_STATE, "rt_comm_info: no communicator (rt_comm_init first)");
    int n = 0, r = 0;
    ncclResult_t res = ncclCommCount(c->comm, &n);
    if (res != ncclSuccess) return nccl_fail(m, "ncclCommCount", res);
    res = ncclCommUserRank(c->comm, &r);
    if (res != ncclSuccess) return nccl_fail(m, "ncclCommUserRank", res);
    *count = n;
    *rank = r;
    return RT_OK;
}

int rt_tile_layout(int32_t width, int32_t height, int32_t world, int32_t rank, uint32_t flags,
                   rt_tile_layout_info* out) {
    if (!out || !tile_args_ok(width, height, world) || rank < 0 || rank >= world)
        return RT_ERR_INVALID_ARG;
    const TileLayout L = tile_layout((uint32_t)width, (uint32_t)height, (uint32_t)world, (uint32_t)rank, flags);
    out->rows = L.rows;
    out->rows_max = L.rows_max;
    out->row_bytes = L.row_bytes;
    out->tile_bytes = L.tile_bytes;
    return RT_OK;
}

int rt_place_tiles(rt_ctx* c, const void* gathered_device, int32_t world, uint32_t flags, void* frame,
                   void* hip_stream) {
    if (!c) return fail(nullptr, RT_ERR_INVALID_ARG, "ctx is null");
    if (!gathered_device || !frame || world < 1) return fail(c, RT_ERR_INVALID_ARG, "null buffer or world < 1");
    if ((flags & RT_OUT_FP16) && (flags & RT_OUT_RGBA8))
        return fail(c, RT_ERR_INVALID_ARG, "RT_OUT_FP16 and RT_OUT_RGBA8 are exclusive");
    DeviceGuard g(c->device);
    // NULL is the HIP null stream (rt_render_async's convention): a caller on
    // the default stream (torch's current stream is handle 0) gets its work
    // ordered after everything it enqueued there
    hipStream_t s = (hipStream_t)hip_stream;
    return place_tiles_impl(c, gathered_device, (uint32_t)world, flags, frame, s);
}

int rt_place_tiles_host(const void* gathered, int32_t width, int32_t height, int32_t world, uint32_t flags,
                        void* frame) {
    if (!gathered || !frame || !tile_args_ok(width, height, world)) return RT_ERR_INVALID_ARG;
    const uint32_t W = (uint32_t)width, H = (uint32_t)height, N = (uint32_t)world;
    for (uint32_t k = 0; k < N && k < H; ++k) {
        const TileLayout L = tile_layout(W, H, N, k, flags);
        for (uint32_t j = 0; j < L.rows; ++j)
            memcpy(static_cast<char*>(frame) + (size_t)(k + j * N) * L.row_bytes,
                   static_cast<const char*>(gathered) + k * L.tile_bytes + j * L.row_bytes, L.row_bytes);
    }
    return RT_OK;
}

int rt_math_selfcheck(uint64_t* mismatches) {
    if (!mismatches) return fail(nullptr, RT_ERR_INVALID_ARG, "null argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(nullptr, RT_ERR_NO_DEVICE, "no HIP device");
    unsigned long long bad[2] = {0, 0};
    const hipError_t e = rt::math_selfcheck(bad);
    if (e != hipSuccess) return hip_fail(nullptr, RT_ERR_LAUNCH, "math_selfcheck", e);
    mismatches[0] = bad[0];
    mismatches[1] = bad[1];
    return RT_OK;
}

int rt_build_info(const rt_ctx* c, rt_build_stats* info) {
    if (!c || !info) return fail(nullptr, RT_ERR_INVALID_ARG, "null argument");
    memset(info, 0, sizeof(*info));
    info->tri_bvh_build = c->tri_bvh_build_used;
    info->tri_bvh_nodes = c->tri_bvh_nodes;
    info->tri_bvh_build_ms = c->tri_bvh_build_ms;
    info->scene_compile_ms = c->scene_compile_ms;
    info->tri_bvh_temp_kib = (uint32_t)((c->tri_bvh_temp_bytes + 1023) / 1024);
    return RT_OK;
}

int rt_last_launch(const rt_ctx* c, rt_launch_info* info) {
    if (!c || !info) return fail(nullptr, RT_ERR_INVALID_ARG, "null argument");
    if (!c->launched) return RT_ERR_STATE;
    memset(info, 0, sizeof(*info));
    static_assert(sizeof(info->kernel) == sizeof(c->launch.kernel), "kernel name buffer");
    memcpy(info->kernel, c->launch.kernel, sizeof(info->kernel));
    info->kernel[sizeof(info->kernel) - 1] = 0;
    info->lanes_per_pixel = c->launch.lanes;
    info->halton_tables = c->launch.tables;
    info->small_index = c->launch.small;
    info->block_threads = c->launch.threads;
    info->grid_x = c->launch.grid_x;
    info->grid_y = c->launch.grid_y;
    info->lds_bytes = c->launch.lds;
    return RT_OK;
}

#ifndef RT_SRC_SHA
#define RT_SRC_SHA "unknown"
#endif
const char* rt_build_sha(void) { return RT_SRC_SHA; }

int rt_destroy(rt_ctx* c) {
    if (!c) return RT_OK;
    release(c);
    delete c;
    return RT_OK;
}

int rt_scene_describe(const rt_scene_desc* d, rt_scene_info* info) {
    return rt_scene_describe_ex(d, nullptr, info);
}

int rt_scene_describe_ex(const rt_scene_desc* d, const rt_create_options* opt, rt_scene_info* info) {
    if (!d || !info || !d->camera || !d->square_lights)
        return fail(nullptr, RT_ERR_INVALID_ARG, "null argument");
    Resolved ro;
    const char* why = nullptr;
    if (!resolve_options(opt, &ro, &why)) return fail(nullptr, RT_ERR_INVALID_ARG, why);
    rt::CompiledScene s;
    const char* err = nullptr;
    if (!rt::compile_scene(*d->camera, d->materials, d->vertices, d->n_triangles,
                           d->square_lights[0], d->spheres, d->n_spheres, &s, &err, ro.build))
        return fail(nullptr, RT_ERR_INVALID_ARG, err);
    info->n_triangles = (uint32_t)s.tri_isect.size();
    info->n_triangle_pairs = (uint32_t)s.pair_isect.size();
    info->n_box_clusters = (uint32_t)(s.clusters.size() / (4 * rt::kCluF4));
    info->pair_free_mask = s.pair_free_mask;
    info->n_spheres = (uint32_t)s.sph_isect.size();
    info->n_sphere_nodes = s.sph_layout_nodes;
    const size_t lds = rt::kernel_lds_bytes(info->n_triangles, info->n_triangle_pairs, info->n_spheres,
                                            s.sph_layout_nodes);
    const size_t lds_single = rt::kernel_lds_bytes(info->n_triangles, 0, 0, 0);
    const bool bvh = info->n_triangles > 0 &&
                     (ro.mem == rt::SceneMem::kTriBvh ||
                      (ro.mem == rt::SceneMem::kAuto && (info->n_triangles > rt::kTriBvhMinTriangles ||
                                                         std::min(lds, lds_single) > rt::kMaxLdsBytes)));
    info->n_triangle_bvh_nodes = bvh ? 2 * info->n_triangles - 1 : 0u;
    // the launcher takes the sphere kernel only for the pair layout (every
    // triangle paired) and no triangle BVH, with its pair copy within 6 KB
    info->sphere_kernel_lds_bytes = (!s.sph_lds.empty() && info->n_triangle_pairs > 0 && !bvh &&
                                     ro.mem == rt::SceneMem::kAuto && lds <= rt::kSphPairLdsMaxBytes)
                                        ? (uint32_t)lds
                                        : 0u;
    // box clusters are staged after the pairs in triangle-only scenes
    const size_t lds_clu =
        lds + (info->n_spheres ? 0u : rt::kCluF4 * sizeof(float) * 4 * info->n_box_clusters);
    info->lds_bytes = (!bvh && lds <= rt::kMaxLdsBytes)
                          ? (uint32_t)(lds_clu <= rt::kMaxLdsBytes ? lds_clu : lds)
                          : 0u;
    // the launcher's own choice (rt::choose_kernel), for a render of >= 1 bounce
    const rt::KernelChoice kc =
        rt::choose_kernel(info->n_triangles, info->n_triangle_pairs, info->n_spheres, info->n_box_clusters,
                          info->n_triangle_bvh_nodes, !s.sph_lds.empty(), 3, ro.mem, ro.walk);
    info->kernel_layout = (uint32_t)kc.layout;
    info->kernel_lds_bytes = (uint32_t)kc.lds_bytes;
    return RT_OK;
}

int rt_debug_stats(rt_ctx* c, uint64_t* out, int n) {
    if (!c || !out || n <= 0) return fail(c, RT_ERR_INVALID_ARG, "null argument");
    DeviceGuard g(c->device);
    hipError_t e = rt::read_debug_stats(reinterpret_cast<unsigned long long*>(out), n);
    if (e == hipErrorNotSupported) return fail(c, RT_ERR_STATE, "not an RT_STATS build");
    if (e != hipSuccess) return hip_fail(c, RT_ERR_LAUNCH, "read stats", e);
    return RT_OK;
}

void rt_seed_splitmix(uint64_t key, uint32_t* seeds, size_t n) {
    if (!seeds) return;
    for (size_t p = 0; p < n; ++p) seeds[p] = rt::seed_splitmix(key, p);
}

static void fill_scene_arrays(const rt::Scene& s, CameraGPU* camera, MaterialGPU* materials,
                              rt_float3* vertices, SquareLightGPU* light) {
    *camera = rt::convert_camera(s.camera);
    for (size_t k = 0; k < s.triangles.size(); ++k) {
        materials[k] = rt::convert_material(s.triangles[k].material);
        for (int v = 0; v < 3; ++v) vertices[3 * k + v] = rt::to_abi(s.triangles[k].vertices[v]);
    }
    *light = rt::convert_square_light(s.light);
}

int rt_scene_cornell_box(int32_t width, int32_t height, CameraGPU* camera, MaterialGPU* materials,
                         rt_float3* vertices, SquareLightGPU* light, uint32_t* n_triangles) {
    if (!camera || !materials || !vertices || !light || !n_triangles || width <= 0 || height <= 0)
        return RT_ERR_INVALID_ARG;
    const rt::Scene s = rt::init_cornell_box(width, height);
    fill_scene_arrays(s, camera, materials, vertices, light);
    *n_triangles = (uint32_t)s.triangles.size();
    return RT_OK;
}

int rt_render_mis(rt_ctx* ctx, const rt_mis_params* params, float* out_rgba32f, uint8_t* out_rgba8) {
    if (!ctx) return fail(nullptr, RT_ERR_INVALID_ARG, "ctx is null");
    DeviceGuard g(ctx->device);
    return render_mis_impl(ctx, params, out_rgba32f, out_rgba8);
}

int rt_scene_cornell_box_mis(int32_t width, int32_t height, CameraGPU* camera, MaterialGPU* materials,
                             rt_float3* vertices, SquareLightGPU* light, uint32_t* n_triangles) {
    if (!camera || !materials || !vertices || !light || !n_triangles || width <= 0 || height <= 0)
        return RT_ERR_INVALID_ARG;
    const rt::Scene s = rt::init_cornell_box_mis(width, height);
    fill_scene_arrays(s, camera, materials, vertices, light);
    *n_triangles = (uint32_t)s.triangles.size();
    return RT_OK;
}

int rt_scene_random_spheres(int32_t width, int32_t height, uint32_t n_spheres, uint64_t seed,
                            CameraGPU* camera, MaterialGPU* materials, rt_float3* vertices,
                            SquareLightGPU* light, uint32_t* n_triangles, SphereGPU* spheres) {
    if (!camera || !materials || !vertices || !light || !n_triangles || width <= 0 ||
        height <= 0 || (n_spheres && !spheres))
        return RT_ERR_INVALID_ARG;
    const rt::Scene s = rt::init_random_spheres(width, height, n_spheres, seed);
    fill_scene_arrays(s, camera, materials, vertices, light);
    *n_triangles = (uint32_t)s.triangles.size();
    for (uint32_t k = 0; k < n_spheres; ++k) spheres[k] = rt::convert_sphere(s.spheres[k]);
    return RT_OK;
}

}  // extern "C"

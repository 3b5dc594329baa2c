// rt_kernel.hpp — launch interface of the gfx950 path-tracing kernel.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "rt_math.h"

namespace rt {

constexpr uint32_t kBlockThreads = 256;  // 4 waves; each wave = 8x8 pixel tile
constexpr uint32_t kTile = 16;           // workgroup = 16x16 pixels
constexpr size_t kMaxLdsBytes = 64 * 1024;
constexpr uint32_t kOutFp16 = 0x2u;
constexpr uint32_t kOutRgba8 = 0x10u;  // fused image.swift:35-65 epilogue, uchar4 store
constexpr uint32_t kPairF4 = 7;  // float4 per pair record: 5 geometry + 2 padded AABB
// The sphere kernel (kGeoSphLds): one-wave workgroups that stage only the
// pair records in LDS and walk the compact sphere BVH (8 octant layouts) from
// global memory (L2-resident).  A workgroup keeps its wave slots until its
// slowest wave ends and sphere walks make wave times differ a lot (config 4:
// 1024 threads 186.1 ms, 512 177.9, 256 162.1, 128 160.5, 64 158.4).  Every
// workgroup stages its own copy of the pair records, so the kernel is taken
// only while they are small (kSphPairLdsMaxBytes; config 4: 672 B): above it
// the pair kernel with the 32-B-node sphere walks serves the scene.  Measured
// on Cornell + 1000 spheres + extra quads, 1080p x 64 spp (tools/bench_mixed.py,
// one-wave vs pair kernel): 37 pairs 47.9 vs 66.7 ms, 48 pairs 59.5 vs 69.4,
// 58 pairs 71.8 vs 71.7, 68 pairs 84.8 vs 73.0: the crossover is ~6.5 KB.
constexpr uint32_t kSphBlockThreads = 64;
constexpr size_t kSphPairLdsMaxBytes = 6 * 1024;
constexpr uint32_t kCluF4 = 7;   // float4 per box cluster (rt_scene.hpp CompiledScene::clusters)
// The path-trace kernel's cluster test reads the face masks of world axes from
// a per-octant table, pre-swapped on the host (rt_trace.hpp cluster_candidates)
#ifndef RT_CLU_OCT
#define RT_CLU_OCT 0
#endif
constexpr uint32_t kCluOctF4 = RT_CLU_OCT ? 16u : 0u;  // float4 per box cluster of the octant mask table (CompiledScene::clu_oct)
// Layouts of the triangle BVH (rt_scene.cpp build_tri_sah / rt_lbvh.hip,
// rt_trace.hpp tri_cbvh_*): one per direction octant, 16 B per node.
constexpr uint32_t kTriCompactLayouts = 8;
// Above this many triangles rt_create builds the triangle BVH (measured crossover
// of the LDS brute-force layouts and the BVH walks on random triangles: ~300).
constexpr uint32_t kTriBvhMinTriangles = 384;

// Kernel arguments (passed by value -> kernarg segment / SGPRs).
struct KParams {
    const float4* tri_isect;  // 3 float4 per triangle (TriIsect)
    const float4* pair_isect; // kPairF4 float4 per shared-edge triangle pair (PairIsect) or null
    const float4* tri_shade;  // 4 float4 per triangle (TriShade)
    const float4* sph_isect;  // 1 float4 per sphere, BVH leaf order (SphIsect)
    const float4* sph_nodes;  // 2 float4 per sphere-BVH node (BvhNode)
    const uint32_t* sph_perm; // BVH leaf order -> sphere id
    const float4* sph_shade;  // 3 float4 per sphere, by id (SphShade)
    const uint32_t* sph_lds;  // compact sphere BVH (8 layouts x nE x 16 B), or null
    const uint16_t* sph_lds_id;  // sphere id per compact entry
    const uint4* sph_box;     // the same BVH with leaf boxes: 8 layouts x nN entries, or null
    const uint4* tri_nodes;   // triangle BVH: 8 compact layouts x nTN nodes, or null
    const float4* tri_sorted; // 3 float4 per triangle, BVH leaf order
    const uint32_t* tri_perm; // BVH leaf order -> triangle id
    const uint32_t* seeds;    // W*H, full frame
    float4* sum;              // running sums (tile layout) or null
    void* out;                // rgba32F / rgba16F tile or null
    uint32_t nT, nP, nS, nN;  // triangles, triangle pairs (0: no pair layout), spheres, BVH nodes
    uint32_t nE;              // entries per layout of the compact sphere BVH
    uint32_t nTN;             // triangle-BVH nodes per layout (0: no triangle BVH)
    float cam_pos[3], cam_u[3], cam_v[3], cam_w[3];
    float halfW, halfH;
    int32_t W, H;
    float light_center[3], light_color[3];
    uint32_t spp, sample_base;
    uint32_t row_start, row_step, row_count;
    uint32_t accumulate;      // read P.sum before adding
    uint32_t samples_total;   // S of `luminance /= samples`
    uint32_t flags;
    uint32_t max_index;       // max Halton index seed+n of this launch (0xFFFFFFFF: unknown/wraps)
    uint32_t lanes;           // lanes per pixel: 0 = auto, else 1, 4 or 16 (rt_create_options)
    uint32_t walk;            // rt_walk_scheduler: 0 auto, 1 lockstep, 2 free-running lanes, 3 sorted
    uint32_t wave_w;          // pixels per wave row (set by the launcher)
    uint32_t walk_leaf_den;   // free-running walks: leaf-round threshold, 0 = default
    uint32_t light_plain;     // light_center.y, .z are not -0 (shade(): q without its zero terms)
    const float4* clusters;   // box clusters, kCluF4 float4 each, or null
    const float4* clu_oct;    // per cluster and octant: pre-swapped face masks, kCluOctF4 float4 per cluster
    uint32_t nC;              // clusters (0: none)
    uint32_t pair_free;       // pairs in no cluster (bit mask)
};

size_t kernel_lds_bytes(uint32_t n_tri, uint32_t n_pairs, uint32_t n_sph, uint32_t n_nodes);

// Kernel layouts the launcher chooses between (0-7 = rt_trace.hpp enum Geo).
enum KernelLayout : int {
    kLayTriLds = 0,      // single-triangle records in LDS
    kLayPairLds = 1,     // shared-edge pair records in LDS
    kLayTriGlobal = 2,   // single-triangle records from global memory
    kLayPairSorted = 3,  // pair records + per-bounce octant sort of the paths
    kLayPairSmem = 4,    // pair records by scalar loads
    kLayTriBvh = 5,      // triangle BVH from global memory
    kLayPairClu = 6,     // pair records + box clusters + Halton tables in LDS (Cornell)
    kLaySphLds = 7,      // pair records in LDS, compact sphere BVH in L2 (config 4)
    kLayFreeSph = 8,     // free-running lanes, sphere scene (rt_free.hpp)
    kLayFreeTri = 9,     // free-running lanes, triangle BVH
    kLaySortSph = 10,    // octant-sorted paths, sphere scene
    kLaySortTri = 11,    // octant-sorted paths, triangle BVH
};
// LDS of the Halton low-digit tables (rt_halton.hpp kHaltonTabFloats) and of
// the sorted kernel's path buffers (rt_kernel.hip kSortF4), static-asserted
// against their definitions.
constexpr uint32_t kHaltonTabLdsFloats = 4679;
constexpr uint32_t kSortLdsF4 = 1097;
// THE dynamic LDS of a workgroup of layout `lay`: the bytes its staging loops
// write (pair / triangle records, then box clusters and their octant mask
// table, then the Halton tables;
// the sorted kernels' path buffers first).  The launcher requests exactly this
// and the kernels place their staged arrays by the same terms; an
// -DRT_LDS_CHECK build also checks it against the dispatch's LDS allocation.
__host__ __device__ constexpr size_t staged_lds_bytes(int lay, uint32_t nT, uint32_t nP, uint32_t nC) {
    return lay == kLayTriLds ? (size_t)48 * nT
           : (lay == kLayPairLds || lay == kLaySphLds || lay == kLayFreeSph) ? (size_t)16 * kPairF4 * nP
           : lay == kLayPairClu ? (size_t)16 * (kPairF4 * nP + (kCluF4 + kCluOctF4) * nC) +
                                      (size_t)4 * kHaltonTabLdsFloats
           : (lay == kLayPairSorted || lay == kLaySortSph) ? (size_t)16 * (kSortLdsF4 + kPairF4 * nP)
           : lay == kLaySortTri ? (size_t)16 * kSortLdsF4
           : (size_t)0;  // TriGlobal, PairSmem, TriBvh, FreeTri: the scene stays in global memory
}
// The kernel layout a launch takes and its dynamic LDS (launch_path_trace and
// rt_scene_describe_ex both ask this one function).  nC: box clusters, nTN:
// triangle-BVH nodes per layout, sph_compact: the compact sphere BVH exists.
struct KernelChoice {
    int layout;
    size_t lds_bytes;
};
// What launch_path_trace launched (rt_last_launch, include/rtpt.h).
struct LaunchInfo {
    char kernel[96];
    uint32_t lanes, tables, small, threads, grid_x, grid_y, lds;
};
// Where the workgroup reads the intersection records from.
// rt_walk_scheduler (include/rtpt.h)
constexpr uint32_t kWalkAuto = 0, kWalkLockstep = 1, kWalkFree = 2, kWalkSorted = 3;
enum class SceneMem { kAuto = 0, kLdsSingle = 1, kSmem = 2, kPairSorted = 3, kPairSmem = 4, kTriBvh = 5, kPairLds = 6 };
hipError_t launch_path_trace(const KParams& P, uint32_t bounces, SceneMem mem, hipStream_t stream,
                             LaunchInfo* info);
KernelChoice choose_kernel(uint32_t nT, uint32_t nP, uint32_t nS, uint32_t nC, uint32_t nTN, bool sph_compact,
                           uint32_t bounces, SceneMem mem, uint32_t walk);
hipError_t read_debug_stats(unsigned long long* out, int n);  // RT_STATS builds only
// -DRT_LDS_CHECK builds: the largest staging end a kernel found past its
// dispatch's dynamic LDS since the last call (0: none; always 0 otherwise).
hipError_t lds_check_result(uint32_t* end);
// Arguments of the MIS integrator kernel (rt_mis.hip; Sources/gpuRaytracer/
// shaders.metal:635-707).
struct MisParams {
    const float4* tri_isect;   // 3 float4 per triangle
    const uint4* tri_nodes;    // triangle BVH or null (as KParams)
    const float4* tri_sorted;
    const uint32_t* tri_perm;
    uint32_t nTN;
    const float4* pair_isect;  // kPairF4 float4 per pair, or null
    const float4* clusters;    // box clusters (as KParams), or null
    uint32_t nC, pair_free;
    const float4* mis_shade;   // 3 float4 per triangle (MisShade)
    const float4* u_tab;       // 3 float4 per MIS sample index i < S (Halton table)
    float4* out;               // (sum over camera rays, camera_rays) per pixel, or null
    uchar4* out8;              // writeToPixelBuffer RGBA8, or null
    uint32_t nT, nP;
    float cam_pos[3], cam_u[3], cam_v[3], cam_w[3];
    float halfW, halfH;
    int32_t W, H;
    float l_center[3], l_tangent[3], l_bitangent[3], l_radiance[3];
    float l_width, l_depth, l_area, exposure;
    uint32_t camera_rays, S;   // S = misSamples / 3 (samples per strategy)
    uint32_t row_start, row_step, row_count;
    float4* part;              // split launches: one float4 per record and pixel, or null (rt_mis.hip SPLIT)
};
hipError_t launch_mis(const MisParams& P, SceneMem mem, hipStream_t stream);
size_t mis_lds_bytes(uint32_t n_tri, uint32_t n_pairs);
size_t mis_part_bytes(uint32_t camera_rays, size_t pixels);  // 0: no split launch

// GPU build of the triangle BVH (rt_lbvh.hip).  d_nodes: 8 * (2n-1) uint4,
// d_sorted: 3n float4, d_perm: n.  Synchronises the stream.
hipError_t build_tri_lbvh(const float4* d_tri, uint32_t n, const float lo[3], const float hi[3],
                          float margin, uint4* d_nodes, float4* d_sorted, uint32_t* d_perm,
                          hipStream_t s);

// GPU binned-SAH build of the triangle BVH (rt_gsah.hip): the host build's
// rules (32 bins, SAH leaf rule) level by level on the device, written in the
// same compact layout.  d_nodes: 8 * (2n-1) uint4 at most, d_sorted: 3n
// float4, d_perm: n; *total_nodes = nodes per layout, *temp_bytes = the peak
// of the build's temporary device memory.  Synchronises the stream.
hipError_t build_tri_gsah(const float4* d_tri, uint32_t n, float margin, uint32_t leaf_max, double trav_cost,
                          uint4* d_nodes, float4* d_sorted, uint32_t* d_perm, uint32_t* total_nodes,
                          size_t* temp_bytes, hipStream_t s);
// Deterministic exclusive scan of n uint32 (rt_gsah.hip); tile_sums holds
// ceil(n / 1024) words.
hipError_t scan_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tile_sums, hipStream_t s);

hipError_t launch_fill_seeds(uint32_t* seeds, uint64_t key, uint64_t n, hipStream_t stream);
// The shipped short sqrt / reciprocal (rt_math.h sqrt_cr, rcp_cr) against IEEE
// sqrtf and 1/x over every float on the current device: mismatch counts.
hipError_t math_selfcheck(unsigned long long bad[2]);

// Rank 0's placement after the gather (rt_place_tiles): frame row y comes from
// tile y mod N, tile row y / N; `gathered` holds N tiles of tile_bytes back to
// back.  One kernel on `stream` (device -> device), row_bytes and tile_bytes
// multiples of 4.
hipError_t launch_place_tiles(const void* gathered, void* frame, size_t row_bytes, size_t tile_bytes,
                              uint32_t H, uint32_t N, hipStream_t stream);

}  // namespace rt

// rt_lbvh.hip — GPU build of the triangle BVH (replaces
// setupAccelerationStructures, RTrace/computeShader.swift:45-97, i.e. the
// MTLAccelerationStructure build).
//
// Linear BVH (Karras 2012): 30-bit Morton codes of the triangle centroids,
// device radix sort (hipCUB, stable: equal codes stay in id order, so the build
// is deterministic), one thread per inner node finds its key range and split,
// leaves are refitted bottom-up with acquire/release counters, and the tree is
// written in the compact stackless layout the triangle walks read (16-B
// entries, rt_trace.hpp tri_cbvh_*): 8 depth-first layouts, one per
// ray-direction octant, near child first along the node's split axis, every
// box padded by the culling margin.  One triangle per leaf.  The default
// build is the host binned-SAH one (rt_scene.cpp build_tri_sah, same layout);
// this GPU build is taken with RTPT_TRI_BUILD=lbvh.  Only speed depends on the tree: the
// walks in rt_trace.hpp return the brute-force (t, id) minimum.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <stdint.h>

#include "rt_kernel.hpp"

namespace rt {

namespace {

__device__ __forceinline__ uint32_t spread10(uint32_t v) {  // 10 bits -> every 3rd bit
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x030000FFu;
    v = (v | (v << 8)) & 0x0300F00Fu;
    v = (v | (v << 4)) & 0x030C30C3u;
    v = (v | (v << 2)) & 0x09249249u;
    return v;
}

// Triangle boxes (from the intersection record, as the test sees the triangle)
// and Morton codes: bit 3i+2 = x_i, 3i+1 = y_i, 3i = z_i.
__global__ void morton_kernel(const float4* __restrict__ tri, uint32_t n, float3 lo, float3 inv_ext,
                              uint32_t* __restrict__ keys, uint32_t* __restrict__ ids) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float4 A = tri[3 * k], Bq = tri[3 * k + 1], C = tri[3 * k + 2];
    const float v0x = A.x, v0y = A.y, v0z = A.z;
    const float cx = v0x + (A.w + Bq.z) * (1.0f / 3.0f);
    const float cy = v0y + (Bq.x + Bq.w) * (1.0f / 3.0f);
    const float cz = v0z + (Bq.y + C.x) * (1.0f / 3.0f);
    auto q = [](float c, float l, float s) {
        const float u = fminf(fmaxf((c - l) * s, 0.0f), 0.9999999f);
        return (uint32_t)(u * 1024.0f);
    };
    keys[k] = (spread10(q(cx, lo.x, inv_ext.x)) << 2) | (spread10(q(cy, lo.y, inv_ext.y)) << 1) |
              spread10(q(cz, lo.z, inv_ext.z));
    ids[k] = k;
}

__device__ __forceinline__ int delta(const uint32_t* keys, uint32_t n, int i, int j) {
    if (j < 0 || j >= (int)n) return -1;
    const uint32_t a = keys[i], b = keys[j];
    if (a == b) return 32 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clz(a ^ b);
}

// Node numbering: inner nodes 0..n-2 (root 0), leaves n-1 .. 2n-2.
__global__ void karras_kernel(const uint32_t* __restrict__ keys, uint32_t n,
                              uint32_t* __restrict__ child, uint32_t* __restrict__ parent,
                              uint32_t* __restrict__ range, uint8_t* __restrict__ axis) {
    const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    if (i >= (int)n - 1) return;
    const int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    const int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    const int j = i + l * d;
    const int dnode = delta(keys, n, i, j);
    int s = 0;
    for (int div = 2;; div *= 2) {
        const int t = (l + div - 1) / div;
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
        if (t <= 1) break;
    }
    const int g = i + s * d + (d < 0 ? -1 : 0);
    const int f = min(i, j), e = max(i, j);
    const uint32_t left = (f == g) ? (n - 1 + g) : (uint32_t)g;
    const uint32_t right = (e == g + 1) ? (n - 1 + g + 1) : (uint32_t)(g + 1);
    child[2 * i] = left;
    child[2 * i + 1] = right;
    parent[left] = (uint32_t)i;
    parent[right] = (uint32_t)i;
    range[2 * i] = (uint32_t)f;
    range[2 * i + 1] = (uint32_t)e;
    // split axis = axis of the highest differing Morton bit of the range
    const uint32_t x = keys[f] ^ keys[e];
    axis[i] = x ? (uint8_t)(2 - (31 - __clz(x)) % 3) : (uint8_t)0;  // bit 3i+2 -> x (0)
}

// Bottom-up boxes: the second child to arrive at a node builds its box.
__global__ void refit_kernel(const float4* __restrict__ tri, const uint32_t* __restrict__ ids,
                             uint32_t n, const uint32_t* __restrict__ child,
                             const uint32_t* __restrict__ parent, uint32_t* __restrict__ flags,
                             float4* __restrict__ box, float margin) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t t = ids[k];
    const float4 A = tri[3 * t], Bq = tri[3 * t + 1], C = tri[3 * t + 2];
    const float x1 = A.x + A.w, y1 = A.y + Bq.x, z1 = A.z + Bq.y;   // v0 + e1
    const float x2 = A.x + Bq.z, y2 = A.y + Bq.w, z2 = A.z + C.x;   // v0 + e2
    uint32_t node = n - 1 + k;
    box[2 * node] = make_float4(fminf(A.x, fminf(x1, x2)) - margin, fminf(A.y, fminf(y1, y2)) - margin,
                                fminf(A.z, fminf(z1, z2)) - margin, 0.0f);
    box[2 * node + 1] = make_float4(fmaxf(A.x, fmaxf(x1, x2)) + margin, fmaxf(A.y, fmaxf(y1, y2)) + margin,
                                    fmaxf(A.z, fmaxf(z1, z2)) + margin, 0.0f);
    if (n == 1) return;
    while (node != 0) {
        node = parent[node];
        __threadfence();
        const uint32_t prev = __hip_atomic_fetch_add(&flags[node], 1u, __ATOMIC_ACQ_REL,
                                                     __HIP_MEMORY_SCOPE_AGENT);
        if (prev == 0) return;  // the sibling subtree is not done yet
        const uint32_t l = child[2 * node], r = child[2 * node + 1];
        const float4 l0 = box[2 * l];
        const float4 l1 = box[2 * l + 1];
        const float4 r0 = box[2 * r];
        const float4 r1 = box[2 * r + 1];
        box[2 * node] = make_float4(fminf(l0.x, r0.x), fminf(l0.y, r0.y), fminf(l0.z, r0.z), 0.0f);
        box[2 * node + 1] = make_float4(fmaxf(l1.x, r1.x), fmaxf(l1.y, r1.y), fmaxf(l1.z, r1.z), 0.0f);
    }
}

__device__ __forceinline__ uint32_t subtree_nodes(const uint32_t* range, uint32_t n, uint32_t v) {
    if (v >= n - 1) return 1u;
    return 2u * (range[2 * v + 1] - range[2 * v] + 1u) - 1u;
}

// Depth-first (preorder) position of node v in the layout of octant `oct`,
// found by walking to the root; then the node is written there.
__global__ void layout_kernel(uint32_t n, const uint32_t* __restrict__ child,
                              const uint32_t* __restrict__ parent,
                              const uint32_t* __restrict__ range, const uint8_t* __restrict__ axis,
                              const float4* __restrict__ box, uint4* __restrict__ nodes) {
    const uint32_t total = 2 * n - 1;
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t oct = blockIdx.y;
    if (v >= total) return;
    uint32_t idx = 0, c = v;
    while (c != 0) {
        const uint32_t p = parent[c];
        const bool neg = (oct >> axis[p]) & 1u;
        const uint32_t first = neg ? child[2 * p + 1] : child[2 * p];
        idx += (c == first) ? 1u : 1u + subtree_nodes(range, n, first);
        c = p;
    }
    const uint32_t escape = idx + subtree_nodes(range, n, v);
    const float4 b0 = box[2 * v], b1 = box[2 * v + 1];
    // compact 16-B entries (rt_trace.hpp tri_cbvh_*): the box in fp16 rounded
    // outward (a superset of the padded box), then escape | 2^31 for an inner
    // node (an entry index over all 8 layouts) or the leaf's triangle index in
    // leaf order (a leaf's escape is the next entry)
    uint4* cn = nodes + (size_t)oct * total + idx;
    uint32_t h[6] = {__half_as_ushort(__float2half_rd(b0.x)), __half_as_ushort(__float2half_rd(b0.y)),
                     __half_as_ushort(__float2half_rd(b0.z)), __half_as_ushort(__float2half_ru(b1.x)),
                     __half_as_ushort(__float2half_ru(b1.y)), __half_as_ushort(__float2half_ru(b1.z))};
    // near/far: the plane a ray of octant `oct` enters through takes the lo slot
#pragma unroll
    for (int a = 0; a < 3; ++a)
        if ((oct >> a) & 1u) {
            const uint32_t x = h[a];
            h[a] = h[3 + a];
            h[3 + a] = x;
        }
    const uint32_t w = (v >= n - 1) ? (v - (n - 1)) : ((oct * total + escape) | 0x80000000u);
    *cn = make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), w);
}

__global__ void gather_kernel(const float4* __restrict__ tri, const uint32_t* __restrict__ ids,
                              uint32_t n, float4* __restrict__ sorted) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t t = ids[k];
    sorted[3 * k] = tri[3 * t];
    sorted[3 * k + 1] = tri[3 * t + 1];
    sorted[3 * k + 2] = tri[3 * t + 2];
}

template <typename T>
hipError_t dalloc(T** p, size_t count) {
    return hipMalloc((void**)p, count * sizeof(T) + 16);
}

}  // namespace

hipError_t build_tri_lbvh(const float4* d_tri, uint32_t n, const float lo[3], const float hi[3],
                          float margin, uint4* d_nodes, float4* d_sorted, uint32_t* d_perm,
                          hipStream_t s) {
    if (n == 0) return hipSuccess;
    if (n >= (1u << 24)) return hipErrorInvalidValue;  // leaf index field is 24 bits
    uint32_t *keys = nullptr, *ids = nullptr, *keys2 = nullptr, *child = nullptr,
             *parent = nullptr, *range = nullptr, *flags = nullptr;
    uint8_t* axis = nullptr;
    float4* box = nullptr;
    void* tmp = nullptr;
    size_t tmp_bytes = 0;
    const uint32_t total = 2 * n - 1;
    hipError_t e = hipSuccess;
    do {
        if ((e = dalloc(&keys, n)) || (e = dalloc(&keys2, n)) || (e = dalloc(&ids, n)) ||
            (e = dalloc(&child, 2 * n)) || (e = dalloc(&parent, total)) ||
            (e = dalloc(&range, 2 * n)) || (e = dalloc(&flags, n)) || (e = dalloc(&axis, n)) ||
            (e = dalloc(&box, 2 * (size_t)total)))
            break;
        const float3 l = make_float3(lo[0], lo[1], lo[2]);
        const float ex = hi[0] - lo[0], ey = hi[1] - lo[1], ez = hi[2] - lo[2];
        const float3 inv = make_float3(ex > 0 ? 1.0f / ex : 0.0f, ey > 0 ? 1.0f / ey : 0.0f,
                                       ez > 0 ? 1.0f / ez : 0.0f);
        const uint32_t T = 256, G = (n + T - 1) / T;
        hipLaunchKernelGGL(morton_kernel, dim3(G), dim3(T), 0, s, d_tri, n, l, inv, keys2, ids);
        if ((e = hipGetLastError())) break;
        // stable LSD radix sort of (code, id); ids start in ascending order
        if ((e = hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys2, keys, ids, d_perm,
                                                    (int)n, 0, 30, s)))
            break;
        if ((e = hipMalloc(&tmp, tmp_bytes + 16))) break;
        if ((e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys2, keys, ids, d_perm,
                                                    (int)n, 0, 30, s)))
            break;
        if ((e = hipMemsetAsync(flags, 0, n * sizeof(uint32_t), s))) break;
        if ((e = hipMemsetAsync(parent, 0, total * sizeof(uint32_t), s))) break;
        if (n > 1) {
            hipLaunchKernelGGL(karras_kernel, dim3((n - 1 + T - 1) / T), dim3(T), 0, s, keys, n,
                               child, parent, range, axis);
            if ((e = hipGetLastError())) break;
        }
        hipLaunchKernelGGL(refit_kernel, dim3(G), dim3(T), 0, s, d_tri, d_perm, n, child, parent,
                           flags, box, margin);
        if ((e = hipGetLastError())) break;
        hipLaunchKernelGGL(layout_kernel, dim3((total + T - 1) / T, 8), dim3(T), 0, s, n, child,
                           parent, range, axis, box, d_nodes);
        if ((e = hipGetLastError())) break;
        hipLaunchKernelGGL(gather_kernel, dim3(G), dim3(T), 0, s, d_tri, d_perm, n, d_sorted);
        if ((e = hipGetLastError())) break;
        e = hipStreamSynchronize(s);
    } while (0);
    (void)hipFree(keys);
    (void)hipFree(keys2);
    (void)hipFree(ids);
    (void)hipFree(child);
    (void)hipFree(parent);
    (void)hipFree(range);
    (void)hipFree(flags);
    (void)hipFree(axis);
    (void)hipFree(box);
    (void)hipFree(tmp);
    return e;
}

}  // namespace rt

// rt_gsah.hip — GPU binned-SAH build of the triangle BVH (SURVEY §8f row 3:
// replaces setupAccelerationStructures, RTrace/computeShader.swift:45-97, the
// MTLAccelerationStructure build on the device).
//
// The same tree rules as the host build (rt_scene.cpp build_tri_sah): 32
// centroid bins per axis, cost area(left) * n_left + area(right) * n_right in
// double precision, the SAH leaf rule for leaves of up to leaf_max triangles,
// a split by index when every centroid coincides -- but built top-down on the
// GPU, one tree level per round:
//   1. bin_kernel     every triangle of a node being split adds itself to its
//                     node's 3 x 32 bins (count, box) with integer atomics
//                     (floats mapped to order-preserving uint32: min/max are
//                     exact and order-free, so the build is deterministic);
//   2. split_kernel   one thread per node evaluates the 93 split candidates
//                     and the leaf rule;
//   3. child numbering and a STABLE partition from exclusive scans (the order
//      of a node's triangles is kept), then the children's exact boxes and
//      centroid boxes from atomic min/max.
// The tree is then emitted in the compact stackless layout the walks read
// (16-B entries, 8 octant layouts, near child first, escape indices over all
// layouts; rt_trace.hpp tri_cbvh_*): subtree sizes bottom-up, preorder
// positions top-down, one thread per node and octant.  Only speed depends
// on the tree (the walks return the brute-force (t, id) answer).
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "rt_kernel.hpp"

namespace rt {

namespace {

constexpr int kBins = 32;
constexpr uint32_t kNoSlot = 0xFFFFFFFFu;

__host__ __device__ __forceinline__ uint32_t fenc(float f) {  // order-preserving float -> uint32
    const uint32_t b = __builtin_bit_cast(uint32_t, f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__host__ __device__ __forceinline__ float fdec(uint32_t u) {
    return __builtin_bit_cast(float, (u & 0x80000000u) ? (u & 0x7FFFFFFFu) : ~u);
}

struct GNode {
    uint32_t lo[3], hi[3];    // encoded box of the node's triangles (unpadded)
    uint32_t clo[3], chi[3];  // encoded centroid box
    uint32_t begin, count;
    int32_t axis;             // split axis (-1: leaf)
    uint32_t left, right;
    uint32_t split;           // first bin of the right child (bin split) or 0xFFFFFFFF (index split)
    uint32_t slot;            // bin slot while being split, else kNoSlot
    uint32_t leaf;            // 1: leaf
};

// Triangle boxes and centroids, as the host build forms them (v0, v0 + e1,
// v0 + e2 from the intersection record; centroid = 0.5 * (lo + hi)).
__global__ void tri_box_kernel(const float4* __restrict__ tri, uint32_t n, float* __restrict__ bl,
                               float* __restrict__ bh, float* __restrict__ cen, uint32_t* __restrict__ ids,
                               uint32_t* __restrict__ seg, GNode* __restrict__ root) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const float4 A = tri[3 * k], Bq = tri[3 * k + 1], C = tri[3 * k + 2];
    const float q[9] = {A.x, A.y, A.z, A.w, Bq.x, Bq.y, Bq.z, Bq.w, C.x};  // v0, e1, e2
    for (int a = 0; a < 3; ++a) {
        const float v0 = q[a], v1 = q[a] + q[3 + a], v2 = q[a] + q[6 + a];
        const float lo = fminf(v0, fminf(v1, v2)), hi = fmaxf(v0, fmaxf(v1, v2));
        const float c = 0.5f * (lo + hi);
        bl[3 * k + a] = lo;
        bh[3 * k + a] = hi;
        cen[3 * k + a] = c;
        atomicMin(&root->lo[a], fenc(lo));
        atomicMax(&root->hi[a], fenc(hi));
        atomicMin(&root->clo[a], fenc(c));
        atomicMax(&root->chi[a], fenc(c));
    }
    ids[k] = k;
    seg[k] = 0;
}

// bins of one slot: count[3][kBins], lo[3][kBins][3], hi[3][kBins][3]
constexpr uint32_t kSlotWords = 3 * kBins * 7;
// Bin slots at a time (2,688 B each: 176 MB): a level with more nodes that
// can split runs its binning and split passes in batches of this many.
constexpr uint32_t kMaxBinSlots = 65536;

// The same binning with the bins of a chunk of kBinChunk consecutive positions
// privatised in LDS when the whole chunk belongs to one node (every chunk of
// the top levels): the global atomics per bin drop from one per triangle to
// one per chunk.  min / max / add are order-free: the same bins.
constexpr uint32_t kBinThreads = 256, kBinChunk = 2048;

__device__ __forceinline__ void bin_one(const GNode& N, uint32_t t, const float* __restrict__ bl,
                                        const float* __restrict__ bh, const float* __restrict__ cen,
                                        uint32_t* B) {
    for (int a = 0; a < 3; ++a) {
        const float clo = fdec(N.clo[a]), ext = fdec(N.chi[a]) - clo;
        if (!(ext > 0.0f)) continue;
        const float scale = (float)kBins / ext;
        const int bi = min(kBins - 1, (int)((cen[3 * t + a] - clo) * scale));
        atomicAdd(&B[a * kBins + bi], 1u);
        uint32_t* lo = B + 3 * kBins + (a * kBins + bi) * 3;
        uint32_t* hi = B + 12 * kBins + (a * kBins + bi) * 3;
        for (int q = 0; q < 3; ++q) {
            atomicMin(&lo[q], fenc(bl[3 * t + q]));
            atomicMax(&hi[q], fenc(bh[3 * t + q]));
        }
    }
}

__global__ __launch_bounds__(kBinThreads) void bin_chunk_kernel(uint32_t n, const uint32_t* __restrict__ ids,
                                                                const uint32_t* __restrict__ seg,
                                                                const GNode* __restrict__ nodes,
                                                                const float* __restrict__ bl,
                                                                const float* __restrict__ bh,
                                                                const float* __restrict__ cen,
                                                                uint32_t* __restrict__ bins) {
    __shared__ uint32_t lb[kSlotWords];
    const uint32_t base = blockIdx.x * kBinChunk;
    const uint32_t end = min(base + kBinChunk, n);
    const uint32_t v0 = seg[base];
    if (v0 == seg[end - 1]) {  // one node (positions are grouped by node)
        const GNode& N = nodes[v0];
        if (N.slot == kNoSlot) return;
        for (uint32_t w = threadIdx.x; w < kSlotWords; w += kBinThreads)
            lb[w] = (w >= 3 * kBins && w < 12 * kBins) ? 0xFFFFFFFFu : 0u;
        __syncthreads();
        for (uint32_t k = base + threadIdx.x; k < end; k += kBinThreads) bin_one(N, ids[k], bl, bh, cen, lb);
        __syncthreads();
        uint32_t* B = bins + (size_t)N.slot * kSlotWords;
        for (uint32_t w = threadIdx.x; w < kSlotWords; w += kBinThreads) {
            const uint32_t v = lb[w];
            if (w < 3 * kBins) {
                if (v) atomicAdd(&B[w], v);
            } else if (w < 12 * kBins) {
                if (v != 0xFFFFFFFFu) atomicMin(&B[w], v);
            } else if (v) {
                atomicMax(&B[w], v);
            }
        }
        return;
    }
    for (uint32_t k = base + threadIdx.x; k < end; k += kBinThreads) {
        const GNode& N = nodes[seg[k]];
        if (N.slot == kNoSlot) continue;
        bin_one(N, ids[k], bl, bh, cen, bins + (size_t)N.slot * kSlotWords);
    }
}

__global__ void clear_bins_kernel(uint32_t* __restrict__ b, uint32_t m) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m * kSlotWords) return;
    const uint32_t w = i % kSlotWords;
    b[i] = (w >= 3 * kBins && w < 12 * kBins) ? 0xFFFFFFFFu : 0u;
}

__device__ __forceinline__ double area(const float* lo, const float* hi) {
    const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
    return x * y + y * z + z * x;
}

// One thread per node of the level: the binned SAH of build_tri_sah for the
// nodes holding a bin slot of this batch; nodes of one triangle (which
// cannot split and hold no slot) become leaves in the first batch.
// split_flag[s] = 1 when the node splits (else it becomes a leaf).
__global__ void split_kernel(uint32_t m, const uint32_t* __restrict__ active, GNode* __restrict__ nodes,
                             const uint32_t* __restrict__ bins, uint32_t leaf_max, double trav_cost,
                             float margin, uint32_t* __restrict__ split_flag, uint32_t first_batch) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= m) return;
    GNode& N = nodes[active[s]];
    if (N.count <= 1) {
        if (first_batch) {
            N.leaf = 1;
            N.axis = -1;
            split_flag[s] = 0;
        }
        return;
    }
    if (N.slot == kNoSlot) return;  // another batch's node
    const uint32_t* B = bins + (size_t)N.slot * kSlotWords;
    double best = INFINITY;
    int best_axis = -1, best_bin = 0;
    for (int a = 0; a < 3; ++a) {
        const float ext = fdec(N.chi[a]) - fdec(N.clo[a]);
        if (!(ext > 0.0f)) continue;
        double right_area[kBins];
        uint32_t right_cnt[kBins];
        float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t rc = 0;
        for (int i = kBins - 1; i >= 1; --i) {  // right part = bins [i, kBins)
            const uint32_t c = B[a * kBins + i];
            rc += c;
            if (c)
                for (int q = 0; q < 3; ++q) {
                    rlo[q] = fminf(rlo[q], fdec(B[3 * kBins + (a * kBins + i) * 3 + q]));
                    rhi[q] = fmaxf(rhi[q], fdec(B[12 * kBins + (a * kBins + i) * 3 + q]));
                }
            right_area[i] = rc ? area(rlo, rhi) : 0.0;
            right_cnt[i] = rc;
        }
        float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
        uint32_t lc = 0;
        for (int i = 1; i < kBins; ++i) {  // left part = bins [0, i)
            const uint32_t c = B[a * kBins + i - 1];
            lc += c;
            if (c)
                for (int q = 0; q < 3; ++q) {
                    llo[q] = fminf(llo[q], fdec(B[3 * kBins + (a * kBins + i - 1) * 3 + q]));
                    lhi[q] = fmaxf(lhi[q], fdec(B[12 * kBins + (a * kBins + i - 1) * 3 + q]));
                }
            if (lc == 0 || right_cnt[i] == 0) continue;
            const double cost = area(llo, lhi) * lc + right_area[i] * right_cnt[i];
            if (cost < best) {
                best = cost;
                best_axis = a;
                best_bin = i;
            }
        }
    }
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = fdec(N.lo[a]) - margin;  // the padded box, as the host rule sees it
        hi[a] = fdec(N.hi[a]) + margin;
    }
    bool leaf = N.count <= 1;
    if (!leaf && N.count <= leaf_max) {
        const double split = best_axis >= 0 ? trav_cost + best / area(lo, hi) : INFINITY;
        leaf = (double)N.count <= split;
    }
    N.slot = kNoSlot;
    if (leaf) {
        N.leaf = 1;
        N.axis = -1;
        split_flag[s] = 0;
        return;
    }
    if (best_axis >= 0) {
        N.axis = best_axis;
        N.split = (uint32_t)best_bin;
    } else {  // every centroid in one point: split by index along the longest extent
        int a = 0;
        for (int q = 1; q < 3; ++q)
            if (fdec(N.hi[q]) - fdec(N.lo[q]) > fdec(N.hi[a]) - fdec(N.lo[a])) a = q;
        N.axis = a;
        N.split = 0xFFFFFFFFu;
    }
    split_flag[s] = 1;
}

__device__ __forceinline__ bool goes_left(const GNode& N, uint32_t k, uint32_t t, const float* cen) {
    if (N.split == 0xFFFFFFFFu) return k - N.begin < N.count / 2;
    const int a = N.axis;
    const float clo = fdec(N.clo[a]), scale = (float)kBins / (fdec(N.chi[a]) - clo);
    return min(kBins - 1, (int)((cen[3 * t + a] - clo) * scale)) < (int)N.split;
}

// Per position: 1 if its triangle goes to the left child of a node being split.
__global__ void left_flag_kernel(uint32_t n, const uint32_t* __restrict__ ids, const uint32_t* __restrict__ seg,
                                 const GNode* __restrict__ nodes, const uint8_t* __restrict__ splitting,
                                 const float* __restrict__ cen, uint32_t* __restrict__ flag) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t v = seg[k];
    flag[k] = splitting[v] ? (goes_left(nodes[v], k, ids[k], cen) ? 1u : 0u) : 0u;
}

// Children of the split nodes: indices from the scan of split flags; the
// left count from the scan of left flags at the node's end.
__global__ void make_children_kernel(uint32_t m, const uint32_t* __restrict__ active, GNode* __restrict__ nodes,
                                     const uint32_t* __restrict__ split_flag, const uint32_t* __restrict__ split_rank,
                                     uint32_t first_child, const uint32_t* __restrict__ lscan,
                                     const uint32_t* __restrict__ lflag, uint32_t* __restrict__ child_list) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= m || !split_flag[s]) return;
    GNode& N = nodes[active[s]];
    const uint32_t e = N.begin + N.count - 1;
    const uint32_t nl = (lscan[e] + lflag[e]) - lscan[N.begin];
    const uint32_t l = first_child + 2 * split_rank[s];
    N.left = l;
    N.right = l + 1;
    GNode* C = nodes + l;
    for (int c = 0; c < 2; ++c) {
        for (int a = 0; a < 3; ++a) {
            C[c].lo[a] = 0xFFFFFFFFu;
            C[c].hi[a] = 0u;
            C[c].clo[a] = 0xFFFFFFFFu;
            C[c].chi[a] = 0u;
        }
        C[c].axis = -1;
        C[c].leaf = 0;
        C[c].slot = kNoSlot;
        C[c].left = C[c].right = 0;
        C[c].split = 0;
    }
    C[0].begin = N.begin;
    C[0].count = nl;
    C[1].begin = N.begin + nl;
    C[1].count = N.count - nl;
    child_list[2 * split_rank[s]] = l;
    child_list[2 * split_rank[s] + 1] = l + 1;
}

// Stable partition of the split nodes' positions into their children, and the
// children's exact boxes and centroid boxes (atomic min / max, privatised in
// LDS when a chunk of positions belongs to one node, as in bin_chunk_kernel).
__device__ __forceinline__ uint32_t part_one(uint32_t k, uint32_t t, const GNode& N, const uint32_t* lscan,
                                             const uint32_t* lflag, uint32_t* ids2, uint32_t* seg2) {
    const uint32_t e = N.begin + N.count - 1;
    const uint32_t nl = (lscan[e] + lflag[e]) - lscan[N.begin];
    const uint32_t before = lscan[k] - lscan[N.begin];  // left triangles before k in the node
    uint32_t dst, c;
    if (lflag[k]) {
        dst = N.begin + before;
        c = N.left;
    } else {
        dst = N.begin + nl + (k - N.begin - before);
        c = N.right;
    }
    ids2[dst] = t;
    seg2[dst] = c;
    return c;
}

__device__ __forceinline__ void grow_bounds(uint32_t* w, uint32_t t, const float* bl, const float* bh,
                                            const float* cen) {  // w: lo[3] hi[3] clo[3] chi[3]
    for (int a = 0; a < 3; ++a) {
        atomicMin(&w[a], fenc(bl[3 * t + a]));
        atomicMax(&w[3 + a], fenc(bh[3 * t + a]));
        atomicMin(&w[6 + a], fenc(cen[3 * t + a]));
        atomicMax(&w[9 + a], fenc(cen[3 * t + a]));
    }
}

__global__ __launch_bounds__(kBinThreads) void partition_kernel(
    uint32_t n, const uint32_t* __restrict__ ids, const uint32_t* __restrict__ seg, GNode* __restrict__ nodes,
    const uint8_t* __restrict__ splitting, const uint32_t* __restrict__ lscan, const uint32_t* __restrict__ lflag,
    const float* __restrict__ bl, const float* __restrict__ bh, const float* __restrict__ cen,
    uint32_t* __restrict__ ids2, uint32_t* __restrict__ seg2) {
    static_assert(offsetof(GNode, hi) == offsetof(GNode, lo) + 12 && offsetof(GNode, clo) == offsetof(GNode, lo) + 24 &&
                      offsetof(GNode, chi) == offsetof(GNode, lo) + 36,
                  "GNode bounds are 12 consecutive words");
    __shared__ uint32_t cb[2][12];
    const uint32_t base = blockIdx.x * kBinChunk;
    const uint32_t end = min(base + kBinChunk, n);
    const uint32_t v0 = seg[base];
    if (v0 == seg[end - 1] && splitting[v0]) {  // one node being split
        const GNode N = nodes[v0];
        if (threadIdx.x < 24) cb[threadIdx.x / 12][threadIdx.x % 12] = (threadIdx.x % 6 < 3) ? 0xFFFFFFFFu : 0u;
        __syncthreads();
        for (uint32_t k = base + threadIdx.x; k < end; k += kBinThreads) {
            const uint32_t t = ids[k];
            const uint32_t c = part_one(k, t, N, lscan, lflag, ids2, seg2);
            grow_bounds(cb[c == N.left ? 0 : 1], t, bl, bh, cen);
        }
        __syncthreads();
        if (threadIdx.x < 24) {
            const uint32_t side = threadIdx.x / 12, w = threadIdx.x % 12;
            uint32_t* dst = nodes[side ? N.right : N.left].lo + w;
            const uint32_t v = cb[side][w];
            if (w % 6 < 3) {
                if (v != 0xFFFFFFFFu) atomicMin(dst, v);
            } else if (v) {
                atomicMax(dst, v);
            }
        }
        return;
    }
    for (uint32_t k = base + threadIdx.x; k < end; k += kBinThreads) {
        const uint32_t v = seg[k], t = ids[k];
        if (!splitting[v]) {
            ids2[k] = t;
            seg2[k] = v;
            continue;
        }
        const GNode& N = nodes[v];
        const uint32_t c = part_one(k, t, N, lscan, lflag, ids2, seg2);
        grow_bounds(nodes[c].lo, t, bl, bh, cen);
    }
}

__global__ void mark_kernel(uint32_t m, const uint32_t* __restrict__ list, const uint32_t* __restrict__ flag,
                            uint8_t* __restrict__ splitting) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < m) splitting[list[s]] = flag ? (uint8_t)flag[s] : (uint8_t)0;
}

// need[s] = 1 for a node of the level that can split (two or more triangles)
__global__ void need_bins_kernel(uint32_t m, const uint32_t* __restrict__ list, const GNode* __restrict__ nodes,
                                 uint32_t* __restrict__ need) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < m) need[s] = nodes[list[s]].count > 1 ? 1u : 0u;
}

// bin slots of one batch: the nodes of need rank [b0, b0 + nb)
__global__ void assign_slots_kernel(uint32_t m, const uint32_t* __restrict__ list, const uint32_t* __restrict__ need,
                                    const uint32_t* __restrict__ rank, uint32_t b0, uint32_t nb,
                                    GNode* __restrict__ nodes) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= m) return;
    const uint32_t r = rank[s];
    nodes[list[s]].slot = (need[s] && r >= b0 && r - b0 < nb) ? r - b0 : kNoSlot;
}

// ---- exclusive scan of uint32 (deterministic, three passes) ----------------
constexpr uint32_t kScanBlock = 256, kScanItems = 4, kScanTile = kScanBlock * kScanItems;

__global__ void scan_tiles_kernel(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, uint32_t n,
                                  uint32_t* __restrict__ tile_sums) {
    __shared__ uint32_t s[kScanBlock];
    const uint32_t base = blockIdx.x * kScanTile + threadIdx.x * kScanItems;
    uint32_t v[kScanItems], sum = 0;
    for (uint32_t i = 0; i < kScanItems; ++i) {
        v[i] = base + i < n ? in[base + i] : 0u;
        sum += v[i];
    }
    s[threadIdx.x] = sum;
    __syncthreads();
    for (uint32_t off = 1; off < kScanBlock; off <<= 1) {
        const uint32_t x = threadIdx.x >= off ? s[threadIdx.x - off] : 0u;
        __syncthreads();
        s[threadIdx.x] += x;
        __syncthreads();
    }
    uint32_t run = s[threadIdx.x] - sum;  // exclusive prefix of this thread's items
    for (uint32_t i = 0; i < kScanItems; ++i) {
        if (base + i < n) out[base + i] = run;
        run += v[i];
    }
    if (threadIdx.x == kScanBlock - 1) tile_sums[blockIdx.x] = s[threadIdx.x];
}

__global__ void scan_sums_kernel(uint32_t* __restrict__ sums, uint32_t tiles) {  // one block, serial chunks
    __shared__ uint32_t s[kScanBlock];
    __shared__ uint32_t carry;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (uint32_t b = 0; b < tiles; b += kScanBlock) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < tiles ? sums[i] : 0u;
        s[threadIdx.x] = v;
        __syncthreads();
        for (uint32_t off = 1; off < kScanBlock; off <<= 1) {
            const uint32_t x = threadIdx.x >= off ? s[threadIdx.x - off] : 0u;
            __syncthreads();
            s[threadIdx.x] += x;
            __syncthreads();
        }
        if (i < tiles) sums[i] = carry + s[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == kScanBlock - 1) carry += s[threadIdx.x];
        __syncthreads();
    }
}

__global__ void scan_add_kernel(uint32_t* __restrict__ out, uint32_t n, const uint32_t* __restrict__ sums) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) out[k] += sums[k / kScanTile];
}

// ---- emission --------------------------------------------------------------
// subtree entry counts, bottom-up over one level's node list
__global__ void size_kernel(uint32_t m, const uint32_t* __restrict__ list, const GNode* __restrict__ nodes,
                            uint32_t* __restrict__ size) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= m) return;
    const uint32_t v = list[s];
    const GNode& N = nodes[v];
    size[v] = N.leaf ? 1u : 1u + size[N.left] + size[N.right];
}

// preorder position of the children of one level's nodes in each octant layout
__global__ void pos_kernel(uint32_t m, const uint32_t* __restrict__ list, const GNode* __restrict__ nodes,
                           const uint32_t* __restrict__ size, uint32_t* __restrict__ pos, uint32_t cap) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t oct = blockIdx.y;
    if (s >= m) return;
    const GNode& N = nodes[list[s]];
    if (N.leaf) return;
    const bool neg = (oct >> N.axis) & 1u;  // moving toward lower coordinates: right child first
    const uint32_t near = neg ? N.right : N.left, far = neg ? N.left : N.right;
    const uint32_t p = pos[(size_t)oct * cap + list[s]];
    pos[(size_t)oct * cap + near] = p + 1;
    pos[(size_t)oct * cap + far] = p + 1 + size[near];
}

__global__ void emit_kernel(uint32_t total, const GNode* __restrict__ nodes, const uint32_t* __restrict__ size,
                            const uint32_t* __restrict__ pos, uint32_t cap, float margin, uint4* __restrict__ out) {
    const uint32_t v = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t oct = blockIdx.y;
    if (v >= total) return;
    const GNode& N = nodes[v];
    const uint32_t p = pos[(size_t)oct * cap + v];
    const float lx = fdec(N.lo[0]) - margin, ly = fdec(N.lo[1]) - margin, lz = fdec(N.lo[2]) - margin;
    const float hx = fdec(N.hi[0]) + margin, hy = fdec(N.hi[1]) + margin, hz = fdec(N.hi[2]) + margin;
    // the box in fp16 rounded outward (a superset of the padded box)
    uint32_t h[6] = {__half_as_ushort(__float2half_rd(lx)), __half_as_ushort(__float2half_rd(ly)),
                     __half_as_ushort(__float2half_rd(lz)), __half_as_ushort(__float2half_ru(hx)),
                     __half_as_ushort(__float2half_ru(hy)), __half_as_ushort(__float2half_ru(hz))};
    // near/far: in the layout of octant `oct` the plane a ray of that octant
    // enters through takes the lo slot (rt_trace.hpp lds_node_hit_nf)
#pragma unroll
    for (int a = 0; a < 3; ++a)
        if ((oct >> a) & 1u) {
            const uint32_t x = h[a];
            h[a] = h[3 + a];
            h[3 + a] = x;
        }
    const uint32_t w = N.leaf ? (N.begin | (N.count - 1u) << 24) : ((oct * total + p + size[v]) | 0x80000000u);
    out[(size_t)oct * total + p] = make_uint4(h[0] | (h[1] << 16), h[2] | (h[3] << 16), h[4] | (h[5] << 16), w);
}

__global__ void gather_sorted_kernel(const float4* __restrict__ tri, const uint32_t* __restrict__ ids, uint32_t n,
                                     float4* __restrict__ sorted, uint32_t* __restrict__ perm) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint32_t t = ids[k];
    sorted[3 * k] = tri[3 * t];
    sorted[3 * k + 1] = tri[3 * t + 1];
    sorted[3 * k + 2] = tri[3 * t + 2];
    perm[k] = t;
}

template <typename T>
hipError_t dalloc(T** p, size_t count) {
    return hipMalloc((void**)p, (count ? count : 1) * sizeof(T) + 16);
}

inline dim3 grid1(uint32_t n, uint32_t t = 256) { return dim3((n + t - 1) / t); }

}  // namespace

hipError_t scan_u32(const uint32_t* in, uint32_t* out, uint32_t n, uint32_t* tile_sums, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t tiles = (n + kScanTile - 1) / kScanTile;
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(tiles), dim3(kScanBlock), 0, s, in, out, n, tile_sums);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(kScanBlock), 0, s, tile_sums, tiles);
    hipLaunchKernelGGL(scan_add_kernel, grid1(n), dim3(256), 0, s, out, n, tile_sums);
    return hipGetLastError();
}

hipError_t build_tri_gsah(const float4* d_tri, uint32_t n, float margin, uint32_t leaf_max, double trav_cost,
                          uint4* d_nodes, float4* d_sorted, uint32_t* d_perm, uint32_t* total_nodes,
                          size_t* temp_bytes, hipStream_t s) {
    *total_nodes = 0;
    if (temp_bytes) *temp_bytes = 0;
    if (n == 0) return hipSuccess;
    if (n >= (1u << 24)) return hipErrorInvalidValue;  // leaf index field is 24 bits
    const uint32_t cap = 2 * n - 1;                    // nodes at most
    float *bl = nullptr, *bh = nullptr, *cen = nullptr;
    uint32_t *ids = nullptr, *ids2 = nullptr, *seg = nullptr, *seg2 = nullptr, *lflag = nullptr, *lscan = nullptr,
             *tiles = nullptr, *bins = nullptr, *split_flag = nullptr, *split_rank = nullptr, *lists = nullptr,
             *size = nullptr, *pos = nullptr, *need = nullptr, *need_rank = nullptr;
    uint8_t* splitting = nullptr;
    GNode* nodes = nullptr;
    hipError_t e = hipSuccess;
    size_t bins_cap = 0, bins_peak = 0;  // words, bytes
    std::vector<uint32_t> level_off, level_cnt;  // node lists of every level (in `lists`)
    do {
        const uint32_t nt = (n + kScanTile - 1) / kScanTile + 1;
        if ((e = dalloc(&bl, 3 * (size_t)n)) || (e = dalloc(&bh, 3 * (size_t)n)) || (e = dalloc(&cen, 3 * (size_t)n)) ||
            (e = dalloc(&ids, n)) || (e = dalloc(&ids2, n)) || (e = dalloc(&seg, n)) || (e = dalloc(&seg2, n)) ||
            (e = dalloc(&lflag, n)) || (e = dalloc(&lscan, n)) || (e = dalloc(&tiles, nt + kScanTile)) ||
            (e = dalloc(&nodes, cap)) || (e = dalloc(&splitting, cap)) || (e = dalloc(&lists, cap)) ||
            (e = dalloc(&split_flag, n)) || (e = dalloc(&split_rank, n)) || (e = dalloc(&size, cap)) ||
            (e = dalloc(&need, n)) || (e = dalloc(&need_rank, n)))
            break;
        // fixed temporaries (the bins and the layout positions are added below)
        size_t temp = (size_t)n * (9 * sizeof(float) + 10 * sizeof(uint32_t)) +
                      (size_t)cap * (sizeof(GNode) + 1 + 2 * sizeof(uint32_t)) + (nt + kScanTile) * sizeof(uint32_t);
        // root: node 0 = every triangle
        GNode root{};
        for (int a = 0; a < 3; ++a) {
            root.lo[a] = root.clo[a] = 0xFFFFFFFFu;
            root.hi[a] = root.chi[a] = 0u;
        }
        root.begin = 0;
        root.count = n;
        root.axis = -1;
        root.slot = kNoSlot;
        if ((e = hipMemcpyAsync(nodes, &root, sizeof(root), hipMemcpyHostToDevice, s))) break;
        if ((e = hipMemsetAsync(splitting, 0, cap, s))) break;
        hipLaunchKernelGGL(tri_box_kernel, grid1(n), dim3(256), 0, s, d_tri, n, bl, bh, cen, ids, seg, nodes);
        const uint32_t zero = 0;
        if ((e = hipMemcpyAsync(lists, &zero, 4, hipMemcpyHostToDevice, s))) break;
        uint32_t m = 1, next_free = 1, list_off = 0;  // level's nodes at lists[list_off, +m)
        while (m > 0) {
            level_off.push_back(list_off);
            level_cnt.push_back(m);
            const uint32_t* active = lists + list_off;
            // bin slots only for the nodes that can split (a node of one
            // triangle becomes a leaf without reading bins), at most
            // kMaxBinSlots at a time: the level runs in batches of slots
            hipLaunchKernelGGL(need_bins_kernel, grid1(m), dim3(256), 0, s, m, active, nodes, need);
            if ((e = scan_u32(need, need_rank, m, tiles, s))) break;
            uint32_t nlast[2];
            if ((e = hipMemcpyAsync(&nlast[0], need_rank + m - 1, 4, hipMemcpyDeviceToHost, s)) ||
                (e = hipMemcpyAsync(&nlast[1], need + m - 1, 4, hipMemcpyDeviceToHost, s)) ||
                (e = hipStreamSynchronize(s)))
                break;
            const uint32_t nneed = nlast[0] + nlast[1];
            const uint32_t slots = nneed < kMaxBinSlots ? nneed : kMaxBinSlots;
            if ((size_t)slots * kSlotWords > bins_cap) {
                (void)hipFree(bins);
                bins = nullptr;
                bins_cap = (size_t)slots * kSlotWords;
                if ((e = hipMalloc((void**)&bins, bins_cap * sizeof(uint32_t)))) break;
                if (bins_cap * sizeof(uint32_t) > bins_peak) bins_peak = bins_cap * sizeof(uint32_t);
            }
            for (uint32_t b0 = 0; b0 == 0 || b0 < nneed; b0 += kMaxBinSlots) {
                const uint32_t nb = nneed - b0 < kMaxBinSlots ? nneed - b0 : kMaxBinSlots;
                // bins: counts 0, lo = +inf (0xFFFFFFFF), hi = -inf (0)
                if (nb) hipLaunchKernelGGL(clear_bins_kernel, grid1(nb * kSlotWords), dim3(256), 0, s, bins, nb);
                hipLaunchKernelGGL(assign_slots_kernel, grid1(m), dim3(256), 0, s, m, active, need, need_rank, b0, nb,
                                   nodes);
                if (nb)
                    hipLaunchKernelGGL(bin_chunk_kernel, dim3((n + kBinChunk - 1) / kBinChunk), dim3(kBinThreads), 0,
                                       s, n, ids, seg, nodes, bl, bh, cen, bins);
                hipLaunchKernelGGL(split_kernel, grid1(m, 64), dim3(64), 0, s, m, active, nodes, bins, leaf_max,
                                   trav_cost, margin, split_flag, b0 == 0 ? 1u : 0u);
            }
            if ((e = scan_u32(split_flag, split_rank, m, tiles, s))) break;
            hipLaunchKernelGGL(mark_kernel, grid1(m), dim3(256), 0, s, m, active, split_flag, splitting);
            hipLaunchKernelGGL(left_flag_kernel, grid1(n), dim3(256), 0, s, n, ids, seg, nodes, splitting, cen, lflag);
            if ((e = scan_u32(lflag, lscan, n, tiles, s))) break;
            // number of splitting nodes = rank of the last + its flag
            uint32_t last[2];
            if ((e = hipMemcpyAsync(&last[0], split_rank + m - 1, 4, hipMemcpyDeviceToHost, s)) ||
                (e = hipMemcpyAsync(&last[1], split_flag + m - 1, 4, hipMemcpyDeviceToHost, s)) ||
                (e = hipStreamSynchronize(s)))
                break;
            const uint32_t nsplit = last[0] + last[1];
            const uint32_t child_off = list_off + m;
            hipLaunchKernelGGL(make_children_kernel, grid1(m), dim3(256), 0, s, m, active, nodes, split_flag,
                               split_rank, next_free, lscan, lflag, lists + child_off);
            hipLaunchKernelGGL(partition_kernel, dim3((n + kBinChunk - 1) / kBinChunk), dim3(kBinThreads), 0, s,
                               n, ids, seg, nodes, splitting, lscan, lflag, bl, bh, cen, ids2, seg2);
            hipLaunchKernelGGL(mark_kernel, grid1(m), dim3(256), 0, s, m, active, (const uint32_t*)nullptr, splitting);
            if ((e = hipGetLastError())) break;
            std::swap(ids, ids2);
            std::swap(seg, seg2);
            next_free += 2 * nsplit;
            list_off = child_off;
            m = 2 * nsplit;
        }
        if (e) break;
        const uint32_t total = next_free;
        // subtree sizes bottom-up, positions top-down
        for (size_t L = level_cnt.size(); L-- > 0;)
            hipLaunchKernelGGL(size_kernel, grid1(level_cnt[L]), dim3(256), 0, s, level_cnt[L], lists + level_off[L],
                               nodes, size);
        if ((e = dalloc(&pos, 8 * (size_t)cap))) break;
        temp += 8 * (size_t)cap * sizeof(uint32_t);
        if (temp_bytes) *temp_bytes = temp + bins_peak;
        if ((e = hipMemsetAsync(pos, 0, 8 * (size_t)cap * 4, s))) break;  // the root at 0 in every layout
        for (size_t L = 0; L < level_cnt.size(); ++L)
            hipLaunchKernelGGL(pos_kernel, dim3((level_cnt[L] + 255) / 256, 8), dim3(256), 0, s, level_cnt[L],
                               lists + level_off[L], nodes, size, pos, cap);
        hipLaunchKernelGGL(emit_kernel, dim3((total + 255) / 256, 8), dim3(256), 0, s, total, nodes, size, pos, cap,
                           margin, d_nodes);
        hipLaunchKernelGGL(gather_sorted_kernel, grid1(n), dim3(256), 0, s, d_tri, ids, n, d_sorted, d_perm);
        if ((e = hipGetLastError())) break;
        if ((e = hipStreamSynchronize(s))) break;
        *total_nodes = total;
    } while (0);
    (void)hipFree(bl);
    (void)hipFree(bh);
    (void)hipFree(cen);
    (void)hipFree(ids);
    (void)hipFree(ids2);
    (void)hipFree(seg);
    (void)hipFree(seg2);
    (void)hipFree(lflag);
    (void)hipFree(lscan);
    (void)hipFree(tiles);
    (void)hipFree(bins);
    (void)hipFree(split_flag);
    (void)hipFree(split_rank);
    (void)hipFree(lists);
    (void)hipFree(size);
    (void)hipFree(pos);
    (void)hipFree(splitting);
    (void)hipFree(nodes);
    (void)hipFree(need);
    (void)hipFree(need_rank);
    return e;
}

}  // namespace rt

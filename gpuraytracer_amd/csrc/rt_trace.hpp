// rt_trace.hpp — ray/primitive tests and scene queries shared by the
// pathTrace kernel (rt_kernel.hip) and the MIS kernel (rt_mis.hip).
// Device-only; every function follows the arithmetic contract of DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>

#include "rt_kernel.hpp"

namespace rt {
namespace {

__device__ __forceinline__ f3 ld_f3(const float* p) { return f3{p[0], p[1], p[2]}; }

// Ray/triangle test of DESIGN.md §3.5 (stands in for Metal's intersector).
// The oracle negates (bu, bv, tn, den) when den < 0; here the same exact
// negation is an XOR with den's sign bit, |den| folds into the compare, and tn
// (with the IEEE division) is only formed for lanes inside the triangle.
__device__ __forceinline__ bool tri_test(const float4& A, const float4& Bq, const float4& C, f3 o,
                                         f3 d, float tmin, float tmax, float* t_out) {
    const f3 v0{A.x, A.y, A.z}, e1{A.w, Bq.x, Bq.y}, e2{Bq.z, Bq.w, C.x}, n{C.y, C.z, C.w};
    const f3 tv = o - v0;
    const f3 c = cross(tv, d);
    const float den = dot(n, d);
    const uint32_t sgn = __float_as_uint(den) & 0x80000000u;
    const uint32_t nsgn = sgn ^ 0x80000000u;
    const float bu = __uint_as_float(__float_as_uint(dot(e2, c)) ^ nsgn);  // -dot(e2,c), sign-normalised
    const float bv = __uint_as_float(__float_as_uint(dot(e1, c)) ^ sgn);
    const float aden = fabsf(den);
    if (aden > 0.0f && bu >= 0.0f && bv >= 0.0f && bu + bv <= aden) {
        const float tn = __uint_as_float(__float_as_uint(dot(n, tv)) ^ nsgn);  // -dot(n,tv)
        const float t = tn / aden;
        if (t > tmin && t < tmax) {
            *t_out = t;
            return true;
        }
    }
    return false;
}

// Two consecutive triangles A=(v0,..), B=(v0,..) that share v0 and one edge S
// (every quad of the reference scene, scene.swift:81-138, :212-240).  The
// per-triangle test above is evaluated for A then B with the common terms
// tv = o - v0, c = cross(tv, d) and dot(S, c) computed once: bit-identical to
// two tri_test calls, ~25% fewer VALU operations.  Record (5 x float4):
//   r0 = (v0.xyz, S.x)  r1 = (S.yz, eA.xy)  r2 = (eA.z, nA.xyz)
//   r3 = (eB.xyz, nB.x) r4 = (nB.yz, m, 0)
// m = 0 when A.e1 == S == B.e2, 0x80000000 when A.e2 == S == B.e1; eA / eB
// are the other edges.  bu+bv and the bu,bv >= 0 tests are symmetric in
// (bu, bv), so only the signs of the two terms matter.
struct PairDots {
    float denA, denB;  // dot(n, d)
    uint32_t a1, a2, b1, b2;  // sign-normalised barycentric terms (bits)
    f3 tv;
};

__device__ __forceinline__ PairDots pair_dots(const float4& r0, const float4& r1,
                                              const float4& r2, const float4& r3,
                                              const float4& r4, f3 o, f3 d) {
    PairDots q;
    const f3 v0{r0.x, r0.y, r0.z}, S{r0.w, r1.x, r1.y}, eA{r1.z, r1.w, r2.x};
    const f3 nA{r2.y, r2.z, r2.w}, eB{r3.x, r3.y, r3.z}, nB{r3.w, r4.x, r4.y};
    const uint32_t m = __float_as_uint(r4.z);
    q.tv = o - v0;
    const f3 c = cross(q.tv, d);
    const uint32_t s = __float_as_uint(dot(S, c));
    const uint32_t ea = __float_as_uint(dot(eA, c));
    const uint32_t eb = __float_as_uint(dot(eB, c));
    q.denA = dot(nA, d);
    q.denB = dot(nB, d);
    const uint32_t sA = (__float_as_uint(q.denA) & 0x80000000u) ^ m;
    const uint32_t sB = (__float_as_uint(q.denB) & 0x80000000u) ^ m;
    q.a1 = s ^ sA;
    q.a2 = ea ^ sA ^ 0x80000000u;
    q.b1 = s ^ sB ^ 0x80000000u;
    q.b2 = eb ^ sB;
    return q;
}

__device__ __forceinline__ bool bary_ok(float den, uint32_t t1, uint32_t t2) {
    const float u = __uint_as_float(t1), v = __uint_as_float(t2);
    return fabsf(den) > 0.0f && u >= 0.0f && v >= 0.0f && u + v <= fabsf(den);
}

// t of a triangle whose barycentric test passed: -dot(n, tv) / den, sign-normalised
__device__ __forceinline__ float pair_t(f3 n, f3 tv, float den) {
    const uint32_t nsgn = (__float_as_uint(den) & 0x80000000u) ^ 0x80000000u;
    const float tn = __uint_as_float(__float_as_uint(dot(n, tv)) ^ nsgn);
    return tn / fabsf(den);
}

// intersectSphere (shaders_old.metal:108-136) with the DESIGN.md §3.6 root rule.
__device__ __forceinline__ bool sph_test(const float4& S, f3 o, f3 d, float a, float tmin,
                                         float tmax, float* t_out) {
    const f3 oc = o - f3{S.x, S.y, S.z};
    const float b = 2.0f * dot(oc, d);
    const float cc = dot(oc, oc) - S.w;
    const float disc = b * b - (4.0f * a) * cc;
    if (disc > 0.0f) {
        const float sq = sqrtf(disc);
        const float a2 = 2.0f * a;
        float t = (-b - sq) / a2;                 // t1
        if (!(t > tmin)) t = (-b + sq) / a2;      // t2, divided only when it is the root taken
        if (t > tmin && t < tmax) {
            *t_out = t;
            return true;
        }
    }
    return false;
}

// Diagnostic counters (only in an -DRT_STATS instrumentation build, read with
// rt_debug_stats by tools/kernel_stats.py and tools/sphere_stats.py).
// Slot groups of 4 per query kind q (0: camera closest hit, 1: bounce closest
// hit, 2: shadow any-hit): [4q] pair records visited per wave, [4q+1] records
// tested, [4q+2] active lanes summed over tested records, [4q+3] division blocks.
// Box-cluster queries: [12] queries per wave, [13] candidate rounds per wave,
// [14] lanes summed over rounds, [15] lanes summed over queries.
// Sphere walks (sphere_walk), base 16 closest / 24 any-hit: [+0] walks per
// wave, [+1] lanes summed over walks, [+2] walk-loop iterations, [+3] lanes
// summed over them, [+4] unused, [+5] root rounds, [+6] parked lanes summed
// over them.
#ifdef RT_STATS
__device__ unsigned long long g_rt_stats[32];
__device__ __forceinline__ void stat_wave(int slot, unsigned long long v) {
    const unsigned long long m = __ballot(1);
    if ((threadIdx.x & 63u) == (unsigned)(__ffsll((long long)m) - 1)) atomicAdd(&g_rt_stats[slot], v);
}
#define RT_STAT(slot, v) stat_wave((slot), (v))
#else
#define RT_STAT(slot, v) ((void)0)
#endif

// Where the intersection records live for one launch.
enum Geo : int {
    kGeoTriLds = 0,     // single-triangle records staged in LDS
    kGeoPairLds = 1,    // shared-edge pair records staged in LDS
    kGeoPairSmem = 4,   // shared-edge pair records read with scalar loads (no LDS)
    kGeoTriBvh = 5,     // GPU-built triangle BVH (rt_lbvh.hip), records from global
    kGeoTriGlobal = 2,  // single-triangle records read from global (big scenes)
    kGeoPairClu = 6,    // pair records in LDS + box clusters
    kGeoSphLds = 7,     // pair records in LDS + the compact sphere BVH in L2 (one-wave workgroups)
};

constexpr bool geo_pairs(int g) { return g == kGeoPairLds || g == kGeoPairSmem || g == kGeoSphLds; }

struct SceneView {
    const float4* tri;        // 3 float4 per triangle (single layout)
    const float4* pair;       // kPairF4 float4 per triangle pair (pair layout)
    const float4* sph;        // 1 float4 per sphere, BVH leaf order
    const float4* node;       // 2 float4 per sphere-BVH node
    const uint32_t* sph_perm; // leaf order -> sphere id (global memory)
    const uint4* tnode;       // triangle BVH: 8 compact octant layouts of nTN nodes
    const float4* tsorted;    // 3 float4 per triangle, BVH leaf order
    const uint32_t* tperm;    // leaf order -> triangle id
    uint32_t nTN;
    uint32_t nT, nP, nS, nN;
    const float4* clu;        // box clusters, kCluF4 float4 each (kGeoPairClu)
    const float4* clu_oct = nullptr;  // per cluster, 8 octants x 2 float4 of pre-swapped face masks, or null
    uint32_t nC;
    uint32_t pair_free;       // pairs in no cluster: tested by every lane
    const float* htab;        // Halton low-digit tables in LDS (kGeoPairClu)
    const uint4* sent;        // compact sphere BVH entries (kGeoSphLds): 8 octant layouts, global
    const uint16_t* sid;      // sphere id of each compact entry (leaves), global
    const uint4* sbox;        // the sphere BVH with leaf boxes (RT_SPH_LEAFBOX): 8 layouts of nSB entries
    uint32_t nSB;
    const float4* shade;      // MIS shading records, 3 float4 per triangle (rt_mis.hip)
    float* xstash;            // MIS: per-lane primary hit (p, din), SoA in LDS (rt_mis.hip)
};

// min / max of the culling tests, issued directly.  fminf/fmaxf lower to
// v_min/v_max_f32 plus a v_max_f32 x,x "canonicalize" of every operand the
// compiler cannot prove canonical (loads, values through phis: the
// loop-carried best, the branch-merged slab terms) -- 8 extra VALU per box
// cluster and 2 per BVH step.  The operands here are results of arithmetic on
// finite scene data (no signalling NaNs), for which v_min/v_max_f32 return
// exactly fminf/fmaxf; and these values only decide what is culled, never a
// result.
__device__ __forceinline__ float vmin(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float vmin3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// Per-ray data of the slab test.  1/d uses the 1-ulp hardware reciprocal: the
// node boxes carry the culling margin, so only speed depends on its rounding.
struct RayBox {
    f3 invd, oinv;
};

// 1/v clamped to +-1e20 (v = +-0 gives +-1e20): one v_rcp + one v_med3.
// Feeds only conservative slab tests (speed, not results, depends on it).
__device__ __forceinline__ float safe_rcp(float v) {
    return __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf(v), -1e20f, 1e20f);
}

__device__ __forceinline__ RayBox ray_box(f3 o, f3 d) {
    RayBox r;
    r.invd = f3{safe_rcp(d.x), safe_rcp(d.y), safe_rcp(d.z)};
    r.oinv = f3{o.x * r.invd.x, o.y * r.invd.y, o.z * r.invd.z};
    return r;
}

// Conservative ray/box overlap on (tmin, tmax): false only if no point of the
// padded box lies on the ray inside that range.
__device__ __forceinline__ bool node_hit(const float4& n0, const float4& n1, const RayBox& rb,
                                         float tmin, float tmax) {
    const float tx0 = fmaf(n0.x, rb.invd.x, -rb.oinv.x), tx1 = fmaf(n1.x, rb.invd.x, -rb.oinv.x);
    const float ty0 = fmaf(n0.y, rb.invd.y, -rb.oinv.y), ty1 = fmaf(n1.y, rb.invd.y, -rb.oinv.y);
    const float tz0 = fmaf(n0.z, rb.invd.z, -rb.oinv.z), tz1 = fmaf(n1.z, rb.invd.z, -rb.oinv.z);
    const float tnear = vmax3(vmin(tx0, tx1), vmin(ty0, ty1), vmax(vmin(tz0, tz1), tmin));
    const float tfar = vmin3(vmax(tx0, tx1), vmax(ty0, ty1), vmin(vmax(tz0, tz1), tmax));
    return tnear <= tfar;
}

// BVH layout of a ray direction: bit a set when component a is negative.
__device__ __forceinline__ uint32_t octant(f3 d) {
    return (__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 31) << 1) |
           ((__float_as_uint(d.z) >> 31) << 2);
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Sphere-BVH walks over the 32-B nodes (the sphere scenes of the pair, single
// and global layouts; the default sphere kernel walks the compact BVH below).
// One stackless depth-first walk per lane through the escape-index tree of
// the ray's direction octant (near child first); a node is entered when the
// ray may hit its padded box.  Candidates are ranked by (t, sphere id) exactly
// like the oracle's id-ordered scan with strict '<', so the visiting order is
// free.
__device__ __forceinline__ void sphere_closest(const float4* __restrict__ node,
                                               const float4* __restrict__ sph,
                                               const uint32_t* __restrict__ perm, uint32_t nN,
                                               uint32_t nT, f3 o, f3 d, float tmin, float& best,
                                               int& id) {
    const float a = dot(d, d);
    const RayBox rb = ray_box(o, d);
    node += 2u * nN * octant(d);
    uint32_t idx = 0;
    while (idx < nN) {
        const float4 n0 = node[2 * idx], n1 = node[2 * idx + 1];
        uint32_t next = __float_as_uint(n0.w);
        if (node_hit(n0, n1, rb, tmin, best)) {
            const uint32_t leaf = __float_as_uint(n1.w);
            if (leaf == 0u) {
                next = idx + 1;
            } else {
                const uint32_t first = leaf & 0xFFFFFFu, end = first + (leaf >> 24);
                for (uint32_t k = first; k < end; ++k) {
                    float t;
                    if (sph_test(sph[k], o, d, a, tmin, 3.0e38f, &t) && t <= best) {
                        const int sid = (int)(nT + perm[k]);
                        if (t < best || sid < id) {
                            best = t;
                            id = sid;
                        }
                    }
                }
            }
        }
        idx = next;
    }
}

__device__ __forceinline__ bool sphere_any(const float4* __restrict__ node,
                                           const float4* __restrict__ sph, uint32_t nN, f3 o,
                                           f3 d, float tmin, float tmax) {
    const float a = dot(d, d);
    const RayBox rb = ray_box(o, d);
    node += 2u * nN * octant(d);
    uint32_t idx = 0;
    while (idx < nN) {
        const float4 n0 = node[2 * idx], n1 = node[2 * idx + 1];
        uint32_t next = __float_as_uint(n0.w);
        if (node_hit(n0, n1, rb, tmin, tmax)) {
            const uint32_t leaf = __float_as_uint(n1.w);
            if (leaf == 0u) {
                next = idx + 1;
            } else {
                const uint32_t first = leaf & 0xFFFFFFu, end = first + (leaf >> 24);
                for (uint32_t k = first; k < end; ++k) {
                    float t;
                    if (sph_test(sph[k], o, d, a, tmin, tmax, &t)) return true;
                }
            }
        }
        idx = next;
    }
    return false;
}

// Compact BVH entries (rt_scene.cpp build_sphere_lds, rt_lbvh.hip): 16 B per
// node, an fp16 box rounded outward (still conservative) and one word --
// escape | 2^31 for an inner node (the escape is an entry index over all
// layouts, so a walk's position names its layout); a sphere leaf stores the
// sphere (c, r*r) itself (a leaf's escape is the next entry).
__device__ __forceinline__ float h2f(uint32_t b16) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)b16);
}

__device__ __forceinline__ bool lds_node_hit(const uint4& e, const RayBox& rb, float tmin,
                                             float tmax) {
    const float4 n0 = make_float4(h2f(e.x & 0xFFFFu), h2f(e.x >> 16), h2f(e.y & 0xFFFFu), 0.0f);
    const float4 n1 = make_float4(h2f(e.y >> 16), h2f(e.z & 0xFFFFu), h2f(e.z >> 16), 0.0f);
    return node_hit(n0, n1, rb, tmin, tmax);
}

// Slab test of a near/far entry: in the layout of direction octant k the lo
// slots hold the planes a ray of that octant enters through.  Equal to
// lds_node_hit for such rays: fma(p, invd, -oinv) is monotone in p and
// sign(invd) orders the two planes of each axis, so the min/max pairs of
// node_hit select exactly these values.
__device__ __forceinline__ bool lds_node_hit_nf(const uint4& e, const RayBox& rb, float tmin,
                                                float tmax) {
    const float nx = fmaf(h2f(e.x & 0xFFFFu), rb.invd.x, -rb.oinv.x);
    const float ny = fmaf(h2f(e.x >> 16), rb.invd.y, -rb.oinv.y);
    const float nz = fmaf(h2f(e.y & 0xFFFFu), rb.invd.z, -rb.oinv.z);
    const float fx = fmaf(h2f(e.y >> 16), rb.invd.x, -rb.oinv.x);
    const float fy = fmaf(h2f(e.z & 0xFFFFu), rb.invd.y, -rb.oinv.y);
    const float fz = fmaf(h2f(e.z >> 16), rb.invd.z, -rb.oinv.z);
    return vmax3(nx, ny, vmax(nz, tmin)) <= vmin3(fx, fy, vmin(fz, tmax));
}

// Per-lane walk of the compact sphere BVH with POSTPONED ROOTS (DESIGN.md
// §3.10; after Aila & Laine's postponed leaf processing, stackless form).
// Each lane walks the layout of its ray's direction octant.  Each step of a
// lane is cheap and of similar cost whatever the entry: a near/far box test
// for an inner node, the discriminant of sph_test for a leaf.  A leaf whose
// discriminant is positive (a real hit candidate) parks the lane with (b, disc);
// the others walk on until at least 1/kSphParkDen of the lanes still
// walking are parked (or none can move), then the wave runs the expensive part
// of the sphere test -- the IEEE sqrt and divisions -- for all parked lanes
// together.  Per lane the entries are visited in the same order and every
// value is sph_test's, ranked by (t, id): the same result.  ANY: *id becomes
// >= 0 on the first accepted hit (and that lane stops).
// the parked roots run once they are >= 1/kSphParkDen of the live lanes
// (config 4: 2 157.3 ms, 4 158.4, 6 161.1; round 5: 3 149.7-149.8, 2 150.2-150.3,
// 1 207.4 -- 1/2 kept: with 1/3 the profiled HBM traffic rose from 69 to 110 MB)
#ifndef RT_SPH_PARK_DEN
#define RT_SPH_PARK_DEN 2
#endif
constexpr int kSphParkDen = RT_SPH_PARK_DEN;
// RT_SPH_SEL: every lane runs both halves of a step (box test and
// discriminant) and keeps its entry's by selects; RT_SPH_CHK: steps between
// two checks of the parking condition (a lane that parks in between holds
// still).  Round 6, config 4 (Msamples/s): every step 3,512-3,520; selects
// 3,059 (selects + every 2 / 3 steps 3,112 / 3,127); branch-form steps checked
// every 2 / 3 / 4 / 5 / 6 / 8 / 12 steps 3,738 / 3,811 / 3,832 / 3,845 / 3,868 /
// 3,829 / 3,791, every 6 or 8 with the roots at 1/3 3,885 / 3,893
// (profiles/r6/ab_results.md)
#ifndef RT_SPH_SEL
#define RT_SPH_SEL 0
#endif
#ifndef RT_SPH_CHK
#define RT_SPH_CHK 6
#endif
// One step of a lane's compact sphere-BVH walk in select form (RT_SPH_SEL).
__device__ __forceinline__ void sphere_step_sel(const uint4* __restrict__ ent, uint32_t& idx, uint32_t& leaf,
                                                float& pb, float& pdisc, const RayBox& rb, f3 o, f3 d,
                                                float a, float tmin, float best) {
    const uint4 e = ent[idx];
    const bool inner = (e.w & 0x80000000u) != 0u;
    const bool h = lds_node_hit_nf(e, rb, tmin, best);
    const f3 oc = o - f3{__uint_as_float(e.x), __uint_as_float(e.y), __uint_as_float(e.z)};
    const float bq = 2.0f * dot(oc, d);
    const float cc = dot(oc, oc) - __uint_as_float(e.w);
    const float disc = bq * bq - (4.0f * a) * cc;
    const bool park = !inner && disc > 0.0f;  // sph_test up to the discriminant (shaders_old.metal:108-136)
    leaf = park ? idx : leaf;
    pb = park ? bq : pb;
    pdisc = park ? disc : pdisc;
    idx = (inner && !h) ? (e.w & 0x7FFFFFFFu) : idx + 1;
}
// The same step with the kernel's branches (the shipped form).
__device__ __forceinline__ void sphere_step_br(const uint4* __restrict__ ent, uint32_t& idx, uint32_t& leaf,
                                               float& pb, float& pdisc, const RayBox& rb, f3 o, f3 d,
                                               float a, float tmin, float best) {
    const uint4 e = ent[idx];
    if (e.w & 0x80000000u) {
        idx = lds_node_hit_nf(e, rb, tmin, best) ? idx + 1 : (e.w & 0x7FFFFFFFu);
    } else {  // sph_test up to the discriminant (shaders_old.metal:108-136)
        const f3 oc = o - f3{__uint_as_float(e.x), __uint_as_float(e.y), __uint_as_float(e.z)};
        const float bq = 2.0f * dot(oc, d);
        const float cc = dot(oc, oc) - __uint_as_float(e.w);
        const float disc = bq * bq - (4.0f * a) * cc;
        if (disc > 0.0f) {
            leaf = idx;
            pb = bq;
            pdisc = disc;
        }
        idx = idx + 1;  // a leaf's escape is the next entry
    }
}
template <bool ANY>
__device__ __forceinline__ void sphere_walk(const uint4* __restrict__ ent, const uint16_t* __restrict__ ids,
                                            uint32_t nN, uint32_t nT, f3 o, f3 d, float tmin, float& best,
                                            int& id) {
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    const float a = dot(d, d);
    const RayBox rb = ray_box(o, d);
    // entry range of this lane's walk over the concatenated layouts
    uint32_t idx = octant(d) * nN;
    const uint32_t end = idx + nN;
    if (ANY && id >= 0) idx = end;
    uint32_t leaf = kNone;                      // the parked leaf
    float pb = 0.0f, pdisc = 0.0f;              // its b and discriminant
    [[maybe_unused]] constexpr int ST = ANY ? 24 : 16;
    RT_STAT(ST, 1);
    RT_STAT(ST + 1, __popcll(__ballot(1)));
    for (;;) {
        for (;;) {  // cheap steps until the lane parks a leaf or leaves its range
            const bool adv = idx < end && leaf == kNone;
            if (__builtin_amdgcn_ballot_w64(adv) == 0) break;
            RT_STAT(ST + 2, 1);
            RT_STAT(ST + 3, __popcll(__builtin_amdgcn_ballot_w64(adv)));
#if RT_SPH_SEL
            if (adv) sphere_step_sel(ent, idx, leaf, pb, pdisc, rb, o, d, a, tmin, best);
            if (false) {
#else
            if (adv) {
#endif
                const uint4 e = ent[idx];
                if (e.w & 0x80000000u) {
                    idx = lds_node_hit_nf(e, rb, tmin, best) ? idx + 1 : (e.w & 0x7FFFFFFFu);
                } else {  // sph_test up to the discriminant (shaders_old.metal:108-136)
                    const f3 oc = o - f3{__uint_as_float(e.x), __uint_as_float(e.y),
                                         __uint_as_float(e.z)};
                    const float bq = 2.0f * dot(oc, d);
                    const float cc = dot(oc, oc) - __uint_as_float(e.w);
                    const float disc = bq * bq - (4.0f * a) * cc;
                    if (disc > 0.0f) {
                        leaf = idx;
                        pb = bq;
                        pdisc = disc;
                    }
                    idx = idx + 1;  // a leaf's escape is the next entry
                }
            }
#if RT_SPH_CHK > 1
#pragma unroll
            for (int q = 1; q < RT_SPH_CHK; ++q) {  // more steps before the next check
                RT_STAT(ST + 2, 1);
                RT_STAT(ST + 3, __popcll(__builtin_amdgcn_ballot_w64(idx < end && leaf == kNone)));
                if (idx < end && leaf == kNone) {
                    if (RT_SPH_SEL)
                        sphere_step_sel(ent, idx, leaf, pb, pdisc, rb, o, d, a, tmin, best);
                    else
                        sphere_step_br(ent, idx, leaf, pb, pdisc, rb, o, d, a, tmin, best);
                }
            }
#endif
            const int parked = __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone));
            const int live = __popcll(__builtin_amdgcn_ballot_w64(idx < end || leaf != kNone));
            if (kSphParkDen * parked >= live) break;
        }
        if (__builtin_amdgcn_ballot_w64(leaf != kNone) == 0) break;
        RT_STAT(ST + 5, 1);
        RT_STAT(ST + 6, __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone)));
        if (leaf != kNone) {  // the roots of the parked leaves (sph_test)
            const float sq = sqrtf(pdisc);
            const float a2 = 2.0f * a;
            float t = (-pb - sq) / a2;
            if (!(t > tmin)) t = (-pb + sq) / a2;
            if (ANY) {
                if (t > tmin && t < best) {
                    id = 0;
                    idx = end;
                }
            } else if (t > tmin && t < 3.0e38f && t <= best) {
                const int s = (int)(nT + ids[leaf]);
                if (t < best || s < id) {
                    best = t;
                    id = s;
                }
            }
            leaf = kNone;
        }
    }
}

// Per-lane walk of the sphere BVH with LEAF BOXES (rt_scene.cpp
// build_sphere_box; RT_SPH_LEAFBOX): every entry is a near/far fp16 box -- a
// leaf's box is its padded sphere box, like any node's -- so every step of
// every lane is the same select-form box test (the compact walk above runs
// the box test and the discriminant side by side whenever a wave holds lanes
// at both kinds of entry, ~33 VALU a step).  A lane whose leaf box is hit
// parks the leaf; the parked lanes' spheres are tested with sph_test (the
// discriminant, then the IEEE roots) once they are >= 1/kSphBoxParkDen of the
// walkers, checked every kSphBoxChk steps.  Candidates are ranked by
// (t, sphere id) as in every walk: the brute-force answer.
// Config 4 (Msamples/s, profiles/r6/ab_results.md): the compact walk checked
// every step 3,512-3,520, every 6 steps 3,867-3,874; leaf boxes checked every
// 2 / 4 / 5 / 6 / 8 steps 3,883 / 4,018 / 4,027 / 4,042-4,044 / 4,037 with the
// roots at 1/3 (1/2 and 1/4 at every 6: 3,989 / 4,038); leaves of 2 / 3 / 4
// spheres 3,883 / 3,734 / 3,591
#ifndef RT_SPH_LEAFBOX
#define RT_SPH_LEAFBOX 1
#endif
#ifndef RT_SPH_BOX_PARK_DEN
#define RT_SPH_BOX_PARK_DEN 3
#endif
#ifndef RT_SPH_BOX_CHK
#define RT_SPH_BOX_CHK 6
#endif
template <bool ANY>
__device__ __forceinline__ void sphere_walk_box(const uint4* __restrict__ ent, const float4* __restrict__ sph,
                                                const uint32_t* __restrict__ perm, uint32_t nN, uint32_t nT, f3 o,
                                                f3 d, float tmin, float& best, int& id) {
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    const float a = dot(d, d);
    const RayBox rb = ray_box(o, d);
    uint32_t idx = octant(d) * nN;
    const uint32_t end = idx + nN;
    if (ANY && id >= 0) idx = end;
    uint32_t leaf = kNone;
    [[maybe_unused]] constexpr int ST = ANY ? 24 : 16;
    RT_STAT(ST, 1);
    RT_STAT(ST + 1, __popcll(__ballot(1)));
    for (;;) {
        for (;;) {
            if (__builtin_amdgcn_ballot_w64(idx < end && leaf == kNone) == 0) break;
#pragma unroll
            for (int q = 0; q < RT_SPH_BOX_CHK; ++q) {
                RT_STAT(ST + 2, 1);
                RT_STAT(ST + 3, __popcll(__builtin_amdgcn_ballot_w64(idx < end && leaf == kNone)));
                if (idx < end && leaf == kNone) {
                    const uint4 e = ent[idx];
                    const bool inner = (e.w & 0x80000000u) != 0u;
                    const bool h = lds_node_hit_nf(e, rb, tmin, best);
                    leaf = (h && !inner) ? e.w : leaf;
                    idx = (h || !inner) ? idx + 1 : (e.w & 0x7FFFFFFFu);
                }
            }
            const int parked = __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone));
            const int live = __popcll(__builtin_amdgcn_ballot_w64(idx < end || leaf != kNone));
            if (RT_SPH_BOX_PARK_DEN * parked >= live) break;
        }
        if (__builtin_amdgcn_ballot_w64(leaf != kNone) == 0) break;
        RT_STAT(ST + 5, 1);
        RT_STAT(ST + 6, __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone)));
        if (leaf != kNone) {  // the parked leaf's spheres (shaders_old.metal:108-136)
            const uint32_t first = leaf & 0xFFFFFFu, cnt = (leaf >> 24) + 1u;
            for (uint32_t k = first; k < first + cnt; ++k) {
                float t;
                if (ANY) {
                    if (sph_test(sph[k], o, d, a, tmin, best, &t)) {
                        id = 0;
                        idx = end;
                        break;
                    }
                } else if (sph_test(sph[k], o, d, a, tmin, 3.0e38f, &t) && t <= best) {
                    const int s = (int)(nT + perm[k]);
                    if (t < best || s < id) {
                        best = t;
                        id = s;
                    }
                }
            }
            leaf = kNone;
        }
    }
}

// Triangle-BVH walks over the compact entries (rt_scene.cpp build_tri_sah or
// rt_lbvh.hip, rt_gsah.hip: 16 B per node, fp16 near/far boxes rounded
// outward, one layout per direction octant, near child first): stackless
// depth-first walks with conservative boxes and (t, id) ranking (DESIGN.md
// §3.10).  A per-lane walk is in its own octant's layout and tests near/far
// (lds_node_hit_nf); the wave-packet walks below use the lane-0 layout for
// every lane and the min/max test, which does not depend on the slot order.

// A leaf of the triangle BVH: up to 128 consecutive triangles in leaf order,
// word = first | (count - 1) << 24 (build_tri_sah makes leaves of up to
// RTPT_TRI_LEAF; the LBVH leaves hold one).  Every triangle is tested with
// the exact test and ranked by (t, id).
__device__ __forceinline__ void tri_leaf_closest(const float4* __restrict__ tri, const uint32_t* __restrict__ perm,
                                                 uint32_t w, f3 o, f3 d, float tmin, float& best, int& id) {
    const uint32_t first = w & 0xFFFFFFu, cnt = (w >> 24) + 1u;
    for (uint32_t k = first; k < first + cnt; ++k) {
        float t;
        if (tri_test(tri[3 * k], tri[3 * k + 1], tri[3 * k + 2], o, d, tmin, 3.0e38f, &t) && t <= best) {
            const int tid = (int)perm[k];
            if (t < best || tid < id) {
                best = t;
                id = tid;
            }
        }
    }
}
__device__ __forceinline__ bool tri_leaf_any(const float4* __restrict__ tri, uint32_t w, f3 o, f3 d, float tmin,
                                             float tmax) {
    const uint32_t first = w & 0xFFFFFFu, cnt = (w >> 24) + 1u;
    bool found = false;
    for (uint32_t k = first; k < first + cnt && !found; ++k) {
        float t;
        found = tri_test(tri[3 * k], tri[3 * k + 1], tri[3 * k + 2], o, d, tmin, tmax, &t);
    }
    return found;
}

// Wave-packet walks for the coherent camera rays and bounce-0 shadow rays: the
// wave walks ONE path (the layout of its first lane's octant) and enters a node
// when any lane's box test passes; the node index is wave uniform.  A lane whose
// own test failed still tests the leaf's triangle, which cannot change its result.
__device__ __forceinline__ void tri_cbvh_closest_packet(const uint4* __restrict__ cn,
                                                        const float4* __restrict__ tri,
                                                        const uint32_t* __restrict__ perm, uint32_t nN,
                                                        f3 o, f3 d, float tmin, float& best, int& id) {
    const RayBox rb = ray_box(o, d);
    uint32_t idx = wave_uniform(octant(d)) * nN;
    const uint32_t end = idx + nN;
    RT_STAT(23, 1);  // packet walks (camera and bounce-0 shadow rays)
    while (idx < end) {
        RT_STAT(31, 1);
        const uint4 e = cn[idx];
        const bool inner = (e.w & 0x80000000u) != 0u;  // wave-uniform
        const bool h = lds_node_hit(e, rb, tmin, best);
        uint32_t next = idx + 1;
        if (__builtin_amdgcn_ballot_w64(h) == 0) {
            if (inner) next = e.w & 0x7FFFFFFFu;
        } else if (!inner) {
            tri_leaf_closest(tri, perm, e.w, o, d, tmin, best, id);
        }
        idx = wave_uniform(next);
    }
}

__device__ __forceinline__ bool tri_cbvh_any_packet(const uint4* __restrict__ cn,
                                                    const float4* __restrict__ tri, uint32_t nN, f3 o,
                                                    f3 d, float tmin, float tmax) {
    const RayBox rb = ray_box(o, d);
    uint32_t idx = wave_uniform(octant(d)) * nN;
    const uint32_t end = idx + nN;
    bool found = false;
    RT_STAT(23, 1);  // packet walks (camera and bounce-0 shadow rays)
    while (idx < end) {
        RT_STAT(31, 1);
        const uint4 e = cn[idx];
        const bool inner = (e.w & 0x80000000u) != 0u;
        const bool h = !found && lds_node_hit(e, rb, tmin, tmax);
        uint32_t next = idx + 1;
        if (__builtin_amdgcn_ballot_w64(h) == 0) {
            if (inner) next = e.w & 0x7FFFFFFFu;
        } else if (!inner) {
            found = found || tri_leaf_any(tri, e.w, o, d, tmin, tmax);
            if (__builtin_amdgcn_ballot_w64(!found) == 0) break;
        }
        idx = wave_uniform(next);
    }
    return found;
}

// Per-lane compact-BVH walks with POSTPONED LEAVES (as sphere_walk parks its
// roots): a lane whose box test passes at a leaf parks the leaf and
// stops; the others walk on until at least 1/kTriParkDen of the lanes
// still walking are parked, then the wave runs the triangle tests of all
// parked lanes together -- instead of every mixed step paying for the box
// test AND the three record loads and the test of a triangle.  Per lane the
// entries are visited in the same order and ranked by (t, id): the same result.
// the parked leaves are tested once they are >= 1/kTriParkDen of the live lanes
// (100k triangles: 1/4 738, 1/2 701, 3/4 570, 1/8 707 Msamples/s; round 5 with
// near/far boxes: 1/3 894-896, 1/4 887-890, 1/2 872, 1/6 865, 1/8 843; round 6
// with select-form steps checked every 4: 1/4 1,115, 1/3 1,111, 1/2 1,078)
#ifndef RT_TRI_PARK_DEN
#define RT_TRI_PARK_DEN 4
#endif
constexpr int kTriParkDen = RT_TRI_PARK_DEN;
// RT_TRI_LOOKAHEAD: the next sequential entry requested one step early
// (100k triangles 888 -> 787 Msamples/s: 4 more VGPRs, 20 spilled; off)
#ifndef RT_TRI_LOOKAHEAD
#define RT_TRI_LOOKAHEAD 0
#endif
// RT_TRI_SEL: the step's outcome by selects (no exec-mask branches around the
// box test); RT_TRI_CHK: steps between two checks of the parking condition
// (the two ballots, popcounts and compares of the check are a third of a
// step's instructions; a lane that parks in between holds still).  Round 6,
// 100k triangles (Msamples/s): branch form, check every step 988-990;
// selects 1,029; check every 2 steps 1,068; both: every 2 / 3 / 4 / 6 / 8
// steps 1,082-1,093 / 1,103 / 1,111 / 1,109 / 1,086 (profiles/r6/ab_results.md)
#ifndef RT_TRI_SEL
#define RT_TRI_SEL 1
#endif
#ifndef RT_TRI_CHK
#define RT_TRI_CHK 4
#endif
template <bool ANY>
__device__ __forceinline__ void tri_cbvh_walk(const uint4* __restrict__ cn, const float4* __restrict__ tri,
                                              const uint32_t* __restrict__ perm, uint32_t nN, f3 o, f3 d,
                                              float tmin, float& best, int& id) {
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    const RayBox rb = ray_box(o, d);
#if RT_TRI_ONE_LAYOUT  // experiment: every lane in the octant-0 layout (min/max box test)
    uint32_t idx = 0;
#else
    uint32_t idx = octant(d) * nN;
#endif
    const uint32_t end = idx + nN;
    if (ANY && id >= 0) idx = end;
    uint32_t leaf = kNone;
    [[maybe_unused]] constexpr int ST = ANY ? 24 : 16;  // the sphere_walk slots (no spheres here)
    RT_STAT(ST, 1);
    RT_STAT(ST + 1, __popcll(__ballot(1)));
#if RT_TRI_LOOKAHEAD
    // one entry of lookahead: `seq` is the entry after the current one, loaded
    // one step early, so a step that goes on to idx + 1 (a box hit, or a
    // missed leaf) finds its entry already requested
    const uint32_t last = end - 1u;
    uint4 cur = cn[idx < last ? idx : last];
    uint4 seq = cn[idx + 1u < last ? idx + 1u : last];
#endif
    for (;;) {
        for (;;) {
            const bool adv = idx < end && leaf == kNone;
            if (__builtin_amdgcn_ballot_w64(adv) == 0) break;
            RT_STAT(ST + 2, 1);
            RT_STAT(ST + 3, __popcll(__builtin_amdgcn_ballot_w64(adv)));
            if (adv) {
#if RT_TRI_LOOKAHEAD
                const uint4 e = cur;
                const bool inner = (e.w & 0x80000000u) != 0u;
                const bool h = lds_node_hit_nf(e, rb, tmin, best);
                if (h && !inner) leaf = e.w;
                if (h || !inner) {
                    idx = idx + 1u;
                    cur = seq;
                } else {
                    idx = e.w & 0x7FFFFFFFu;
                    cur = cn[idx < last ? idx : last];
                }
                seq = cn[idx + 1u < last ? idx + 1u : last];
#elif RT_TRI_SEL
                const uint4 e = cn[idx];
                const bool inner = (e.w & 0x80000000u) != 0u;
                const bool h = lds_node_hit_nf(e, rb, tmin, best);
                leaf = (h && !inner) ? e.w : leaf;
                idx = (h || !inner) ? idx + 1 : (e.w & 0x7FFFFFFFu);
#else
                const uint4 e = cn[idx];
                const bool inner = (e.w & 0x80000000u) != 0u;
#if RT_TRI_ONE_LAYOUT
                if (!lds_node_hit(e, rb, tmin, best)) {
#else
                if (!lds_node_hit_nf(e, rb, tmin, best)) {
#endif
                    idx = inner ? (e.w & 0x7FFFFFFFu) : idx + 1;
                } else {
                    if (!inner) leaf = e.w;
                    idx = idx + 1;
                }
#endif
            }
#if RT_TRI_CHK > 1
            // more steps before the next check (a parked lane holds still)
#pragma unroll
            for (int q = 1; q < RT_TRI_CHK; ++q) {
                RT_STAT(ST + 2, 1);
                RT_STAT(ST + 3, __popcll(__builtin_amdgcn_ballot_w64(idx < end && leaf == kNone)));
                if (idx < end && leaf == kNone) {
                    const uint4 e = cn[idx];
                    const bool inner = (e.w & 0x80000000u) != 0u;
                    const bool h = lds_node_hit_nf(e, rb, tmin, best);
                    leaf = (h && !inner) ? e.w : leaf;
                    idx = (h || !inner) ? idx + 1 : (e.w & 0x7FFFFFFFu);
                }
            }
#endif
            const int parked = __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone));
            const int live = __popcll(__builtin_amdgcn_ballot_w64(idx < end || leaf != kNone));
            if (kTriParkDen * parked >= live) break;
        }
        if (__builtin_amdgcn_ballot_w64(leaf != kNone) == 0) break;
        RT_STAT(ST + 5, 1);
        RT_STAT(ST + 6, __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone)));
        if (leaf != kNone) {
            if (ANY) {
                if (tri_leaf_any(tri, leaf, o, d, tmin, best)) {
                    id = 0;
                    idx = end;
                }
            } else {
                tri_leaf_closest(tri, perm, leaf, o, d, tmin, best, id);
            }
            leaf = kNone;
        }
    }
}

// ---- box clusters ------------------------------------------
// Candidate pairs of one ray among the clustered pairs: bit k set when pair k
// can hold an accepted hit with t in (tmin, tmax).  Per cluster: slab test of
// the padded box along its three axes ([Tlo, Thi], widened by a relative
// slack for the approximate rcp arithmetic), then a face is a candidate when
// its plane's interval [t_plane -/+ w] meets [Tlo, Thi] — in a box that is the
// face the ray enters through and the one it leaves through (two or three more
// near an edge or corner).  Only speed depends on the rounding here.
// SEG (shadow any-hit): a container cluster (flags bit 3: all axes world axes,
// a box with volume, e.g. the room) is skipped for the whole wave when every
// lane's segment [o, o + d*tmax] lies inside the box shrunk to more than the
// normal tolerance from each face plane: the box is convex, so the segment
// stays away from every face and no face can accept a hit.  The shrunk box
// is precomputed on the host into the container's unused axis slots.
template <bool SEG = false>
__device__ __forceinline__ uint32_t cluster_candidates(const SceneView& sv, f3 o, f3 d, float tmin,
                                                       float tmax) {
    constexpr float kEps = 1.52587890625e-05f;  // 2^-16 relative slack
    // containers the whole wave's segments stay inside (wave-uniform bit mask),
    // decided before the slab terms are live
    uint32_t skip = 0;
    if (SEG) {
        const f3 e = o + d * tmax;
        for (uint32_t c = 0; c < sv.nC; ++c) {
            const float4* r = sv.clu + kCluF4 * c;
            if (!(__float_as_uint(r[3].w) & 8u)) continue;
            // the shrunk box (rt_scene.cpp): face plane + tol_seg, with a 2^-20
            // relative slack for the rounding of o + d*tmax and of the bounds
            const float4 X = r[0], Y = r[1], Z = r[2];
            const bool inside = o.x > X.x && o.x < X.y && e.x > X.x && e.x < X.y &&
                                o.y > Y.x && o.y < Y.y && e.y > Y.x && e.y < Y.y &&
                                o.z > Z.x && o.z < Z.y && e.z > Z.x && e.z < Z.y;
            if (__builtin_amdgcn_ballot_w64(!inside) == 0) skip |= 1u << c;
        }
    }
    // per-ray terms of world-aligned box axes: t = lo * invd - o * invd
    const RayBox rb = ray_box(o, d);
    const float iv[3] = {rb.invd.x, rb.invd.y, rb.invd.z};
    const float oi[3] = {rb.oinv.x, rb.oinv.y, rb.oinv.z};
    uint32_t mask = 0;
    uint32_t c = 0;
    // the face masks: the cluster record's, or with the octant table the row of
    // this ray's octant, where world axes need no select (rt_scene.cpp clu_oct)
    const bool oct = RT_CLU_OCT && sv.clu_oct != nullptr;  // wave-uniform
    const uint32_t octant = (iv[0] < 0.0f ? 1u : 0u) | (iv[1] < 0.0f ? 2u : 0u) | (iv[2] < 0.0f ? 4u : 0u);
    const float4* mrow = oct ? sv.clu_oct + 2u * octant : sv.clu + 4;
    const uint32_t mstride = oct ? kCluOctF4 : kCluF4;
    for (; c < sv.nC; ++c) {
        if (SEG && ((skip >> c) & 1u)) continue;
        const float4* r = sv.clu + kCluF4 * c;
        const float4 H = r[3], W = r[6];
        const float4 M0 = mrow[mstride * c], M1 = mrow[mstride * c + 1];
        const uint32_t flags = __float_as_uint(H.w);
        if (flags & 16u) break;  // single-face clusters come last (rt_scene.cpp)
        const float hi[3] = {H.x, H.y, H.z}, wf[3] = {W.x, W.y, W.z};
        float en[3], ex[3], ida[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float4 A = r[a];
            float t0, t1;
            if (flags & (1u << a)) {  // wave-uniform
                ida[a] = iv[a];
                t0 = fmaf(A.w, iv[a], -oi[a]);
                t1 = fmaf(hi[a], iv[a], -oi[a]);
            } else {
                const float oa = dot(f3{A.x, A.y, A.z}, o), da = dot(f3{A.x, A.y, A.z}, d);
                ida[a] = safe_rcp(da);
                t0 = (A.w - oa) * ida[a];
                t1 = (hi[a] - oa) * ida[a];
            }
            en[a] = vmin(t0, t1);
            ex[a] = vmax(t0, t1);
        }
        const float tlo0 = vmax3(en[0], en[1], vmax(en[2], tmin));
        const float thi0 = vmin3(ex[0], ex[1], vmin(ex[2], tmax));
        const float tlo = fmaf(-kEps, fabsf(tlo0), tlo0), thi = fmaf(kEps, fabsf(thi0), thi0);  // kEps*|x| is exact: the same values
        if (!__builtin_amdgcn_ballot_w64(tlo <= thi)) continue;  // no lane meets the box
        const uint32_t m[6] = {__float_as_uint(M0.x), __float_as_uint(M0.y), __float_as_uint(M0.z),
                               __float_as_uint(M0.w), __float_as_uint(M1.x), __float_as_uint(M1.y)};
        uint32_t cm = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            // a ray with d_a >= 0 enters through the low face (slot 2a) and
            // leaves through the high one (2a + 1); the face plane lies
            // wf * |1/d_a| inside the padded slab, +- the tolerance
            uint32_t m_en = m[2 * a], m_ex = m[2 * a + 1];
            if (!(RT_CLU_OCT && oct && (flags & (1u << a)))) {  // wave-uniform
                const bool neg = ida[a] < 0.0f;
                m_en = neg ? m[2 * a + 1] : m[2 * a];
                m_ex = neg ? m[2 * a] : m[2 * a + 1];
            }
            const float wa = wf[a] * fabsf(ida[a]);
            cm |= (en[a] + fmaf(fabsf(en[a]), kEps, wa) >= tlo) ? m_en : 0u;
            cm |= (ex[a] - fmaf(fabsf(ex[a]), kEps, wa) <= thi) ? m_ex : 0u;
        }
        mask |= (tlo <= thi) ? cm : 0u;
    }
    // single-face clusters (the light, lone rectangles): the face is a
    // candidate whenever the padded box is hit (a superset of its face test)
    for (; c < sv.nC; ++c) {
        const float4* r = sv.clu + kCluF4 * c;
        const float4 A0 = r[0], A1 = r[1], A2 = r[2], H = r[3];
        const uint32_t flags = __float_as_uint(H.w);
        const float4 A[3] = {A0, A1, A2};
        const float hi[3] = {H.x, H.y, H.z};
        float tlo0 = tmin, thi0 = tmax;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float t0, t1;
            if (flags & (1u << a)) {  // wave-uniform
                t0 = fmaf(A[a].w, iv[a], -oi[a]);
                t1 = fmaf(hi[a], iv[a], -oi[a]);
            } else {
                const float oa = dot(f3{A[a].x, A[a].y, A[a].z}, o);
                const float ida = safe_rcp(dot(f3{A[a].x, A[a].y, A[a].z}, d));
                t0 = (A[a].w - oa) * ida;
                t1 = (hi[a] - oa) * ida;
            }
            tlo0 = vmax(tlo0, vmin(t0, t1));
            thi0 = vmin(thi0, vmax(t0, t1));
        }
        const float tlo = fmaf(-kEps, fabsf(tlo0), tlo0), thi = fmaf(kEps, fabsf(thi0), thi0);  // kEps*|x| is exact: the same values
        mask |= (tlo <= thi) ? __float_as_uint(r[5].z) : 0u;
    }
    return mask;
}

#ifndef RT_PAIR_SEL
#define RT_PAIR_SEL 0
#endif
// Exact pair test (the same arithmetic as the brute-force loops) with the
// hit ranked lexicographically by (t, triangle id): pairs are visited out of
// id order here, and (t, id) order is what the id-ordered scan with strict
// '<' computes.  ANY = shadow any-hit: *id becomes >= 0 on any accepted hit.
template <bool ANY>
__device__ __forceinline__ void pair_test_rank(const float4* r, uint32_t k, f3 o, f3 d, float tmin,
                                               float* best, int* id) {
    const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
    const PairDots q = pair_dots(r0, r1, r2, r3, r4, o, d);
    const bool pa = bary_ok(q.denA, q.a1, q.a2);
    const bool pb = bary_ok(q.denB, q.b1, q.b2);
#if RT_PAIR_SEL  // A/B: the first division by every lane, kept by selects (no exec branch)
    {
        const f3 nsel = pa ? f3{r2.y, r2.z, r2.w} : f3{r3.w, r4.x, r4.y};
        const float t = pair_t(nsel, q.tv, pa ? q.denA : q.denB);
        const int ia = (int)(pa ? 2 * k : 2 * k + 1);
        const bool take = (pa || pb) && t > tmin && (t < *best || (!ANY && t == *best && ia < *id));
        if (!ANY) *best = take ? t : *best;
        *id = take ? ia : *id;
    }
    if (pa && pb) {
        {
#else
    if (pa || pb) {
        const f3 nsel = pa ? f3{r2.y, r2.z, r2.w} : f3{r3.w, r4.x, r4.y};
        const float t = pair_t(nsel, q.tv, pa ? q.denA : q.denB);
        const int ia = (int)(pa ? 2 * k : 2 * k + 1);
        if (t > tmin && (t < *best || (!ANY && t == *best && ia < *id))) {
            if (!ANY) *best = t;
            *id = ia;
        }
        if (pa && pb) {
#endif
            const float t2 = pair_t(f3{r3.w, r4.x, r4.y}, q.tv, q.denB);
            const int ib = (int)(2 * k + 1);
            if (t2 > tmin && (t2 < *best || (!ANY && t2 == *best && ib < *id))) {
                if (!ANY) *best = t2;
                *id = ib;
            }
        }
    }
}

#ifndef RT_CLU_HELP
#define RT_CLU_HELP 0
#endif
// Position of the (r+1)-th set bit of a 64-bit mask (r < popcount).
__device__ __forceinline__ uint32_t select_bit64(uint64_t m, uint32_t r) {
    uint32_t pos = 0;
    uint32_t lo = (uint32_t)m;
    uint32_t c = (uint32_t)__builtin_popcount(lo);
    if (r >= c) {
        r -= c;
        pos = 32;
        lo = (uint32_t)(m >> 32);
    }
#pragma unroll
    for (uint32_t w = 16; w >= 1; w >>= 1) {
        c = (uint32_t)__builtin_popcount(lo & ((1u << w) - 1u));
        if (r >= c) {
            r -= c;
            pos += w;
            lo >>= w;
        }
    }
    return pos;
}

// Closest hit / any hit over the pair records with box clusters: the
// unclustered pairs by every lane (wave-uniform records, LDS broadcast), then
// each lane's own candidate pairs (per-lane LDS reads).  For ANY, *best is
// tmax and is not changed.
// SEG: skip containers the wave's segments [o, o + d*tmax] stay inside (any
// hit, and the MIS light queries: closest hits that only matter up to tmax).
template <bool ANY, bool SEG = ANY>
__device__ __forceinline__ void cluster_query(const SceneView& sv, f3 o, f3 d, float tmin,
                                              float* best, int* id) {
    for (uint32_t free = sv.pair_free; free != 0u; free &= free - 1u) {
        const uint32_t k = (uint32_t)__builtin_ctz(free);
        pair_test_rank<ANY>(sv.pair + kPairF4 * k, k, o, d, tmin, best, id);
    }
    uint32_t cand = cluster_candidates<SEG>(sv, o, d, tmin, *best);
    RT_STAT(12, 1);
    RT_STAT(15, __popcll(__ballot(1)));
#if RT_CLU_HELP
    // A/B variant: candidate-round compaction.  In
    // every round the lanes of the query with no candidate left help the
    // lanes with two or more: a helper pulls its owner's ray, best and
    // candidate mask (ds_bpermute), tests the owner's SECOND candidate while
    // the owner tests its first, and the owner merges the two (t, id)-ranked
    // results -- both started from the same (best, id), so their
    // lexicographic minimum is the result of testing both in any order.
    const uint32_t me = __lane_id();
    for (;;) {
        const bool want = cand != 0u && !(ANY && *id >= 0);
        if (__builtin_amdgcn_ballot_w64(want) == 0) break;
        const bool two = want && (cand & (cand - 1u)) != 0u;
        const uint64_t m2 = __builtin_amdgcn_ballot_w64(two);
        const uint64_t idle = __builtin_amdgcn_ballot_w64(!want);
        const uint32_t n2 = (uint32_t)__popcll(m2), ni = (uint32_t)__popcll(idle);
        uint32_t partner = me;
        bool helped = false, helping = false;
        if (two) {
            const uint32_t q = (uint32_t)__popcll(m2 & ((1ull << me) - 1ull));
            if (q < ni) {
                partner = select_bit64(idle, q);
                helped = true;
            }
        } else if (!want) {
            const uint32_t r = (uint32_t)__popcll(idle & ((1ull << me) - 1ull));
            if (r < n2) {
                partner = select_bit64(m2, r);
                helping = true;
            }
        }
        const f3 po{__shfl(o.x, (int)partner), __shfl(o.y, (int)partner), __shfl(o.z, (int)partner)};
        const f3 pd{__shfl(d.x, (int)partner), __shfl(d.y, (int)partner), __shfl(d.z, (int)partner)};
        const uint32_t pc = (uint32_t)__shfl((int)cand, (int)partner);
        const float ob = __shfl(*best, (int)partner);
        const int oid = __shfl(*id, (int)partner);
        float tb = helping ? ob : *best;  // a helper starts from its owner's (best, id)
        int tid = helping ? oid : *id;
        RT_STAT(13, 1);
        RT_STAT(14, __popcll(__ballot(want || helping)));
        if (want || helping) {
            const uint32_t k = (uint32_t)__builtin_ctz(helping ? (pc & (pc - 1u)) : cand);
            pair_test_rank<ANY>(sv.pair + kPairF4 * k, k, helping ? po : o, helping ? pd : d, tmin, &tb, &tid);
        }
        const float rb = __shfl(tb, (int)partner);
        const int rid = __shfl(tid, (int)partner);
        if (want) {
            cand &= cand - 1u;
            *best = tb;
            *id = tid;
            if (helped) {
                cand &= cand - 1u;
                if (ANY) {
                    if (rid >= 0) *id = rid;
                } else if (rb < *best || (rb == *best && rid < *id)) {
                    *best = rb;
                    *id = rid;
                }
            }
        }
    }
#else
    while (cand != 0u && !(ANY && *id >= 0)) {
        RT_STAT(13, 1);
        RT_STAT(14, __popcll(__ballot(1)));
        const uint32_t k = (uint32_t)__builtin_ctz(cand);
        cand &= cand - 1u;
        pair_test_rank<ANY>(sv.pair + kPairF4 * k, k, o, d, tmin, best, id);
    }
#endif
}

// closest hit, accept_any_intersection(false) (raytrace.metal:48-49).
// Primitives are tested in id order; a strictly smaller t wins (ties keep the
// lower id), exactly as the oracle.
// With CULL (used for coherent camera rays) a pair is skipped when no lane's
// box around its current candidate segment [o, o + d*best] touches the pair's
// padded AABB: any hit that could still win has t < best and lies inside it.
template <int GEO, bool SPH, bool CULL, int QT = 0>
__device__ __forceinline__ int closest_hit(const SceneView& sv, f3& o, f3& d, float tmin,
                                           float* t_io) {
    float best = *t_io;
    int id = -1;
    if (GEO == kGeoPairClu) {
        cluster_query<false>(sv, o, d, tmin, &best, &id);
    } else if (geo_pairs(GEO)) {
        f3 seg_lo, seg_hi;
        if (CULL) {
            const f3 e = o + d * best;
            seg_lo = f3{fminf(o.x, e.x), fminf(o.y, e.y), fminf(o.z, e.z)};
            seg_hi = f3{fmaxf(o.x, e.x), fmaxf(o.y, e.y), fmaxf(o.z, e.z)};
        }
        for (uint32_t k = 0; k < sv.nP; ++k) {
            const float4* r = sv.pair + kPairF4 * k;
            RT_STAT(4 * QT, 1);
            if (CULL) {
                const float4 b0 = r[5], b1 = r[6];
                const bool overlap = seg_lo.x <= b0.w && seg_hi.x >= b0.x && seg_lo.y <= b1.x &&
                                     seg_hi.y >= b0.y && seg_lo.z <= b1.y && seg_hi.z >= b0.z;
                if (!__any(overlap)) continue;
            }
            RT_STAT(4 * QT + 1, 1);
            RT_STAT(4 * QT + 2, __popcll(__ballot(1)));
            const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
            const PairDots q = pair_dots(r0, r1, r2, r3, r4, o, d);
            const bool pa = bary_ok(q.denA, q.a1, q.a2);
            const bool pb = bary_ok(q.denB, q.b1, q.b2);
            if (pa || pb) {
                RT_STAT(4 * QT + 3, 1);
                // One division for whichever of A, B the ray passes (A first);
                // a ray on the shared edge passes both and also runs B after.
                const f3 nsel = pa ? f3{r2.y, r2.z, r2.w} : f3{r3.w, r4.x, r4.y};
                const float t = pair_t(nsel, q.tv, pa ? q.denA : q.denB);
                if (t > tmin && t < best) {
                    best = t;
                    id = (int)(pa ? 2 * k : 2 * k + 1);
                }
                if (pa && pb) {
                    const float t2 = pair_t(f3{r3.w, r4.x, r4.y}, q.tv, q.denB);
                    if (t2 > tmin && t2 < best) {
                        best = t2;
                        id = (int)(2 * k + 1);
                    }
                }
                if (CULL) {
                    const f3 e = o + d * best;
                    seg_lo = f3{fminf(o.x, e.x), fminf(o.y, e.y), fminf(o.z, e.z)};
                    seg_hi = f3{fmaxf(o.x, e.x), fmaxf(o.y, e.y), fmaxf(o.z, e.z)};
                }
            }
        }
    } else if (GEO == kGeoTriBvh) {
        // camera rays: wave packets; bounce rays: per-lane walks with parked leaves
        if (CULL)
            tri_cbvh_closest_packet(sv.tnode, sv.tsorted, sv.tperm, sv.nTN, o, d, tmin,
                                    best, id);
        else
            tri_cbvh_walk<false>(sv.tnode, sv.tsorted, sv.tperm, sv.nTN, o, d, tmin,
                                 best, id);
    } else {
        for (uint32_t k = 0; k < sv.nT; ++k) {
            float t;
            if (tri_test(sv.tri[3 * k], sv.tri[3 * k + 1], sv.tri[3 * k + 2], o, d, tmin, best,
                         &t)) {
                best = t;
                id = (int)k;
            }
        }
    }
    if (SPH && GEO == kGeoSphLds && RT_SPH_LEAFBOX)
        sphere_walk_box<false>(sv.sbox, sv.sph, sv.sph_perm, sv.nSB, sv.nT, o, d, tmin, best, id);
    else if (SPH && GEO == kGeoSphLds)
        sphere_walk<false>(sv.sent, sv.sid, sv.nN, sv.nT, o, d, tmin, best, id);
    else if (SPH)
        sphere_closest(sv.node, sv.sph, sv.sph_perm, sv.nN, sv.nT, o, d, tmin, best, id);
    *t_io = best;
    return id;
}

// any hit, accept_any_intersection(true) (raytrace.metal:79-85).  The boolean
// result does not depend on the order of the tests.
// seg_lo/seg_hi bound every point the ray can accept (t in (tmin, tmax)); a
// pair whose padded AABB no lane's segment box touches cannot be hit by any
// lane of the wave and is skipped as a whole.
template <int GEO, bool SPH, bool PACKET>
__device__ __forceinline__ bool any_hit(const SceneView& sv, f3& o, f3& d, float tmin, float tmax,
                                        f3 seg_lo, f3 seg_hi) {
    if (GEO == kGeoPairClu) {
        float tm = tmax;
        int id = -1;
        cluster_query<true>(sv, o, d, tmin, &tm, &id);
        if (id >= 0) return true;
    } else if (geo_pairs(GEO)) {
        for (uint32_t k = 0; k < sv.nP; ++k) {
            const float4* r = sv.pair + kPairF4 * k;
            const float4 b0 = r[5], b1 = r[6];
            const bool overlap = seg_lo.x <= b0.w && seg_hi.x >= b0.x && seg_lo.y <= b1.x &&
                                 seg_hi.y >= b0.y && seg_lo.z <= b1.y && seg_hi.z >= b0.z;
            RT_STAT(8, 1);
            if (!__any(overlap)) continue;
            RT_STAT(9, 1);
            RT_STAT(10, __popcll(__ballot(1)));
            const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
            const PairDots q = pair_dots(r0, r1, r2, r3, r4, o, d);
            const bool pa = bary_ok(q.denA, q.a1, q.a2);
            const bool pb = bary_ok(q.denB, q.b1, q.b2);
            if (pa || pb) {
                RT_STAT(11, 1);
                const f3 nsel = pa ? f3{r2.y, r2.z, r2.w} : f3{r3.w, r4.x, r4.y};
                const float t = pair_t(nsel, q.tv, pa ? q.denA : q.denB);
                if (t > tmin && t < tmax) return true;
                if (pa && pb) {
                    const float t2 = pair_t(f3{r3.w, r4.x, r4.y}, q.tv, q.denB);
                    if (t2 > tmin && t2 < tmax) return true;
                }
            }
        }
    } else if (GEO == kGeoTriBvh) {
        if (PACKET) {  // bounce-0 shadow rays: wave packets
            if (tri_cbvh_any_packet(sv.tnode, sv.tsorted, sv.nTN, o, d, tmin, tmax))
                return true;
        } else {
            float tm = tmax;
            int hid = -1;
            tri_cbvh_walk<true>(sv.tnode, sv.tsorted, sv.tperm, sv.nTN, o, d, tmin,
                                tm, hid);
            if (hid >= 0) return true;
        }
    } else {
        for (uint32_t k = 0; k < sv.nT; ++k) {
            float t;
            if (tri_test(sv.tri[3 * k], sv.tri[3 * k + 1], sv.tri[3 * k + 2], o, d, tmin, tmax,
                         &t))
                return true;
        }
    }
    if (SPH && GEO == kGeoSphLds) {
        float tm = tmax;
        int id = -1;
        if (RT_SPH_LEAFBOX)
            sphere_walk_box<true>(sv.sbox, sv.sph, sv.sph_perm, sv.nSB, sv.nT, o, d, tmin, tm, id);
        else
            sphere_walk<true>(sv.sent, sv.sid, sv.nN, sv.nT, o, d, tmin, tm, id);
        return id >= 0;
    }
    if (SPH) return sphere_any(sv.node, sv.sph, sv.nN, o, d, tmin, tmax);
    return false;
}

// Fused queries of one bounce (pair layout, triangles only): the shadow any-hit
// of bounce b from p toward the light sample, and the closest hit of bounce
// b+1 from the same p along the new direction d2.  Both are evaluated pair by
// pair over ONE load of each record; every lane's two results are exactly
// those of any_hit and closest_hit (same tests, same order, same culling rule
// for the shadow segment), so the path's arithmetic is unchanged.
struct FusedHit {
    bool occluded;
    int id;     // closest hit of (p, d2), -1 if none
    float t;
};

__device__ __forceinline__ FusedHit fused_shadow_closest(const SceneView& sv, f3 p, f3 L,
                                                         float smax, f3 seg_lo, f3 seg_hi,
                                                         f3 d2) {
    FusedHit h{false, -1, 1000.0f};  // max_distance (sampling.metal:155)
    for (uint32_t k = 0; k < sv.nP; ++k) {
        const float4* r = sv.pair + kPairF4 * k;
        const float4 r0 = r[0], r1 = r[1], r2 = r[2], r3 = r[3], r4 = r[4];
        // shadow ray: segment-box cull, then the any-hit test for lanes still open
        const float4 b0 = r[5], b1 = r[6];
        const bool overlap = !h.occluded && seg_lo.x <= b0.w && seg_hi.x >= b0.x &&
                             seg_lo.y <= b1.x && seg_hi.y >= b0.y && seg_lo.z <= b1.y &&
                             seg_hi.z >= b0.z;
        if (__any(overlap)) {
            const PairDots q = pair_dots(r0, r1, r2, r3, r4, p, L);
            const bool pa = overlap && bary_ok(q.denA, q.a1, q.a2);
            const bool pb = overlap && bary_ok(q.denB, q.b1, q.b2);
            if (pa || pb) {
                const f3 nsel = pa ? f3{r2.y, r2.z, r2.w} : f3{r3.w, r4.x, r4.y};
                const float t = pair_t(nsel, q.tv, pa ? q.denA : q.denB);
                bool hit = t > 0.0f && t < smax;
                if (pa && pb && !hit) {
                    const float t2 = pair_t(f3{r3.w, r4.x, r4.y}, q.tv, q.denB);
                    hit = t2 > 0.0f && t2 < smax;
                }
                h.occluded = h.occluded || hit;
            }
        }
        // next-bounce closest hit (no culling: bounce rays are incoherent)
        const PairDots q = pair_dots(r0, r1, r2, r3, r4, p, d2);
        const bool pa = bary_ok(q.denA, q.a1, q.a2);
        const bool pb = bary_ok(q.denB, q.b1, q.b2);
        if (pa || pb) {
            const f3 nsel = pa ? f3{r2.y, r2.z, r2.w} : f3{r3.w, r4.x, r4.y};
            const float t = pair_t(nsel, q.tv, pa ? q.denA : q.denB);
            if (t > 0.001f && t < h.t) {
                h.t = t;
                h.id = (int)(pa ? 2 * k : 2 * k + 1);
            }
            if (pa && pb) {
                const float t2 = pair_t(f3{r3.w, r4.x, r4.y}, q.tv, q.denB);
                if (t2 > 0.001f && t2 < h.t) {
                    h.t = t2;
                    h.id = (int)(2 * k + 1);
                }
            }
        }
    }
    return h;
}

// Dual walk of the triangle BVH (A/B variant RT_TRI_DUAL, round 5): the
// shadow any-hit of bounce b (from p toward the light sample, A) and the
// closest hit of bounce b + 1 (from the same p along the next direction, B)
// are independent, so one loop walks both per lane, loading both rays' next
// entries before testing either: two dependent-load chains in flight per lane
// instead of one (the 100k-triangle walks wait on memory, not on issue).
// Each ray visits the same entries in the same order as tri_cbvh_walk and is
// ranked the same way: the same results.
__device__ __forceinline__ FusedHit tri_walk_dual(const SceneView& sv, f3 p, f3 dA, float tmaxA, bool litA, f3 dB) {
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    const uint4* __restrict__ cn = sv.tnode;
    const uint32_t nN = sv.nTN;
    const RayBox ra = ray_box(p, dA), rb = ray_box(p, dB);
    uint32_t ia = octant(dA) * nN;
    const uint32_t ea = ia + nN;
    if (!litA) ia = ea;
    uint32_t ib = octant(dB) * nN;
    const uint32_t eb = ib + nN;
    uint32_t la = kNone, lb = kNone;
    FusedHit h{false, -1, 1000.0f};  // max_distance (sampling.metal:155)
    for (;;) {
        for (;;) {
            const bool aa = ia < ea && la == kNone, ab = ib < eb && lb == kNone;
            if (__builtin_amdgcn_ballot_w64(aa || ab) == 0) break;
            // both entries requested before either is tested (clamped indices:
            // a finished ray re-reads an entry of its own layout, unused)
            const uint4 na = cn[aa ? ia : ea - 1u];
            const uint4 nb = cn[ab ? ib : eb - 1u];
            if (aa) {
                const bool inner = (na.w & 0x80000000u) != 0u;
                if (!lds_node_hit_nf(na, ra, 0.0f, tmaxA)) {
                    ia = inner ? (na.w & 0x7FFFFFFFu) : ia + 1;
                } else {
                    if (!inner) la = na.w;
                    ia = ia + 1;
                }
            }
            if (ab) {
                const bool inner = (nb.w & 0x80000000u) != 0u;
                if (!lds_node_hit_nf(nb, rb, 0.001f, h.t)) {
                    ib = inner ? (nb.w & 0x7FFFFFFFu) : ib + 1;
                } else {
                    if (!inner) lb = nb.w;
                    ib = ib + 1;
                }
            }
            const int parked = __popcll(__builtin_amdgcn_ballot_w64(la != kNone)) +
                               __popcll(__builtin_amdgcn_ballot_w64(lb != kNone));
            const int live = __popcll(__builtin_amdgcn_ballot_w64(ia < ea || la != kNone)) +
                             __popcll(__builtin_amdgcn_ballot_w64(ib < eb || lb != kNone));
            if (kTriParkDen * parked >= live) break;
        }
        if (__builtin_amdgcn_ballot_w64(la != kNone || lb != kNone) == 0) break;
        if (la != kNone) {
            if (tri_leaf_any(sv.tsorted, la, p, dA, 0.0f, tmaxA)) {
                h.occluded = true;
                ia = ea;
            }
            la = kNone;
        }
        if (lb != kNone) {
            tri_leaf_closest(sv.tsorted, sv.tperm, lb, p, dB, 0.001f, h.t, h.id);
            lb = kNone;
        }
    }
    return h;
}

}  // namespace
}  // namespace rt

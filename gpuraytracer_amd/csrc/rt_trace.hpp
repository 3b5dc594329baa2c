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
#ifdef RT_TIMING_APPROX_DIV  // timing-only experiment, NOT bit-exact
    return tn * __builtin_amdgcn_rcpf(fabsf(den));
#else
    return tn / fabsf(den);
#endif
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

// Diagnostic counters (only in an -DRT_STATS build; read with rt_debug_stats).
// Slot groups of 4 per query kind q (0: camera closest hit, 1: bounce closest
// hit, 2: shadow any-hit): [4q] pair records visited per wave, [4q+1] records
// tested, [4q+2] active lanes summed over tested records, [4q+3] division blocks.
// Box-cluster queries: [12] queries per wave, [13] candidate rounds per wave,
// [14] lanes summed over rounds, [15] lanes summed over queries.
// Sphere walks (sphere_walk_lds), base 16 closest / 24 any-hit: [+0] walks per
// wave, [+1] lanes summed over walks, [+2] cheap-step iterations, [+3] lanes
// summed over them, [+4] unused, [+5] root rounds, [+6] parked lanes summed
// over them.  [23] packet walks, [31] packet walk iterations.
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
    kGeoSphLds = 7,     // pair records + the compact sphere BVH in LDS (1024-thread workgroups)
};

constexpr bool geo_pairs(int g) { return g == kGeoPairLds || g == kGeoPairSmem || g == kGeoSphLds; }

struct SceneView {
    const float4* tri;        // 3 float4 per triangle (single layout)
    const float4* pair;       // kPairF4 float4 per triangle pair (pair layout)
    const float4* sph;        // 1 float4 per sphere, BVH leaf order
    const float4* node;       // 2 float4 per sphere-BVH node
    const uint32_t* sph_perm; // leaf order -> sphere id (global memory)
    const float4* tnode;      // triangle BVH: 8 octant layouts of nTN nodes
    const float4* tsorted;    // 3 float4 per triangle, BVH leaf order
    const uint32_t* tperm;    // leaf order -> triangle id
    uint32_t nTN;
    uint32_t nT, nP, nS, nN;
    const float4* clu;        // box clusters, 4 float4 each (kGeoPairClu)
    uint32_t nC;
    uint32_t pair_free;       // pairs in no cluster: tested by every lane
    const float* htab;        // Halton low-digit tables in LDS (kGeoPairClu)
    const uint4* sent;        // compact sphere BVH entries in LDS (kGeoSphLds), 2 layouts
    const uint16_t* sid;      // sphere id of each entry (leaves): LDS, or global with RT_SPH_SPLIT
    uint8_t* wscr;            // this wave's LDS scratch for split walks (kWaveScratchBytes)
    uint8_t* pool;            // the workgroup's walk pool in LDS (RT_SPH_POOL, sphere_pool_bytes)
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
#ifndef RT_ASM_MINMAX
#define RT_ASM_MINMAX 1
#endif
__device__ __forceinline__ float vmin(float a, float b) {
#if RT_ASM_MINMAX
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fminf(a, b);
#endif
}
__device__ __forceinline__ float vmax(float a, float b) {
#if RT_ASM_MINMAX
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return fmaxf(a, b);
#endif
}
__device__ __forceinline__ float vmin3(float a, float b, float c) {
#if RT_ASM_MINMAX
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return fminf(fminf(a, b), c);
#endif
}
__device__ __forceinline__ float vmax3(float a, float b, float c) {
#if RT_ASM_MINMAX
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return fmaxf(fmaxf(a, b), c);
#endif
}

// Per-ray data of the slab test.  1/d uses the 1-ulp hardware reciprocal: the
// node boxes carry the culling margin, so only speed depends on its rounding.
struct RayBox {
    f3 invd, oinv;
};

__device__ __forceinline__ float safe_rcp(float v) {
    return __builtin_amdgcn_rcpf(fabsf(v) < 1e-20f ? copysignf(1e-20f, v) : v);
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

#ifndef RT_SPH_PACKET
// sphere scenes: 1: wave-packet walks for camera and bounce-0 shadow rays;
// 2: + all shadow rays; 3: all; 0 (round 3): per-lane walks for every ray --
// with the near/far L2 tree and one-wave workgroups 155.8 vs 158.4 ms on
// config 4.  (Triangle-BVH scenes keep packets for bounce-0 shadow rays.)
#define RT_SPH_PACKET 0
#endif

// BVH layout of a ray direction: bit a set when component a is negative.
__device__ __forceinline__ uint32_t octant(f3 d) {
    return (__float_as_uint(d.x) >> 31) | ((__float_as_uint(d.y) >> 31) << 1) |
           ((__float_as_uint(d.z) >> 31) << 2);
}

__device__ __forceinline__ uint32_t wave_uniform(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// Sphere-BVH walks.  The wave walks ONE stackless
// depth-first path through the escape-index tree: a node is entered when any
// active lane's ray may hit its padded box.  The node index is therefore wave
// uniform, node and sphere records are fetched with scalar loads from global
// memory (no LDS footprint, no bank conflicts) and every lane stays busy; a
// lane whose own box test failed still tests the leaf's spheres, which cannot
// change its result because the boxes are conservative.
template <bool PACKET>
__device__ __forceinline__ void sphere_closest(const float4* __restrict__ node,
                                               const float4* __restrict__ sph,
                                               const uint32_t* __restrict__ perm, uint32_t nN,
                                               uint32_t nT, f3 o, f3 d, float tmin, float& best,
                                               int& id) {
    // Candidates are ranked by (t, sphere id) exactly like the oracle's
    // id-ordered scan with strict '<', so the visiting order is free.
    const float a = dot(d, d);
    const RayBox rb = ray_box(o, d);
    node += 2u * nN * (PACKET ? wave_uniform(octant(d)) : octant(d));
    uint32_t idx = 0;
    while (idx < nN) {
        const float4 n0 = node[2 * idx], n1 = node[2 * idx + 1];
        uint32_t next = PACKET ? wave_uniform(__float_as_uint(n0.w)) : __float_as_uint(n0.w);
        const bool h = node_hit(n0, n1, rb, tmin, best);
        if (PACKET ? __builtin_amdgcn_ballot_w64(h) != 0 : h) {
            const uint32_t leaf = PACKET ? wave_uniform(__float_as_uint(n1.w)) : __float_as_uint(n1.w);
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

template <bool PACKET>
__device__ __forceinline__ bool sphere_any(const float4* __restrict__ node,
                                           const float4* __restrict__ sph, uint32_t nN, f3 o,
                                           f3 d, float tmin, float tmax) {
    const float a = dot(d, d);
    const RayBox rb = ray_box(o, d);
    node += 2u * nN * (PACKET ? wave_uniform(octant(d)) : octant(d));
    bool found = false;
    uint32_t idx = 0;
    while (idx < nN) {
        const float4 n0 = node[2 * idx], n1 = node[2 * idx + 1];
        if (PACKET) {
            uint32_t next = wave_uniform(__float_as_uint(n0.w));
            if (__builtin_amdgcn_ballot_w64(!found && node_hit(n0, n1, rb, tmin, tmax)) != 0) {
                const uint32_t leaf = wave_uniform(__float_as_uint(n1.w));
                if (leaf == 0u) {
                    next = idx + 1;
                } else {
                    const uint32_t first = leaf & 0xFFFFFFu, end = first + (leaf >> 24);
                    for (uint32_t k = first; k < end; ++k) {
                        float t;
                        found = found || sph_test(sph[k], o, d, a, tmin, tmax, &t);
                    }
                    if (__builtin_amdgcn_ballot_w64(!found) == 0) break;
                }
            }
            idx = next;
        } else {
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
    }
    return found;
}

// Sphere-BVH walks over the compact LDS entries (rt_scene.cpp build_sphere_lds):
// the same stackless depth-first walk and (t, id) ranking as sphere_closest /
// sphere_any, with fp16 boxes rounded outward (still conservative) and the
// sphere of a leaf stored in the entry itself (a leaf's escape is the next
// entry).  Two layouts: near child first for (+,+,+) and for (-,-,-); a ray
// takes the one matching most of its direction signs.
__device__ __forceinline__ float h2f(uint32_t b16) {
    return (float)__builtin_bit_cast(_Float16, (uint16_t)b16);
}

__device__ __forceinline__ uint32_t lds_layout(f3 d) {
#ifdef RT_SPH_ONE_LAYOUT  // experiment: every ray walks layout (+,+,+) (speed only)
    return 0u;
#endif
    return __builtin_popcount(octant(d)) >= 2 ? 1u : 0u;
}
// layout of the compact sphere BVH a ray walks (RT_SPH_LAYOUTS)
__device__ __forceinline__ uint32_t sph_layout(f3 d) { return RT_SPH_LAYOUTS == 8 ? octant(d) : lds_layout(d); }

__device__ __forceinline__ bool lds_node_hit(const uint4& e, const RayBox& rb, float tmin,
                                             float tmax) {
    const float4 n0 = make_float4(h2f(e.x & 0xFFFFu), h2f(e.x >> 16), h2f(e.y & 0xFFFFu), 0.0f);
    const float4 n1 = make_float4(h2f(e.y >> 16), h2f(e.z & 0xFFFFu), h2f(e.z >> 16), 0.0f);
    return node_hit(n0, n1, rb, tmin, tmax);
}

// Slab test of a near/far entry (RT_SPH_NEARFAR): the lo slots hold the planes
// the ray enters through, which holds for every ray whose direction octant is
// the layout's.  Equal to lds_node_hit for such rays: fma(p, invd, -oinv) is
// monotone in p and sign(invd) orders the two planes of each axis, so the
// min/max pairs of node_hit select exactly these values.
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

template <bool PACKET>
__device__ __forceinline__ void sphere_closest_lds(const uint4* ent, const uint16_t* ids,
                                                   uint32_t nN, uint32_t nT, f3 o, f3 d,
                                                   float tmin, float& best, int& id) {
    const float a = dot(d, d);
    const RayBox rb = ray_box(o, d);
    const uint32_t lay = PACKET ? wave_uniform(sph_layout(d)) : sph_layout(d);
    // entry indices (and escapes) run over both layouts: layout `lay` is
    // [lay * nN, (lay + 1) * nN)
    uint32_t idx = lay * nN;
    const uint32_t end = idx + nN;
    if (PACKET) RT_STAT(23, 1);
    while (idx < end) {
        if (PACKET) RT_STAT(31, 1);
        const uint4 e = ent[idx];
        uint32_t next = idx + 1;
        if (e.w & 0x80000000u) {  // inner node (wave-uniform for PACKET)
            const bool h = lds_node_hit(e, rb, tmin, best);
            if (PACKET ? __builtin_amdgcn_ballot_w64(h) == 0 : !h) next = e.w & 0x7FFFFFFFu;
        } else {  // leaf: the sphere (c, r*r)
            float t;
            if (sph_test(make_float4(__uint_as_float(e.x), __uint_as_float(e.y),
                                     __uint_as_float(e.z), __uint_as_float(e.w)),
                         o, d, a, tmin, 3.0e38f, &t) && t <= best) {
                const int s = (int)(nT + ids[idx]);
                if (t < best || s < id) {
                    best = t;
                    id = s;
                }
            }
        }
        idx = PACKET ? wave_uniform(next) : next;
    }
}

// Per-lane walk of the compact LDS BVH with POSTPONED ROOTS (DESIGN.md §3.10;
// after Aila & Laine's postponed leaf processing, stackless form).  Each step
// of a lane is cheap and of similar cost whatever the entry: a box test for an
// inner node, the discriminant of sph_test for a leaf.  A leaf whose
// discriminant is positive (a real hit candidate) parks the lane with (b, disc);
// the others walk on until at least half of the lanes still walking are
// parked (or none can move), then the wave runs the expensive part of the
// sphere test -- the IEEE sqrt and divisions -- for all parked lanes together.
// In the plain walk (sphere_closest_lds) a mixed wave pays for the box test,
// the discriminant AND the roots in most steps.  Per lane the entries are
// visited in the same order and every value is sph_test's, ranked by (t, id):
// the same result.  ANY: *id becomes >= 0 on the first accepted hit (and that
// lane stops).
//
// SPLIT: a wave no longer waits with idle lanes for its
// longest walk.  A walk is a range [idx, end) of the depth-first entry order
// (stackless: walking from any entry m to end visits everything of the
// subtrees from m on that the full walk would, plus possibly more).  When at
// least RT_SPH_SPLIT_MIN lanes of the wave have finished, every walking lane
// offers the rest of its range after the current subtree ([escape, end); or
// after the first child when the subtree is all that is left), and the k-th
// idle lane takes the k-th offer: it pulls the ray, the running (best, id) and
// the range through cross-lane reads (ds_bpermute), the giver keeps
// [idx, split).  Takers may be split again.  At the end every lane delivers
// its (t, id) to the walk's original lane with an LDS atomic min of the key
// (t bits << 32 | id + 1) -- exactly the (t, id) ranking, since every t here
// is positive -- and every lane reads back its own query's result.  Extra
// entries visited by a split walk can only add candidates that are real hits
// in (tmin, tmax), so the minimum is the brute-force one.
#ifndef RT_SPH_PARK_DEN
#define RT_SPH_PARK_DEN 2  // the parked roots run once they are >= 1/DEN of the live lanes (L2 tree: 2 157.3 ms, 4 158.4, 6 161.1)
#endif
#ifndef RT_SPH_SPLIT_CLOSEST_ONLY
#define RT_SPH_SPLIT_CLOSEST_ONLY 0  // 1: shadow (any-hit) walks are not split
#endif
#ifndef RT_SPH_SPLIT_MIN
#define RT_SPH_SPLIT_MIN 16  // idle lanes of a wave that trigger a split round
#endif
__device__ __forceinline__ unsigned long long walk_key(float best, int id) {
    return ((unsigned long long)__float_as_uint(best) << 32) | (uint32_t)(id + 1);
}

template <bool ANY, bool SPLIT>
__device__ __forceinline__ void sphere_walk_lds(const uint4* ent, const uint16_t* ids, uint32_t nN,
                                                uint32_t nT, f3 o, f3 d, float tmin, float& best,
                                                int& id, uint8_t* wscr) {
    constexpr uint32_t kNone = 0xFFFFFFFFu;
#ifdef RT_TIMING_NO_SPH_WALK  // timing-only experiment (share of the walks), NOT exact
    return;
#endif
#ifdef RT_TIMING_NO_SPH_ANY  // timing-only: share of the per-lane shadow walks, NOT exact
    if (ANY) return;
#endif
#ifdef RT_TIMING_NO_SPH_CLOSEST  // timing-only: share of the per-lane closest walks, NOT exact
    if (!ANY) return;
#endif
    float a = dot(d, d);
    RayBox rb = ray_box(o, d);
    // entry range of this lane's walk over the concatenated layouts
    uint32_t idx = sph_layout(d) * nN;
    uint32_t end = idx + nN;
    if (ANY && id >= 0) idx = end;
    uint32_t leaf = kNone;                      // the parked leaf
    float pb = 0.0f, pdisc = 0.0f;              // its b and discriminant
    [[maybe_unused]] const uint32_t lane = __lane_id();
    [[maybe_unused]] uint32_t owner = lane;     // lane whose query this walk serves
    [[maybe_unused]] bool split_any = false;    // wave-uniform
    // the wave scratch as LDS pointers (a generic pointer would become flat
    // accesses): rank map [64] bytes, then 64 result keys
    typedef __attribute__((address_space(3))) uint8_t lds_u8;
    typedef __attribute__((address_space(3))) unsigned long long lds_u64;
    lds_u8* rank_map = (lds_u8*)wscr;
    lds_u64* res = (lds_u64*)(wscr + 64);
    [[maybe_unused]] const int n_exec = __popcll(__builtin_amdgcn_ballot_w64(true));
    // split when RT_SPH_SPLIT_MIN more lanes are idle than the last round
    // left without work (no offer for them): a wave whose remaining walks
    // cannot be split any more does not retry every step
    [[maybe_unused]] int split_at = RT_SPH_SPLIT_MIN;  // wave-uniform
    [[maybe_unused]] constexpr int ST = ANY ? 24 : 16;
    RT_STAT(ST, 1);
    RT_STAT(ST + 1, __popcll(__ballot(1)));
    for (;;) {
        for (;;) {  // cheap steps until the lane parks a leaf or leaves its range
            const bool adv = idx < end && leaf == kNone;
            if (__builtin_amdgcn_ballot_w64(adv) == 0) break;
            RT_STAT(ST + 2, 1);
            RT_STAT(ST + 3, __popcll(__builtin_amdgcn_ballot_w64(adv)));
            if (adv) {
                const uint4 e = ent[idx];
                if (e.w & 0x80000000u) {
                    const bool h = RT_SPH_NEARFAR && !SPLIT ? lds_node_hit_nf(e, rb, tmin, best)
                                                            : lds_node_hit(e, rb, tmin, best);
                    idx = h ? idx + 1 : (e.w & 0x7FFFFFFFu);
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
            const int parked = __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone));
            const int live = __popcll(__builtin_amdgcn_ballot_w64(idx < end || leaf != kNone));
            if (RT_SPH_PARK_DEN * parked >= live) break;
            if constexpr (SPLIT) {
                if (n_exec - live >= split_at) {  // lanes with nothing to walk
                    RT_STAT(ST + 4, 1);
                    const bool idle = idx >= end && leaf == kNone;
                    const unsigned long long idle_m = __builtin_amdgcn_ballot_w64(idle);
                    if (!split_any) {  // first split of this walk: empty result slots
                        res[lane] = ANY ? 0ull : ~0ull;
                        split_any = true;
                    }
                    // offer: the part of the range after the current subtree
                    uint32_t m = end;
                    if (idx < end && leaf == kNone) {
                        const uint4 e = ent[idx];
                        if (e.w & 0x80000000u) {
                            const uint32_t esc = e.w & 0x7FFFFFFFu;
                            if (esc < end) {
                                m = esc;
                            } else {  // the subtree is all that is left: offer its 2nd child on
                                const uint32_t w1 = ent[idx + 1].w;
                                m = (w1 & 0x80000000u) ? (w1 & 0x7FFFFFFFu) : idx + 2;
                            }
                        } else {
                            m = idx + 1;
                        }
                    }
                    const bool can = m < end;
                    const unsigned long long can_m = __builtin_amdgcn_ballot_w64(can);
                    const uint32_t n = (uint32_t)min(__popcll(can_m), __popcll(idle_m));
                    const uint32_t rc = __builtin_amdgcn_mbcnt_hi((uint32_t)(can_m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)can_m, 0u));
                    const uint32_t ri = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle_m >> 32),
                                                                  __builtin_amdgcn_mbcnt_lo((uint32_t)idle_m, 0u));
                    const bool giver = can && rc < n;
                    const bool taker = idle && ri < n;
                    split_at = (__popcll(idle_m) - (int)n) + RT_SPH_SPLIT_MIN;
                    if (giver) rank_map[rc] = (uint8_t)lane;
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    const int src = taker ? (int)rank_map[ri] : (int)lane;
                    // the taker's finished query result goes to its query's lane
                    if (taker) {
                        if (ANY)
                            __hip_atomic_fetch_max(&res[owner], id >= 0 ? 1ull : 0ull, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
                        else
                            __hip_atomic_fetch_min(&res[owner], walk_key(best, id), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
                    }
                    // the giver's ray, running (best, id), split point, range end
                    // and query lane (two 16-bit fields per word where they fit)
                    const f3 o2{__shfl(o.x, src), __shfl(o.y, src), __shfl(o.z, src)};
                    const f3 d2{__shfl(d.x, src), __shfl(d.y, src), __shfl(d.z, src)};
                    const float best2 = __shfl(best, src);
                    const uint32_t range2 = (uint32_t)__shfl((int)(m | (end << 16)), src);
                    const uint32_t who2 = (uint32_t)__shfl((int)(owner | ((uint32_t)(id + 1) << 8)), src);
                    if (taker) {
                        o = o2;
                        d = d2;
                        a = dot(d, d);
                        rb = ray_box(o, d);
                        best = best2;
                        id = (int)(who2 >> 8) - 1;
                        idx = range2 & 0xFFFFu;
                        end = range2 >> 16;
                        owner = who2 & 0xFFu;
                    }
                    if (giver) end = m;
                }
            }
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
    if constexpr (SPLIT) {
        if (split_any) {  // every walk's (t, id) to its query's lane; read back this lane's own
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (ANY)
                __hip_atomic_fetch_max(&res[owner], id >= 0 ? 1ull : 0ull, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WAVEFRONT);
            else
                __hip_atomic_fetch_min(&res[owner], walk_key(best, id), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WAVEFRONT);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const unsigned long long k = res[lane];
            if (ANY) {
                id = k ? 0 : -1;
            } else {
                best = __uint_as_float((uint32_t)(k >> 32));
                id = (int)(uint32_t)k - 1;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Workgroup walk pool (RT_SPH_POOL).  A wave's per-lane walks
// take as long as its longest one (a lane walks ~38 entries, its wave ~103):
// the lanes that finish early idle.  Here every lane's query sits in its own
// LDS slot; once at most RT_SPH_POOL_T walks of a wave are left, the wave hands
// them to the workgroup's pool (slot state + a bit in its `ready` mask) and
// its idle lanes -- like those of every wave of the workgroup that has handed
// over -- claim handed-over walks, of any wave and of either kind, and walk
// them to the end.  The result goes back to the query's slot (and a bit in
// the owner's `done` mask); every lane finally reads its own query back.
// Packing the tails of 16 waves into few dense waves is the point: the
// waiting waves issue nothing (s_sleep) and leave their SIMD to others.
//
// Exactness: a walk is the same sequence of entries and the same arithmetic
// whichever lane runs it (the ray, running best and entry index travel
// bit-exactly through LDS; a and the slab constants are recomputed from d
// by the same code), so results are those of sphere_walk_lds.  tmin of a
// pooled walk is implied by its kind: 0 for shadow (any-hit) walks
// (raytrace.metal:79-85 leaves min_distance at 0) and 1e-3 for closest walks
// (sampling.metal:154) -- the only two queries of the path.  The box tests
// use tmin 0 for both (a superset of the entries: conservative).
//
// Liveness: a claimed walk always ends (entry indices only grow), a wave
// never leaves the walk while it holds claimed walks, and a wave waiting for
// its own handed-over walks claims them itself when nobody else has.
#ifndef RT_SPH_POOL_T
#define RT_SPH_POOL_T 16      // hand over once <= T walks of the wave are left
#endif
#ifndef RT_SPH_POOL_REFILL
#define RT_SPH_POOL_REFILL 8  // idle lanes (beyond the last claim) that trigger another claim
#endif

typedef __attribute__((address_space(3))) float4 lds_f4_t;
typedef __attribute__((address_space(3))) float lds_f32_t;
typedef __attribute__((address_space(3))) uint32_t lds_u32_t;
typedef __attribute__((address_space(3))) unsigned long long lds_u64_t;

struct PoolView {
    lds_f4_t* a;      // [NT] o, best
    lds_f4_t* b;      // [NT] d, entry index (bits)
    lds_u32_t* c;     // [NT] id + 1 | any-hit << 31
    lds_u64_t* ready; // [NW] handed-over walks not claimed yet (bit = lane)
    lds_u64_t* done;  // [NW] handed-over walks finished
    lds_u32_t* sum;   // waves with ready walks (bit = wave)
};

template <uint32_t NT>
__device__ __forceinline__ PoolView pool_view(uint8_t* base) {
    typedef __attribute__((address_space(3))) uint8_t lds_u8_t;
    lds_u8_t* p = (lds_u8_t*)base;
    PoolView v;
    v.a = (lds_f4_t*)p;
    v.b = (lds_f4_t*)(p + 16u * NT);
    v.c = (lds_u32_t*)(p + 32u * NT);
    v.ready = (lds_u64_t*)(p + 36u * NT);
    v.done = (lds_u64_t*)(p + 36u * NT + 8u * (NT / 64u));
    v.sum = (lds_u32_t*)(p + 36u * NT + 16u * (NT / 64u));
    return v;
}

// Zero the masks (every thread of the workgroup calls it before the first
// __syncthreads of the kernel).
template <uint32_t NT>
__device__ __forceinline__ void pool_init(uint8_t* base, uint32_t tid) {
#if defined(__HIP_DEVICE_COMPILE__)
    const PoolView v = pool_view<NT>(base);
    if (tid < NT / 64u) {
        v.ready[tid] = 0ull;
        v.done[tid] = 0ull;
    }
    if (tid == 0) *v.sum = 0u;
#endif
}

// Claim handed-over walks for the idle lanes (`idle`, wave-uniform).  Returns,
// per lane, the claimed slot or 0xFFFFFFFF.  Own wave first (liveness), then
// the waves the summary names.  Called by the whole wave (uniform control).
template <uint32_t NT>
__device__ __forceinline__ uint32_t pool_claim(const PoolView& v, uint32_t wave, bool own_first,
                                               unsigned long long idle) {
    uint32_t got = 0xFFFFFFFFu;
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr uint32_t NW = NT / 64u;
    uint32_t cand = __hip_atomic_load(v.sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    cand = wave_uniform(cand);
    if (own_first) cand |= 1u << wave;
    // rotate so the scan starts at this wave
    cand = ((cand >> wave) | (cand << ((NW - wave) % NW))) & ((1u << NW) - 1u);
    while (cand != 0u && idle != 0ull) {
        const uint32_t k = (uint32_t)__builtin_ctz(cand);
        cand &= cand - 1u;
        const uint32_t w = (wave + k) % NW;
        // take at most as many walks as there are idle lanes: the lowest bits
        const uint32_t n_idle = (uint32_t)__popcll(idle);
        unsigned long long want = ~0ull;
        {
            unsigned long long r = __hip_atomic_load(&v.ready[w], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
            r = ((unsigned long long)wave_uniform((uint32_t)(r >> 32)) << 32) | wave_uniform((uint32_t)r);
            if (r == 0ull) continue;
            want = r;
            while ((uint32_t)__popcll(want) > n_idle) want &= ~(1ull << (63 - __builtin_clzll(want)));
        }
        unsigned long long old = 0ull;
        if (__lane_id() == (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))
            old = __hip_atomic_fetch_and(&v.ready[w], ~want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        old = ((unsigned long long)wave_uniform((uint32_t)(old >> 32)) << 32) | wave_uniform((uint32_t)old);
        unsigned long long cl = old & want;
        if (old != 0ull && (old & ~want) == 0ull &&
            __lane_id() == (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))
            __hip_atomic_fetch_and(v.sum, ~(1u << w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // deal the claimed walks to idle lanes in order
        while (cl != 0ull) {
            const uint32_t s = (uint32_t)__builtin_ctzll(cl);
            const uint32_t l = (uint32_t)__builtin_ctzll(idle);
            cl &= cl - 1ull;
            idle &= idle - 1ull;
            got = (__lane_id() == l) ? w * 64u + s : got;
        }
    }
#endif
    return got;
}

template <bool ANY>
__device__ __forceinline__ void sphere_walk_pool(const uint4* __restrict__ ent,
                                                 const uint16_t* __restrict__ ids, uint32_t nN,
                                                 uint32_t nT, uint8_t* pool_base, f3& o, f3& d,
                                                 float& best, int& id) {
#if defined(__HIP_DEVICE_COMPILE__)
    constexpr uint32_t NT = RT_SPH_BLOCK;
    constexpr uint32_t kNone = 0xFFFFFFFFu, kClaimed = 0x10000u, kAnyBit = 0x20000u;
#ifdef RT_TIMING_NO_SPH_WALK
    return;
#endif
    const PoolView v = pool_view<NT>(pool_base);
    // threadIdx.x through an opaque copy at each use: slot addresses hoisted
    // out of the sample loop would hold VGPRs (and spill) for the whole launch
    auto opaque_me = []() {
        uint32_t t = threadIdx.x;
        asm volatile("" : "+v"(t));
        return t;
    };
    uint32_t me = opaque_me();
    const uint32_t wave = wave_uniform(me >> 6);
    const uint32_t lane = __lane_id();
    // this lane's query in its slot: read back at the end, whoever walked it
    v.a[me] = make_float4(o.x, o.y, o.z, best);
    v.b[me] = make_float4(d.x, d.y, d.z, 0.0f);
    float a = dot(d, d);
    RayBox rb = ray_box(o, d);
    uint32_t idx = octant(d) * nN;
    uint32_t end = idx + nN;
    if (ANY && id >= 0) idx = end;
    uint32_t cur = me | (ANY ? kAnyBit : 0u);   // slot of the walk this lane runs (+ kind bits)
    float pb = 0.0f, pdisc = 0.0f;               // parked leaf idx - 1 while pdisc > 0
    unsigned long long handed = 0ull;            // wave-uniform: walks this wave handed over
    bool over = false;                           // wave-uniform: handed over (once per query)
    const int n_exec = __popcll(__builtin_amdgcn_ballot_w64(true));
    int refill_at = 0;                           // wave-uniform
    uint32_t guard = 0;                          // wave-uniform: polls while waiting
    for (;;) {
        for (;;) {  // cheap steps
            const bool adv = idx < end && !(pdisc > 0.0f);
            if (__builtin_amdgcn_ballot_w64(adv) == 0) break;
            if (adv) {
                const uint4 e = ent[idx];
                if (e.w & 0x80000000u) {
                    idx = lds_node_hit(e, rb, 0.0f, best) ? idx + 1 : (e.w & 0x7FFFFFFFu);
                } else {  // sph_test up to the discriminant (shaders_old.metal:108-136)
                    const f3 oc = o - f3{__uint_as_float(e.x), __uint_as_float(e.y), __uint_as_float(e.z)};
                    const float bq = 2.0f * dot(oc, d);
                    const float cc = dot(oc, oc) - __uint_as_float(e.w);
                    const float disc = bq * bq - (4.0f * a) * cc;
                    if (disc > 0.0f) {
                        pb = bq;
                        pdisc = disc;
                    }
                    idx = idx + 1;
                }
            }
            const int parked = __popcll(__builtin_amdgcn_ballot_w64(pdisc > 0.0f));
            const int live = __popcll(__builtin_amdgcn_ballot_w64(idx < end || pdisc > 0.0f));
            if (RT_SPH_PARK_DEN * parked >= live) break;
            if (!over ? live <= RT_SPH_POOL_T : n_exec - live >= refill_at) break;
        }
        if (__builtin_amdgcn_ballot_w64(pdisc > 0.0f) != 0) {  // roots of the parked leaves
            if (pdisc > 0.0f) {
                const bool any = (cur & kAnyBit) != 0u;
                const float tmin = any ? 0.0f : 1e-3f;
                const float sq = sqrtf(pdisc);
                const float a2 = 2.0f * a;
                float t = (-pb - sq) / a2;
                if (!(t > tmin)) t = (-pb + sq) / a2;
                if (any) {
                    if (t > tmin && t < best) {
                        id = 0;
                        idx = end;
                    }
                } else if (t > tmin && t < 3.0e38f && t <= best) {
                    const int s = (int)(nT + ids[idx - 1u]);
                    if (t < best || s < id) {
                        best = t;
                        id = s;
                    }
                }
                pdisc = 0.0f;
            }
        }
        // finished walks: the result to the query's slot (claimed: + the owner's done bit)
        const bool fin = cur != kNone && idx >= end;
        if (fin) {
            const uint32_t s = cur & 0xFFFFu;
            ((lds_f32_t*)&v.a[s])[3] = best;
            v.c[s] = (uint32_t)(id + 1);
        }
        if (__builtin_amdgcn_ballot_w64(fin && (cur & kClaimed)) != 0ull) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (fin && (cur & kClaimed))
                __hip_atomic_fetch_or(&v.done[(cur & 0xFFFFu) >> 6], 1ull << (cur & 63u), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        if (fin) {
            cur = kNone;
            idx = end = 0u;
        }
        // hand over this wave's last walks (all of them are its own until now)
        if (!over) {
            const unsigned long long give = __builtin_amdgcn_ballot_w64(cur != kNone);
            if (__popcll(give) <= RT_SPH_POOL_T) {
                over = true;
                handed = give;
                if (give != 0ull) {
                    if (cur != kNone) {
                        me = cur & 0xFFFFu;  // (own walks only before the hand-over)
                        ((lds_f32_t*)&v.a[me])[3] = best;
                        ((lds_u32_t*)&v.b[me])[3] = idx;
                        v.c[me] = (uint32_t)(id + 1) | ((cur & kAnyBit) ? 0x80000000u : 0u);
                        cur = kNone;
                        idx = end = 0u;
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    if (lane == (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(true))) {
                        __hip_atomic_fetch_or(&v.ready[wave], give, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_or(v.sum, 1u << wave, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
        }
        if (!over) continue;
        // idle lanes claim handed-over walks (this wave's first)
        const unsigned long long idle = __builtin_amdgcn_ballot_w64(cur == kNone);
        bool waiting = false;
        if (idle != 0ull) {
            const uint32_t got = pool_claim<NT>(v, wave, handed != 0ull, idle);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (got != kNone) {
                const float4 qa = v.a[got], qb = v.b[got];
                const uint32_t qc = v.c[got];
                o = f3{qa.x, qa.y, qa.z};
                best = qa.w;
                d = f3{qb.x, qb.y, qb.z};
                idx = __float_as_uint(qb.w);
                id = (int)(qc & 0x7FFFFFFFu) - 1;
                cur = got | kClaimed | ((qc >> 31) ? kAnyBit : 0u);
                a = dot(d, d);
                rb = ray_box(o, d);
                end = (octant(d) + 1u) * nN;
            }
            refill_at = n_exec - __popcll(__builtin_amdgcn_ballot_w64(idx < end)) + RT_SPH_POOL_REFILL;
        }
        if (__builtin_amdgcn_ballot_w64(cur != kNone) == 0ull) {
            // nothing to walk: done once every handed-over walk of this wave is back
            unsigned long long dn = __hip_atomic_load(&v.done[wave], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            dn = ((unsigned long long)wave_uniform((uint32_t)(dn >> 32)) << 32) | wave_uniform((uint32_t)dn);
            if ((dn & handed) == handed) break;
            waiting = true;
        }
        if (waiting) {
            __builtin_amdgcn_s_sleep(1);
            if (++guard > (1u << 18)) {  // liveness guard (never expected): poison the result
                best = __uint_as_float(0x7FC00000u);
                break;
            }
        }
    }
    if (handed != 0ull && lane == (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(true)))
        __hip_atomic_fetch_and(&v.done[wave], ~handed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    me = opaque_me();
    const float4 qa = v.a[me], qb = v.b[me];
    const uint32_t qc = v.c[me];
    const float b0 = best;
    o = f3{qa.x, qa.y, qa.z};
    d = f3{qb.x, qb.y, qb.z};
    best = (b0 != b0) ? b0 : qa.w;
    id = (int)(qc & 0x7FFFFFFFu) - 1;
#endif
}

template <bool PACKET>
__device__ __forceinline__ bool sphere_any_lds(const uint4* ent, uint32_t nN, f3 o, f3 d,
                                               float tmin, float tmax) {
    const float a = dot(d, d);
    const RayBox rb = ray_box(o, d);
    const uint32_t lay = PACKET ? wave_uniform(sph_layout(d)) : sph_layout(d);
    bool found = false;
    uint32_t idx = lay * nN;
    const uint32_t end = idx + nN;
    while (idx < end) {
        const uint4 e = ent[idx];
        uint32_t next = idx + 1;
        if (e.w & 0x80000000u) {
            const bool h = !found && lds_node_hit(e, rb, tmin, tmax);
            if (PACKET ? __builtin_amdgcn_ballot_w64(h) == 0 : !h) next = e.w & 0x7FFFFFFFu;
        } else {
            float t;
            found = found || sph_test(make_float4(__uint_as_float(e.x), __uint_as_float(e.y),
                                                  __uint_as_float(e.z), __uint_as_float(e.w)),
                                      o, d, a, tmin, tmax, &t);
            if (!PACKET && found) return true;
            if (PACKET && __builtin_amdgcn_ballot_w64(!found) == 0) break;
        }
        idx = PACKET ? wave_uniform(next) : next;
    }
    return found;
}

// Triangle-BVH walks: the sphere walks above with the triangle test in the
// leaves (one triangle per leaf) — same conservative boxes, same (t, id)
// ranking, so the result is the id-ordered brute-force scan's.
template <bool PACKET>
__device__ __forceinline__ void tri_bvh_closest(const float4* __restrict__ node,
                                                const float4* __restrict__ tri,
                                                const uint32_t* __restrict__ perm, uint32_t nN,
                                                f3 o, f3 d, float tmin, float& best, int& id) {
    const RayBox rb = ray_box(o, d);
    node += 2u * nN * (PACKET ? wave_uniform(octant(d)) : octant(d));
    uint32_t idx = 0;
    while (idx < nN) {
        const float4 n0 = node[2 * idx], n1 = node[2 * idx + 1];
        uint32_t next = PACKET ? wave_uniform(__float_as_uint(n0.w)) : __float_as_uint(n0.w);
        const bool h = node_hit(n0, n1, rb, tmin, best);
        if (PACKET ? __builtin_amdgcn_ballot_w64(h) != 0 : h) {
            const uint32_t leaf = PACKET ? wave_uniform(__float_as_uint(n1.w)) : __float_as_uint(n1.w);
            if (leaf == 0u) {
                next = idx + 1;
            } else {
                const uint32_t first = leaf & 0xFFFFFFu, end = first + (leaf >> 24);
                for (uint32_t k = first; k < end; ++k) {
                    float t;
                    if (tri_test(tri[3 * k], tri[3 * k + 1], tri[3 * k + 2], o, d, tmin, 3.0e38f,
                                 &t) && t <= best) {
                        const int tid = (int)perm[k];
                        if (t < best || tid < id) {
                            best = t;
                            id = tid;
                        }
                    }
                }
            }
        }
        idx = next;
    }
}

template <bool PACKET>
__device__ __forceinline__ bool tri_bvh_any(const float4* __restrict__ node,
                                            const float4* __restrict__ tri, uint32_t nN, f3 o,
                                            f3 d, float tmin, float tmax) {
    const RayBox rb = ray_box(o, d);
    node += 2u * nN * (PACKET ? wave_uniform(octant(d)) : octant(d));
    bool found = false;
    uint32_t idx = 0;
    while (idx < nN) {
        const float4 n0 = node[2 * idx], n1 = node[2 * idx + 1];
        if (PACKET) {
            uint32_t next = wave_uniform(__float_as_uint(n0.w));
            if (__builtin_amdgcn_ballot_w64(!found && node_hit(n0, n1, rb, tmin, tmax)) != 0) {
                const uint32_t leaf = wave_uniform(__float_as_uint(n1.w));
                if (leaf == 0u) {
                    next = idx + 1;
                } else {
                    const uint32_t first = leaf & 0xFFFFFFu, end = first + (leaf >> 24);
                    for (uint32_t k = first; k < end; ++k) {
                        float t;
                        found = found || tri_test(tri[3 * k], tri[3 * k + 1], tri[3 * k + 2], o, d,
                                                  tmin, tmax, &t);
                    }
                    if (__builtin_amdgcn_ballot_w64(!found) == 0) break;
                }
            }
            idx = next;
        } else {
            uint32_t next = __float_as_uint(n0.w);
            if (node_hit(n0, n1, rb, tmin, tmax)) {
                const uint32_t leaf = __float_as_uint(n1.w);
                if (leaf == 0u) {
                    next = idx + 1;
                } else {
                    const uint32_t first = leaf & 0xFFFFFFu, end = first + (leaf >> 24);
                    for (uint32_t k = first; k < end; ++k) {
                        float t;
                        if (tri_test(tri[3 * k], tri[3 * k + 1], tri[3 * k + 2], o, d, tmin, tmax,
                                     &t))
                            return true;
                    }
                }
            }
            idx = next;
        }
    }
    return found;
}

// Triangle-BVH walks over the compact entries (rt_lbvh.hip: 16 B per node, fp16
// boxes rounded outward, two layouts -- near child first for (+,+,+) and for
// (-,-,-), a ray takes the one matching most of its direction signs -- stored
// after the 8 full layouts): the same stackless depth-first walks, conservative
// boxes and (t, id) ranking as tri_bvh_*, with half the bytes per step and a
// quarter of the layouts in the caches.
__device__ __forceinline__ const uint4* tri_compact(const float4* node, uint32_t nN) {
    return reinterpret_cast<const uint4*>(node + 16u * nN);
}
__device__ __forceinline__ uint32_t tri_compact_layout(f3 d) {
    return RT_TRI_COMPACT_LAYOUTS == 8 ? octant(d) : lds_layout(d);
}

template <bool PACKET>
__device__ __forceinline__ void tri_cbvh_closest(const uint4* __restrict__ cn,
                                                 const float4* __restrict__ tri,
                                                 const uint32_t* __restrict__ perm, uint32_t nN,
                                                 f3 o, f3 d, float tmin, float& best, int& id) {
    const RayBox rb = ray_box(o, d);
    uint32_t idx = (PACKET ? wave_uniform(tri_compact_layout(d)) : tri_compact_layout(d)) * nN;
    const uint32_t end = idx + nN;
    while (idx < end) {
        const uint4 e = cn[idx];
        const bool inner = (e.w & 0x80000000u) != 0u;  // wave-uniform for PACKET
        const bool h = lds_node_hit(e, rb, tmin, best);
        uint32_t next = idx + 1;
        if (PACKET ? __builtin_amdgcn_ballot_w64(h) == 0 : !h) {
            if (inner) next = e.w & 0x7FFFFFFFu;
        } else if (!inner) {
            const uint32_t k = e.w;
            float t;
            if (tri_test(tri[3 * k], tri[3 * k + 1], tri[3 * k + 2], o, d, tmin, 3.0e38f, &t) &&
                t <= best) {
                const int tid = (int)perm[k];
                if (t < best || tid < id) {
                    best = t;
                    id = tid;
                }
            }
        }
        idx = PACKET ? wave_uniform(next) : next;
    }
}

template <bool PACKET>
__device__ __forceinline__ bool tri_cbvh_any(const uint4* __restrict__ cn, const float4* __restrict__ tri,
                                             uint32_t nN, f3 o, f3 d, float tmin, float tmax) {
    const RayBox rb = ray_box(o, d);
    uint32_t idx = (PACKET ? wave_uniform(tri_compact_layout(d)) : tri_compact_layout(d)) * nN;
    const uint32_t end = idx + nN;
    bool found = false;
    while (idx < end) {
        const uint4 e = cn[idx];
        const bool inner = (e.w & 0x80000000u) != 0u;
        const bool h = !found && lds_node_hit(e, rb, tmin, tmax);
        uint32_t next = idx + 1;
        if (PACKET ? __builtin_amdgcn_ballot_w64(h) == 0 : !h) {
            if (inner) next = e.w & 0x7FFFFFFFu;
        } else if (!inner) {
            const uint32_t k = e.w;
            float t;
            found = found || tri_test(tri[3 * k], tri[3 * k + 1], tri[3 * k + 2], o, d, tmin, tmax, &t);
            if (!PACKET && found) return true;
            if (PACKET && __builtin_amdgcn_ballot_w64(!found) == 0) break;
        }
        idx = PACKET ? wave_uniform(next) : next;
    }
    return found;
}

// Per-lane compact-BVH walks with POSTPONED LEAVES (as sphere_walk_lds parks
// its roots): a lane whose box test passes at a leaf parks the triangle and
// stops; the others walk on until at least half of the lanes still walking
// are parked, then the wave runs the triangle tests of all parked lanes
// together -- instead of every mixed step paying for the box test AND the
// three record loads and the test of a triangle.  Per lane the entries are
// visited in the same order and ranked by (t, id): the same result.
#ifndef RT_TRI_PARK_DEN
#define RT_TRI_PARK_DEN 4  // the parked leaves are tested once they are >= 1/DEN of the live lanes
#endif
template <bool ANY>
__device__ __forceinline__ void tri_cbvh_walk(const uint4* __restrict__ cn, const float4* __restrict__ tri,
                                              const uint32_t* __restrict__ perm, uint32_t nN, f3 o, f3 d,
                                              float tmin, float& best, int& id) {
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    const RayBox rb = ray_box(o, d);
    uint32_t idx = tri_compact_layout(d) * nN;
    const uint32_t end = idx + nN;
    if (ANY && id >= 0) idx = end;
    uint32_t leaf = kNone;
    for (;;) {
        for (;;) {
            const bool adv = idx < end && leaf == kNone;
            if (__builtin_amdgcn_ballot_w64(adv) == 0) break;
            if (adv) {
                const uint4 e = cn[idx];
                const bool inner = (e.w & 0x80000000u) != 0u;
                if (!lds_node_hit(e, rb, tmin, best)) {
                    idx = inner ? (e.w & 0x7FFFFFFFu) : idx + 1;
                } else {
                    if (!inner) leaf = e.w;
                    idx = idx + 1;
                }
            }
            const int parked = __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone));
            const int live = __popcll(__builtin_amdgcn_ballot_w64(idx < end || leaf != kNone));
            if (RT_TRI_PARK_DEN * parked >= live) break;
        }
        if (__builtin_amdgcn_ballot_w64(leaf != kNone) == 0) break;
        if (leaf != kNone) {
            float t;
            if (tri_test(tri[3 * leaf], tri[3 * leaf + 1], tri[3 * leaf + 2], o, d, tmin,
                         ANY ? best : 3.0e38f, &t)) {
                if (ANY) {
                    id = 0;
                    idx = end;
                } else if (t <= best) {
                    const int tid = (int)perm[leaf];
                    if (t < best || tid < id) {
                        best = t;
                        id = tid;
                    }
                }
            }
            leaf = kNone;
        }
    }
}

#ifndef RT_TRI_PARK
#define RT_TRI_PARK 1  // per-lane triangle-BVH walks with postponed leaves (tri_cbvh_walk)
#endif
#ifndef RT_TRI_PARK_ALL
#define RT_TRI_PARK_ALL 0  // 1: also camera and bounce-0 shadow rays (else wave-packet walks)
#endif

#ifndef RT_TRI_COMPACT
#define RT_TRI_COMPACT 1  // triangle-BVH walks over the compact 16-B entries
#endif

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
// stays away from every face and no face can accept a hit.
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
            const float4 H = r[3];
            if (!(__float_as_uint(H.w) & 8u)) continue;
            const float4 W = r[6];
            const float lo[3] = {r[0].w, r[1].w, r[2].w}, hi[3] = {H.x, H.y, H.z};
            const float wf[3] = {W.x, W.y, W.z};
            const float oo[3] = {o.x, o.y, o.z}, ee[3] = {e.x, e.y, e.z};
            bool inside = true;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                // lo' + w = face plane + tol_n; 2^-16 relative slack for the
                // rounding of o + d*tmax and of the bounds
                const float in_lo = lo[a] + wf[a] + kEps * (fabsf(lo[a]) + fabsf(ee[a]));
                const float in_hi = hi[a] - wf[a] - kEps * (fabsf(hi[a]) + fabsf(ee[a]));
                inside = inside && oo[a] > in_lo && oo[a] < in_hi && ee[a] > in_lo && ee[a] < in_hi;
            }
            if (__builtin_amdgcn_ballot_w64(!inside) == 0) skip |= 1u << c;
        }
    }
    // per-ray terms of world-aligned box axes: t = lo * invd - o * invd
    const RayBox rb = ray_box(o, d);
    const float iv[3] = {rb.invd.x, rb.invd.y, rb.invd.z};
    const float oi[3] = {rb.oinv.x, rb.oinv.y, rb.oinv.z};
    uint32_t mask = 0;
    uint32_t c = 0;
    for (; c < sv.nC; ++c) {
        if (SEG && ((skip >> c) & 1u)) continue;
        const float4* r = sv.clu + kCluF4 * c;
        const float4 H = r[3], M0 = r[4], M1 = r[5], W = r[6];
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
        const float tlo = tlo0 - kEps * fabsf(tlo0), thi = thi0 + kEps * fabsf(thi0);
#ifndef RT_NO_CLU_WAVE_SKIP
        if (!__builtin_amdgcn_ballot_w64(tlo <= thi)) continue;  // no lane meets the box
#endif
        const uint32_t m[6] = {__float_as_uint(M0.x), __float_as_uint(M0.y), __float_as_uint(M0.z),
                               __float_as_uint(M0.w), __float_as_uint(M1.x), __float_as_uint(M1.y)};
        uint32_t cm = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            // a ray with d_a >= 0 enters through the low face (slot 2a) and
            // leaves through the high one (2a + 1); the face plane lies
            // wf * |1/d_a| inside the padded slab, +- the tolerance
            const bool neg = ida[a] < 0.0f;
            const uint32_t m_en = neg ? m[2 * a + 1] : m[2 * a], m_ex = neg ? m[2 * a] : m[2 * a + 1];
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
        const float tlo = tlo0 - kEps * fabsf(tlo0), thi = thi0 + kEps * fabsf(thi0);
        mask |= (tlo <= thi) ? __float_as_uint(r[5].z) : 0u;
    }
    return mask;
}

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
    if (pa || pb) {
        const f3 nsel = pa ? f3{r2.y, r2.z, r2.w} : f3{r3.w, r4.x, r4.y};
        const float t = pair_t(nsel, q.tv, pa ? q.denA : q.denB);
        const int ia = (int)(pa ? 2 * k : 2 * k + 1);
        if (t > tmin && (t < *best || (!ANY && t == *best && ia < *id))) {
            if (!ANY) *best = t;
            *id = ia;
        }
        if (pa && pb) {
            const float t2 = pair_t(f3{r3.w, r4.x, r4.y}, q.tv, q.denB);
            const int ib = (int)(2 * k + 1);
            if (t2 > tmin && (t2 < *best || (!ANY && t2 == *best && ib < *id))) {
                if (!ANY) *best = t2;
                *id = ib;
            }
        }
    }
}

// Closest hit / any hit over the pair records with box clusters: the
// unclustered pairs by every lane (wave-uniform records, LDS broadcast), then
// each lane's own candidate pairs (per-lane LDS reads).  For ANY, *best is
// tmax and is not changed.
template <bool ANY>
__device__ __forceinline__ void cluster_query(const SceneView& sv, f3 o, f3 d, float tmin,
                                              float* best, int* id) {
    for (uint32_t free = sv.pair_free; free != 0u; free &= free - 1u) {
        const uint32_t k = (uint32_t)__builtin_ctz(free);
        pair_test_rank<ANY>(sv.pair + kPairF4 * k, k, o, d, tmin, best, id);
    }
    uint32_t cand = cluster_candidates<ANY>(sv, o, d, tmin, *best);
    RT_STAT(12, 1);
    RT_STAT(15, __popcll(__ballot(1)));
    while (cand != 0u && !(ANY && *id >= 0)) {
        RT_STAT(13, 1);
        RT_STAT(14, __popcll(__ballot(1)));
        const uint32_t k = (uint32_t)__builtin_ctz(cand);
        cand &= cand - 1u;
        pair_test_rank<ANY>(sv.pair + kPairF4 * k, k, o, d, tmin, best, id);
    }
}

// closest hit, accept_any_intersection(false) (raytrace.metal:48-49).
// Primitives are tested in id order; a strictly smaller t wins (ties keep the
// lower id), exactly as the oracle.
// With CULL (used for coherent camera rays) a pair is skipped when no lane's
// box around its current candidate segment [o, o + d*best] touches the pair's
// padded AABB: any hit that could still win has t < best and lies inside it.
// o and d are references so that the pooled sphere walk (which hands them
// back bit-identical) does not make the caller keep a second copy live.
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
        if (RT_TRI_COMPACT && RT_TRI_PARK && (!CULL || RT_TRI_PARK_ALL))
            tri_cbvh_walk<false>(tri_compact(sv.tnode, sv.nTN), sv.tsorted, sv.tperm, sv.nTN, o, d, tmin,
                                 best, id);
        else if (RT_TRI_COMPACT)
            tri_cbvh_closest<CULL>(tri_compact(sv.tnode, sv.nTN), sv.tsorted, sv.tperm, sv.nTN, o, d,
                                   tmin, best, id);
        else
            tri_bvh_closest<CULL>(sv.tnode, sv.tsorted, sv.tperm, sv.nTN, o, d, tmin, best, id);
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
    if (SPH && GEO == kGeoSphLds && ((CULL && RT_SPH_PACKET) || RT_SPH_PACKET >= 3))
        sphere_closest_lds<true>(sv.sent, sv.sid, sv.nN, sv.nT, o, d, tmin, best, id);
    else if (SPH && GEO == kGeoSphLds && RT_SPH_POOL)
        sphere_walk_pool<false>(sv.sent, sv.sid, sv.nN, sv.nT, sv.pool, o, d, best, id);
    else if (SPH && GEO == kGeoSphLds)
        sphere_walk_lds<false, RT_SPH_SPLIT != 0>(sv.sent, sv.sid, sv.nN, sv.nT, o, d, tmin, best, id,
                                                  sv.wscr);
    else if (SPH)
        sphere_closest<(CULL && RT_SPH_PACKET) || RT_SPH_PACKET >= 3>(sv.node, sv.sph, sv.sph_perm, sv.nN, sv.nT, o, d, tmin, best, id);
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
        if (RT_TRI_COMPACT && RT_TRI_PARK && (!PACKET || RT_TRI_PARK_ALL)) {
            float tm = tmax;
            int hid = -1;
            tri_cbvh_walk<true>(tri_compact(sv.tnode, sv.nTN), sv.tsorted, sv.tperm, sv.nTN, o, d, tmin,
                                tm, hid);
            if (hid >= 0) return true;
        } else if (RT_TRI_COMPACT ? tri_cbvh_any<PACKET>(tri_compact(sv.tnode, sv.nTN), sv.tsorted, sv.nTN, o,
                                                         d, tmin, tmax)
                                  : tri_bvh_any<PACKET>(sv.tnode, sv.tsorted, sv.nTN, o, d, tmin, tmax)) {
            return true;
        }
    } else {
        for (uint32_t k = 0; k < sv.nT; ++k) {
            float t;
            if (tri_test(sv.tri[3 * k], sv.tri[3 * k + 1], sv.tri[3 * k + 2], o, d, tmin, tmax,
                         &t))
                return true;
        }
    }
    if (SPH && GEO == kGeoSphLds && PACKET) return sphere_any_lds<true>(sv.sent, sv.nN, o, d, tmin, tmax);
    if (SPH && GEO == kGeoSphLds && RT_SPH_POOL) {
        float tm = tmax;
        int id = -1;
        sphere_walk_pool<true>(sv.sent, sv.sid, sv.nN, sv.nT, sv.pool, o, d, tm, id);
        return id >= 0;
    }
    if (SPH && GEO == kGeoSphLds) {
        float tm = tmax;
        int id = -1;
        sphere_walk_lds<true, RT_SPH_SPLIT != 0 && !RT_SPH_SPLIT_CLOSEST_ONLY>(
            sv.sent, sv.sid, sv.nN, sv.nT, o, d, tmin, tm, id, sv.wscr);
        return id >= 0;
    }
    if (SPH) return sphere_any<PACKET>(sv.node, sv.sph, sv.nN, o, d, tmin, tmax);
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

// Fused shadow any-hit of bounce b and closest hit of bounce b+1 over the box
// clusters (kGeoPairClu; the cluster twin of fused_shadow_closest): both rays
// start at p, so after both candidate masks are formed each lane tests ONE
// candidate pair per round -- a shadow candidate while its shadow ray is not yet
// occluded, else a closest candidate -- instead of running the shadow rounds
// and then the closest rounds each to the wave's longest list.  Every test is
// pair_test_rank's (same arithmetic, same (t, id) ranking, candidates visited
// out of id order as there), so each lane's two results are exactly those of
// cluster_query<true> and cluster_query<false>.
__device__ __forceinline__ FusedHit fused_cluster_query(const SceneView& sv, f3 p, f3 L, float smax,
                                                        f3 d2) {
    FusedHit h{false, -1, 1000.0f};  // max_distance (sampling.metal:155)
    float tm = smax;
    int sid = -1;
    for (uint32_t free = sv.pair_free; free != 0u; free &= free - 1u) {
        const uint32_t k = (uint32_t)__builtin_ctz(free);
        pair_test_rank<true>(sv.pair + kPairF4 * k, k, p, L, 0.0f, &tm, &sid);
        pair_test_rank<false>(sv.pair + kPairF4 * k, k, p, d2, 0.001f, &h.t, &h.id);
    }
    uint32_t cs = sid >= 0 ? 0u : cluster_candidates<true>(sv, p, L, 0.0f, smax);
    uint32_t cc = cluster_candidates<false>(sv, p, d2, 0.001f, h.t);
    while ((cs | cc) != 0u) {
        const bool shadow = cs != 0u;
        const uint32_t k = (uint32_t)__builtin_ctz(shadow ? cs : cc);
        if (shadow)
            cs &= cs - 1u;
        else
            cc &= cc - 1u;
        // pair_test_rank with the mode chosen per lane
        const f3 dir = shadow ? L : d2;
        const float tmin = shadow ? 0.0f : 0.001f;
        const float4* rr = sv.pair + kPairF4 * k;
        const float4 r0 = rr[0], r1 = rr[1], r2 = rr[2], r3 = rr[3], r4 = rr[4];
        const PairDots q = pair_dots(r0, r1, r2, r3, r4, p, dir);
        const bool pa = bary_ok(q.denA, q.a1, q.a2);
        const bool pb = bary_ok(q.denB, q.b1, q.b2);
        if (pa || pb) {
            const float best = shadow ? smax : h.t;
            const f3 nsel = pa ? f3{r2.y, r2.z, r2.w} : f3{r3.w, r4.x, r4.y};
            const float t = pair_t(nsel, q.tv, pa ? q.denA : q.denB);
            const int ia = (int)(pa ? 2 * k : 2 * k + 1);
            bool hit = t > tmin && (t < best || (!shadow && t == best && ia < h.id));
            float tb = t;
            int ib = ia;
            if (pa && pb) {
                const float t2 = pair_t(f3{r3.w, r4.x, r4.y}, q.tv, q.denB);
                const int i2 = (int)(2 * k + 1);
                const float best2 = hit ? tb : best;
                const int id2 = hit ? ib : h.id;
                if (t2 > tmin && (t2 < best2 || (!shadow && t2 == best2 && i2 < id2))) {
                    hit = true;
                    tb = t2;
                    ib = i2;
                }
            }
            if (hit) {
                if (shadow) {
                    h.occluded = true;
                    cs = 0u;  // any hit ends the shadow query (cluster_query<true>)
                } else {
                    h.t = tb;
                    h.id = ib;
                }
            }
        }
    }
    h.occluded = h.occluded || sid >= 0;
    return h;
}

}  // namespace
}  // namespace rt

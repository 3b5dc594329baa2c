// rt_kernel.hip — gfx950 path-tracing kernel (the hot path) and its launcher.
//
// Rebuilds `kernel pathTrace` (RTrace/raytrace.metal:11-111) for CDNA4:
//   * the scene's intersection records (shared-edge triangle pairs, box
//     clusters) and the Halton low-digit tables are staged into LDS once per
//     workgroup; the sphere and triangle BVHs are read from global memory
//     (L2-resident); shading records are fetched from global only on a hit;
//   * L = 4 or 16 lanes per pixel: a wave traces 64/L pixels (a 4x4 or 2x2
//     tile, or one row of interleaved rows), lane `sub` traces samples
//     n = r*L + sub, and the colours are summed at the pixel's leader in
//     sample order (DPP row shifts or ds_bpermute) -- the additions of one
//     lane per pixel, so the result is unchanged;
//   * the bounce loop is unrolled at compile time (template B) so every Halton
//     dimension, hence every base, is a constant: the digit steps run in float
//     (floor(x*c), fma(q, -b, x): exact for indices < 3^13, rt_halton.hpp);
//   * camera constants are precomputed on the host once (same contract ops);
//   * the per-pixel result is one coalesced float4 / half4 / uchar4 store.
// Arithmetic follows the contract of rt_math.h / DESIGN.md §3 so the result is
// bit-identical to the CPU oracle.
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>

#include <stddef.h>
#include <stdio.h>
#ifdef RT_LDS_CHECK
#include <hsa/hsa.h>
#endif

#include "rt_kernel.hpp"
#include "rt_halton.hpp"
#include "rt_trace.hpp"

namespace rt {

// -DRT_LDS_CHECK diagnostic builds: before staging, every kernel checks that
// the end of what its staging loops write (computed from the kernel's own
// loop bounds) lies within the dynamic LDS of its dispatch
// (hsa_kernel_dispatch_packet_t.group_segment_size, byte 28 = static +
// dynamic LDS).  A short allocation records the end in g_lds_overflow and the
// workgroup returns before writing anything; rt_render then fails with
// RT_ERR_LAUNCH (lds_check_result).  Production builds compile it out: the
// launcher requests staged_lds_bytes (rt_kernel.hpp), the same terms.
#ifdef RT_LDS_CHECK
__device__ uint32_t g_lds_overflow;
__device__ __forceinline__ bool lds_short(size_t end) {
    // word 7 (byte 28) of the AQL packet: group_segment_size (static_assert below)
    const uint32_t grp = ((const uint32_t*)__builtin_amdgcn_dispatch_ptr())[7];
    const size_t dyn = grp - __builtin_amdgcn_groupstaticsize();
    if (end <= dyn) return false;
    if (threadIdx.x == 0) atomicMax(&g_lds_overflow, (uint32_t)end);
    return true;
}
static_assert(offsetof(hsa_kernel_dispatch_packet_t, group_segment_size) == 28, "AQL packet layout");
#define RT_LDS_GUARD(end)            \
    do {                             \
        if (lds_short(end)) return;  \
    } while (0)
#else
#define RT_LDS_GUARD(end) ((void)0)
#endif

namespace {

// -DRT_CENSUS=k: VALU census builds of the box-cluster (Cornell) kernel
// (tools/census.sh).  Build k runs phase k a second time on opaque copies of
// its inputs (the compiler cannot reuse the first result) and discards the
// result through an opaque sink, under the same lanes and control flow: the
// SQ_INSTS_VALU difference to the plain build is the phase's dynamic VALU.
// 1 camera ray (Halton dims 0-1 + generateCameraRay), 2 closest-hit queries,
// 3 shadow queries, 4 Halton dims 2-5 of the bounces, 5 the rest of the
// shading arithmetic (light sample, NEE term, cosine direction), 6 the
// in-order pixel sums.  Timing-invalid by construction; never shipped.
#ifndef RT_CENSUS
#define RT_CENSUS 0
#endif
// RT_LQ: the light sample point and its cosine without their zero terms (shade)
#ifndef RT_LQ
#define RT_LQ 1
#endif
template <typename T>
__device__ __forceinline__ T cz(T v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ f3 cz(f3 v) { return f3{cz(v.x), cz(v.y), cz(v.z)}; }
__device__ __forceinline__ void cz_sink(float v) { asm volatile("" ::"v"(v)); }
__device__ __forceinline__ void cz_sink(f3 v) {
    cz_sink(v.x);
    cz_sink(v.y);
    cz_sink(v.z);
}

struct PathState {
    f3 o, d, acc, thr;
    uint32_t i;  // Halton index seed + n
};

// One bounce b of raytrace.metal:47-101.  Returns false when the path ends.
// Shading of a hit (id, t) at bounce b: raytrace.metal:55-101.  Returns false
// when the path ends (light hit).
// FUSE (pair layout, triangles only): the shadow query of bounce b and the
// closest hit of bounce b+1 run as one pass over the records
// (fused_shadow_closest); the next hit is returned in *nid / *nt.
// STASH (the one-wave sphere kernel): contrib and the next direction wait in
// the per-lane LDS stash sv.xstash across the shadow walk.
template <int b, int B, int GEO, bool SPH, bool SMALL, bool FUSE = false, bool STASH = false>
__device__ __forceinline__ bool shade(const KParams& P, const SceneView& sv, PathState& s, int id,
                                      float t, int* nid = nullptr, float* nt = nullptr) {
    f3 N, right, fwd, diffuse;
    if (!SPH || (uint32_t)id < sv.nT) {
        const float4* sh = P.tri_shade + 4 * id;
        const float4 s0 = sh[0];
        const float4 s3 = sh[3];
        if (s0.w != 0.0f) {                                 // :57-60 light: overwrite, stop
            s.acc = f3{s3.x, s3.y, s3.z};
            return false;
        }
        const float4 s1 = sh[1], s2 = sh[2];
        N = f3{s0.x, s0.y, s0.z};
        right = f3{s1.x, s1.y, s1.z};
        fwd = f3{s2.x, s2.y, s2.z};
        diffuse = f3{s1.w, s2.w, s3.w};
    } else {
        const uint32_t k = (uint32_t)id - sv.nT;
        const float4* sh = P.sph_shade + 3 * k;
        const float4 s0 = sh[0];
        if (s0.w != 0.0f) {
            const float4 s1 = sh[1];
            s.acc = f3{s1.x, s1.y, s1.z};
            return false;
        }
        const float4 S = sh[2];
        N = normalize((s.o + s.d * t) - f3{S.x, S.y, S.z});
        shading_frame(N, &right, &fwd);
        diffuse = f3{s0.x, s0.y, s0.z};
    }
    f3 p = (s.o + s.d * t) + N * 1e-3f;              // :67

#if RT_CENSUS == 4
    {
        const uint32_t i2 = cz(s.i);
        float h = halton_dim<2 + 5 * b, SMALL, GEO == kGeoPairClu>(i2, sv.htab) +
                  halton_dim<3 + 5 * b, SMALL, GEO == kGeoPairClu>(i2, sv.htab);
        if (b + 1 < B)
            h = h + halton_dim<4 + 5 * b, SMALL, GEO == kGeoPairClu>(i2, sv.htab) +
                halton_dim<5 + 5 * b, SMALL, GEO == kGeoPairClu>(i2, sv.htab);
        cz_sink(h);
    }
#endif
    // sampleAreaLight (sampling.metal:198-236), dims 2+5b, 3+5b (:72-74)
    const float ux = halton_dim<2 + 5 * b, SMALL, GEO == kGeoPairClu>(s.i, sv.htab) * 2.0f - 1.0f;
    const float uy = halton_dim<3 + 5 * b, SMALL, GEO == kGeoPairClu>(s.i, sv.htab) * 2.0f - 1.0f;
#if RT_CENSUS == 5
    {
        const f3 o2 = cz(s.o), dd = cz(s.d), N2 = cz(N), r2 = cz(right), f2 = cz(fwd), df = cz(diffuse);
        const float t2 = cz(t), ux2 = cz(ux), uy2 = cz(uy);
        const f3 p2 = (o2 + dd * t2) + N2 * 1e-3f;
        const f3 q2 = (ld_f3(P.light_center) + f3{0.25f, 0.0f, 0.0f} * ux2) + f3{0.0f, 0.0f, 0.25f} * uy2;
        f3 L2 = q2 - p2;
        const float dist2 = length(L2);
        const float inv2 = 1.0f / fmaxf(dist2, 1e-3f);
        L2 = L2 * inv2;
        f3 lc2 = ld_f3(P.light_color) * (inv2 * inv2);
        lc2 = lc2 * saturate(dot(-L2, f3{0.0f, -1.0f, 0.0f}));
        lc2 = lc2 * saturate(dot(N2, L2));
        const f3 c2 = lc2 * (cz(s.thr) * df);
        cz_sink(c2);
        cz_sink(f3{fminf(p2.x, q2.x), fminf(p2.y, q2.y), fminf(p2.z, q2.z)});
        cz_sink(f3{fmaxf(p2.x, q2.x), fmaxf(p2.y, q2.y), fmaxf(p2.z, q2.z)});
        if (b + 1 < B) {
            float sp2, cp2;
            sincos_pt(6.28318548f * cz(ux), &sp2, &cp2);
            const float ct2 = sqrtf(cz(uy));
            const float st2 = sqrtf(1.0f - ct2 * ct2);
            cz_sink((r2 * (st2 * cp2) + N2 * ct2) + f2 * (st2 * sp2));
        }
    }
#endif
    const f3 lcen = ld_f3(P.light_center);
    // q = center + (0.25,0,0)*ux + (0,0,0.25)*uy (sampling.metal:208-213).  The
    // zero terms (0*ux, 0*uy: +-0, ux and uy are finite and never -0) drop out
    // exactly: lcen.x + 0.25ux is never -0, so adding +-0 keeps it, and
    // lcen.y (lcen.z) + +-0 is lcen.y (lcen.z) unless that is -0 -- the
    // host's light_plain flag; otherwise the literal form
    f3 q;
    if (RT_LQ && P.light_plain)
        q = f3{lcen.x + 0.25f * ux, lcen.y, lcen.z + 0.25f * uy};
    else
        q = (lcen + f3{0.25f, 0.0f, 0.0f} * ux) + f3{0.0f, 0.0f, 0.25f} * uy;
    f3 L = q - p;
    // the short correctly rounded forms (rt_math.h) except in the triangle-BVH
    // kernel, where their uniform branches cost spills (scratch 16 -> 36 B)
    constexpr bool CR = GEO != kGeoTriBvh;
    const float dist = CR ? length(L) : length_ieee(L);
    const float inv = CR ? rcp_cr(fmaxf(dist, 1e-3f)) : 1.0f / fmaxf(dist, 1e-3f);
    L = L * inv;
    f3 lc = ld_f3(P.light_color) * (inv * inv);
    // dot(-L, (0,-1,0)) = fma(-L.z, 0, fma(-L.y, -1, -L.x * 0)) is L.y exactly
    // when L.y != 0; when L.y is +-0 either form gives a zero, which makes the
    // light term zero (no shadow query, +0 added: the same result)
    lc = lc * saturate(RT_LQ ? L.y : dot(-L, f3{0.0f, -1.0f, 0.0f}));
    lc = lc * saturate(dot(N, L));                         // :75
    s.thr = s.thr * diffuse;                               // :76
    // the light term lc * throughput (:87-89) and the next direction (:93-100)
    // are formed BEFORE the shadow query: the same operations, but the shading
    // frame N/right/fwd and lc are dead during the walk (6-9 fewer live VGPRs)
    const f3 contrib = lc * s.thr;
    const f3 seg_lo{fminf(p.x, q.x), fminf(p.y, q.y), fminf(p.z, q.z)};
    const f3 seg_hi{fmaxf(p.x, q.x), fmaxf(p.y, q.y), fmaxf(p.z, q.z)};
    f3 d2{0.0f, 0.0f, 0.0f};
    if (b + 1 < B) {                                       // last direction never traced
        const float cu = halton_dim<4 + 5 * b, SMALL, GEO == kGeoPairClu>(s.i, sv.htab);           // :93-94
        const float cv = halton_dim<5 + 5 * b, SMALL, GEO == kGeoPairClu>(s.i, sv.htab);
        float sp, cp;
        sincos_pt(6.28318548f * cu, &sp, &cp);             // sampling.metal:40-48
        const float ct = CR ? sqrt_cr(cv) : sqrtf(cv);
        const float st = CR ? sqrt_cr(1.0f - ct * ct) : sqrtf(1.0f - ct * ct);
        d2 = (right * (st * cp) + N * ct) + fwd * (st * sp);  // sampling.metal:65
    }
    if (FUSE && b + 1 < B) {
        FusedHit h;
        if constexpr (GEO == kGeoTriBvh) {
            const bool lit = contrib.x != 0.0f || contrib.y != 0.0f || contrib.z != 0.0f;
            h = tri_walk_dual(sv, p, L, dist - 1e-3f, lit, d2);
        } else {
            h = fused_shadow_closest(sv, p, L, dist - 1e-3f, seg_lo, seg_hi, d2);
        }
        if (!h.occluded) s.acc = s.acc + contrib;          // :79-89
        s.d = d2;
        s.o = p;                                           // :99-100
        *nid = h.id;
        *nt = h.t;
        return true;
    }
    // A zero light term (the light behind the surface or behind its own plane,
    // a black material) adds +0 to acc whatever the shadow query says: acc is a
    // sum of non-negative terms starting at +0, so acc + 0 == acc bit for bit,
    // and such lanes skip the query (whole waves do, e.g. camera rays on the
    // ceiling): Cornell +4.3 %, 1000 spheres +1.8 %, 100k triangles +2.5 %.
    // Bounce-0 shadow rays of the triangle BVH walk as wave packets and keep
    // every lane (skipping there: 100k triangles -8 %).
    const bool lit = (GEO == kGeoTriBvh && b == 0) || contrib.x != 0.0f || contrib.y != 0.0f ||
                     contrib.z != 0.0f;
    if constexpr (STASH) {
        // the BVH kernels park contrib and the next direction in a per-lane
        // LDS stash across the shadow walk (read back through an opaque lane
        // index, so they are not kept in registers): at 64 VGPRs (8 waves/SIMD)
        // they were 5-6 spilled VGPRs, 24-28 B of scratch per lane (round 4)
        constexpr uint32_t SS = GEO == kGeoSphLds ? kSphBlockThreads : kBlockThreads;  // stash stride
        uint32_t t = threadIdx.x;
        asm volatile("" : "+v"(t));
        float* st = sv.xstash;
        st[t] = contrib.x;
        st[SS + t] = contrib.y;
        st[2 * SS + t] = contrib.z;
        if (b + 1 < B) {
            st[3 * SS + t] = d2.x;
            st[4 * SS + t] = d2.y;
            st[5 * SS + t] = d2.z;
        }
        const bool occluded =
            lit && any_hit<GEO, SPH, b == 0 && !SPH>(sv, p, L, 0.0f, dist - 1e-3f, seg_lo, seg_hi);  // :79-85
        uint32_t t2 = threadIdx.x;
        asm volatile("" : "+v"(t2));
        if (lit && !occluded)                              // :87-89
            s.acc = s.acc + f3{st[t2], st[SS + t2], st[2 * SS + t2]};
        if (b + 1 < B) {
            s.d = f3{st[3 * SS + t2], st[4 * SS + t2], st[5 * SS + t2]};
            s.o = p;                                       // :99-100
        }
        return true;
    }
#if RT_CENSUS == 3
    if (lit) {
        f3 p2 = cz(p), L2 = cz(L);
        cz_sink(any_hit<GEO, SPH, b == 0 && !SPH>(sv, p2, L2, 0.0f, cz(dist) - 1e-3f, cz(seg_lo), cz(seg_hi)) ? 1.0f
                                                                                                            : 0.0f);
    }
#endif
    if (lit && !any_hit<GEO, SPH, b == 0 && !SPH>(sv, p, L, 0.0f, dist - 1e-3f, seg_lo, seg_hi))  // :79-85
        s.acc = s.acc + contrib;                           // :87-89
    if (b + 1 < B) {
        s.d = d2;
        s.o = p;                                           // :99-100
    }
    return true;
}

// The triangle-BVH kernel runs WITHOUT the LDS stash of shade(): with it the
// kernel has no scratch (63 VGPRs) but ran 778 vs 846 Msamples/s on 100k
// triangles (round 5, profiles/r5/ab_results.md); without it 18 VGPRs spill
// (16 B of scratch per lane, L2-resident)
#ifndef RT_TRI_STASH
#define RT_TRI_STASH 0
#endif
// One bounce b of raytrace.metal:47-101.  Returns false when the path ends.
template <int b, int B, int GEO, bool SPH, bool SMALL>
__device__ __forceinline__ bool bounce(const KParams& P, const SceneView& sv, PathState& s) {
    float t = 1000.0f;                                      // max_distance (sampling.metal:155)
    // Camera rays of an 8x8 tile are coherent: cull with their segment boxes.
    const int id = closest_hit<GEO, SPH, b == 0, (b == 0 ? 0 : 1)>(sv, s.o, s.d, 0.001f, &t);  // min_distance :154
#if RT_CENSUS == 2
    {
        f3 o2 = cz(s.o), d2 = cz(s.d);
        float t2 = cz(1000.0f);
        const int id2 = closest_hit<GEO, SPH, b == 0, (b == 0 ? 0 : 1)>(sv, o2, d2, 0.001f, &t2);
        cz_sink(t2 + (float)id2);
    }
#endif
    if (id < 0) return false;                               // :51-53
    return shade<b, B, GEO, SPH, SMALL, false, GEO == kGeoSphLds || (RT_TRI_STASH && GEO == kGeoTriBvh)>(P, sv, s, id,
                                                                                                 t);
}

template <int b, int B, int GEO, bool SPH, bool SMALL>
struct BounceChain {
    __device__ __forceinline__ static void run(const KParams& P, const SceneView& sv,
                                               PathState& s) {
#ifdef RT_STATS
        if constexpr (!SPH && GEO != kGeoTriBvh) {  // slots 16-31: the per-lane BVH walks' otherwise
            // lane-slot accounting of the triangle kernels (tools/kernel_stats.py):
            // shader-clock cycles of this bounce per wave, and the same weighted
            // by the lanes whose path is still alive when it starts (16+b, 20+b)
            const unsigned long long t0 = clock64();
            const unsigned long long live = (unsigned long long)__popcll(__ballot(1));
            const bool ok = bounce<b, B, GEO, SPH, SMALL>(P, sv, s);
            const unsigned long long dt = clock64() - t0;
            RT_STAT(16 + b, dt);
            RT_STAT(20 + b, dt * live);
            if (!ok) return;
            BounceChain<b + 1, B, GEO, SPH, SMALL>::run(P, sv, s);
            return;
        }
#endif
        if (!bounce<b, B, GEO, SPH, SMALL>(P, sv, s)) return;
        BounceChain<b + 1, B, GEO, SPH, SMALL>::run(P, sv, s);
    }
};
template <int B, int GEO, bool SPH, bool SMALL>
struct BounceChain<B, B, GEO, SPH, SMALL> {
    __device__ __forceinline__ static void run(const KParams&, const SceneView&, PathState&) {}
};

// Fused bounce chain: enters bounce b with the closest hit (id, t) of its ray.
template <int b, int B, int GEO, bool SMALL>
struct FusedChain {
    __device__ __forceinline__ static void run(const KParams& P, const SceneView& sv,
                                               PathState& s, int id, float t) {
        int nid = -1;
        float nt = 0.0f;
        if (!shade<b, B, GEO, false, SMALL, true>(P, sv, s, id, t, &nid, &nt)) return;
        if (b + 1 < B && nid >= 0) FusedChain<b + 1, B, GEO, SMALL>::run(P, sv, s, nid, nt);
    }
};
template <int B, int GEO, bool SMALL>
struct FusedChain<B, B, GEO, SMALL> {
    __device__ __forceinline__ static void run(const KParams&, const SceneView&, PathState&, int,
                                               float) {}
};

// The pair layouts (triangles only) fuse the shadow query of bounce b with the
// closest hit of bounce b + 1 (fused_shadow_closest).  The box-cluster kernel
// does not: its fused candidate rounds measured 5 % slower on Cornell 1080p
// (DESIGN.md §5).
// Triangle-BVH chain with the dual walks (RT_TRI_DUAL): bounce 0 as usual
// (packet walks), then for b >= 1 the shadow query of b and the closest hit of
// b + 1 in one tri_walk_dual loop.
template <int b, int B, bool SMALL>
struct TriDualChain {
    __device__ __forceinline__ static void run(const KParams& P, const SceneView& sv, PathState& s, int id,
                                               float t) {
        if constexpr (b + 1 < B) {
            int nid = -1;
            float nt = 0.0f;
            if (!shade<b, B, kGeoTriBvh, false, SMALL, true>(P, sv, s, id, t, &nid, &nt)) return;
            if (nid >= 0) TriDualChain<b + 1, B, SMALL>::run(P, sv, s, nid, nt);
        } else {
            (void)shade<b, B, kGeoTriBvh, false, SMALL>(P, sv, s, id, t);
        }
    }
};
template <int B, bool SMALL>
struct TriDualChain<B, B, SMALL> {
    __device__ __forceinline__ static void run(const KParams&, const SceneView&, PathState&, int, float) {}
};

#ifndef RT_TRI_DUAL
#define RT_TRI_DUAL 0
#endif

template <int B, int GEO, bool SPH, bool SMALL>
__device__ __forceinline__ void trace_path(const KParams& P, const SceneView& sv, PathState& s) {
    if constexpr (RT_TRI_DUAL && GEO == kGeoTriBvh && !SPH && B > 1) {
        float t = 1000.0f;                                  // sampling.metal:155
        const int id = closest_hit<GEO, false, true, 0>(sv, s.o, s.d, 0.001f, &t);
        if (id < 0 || !shade<0, B, GEO, false, SMALL>(P, sv, s, id, t)) return;
        float t1 = 1000.0f;
        const int id1 = closest_hit<GEO, false, false, 1>(sv, s.o, s.d, 0.001f, &t1);
        if (id1 >= 0) TriDualChain<1, B, SMALL>::run(P, sv, s, id1, t1);
        return;
    }
    if (geo_pairs(GEO) && !SPH && B > 1) {
        float t = 1000.0f;                                  // sampling.metal:155
        const int id = closest_hit<GEO, false, true, 0>(sv, s.o, s.d, 0.001f, &t);
        if (id >= 0) FusedChain<0, B, GEO, SMALL>::run(P, sv, s, id, t);
    } else {
        BounceChain<0, B, GEO, SPH, SMALL>::run(P, sv, s);
    }
}

// In-order sum of the L colours of a pixel's lanes at its group leader, with
// DPP row shifts (row_shl:k: lane i reads lane i + k of its 16-lane row).  The
// sphere kernel keeps ds_bpermute shuffles (its DPP form spilled 3 more VGPRs:
// 2,715 vs 2,724 Msamples/s).
template <int k>
__device__ __forceinline__ float row_shl(float v) {
    if constexpr (k == 0) {
        return v;
    } else {
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x100 + k, 0xF, 0xF, false));
    }
}
template <int L, int k>
struct row_sum_in_order {
    __device__ __forceinline__ static void run(f3& acc, f3 c, uint32_t n0, uint32_t spp) {
        if (n0 + (uint32_t)k < spp)  // wave-uniform: the round's last samples may be past spp
            acc = acc + f3{row_shl<k>(c.x), row_shl<k>(c.y), row_shl<k>(c.z)};
        row_sum_in_order<L, k + 1>::run(acc, c, n0, spp);
    }
};
template <int L>
struct row_sum_in_order<L, L> {
    __device__ __forceinline__ static void run(f3&, f3, uint32_t, uint32_t) {}
};

// The pixel store (raytrace.metal:109): float4(luminance, 1) as rgba32F, as
// the reference's rgba16F texture (renderer.swift:74-82), or that texture
// tonemapped to the reference's 8-bit image (RTrace/image.swift:35-65: fp16
// read-back, then rt::tonemap_channel) -- 16, 8 or 4 bytes, one store.
__device__ __forceinline__ void store_pixel(const KParams& P, size_t o, float r, float g, float b) {
    if (P.flags & kOutRgba8) {
        const uint8_t cr = tonemap_channel(__half2float(__float2half_rn(r)));
        const uint8_t cg = tonemap_channel(__half2float(__float2half_rn(g)));
        const uint8_t cb = tonemap_channel(__half2float(__float2half_rn(b)));
        reinterpret_cast<uchar4*>(P.out)[o] = make_uchar4(cr, cg, cb, 255);
    } else if (P.flags & kOutFp16) {
        ushort4 h;
        h.x = __half_as_ushort(__float2half_rn(r));
        h.y = __half_as_ushort(__float2half_rn(g));
        h.z = __half_as_ushort(__float2half_rn(b));
        h.w = __half_as_ushort(__float2half_rn(1.0f));
        reinterpret_cast<ushort4*>(P.out)[o] = h;
    } else {
        reinterpret_cast<float4*>(P.out)[o] = make_float4(r, g, b, 1.0f);
    }
}

// ---- sorted-path variant ----------------------------------------------------
// Between bounces the 256 paths of a workgroup are counting-sorted through LDS
// by the octant of their next direction, dead paths last (9 buckets).  Waves
// then hold live rays of one octant: the wave-level segment culling of
// closest_hit works for bounce rays too, and finished paths no longer idle
// lanes.  Each path carries its owner pixel; at the end of a sample every path
// hands its accumulatedColor to its owner through LDS, and the owner adds it
// to its running sum in sample order n = 0, 1, ... exactly as before.
constexpr uint32_t kSortBuckets = 9;
// LDS layout of the sorted kernel: fixed offsets (in float4) from the dynamic
// LDS base, scene records after them.
constexpr uint32_t kSortA = 0;                            // (o.xyz, thr.x)   [256]
constexpr uint32_t kSortB = kBlockThreads;                // (d.xyz, thr.y)   [256]
constexpr uint32_t kSortC = 2 * kBlockThreads;            // (acc.xyz, thr.z) [256]
constexpr uint32_t kSortD = 3 * kBlockThreads;            // uint2 (i, owner)  [256]
constexpr uint32_t kSortLum = kSortD + kBlockThreads / 2;  // float sum x[256], y[256], z[256]
constexpr uint32_t kSortCnt = kSortLum + 3 * kBlockThreads / 4;  // uint [bucket][wave]
constexpr uint32_t kSortF4 = kSortCnt + (kSortBuckets * 4 + 3) / 4;

__device__ __forceinline__ uint32_t sort_octant(f3 d) {
    return (d.x > 0.0f ? 4u : 0u) | (d.y > 0.0f ? 2u : 0u) | (d.z > 0.0f ? 1u : 0u);
}

// Counting sort of the workgroup's live paths by the octant of their next
// direction (buckets 0-7); dead paths (bucket 8) are dropped — they have
// already handed their colour to their pixel.  All 256 threads must call it
// (two barriers).  Afterwards lanes tid < n_live hold a path: o, d, i and owner
// are reloaded here, thr/acc later by load_thr_acc (same slot, valid until the
// next sort), which keeps them out of registers during the intersection loops.
__device__ __forceinline__ void sort_paths(float4* lds, PathState& s, uint32_t& owner,
                                           bool& alive) {
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63u;
    uint32_t* counts = reinterpret_cast<uint32_t*>(lds + kSortCnt);
    const uint32_t key = alive ? sort_octant(s.d) : 8u;
    uint32_t my_count = 0, slot = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSortBuckets - 1; ++k) {
        const unsigned long long m = __ballot(key == k);
        if (lane == k) my_count = (uint32_t)__popcll(m);
        if (key == k) slot = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    }
    if (lane < kSortBuckets - 1) counts[lane * 4u + wave] = my_count;
    __syncthreads();
    // Exclusive scan of the 32 counts in (bucket, wave) order, redundantly in
    // every wave (lanes 32-63 repeat lanes 0-31): entry (key, wave) is where
    // this wave's paths of bucket `key` start.
    const uint32_t idx = lane & 31u;
    const uint32_t c = counts[idx];
    uint32_t v = c;
#pragma unroll
    for (uint32_t off = 1; off < 32; off <<= 1) {
        const uint32_t t = __shfl_up(v, off);
        if (idx >= off) v += t;
    }
    const uint32_t live = __shfl(v, 31);
    slot += __shfl(v - c, (int)(key * 4u + wave));
    if (alive) {
        lds[kSortA + slot] = make_float4(s.o.x, s.o.y, s.o.z, s.thr.x);
        lds[kSortB + slot] = make_float4(s.d.x, s.d.y, s.d.z, s.thr.y);
        lds[kSortC + slot] = make_float4(s.acc.x, s.acc.y, s.acc.z, s.thr.z);
        reinterpret_cast<uint2*>(lds + kSortD)[slot] = make_uint2(s.i, owner);
    }
    // thr/acc now live in LDS only (reloaded by load_thr_acc): end their
    // register live ranges here.
    s.thr = f3{0.0f, 0.0f, 0.0f};
    s.acc = f3{0.0f, 0.0f, 0.0f};
    __syncthreads();
    alive = tid < live;
    if (alive) {
        const float4 a = lds[kSortA + tid], bq = lds[kSortB + tid];
        const uint2 dd = reinterpret_cast<const uint2*>(lds + kSortD)[tid];
        s.o = f3{a.x, a.y, a.z};
        s.d = f3{bq.x, bq.y, bq.z};
        s.i = dd.x;
        owner = dd.y;
    }
}

__device__ __forceinline__ void load_thr_acc(const float4* lds, PathState& s) {
    const uint32_t tid = threadIdx.x;
    const float4 c = lds[kSortC + tid];
    s.thr = f3{lds[kSortA + tid].w, lds[kSortB + tid].w, c.w};
    s.acc = f3{c.x, c.y, c.z};
}

// A finished path adds its accumulatedColor to its pixel's running sum in LDS
// (raytrace.metal:103).  Each pixel gets exactly one path per sample and
// samples are separated by barriers, so the additions keep the order n.
__device__ __forceinline__ void deliver(float4* lds, uint32_t owner, f3 acc) {
    float* sum = reinterpret_cast<float*>(lds + kSortLum);
    sum[owner] = sum[owner] + acc.x;
    sum[kBlockThreads + owner] = sum[kBlockThreads + owner] + acc.y;
    sum[2 * kBlockThreads + owner] = sum[2 * kBlockThreads + owner] + acc.z;
}

// GEO: kGeoPairLds (pair records in LDS, wave-culled loops), kGeoTriBvh
// (triangle BVH: camera rays as wave packets, bounce rays per lane) or
// kGeoSphLds (the room's pairs in LDS + the compact sphere BVH).  For the BVH
// scenes the sort is what the lockstep kernels lack: the waves of a bounce
// walk rays of ONE direction octant, i.e. ONE of the eight BVH layouts.
template <int b, int B, int GEO, bool SPH, bool SMALL>
struct SortedChain {
    __device__ __forceinline__ static void run(const KParams& P, const SceneView& sv, float4* lds,
                                               PathState& s, uint32_t& owner, bool& alive) {
        if (b > 0) sort_paths(lds, s, owner, alive);
        if (alive) {
            float t = 1000.0f;                                   // sampling.metal:154-155
            constexpr bool cull = GEO == kGeoTriBvh ? b == 0 : true;
            const int id = closest_hit<GEO, SPH, cull, (b == 0 ? 0 : 1)>(sv, s.o, s.d, 0.001f, &t);
            if (b > 0) load_thr_acc(lds, s);
            alive = id >= 0 && shade<b, B, GEO, SPH, SMALL>(P, sv, s, id, t);
            if (!alive || b + 1 == B) deliver(lds, owner, s.acc);
        }
        SortedChain<b + 1, B, GEO, SPH, SMALL>::run(P, sv, lds, s, owner, alive);
    }
};
template <int B, int GEO, bool SPH, bool SMALL>
struct SortedChain<B, B, GEO, SPH, SMALL> {
    __device__ __forceinline__ static void run(const KParams&, const SceneView&, float4*,
                                               PathState&, uint32_t&, bool&) {}
};


}  // namespace

constexpr int kMinWavesPerEu = 8;     // 8 waves/SIMD (<= 64 VGPRs): +4.5% measured over 7
constexpr int kMinWavesPerEuSph = 8;  // sphere kernel: 7 / 6 waves 162.2 / 176.3 ms vs 154.3
constexpr uint32_t kHaltonTabMinRounds = 8;  // samples per lane below which no tables
// Whether a launch fills the LDS low-digit Halton tables: box-cluster kernel,
// fixed-digit indices, and every lane tracing enough samples to amortise the
// fill (~700 VALU per thread): config 1 (1 spp) runs without them.  The kernel
// and the launcher's rt_last_launch report share this one definition.
__host__ __device__ constexpr bool halton_tables_on(int geo, bool small, uint32_t spp, uint32_t L) {
    return geo == kGeoPairClu && small && (spp + L - 1) / L >= kHaltonTabMinRounds;
}
// box-cluster kernel: 7 waves/SIMD runs as fast as 8 and spills 6 VGPRs
// instead of 30 (HBM traffic 146 MB instead of 19 GB per 1080p launch)
#ifndef RT_CLU_WAVES
#define RT_CLU_WAVES 7
#endif
constexpr int kMinWavesPerEuClu = RT_CLU_WAVES;
// L lanes per pixel (1, 4 or 16: more lanes when the launch has few pixels,
// e.g. one GPU's share of a multi-GPU frame): lane `sub` of a pixel's
// group traces samples n = r*L + sub of round r, and after every round the L
// colours are shuffled within the wave and added to the pixel's sum in sample
// order n — the same sequence of fp32 additions as one lane per pixel.
// Workgroup size: one wave for the sphere kernel (rt_kernel.hpp
// kSphBlockThreads), 256 threads (2x2 waves) otherwise -- the box-cluster
// kernel at 128 / 64 / 512 threads ran 40.1 / 68.9 / 27.8 ms vs 26.2 (its 22 KB
// of Halton tables per workgroup then cap the waves per CU), the
// triangle-BVH kernel at 64 / 128 threads 204.3 / 192.1 ms vs 180.7.
constexpr uint32_t block_threads(int geo) { return geo == kGeoSphLds ? kSphBlockThreads : kBlockThreads; }
constexpr uint32_t waves_per_row(int geo) { return block_threads(geo) >= 128 ? 2u : 1u; }
constexpr uint32_t waves_per_col(int geo) { return block_threads(geo) / 64u / waves_per_row(geo); }

template <int B, int GEO, bool SPH, bool SMALL, int L = 1>
#ifndef RT_TRI_WAVES
#define RT_TRI_WAVES 8
#endif
__global__ __launch_bounds__(block_threads(GEO),
                             SPH ? kMinWavesPerEuSph
                                 : (GEO == kGeoPairClu ? kMinWavesPerEuClu
                                                       : (GEO == kGeoTriBvh ? RT_TRI_WAVES : kMinWavesPerEu)))
void path_trace_kernel(KParams P) {
    constexpr uint32_t NT = block_threads(GEO), WR = waves_per_row(GEO), WC = waves_per_col(GEO);
    extern __shared__ float4 lds[];
    SceneView sv;
    sv.nT = P.nT;
    sv.nP = P.nP;
    sv.nS = SPH ? P.nS : 0u;
    if (GEO == kGeoPairSmem) {
        sv.tri = nullptr;
        sv.pair = P.pair_isect;
    } else if (GEO != kGeoTriGlobal && GEO != kGeoTriBvh) {
        // Stage the intersection records once per workgroup.
        constexpr bool pairs = GEO == kGeoPairLds || GEO == kGeoPairClu || GEO == kGeoSphLds;
        const uint32_t ng4 = pairs ? kPairF4 * sv.nP : 3u * sv.nT;
        const float4* src = pairs ? P.pair_isect : P.tri_isect;
        RT_LDS_GUARD(16 * (size_t)(ng4 + (GEO == kGeoPairClu ? (kCluF4 + kCluOctF4) * P.nC : 0u)) +
                     (GEO == kGeoPairClu ? 4 * (size_t)kHaltonTabFloats : 0));
        for (uint32_t k = threadIdx.x; k < ng4; k += NT) lds[k] = src[k];
        if (GEO == kGeoSphLds) {  // the compact sphere BVH (8 layouts) stays in global memory (L2)
            sv.sent = reinterpret_cast<const uint4*>(P.sph_lds);
            sv.sid = P.sph_lds_id;
            sv.sbox = P.sph_box;
            sv.nSB = P.nN;
            __shared__ float sph_stash[GEO == kGeoSphLds ? 6 * kSphBlockThreads : 1];
            sv.xstash = sph_stash;
        }
        if (GEO == kGeoPairClu) {  // box clusters after the pair records, then the Halton tables
            for (uint32_t k = threadIdx.x; k < kCluF4 * P.nC; k += NT) lds[ng4 + k] = P.clusters[k];
            for (uint32_t k = threadIdx.x; k < kCluOctF4 * P.nC; k += NT)
                lds[ng4 + kCluF4 * P.nC + k] = P.clu_oct[k];
            sv.clu_oct = kCluOctF4 ? lds + ng4 + kCluF4 * P.nC : nullptr;
            const uint32_t tab0 = ng4 + (kCluF4 + kCluOctF4) * P.nC;
            const bool tab = halton_tables_on(GEO, SMALL, P.spp, L);
            sv.htab = tab ? reinterpret_cast<const float*>(lds + tab0) : nullptr;
            if (tab) fill_halton_tables(reinterpret_cast<float*>(lds + tab0), threadIdx.x, NT);
        }
        __syncthreads();
        sv.tri = lds;
        sv.pair = lds;
        sv.clu = lds + ng4;
        sv.nC = P.nC;
        sv.pair_free = P.pair_free;
    } else {
        sv.tri = P.tri_isect;
        sv.pair = nullptr;
    }
    if (GEO == kGeoTriBvh && RT_TRI_STASH) {  // per-lane stash of shade() across the shadow walks
        __shared__ float tri_stash[GEO == kGeoTriBvh && RT_TRI_STASH ? 6 * kBlockThreads : 1];
        sv.xstash = tri_stash;
    }
    sv.tnode = P.tri_nodes;
    sv.tsorted = P.tri_sorted;
    sv.tperm = P.tri_perm;
    sv.nTN = P.nTN;
    sv.node = P.sph_nodes;  // sphere BVH: scalar loads from global memory
    sv.sph = P.sph_isect;
    // sphere walks: BVH nodes per layout (global walks) or compact LDS entries
    sv.nN = SPH ? (GEO == kGeoSphLds ? P.nE : P.nN) : 0u;
    sv.sph_perm = P.sph_perm;

    // wave = 64/L pixels: 8x8 (L=1), 4x4 (L=4), 2x2 (L=16), or one row of 64/L
    // pixels for interleaved rows (launcher's wave_w); workgroup = 2x2 waves
    const uint32_t kWX = (L == 1) ? 8u : P.wave_w, kWY = (64u / L) / kWX;
    // XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs in
    // dispatch order (p = blockIdx.y * gridDim.x + blockIdx.x; MI355X_MICROARCH.md
    // "Workgroup dispatch"), so the tiles are dealt in runs of kXcdRun: the run
    // of neighbouring tiles that share the 128-B lines of the seed rows goes
    // through ONE XCD's L2 (seed reads 4x -> 1x the seed bytes), while the runs
    // still interleave over the XCDs, which keeps the cheap and the expensive
    // image regions evenly spread (contiguous bands per XCD ran 7 % slower).
    // Speed only: every tile is rendered exactly once.
    uint32_t bx, by;
    {
        constexpr uint32_t kXcdRun = 4;  // runs of 0 (plain order) / 16: 158.9 / 157.6 vs 158.4 ms on config 4
        const uint32_t n = gridDim.x * gridDim.y, full = n / (8u * kXcdRun + (kXcdRun == 0)) * (8u * kXcdRun);
        const uint32_t p = blockIdx.y * gridDim.x + blockIdx.x;
        uint32_t t = p;
        if (kXcdRun > 0 && p < full) {
            const uint32_t xcd = p % 8u, k = p / 8u;
            t = ((k / kXcdRun) * 8u + xcd) * kXcdRun + k % kXcdRun;
        }
        bx = t % gridDim.x;
        by = t / gridDim.x;
    }
    auto pixel_of = [&](uint32_t t, uint32_t& x, uint32_t& j) {
        const uint32_t lane = t & 63u, wave = t >> 6, pix = lane / L;
        x = bx * (WR * kWX) + (wave % WR) * kWX + (pix % kWX);
        j = by * (WC * kWY) + (wave / WR) * kWY + (pix / kWX);
    };
    // Per-lane constants (pixel coordinates, lane roles) are recomputed from an
    // opaque copy of threadIdx.x where they are used, and the seed is kept in
    // LDS: otherwise the compiler hoists them out of the sample loop and spills
    // them to scratch for the whole launch (36 B/lane of scratch writes).
    // Only for the box-cluster and LDS-sphere kernels: the triangle-BVH walk
    // kernel (global-memory nodes) ran 16 % slower with the opaque copies
    // (325 vs 281 ms, 10k triangles) and spills about as much without them.
    constexpr bool kRemat = GEO == kGeoPairClu || GEO == kGeoSphLds;
    auto opaque_tid = []() {
        uint32_t t = threadIdx.x;
        if constexpr (kRemat) asm volatile("" : "+v"(t));
        return t;
    };
    {
        uint32_t x, j;
        pixel_of(threadIdx.x, x, j);
        if (x >= (uint32_t)P.W || j >= P.row_count) return;  // a pixel's L lanes leave together
    }
    __shared__ uint32_t seed_s[NT];        // seed + sample_base of the lane's pixel
    __shared__ float lum_s[L > 1 ? 3 * (NT / L) : 1];
    f3 lum{0.0f, 0.0f, 0.0f};                                    // :32
    {
        const uint32_t t = threadIdx.x, sub = t % L;
        uint32_t x, j;
        pixel_of(t, x, j);
        const uint32_t y = P.row_start + j * P.row_step;
        seed_s[t] = P.seeds[(size_t)y * (size_t)P.W + x] + P.sample_base;  // raytrace.metal:37
        if (P.accumulate) {
            const float4 prev = P.sum[(size_t)j * (size_t)P.W + x];
            lum = f3{prev.x, prev.y, prev.z};
        }
        // L > 1: the pixel's running sum lives in LDS (its group leader adds to
        // it), which keeps three VGPRs free across the path traversal
        const uint32_t slot = t / L;
        if (L > 1 && sub == 0) {
            lum_s[3 * slot] = lum.x;
            lum_s[3 * slot + 1] = lum.y;
            lum_s[3 * slot + 2] = lum.z;
        }
    }
    const f3 cu = ld_f3(P.cam_u), cv = ld_f3(P.cam_v), cw = ld_f3(P.cam_w);
    const float fW = (float)P.W, fH = (float)P.H;
    const uint32_t rounds = (P.spp + (L - 1)) / L;
    for (uint32_t r = 0; r < rounds; ++r) {                      // :34
#ifdef RT_STATS
        const unsigned long long t_round = clock64();  // slot 24: cycles of whole rounds
#endif
        const uint32_t t = opaque_tid(), sub = t % L;
        // a lane past the last sample re-traces the last one (discarded below):
        // no divergent branch around the path
        const uint32_t n = (L == 1) ? r : min(r * L + sub, P.spp - 1u);
        PathState s;
        s.acc = f3{0.0f, 0.0f, 0.0f};
        {
            uint32_t x, j;
            pixel_of(t, x, j);
            const float fx = (float)x, fy = (float)(P.row_start + j * P.row_step);
            s.i = seed_s[t] + n;                                 // seed + (sample_base + n)
            const float jx = halton_dim<0, SMALL>(s.i);                                // :39-40
            const float jy = halton_dim<1, SMALL, GEO == kGeoPairClu>(s.i, sv.htab);
            // generateCameraRay (sampling.metal:125-157)
            const float sx = ((fx + jx) / fW) * 2.0f - 1.0f;
            const float ty = -(((fy + jy) / fH) * 2.0f - 1.0f);
            const float sh = sx * P.halfW, th = ty * P.halfH;
            s.d = GEO != kGeoTriBvh ? normalize((cu * sh + cv * th) - cw) : normalize_ieee((cu * sh + cv * th) - cw);
            s.o = ld_f3(P.cam_pos);
            s.thr = f3{1.0f, 1.0f, 1.0f};
#if RT_CENSUS == 1
            {
                const uint32_t i2 = cz(s.i);
                const float jx2 = halton_dim<0, SMALL>(i2);
                const float jy2 = halton_dim<1, SMALL, GEO == kGeoPairClu>(i2, sv.htab);
                const float sx2 = ((cz(fx) + jx2) / fW) * 2.0f - 1.0f;
                const float ty2 = -(((cz(fy) + jy2) / fH) * 2.0f - 1.0f);
                cz_sink(normalize((cu * (sx2 * P.halfW) + cv * (ty2 * P.halfH)) - cw));
            }
#endif
#ifndef RT_TIMING_NO_TRACE  // timing-only A/B (tools/ab_kernel.sh): camera, Halton jitter and sums alone
            trace_path<B, GEO, SPH, SMALL>(P, sv, s);                       // :47-102
#else
            s.acc = s.d;
#endif
        }
        if (L == 1) {
            lum = lum + s.acc;                                   // :103
#ifndef RT_SPH_DPP
#define RT_SPH_DPP 0
#endif
        } else if (L <= 16 && (!SPH || RT_SPH_DPP)) {
            // a pixel's L lanes are consecutive lanes of one 16-lane DPP row
            // (L = 4: groups at 0, 4, 8, 12; L = 16: the whole row), so its
            // leader reads sample r*L + k from lane +k with a row shift fused
            // into the add (v_add_f32_dpp row_shl:k) -- the same additions in
            // sample order, no LDS-pipe traffic.  Only the leaders' sums are kept.
            const uint32_t t2 = opaque_tid(), sub2 = t2 % L, slot = t2 / L;
            f3 acc{lum_s[3 * slot], lum_s[3 * slot + 1], lum_s[3 * slot + 2]};
#if RT_CENSUS == 6
            {
                f3 a2 = cz(acc);
                row_sum_in_order<L, 0>::run(a2, cz(s.acc), r * L, P.spp);
                cz_sink(a2);
            }
#endif
            row_sum_in_order<L, 0>::run(acc, s.acc, r * L, P.spp);  // :103
            if (sub2 == 0) {
                lum_s[3 * slot] = acc.x;
                lum_s[3 * slot + 1] = acc.y;
                lum_s[3 * slot + 2] = acc.z;
            }
        } else {
            const uint32_t t2 = opaque_tid(), lane = t2 & 63u, sub2 = t2 % L, slot = t2 / L;
            const int base = (int)(lane - sub2);
            f3 c[L];
#pragma unroll
            for (int k = 0; k < L; ++k)                          // samples r*L + k
                c[k] = f3{__shfl(s.acc.x, base + k), __shfl(s.acc.y, base + k),
                          __shfl(s.acc.z, base + k)};
            if (sub2 == 0) {
                f3 acc{lum_s[3 * slot], lum_s[3 * slot + 1], lum_s[3 * slot + 2]};
#pragma unroll
                for (int k = 0; k < L; ++k)                      // in sample order
                    if (r * L + (uint32_t)k < P.spp) acc = acc + c[k];  // :103
                lum_s[3 * slot] = acc.x;
                lum_s[3 * slot + 1] = acc.y;
                lum_s[3 * slot + 2] = acc.z;
            }
        }
#ifdef RT_STATS
        if (!SPH && GEO != kGeoTriBvh) {  // 24-31: the BVH any-hit walks' there
            RT_STAT(24, clock64() - t_round);
            RT_STAT(25, 1);
        }
#endif
    }
    // the pixel of the epilogue, recomputed from an opaque copy of threadIdx.x
    // in every kernel: otherwise the prologue's pixel offsets are kept (and
    // spilled) across the whole sample loop
    uint32_t t = threadIdx.x;
    asm volatile("" : "+v"(t));
    if (L > 1) {
        if (t % L != 0) return;
        const uint32_t slot = t / L;
        lum = f3{lum_s[3 * slot], lum_s[3 * slot + 1], lum_s[3 * slot + 2]};
    }
    uint32_t x, j;
    pixel_of(t, x, j);
    const size_t o = (size_t)j * (size_t)P.W + x;
    if (P.sum) P.sum[o] = make_float4(lum.x, lum.y, lum.z, (float)P.samples_total);
    if (P.out) {
        const float fs = (float)P.samples_total;                 // :106
        const float r = lum.x / fs, g = lum.y / fs, bl = lum.z / fs;
        store_pixel(P, o, r, g, bl);
    }
}

#include "rt_free.hpp"

// waves per SIMD of the sorted kernel: the pair layout keeps 8; the BVH walks
// hold more state (RTPT A/B: sorted_waves)
#ifndef RT_SORTED_BVH_WAVES
#define RT_SORTED_BVH_WAVES 4
#endif
template <int B, int GEO, bool SPH, bool SMALL>
__global__ __launch_bounds__(kBlockThreads, GEO == kGeoPairLds ? kMinWavesPerEu : RT_SORTED_BVH_WAVES)
void path_trace_sorted_kernel(
    KParams P) {
    extern __shared__ float4 lds[];
    SceneView sv;
    sv.nT = P.nT;
    sv.nP = P.nP;
    sv.nS = SPH ? P.nS : 0u;
    sv.nC = 0;
    sv.htab = nullptr;
    const uint32_t ng4 = GEO == kGeoTriBvh ? 0u : kPairF4 * sv.nP;
    RT_LDS_GUARD(16 * (size_t)(kSortF4 + ng4));
    float4* scene = lds + kSortF4;  // sort buffers first: compile-time offsets
    for (uint32_t k = threadIdx.x; k < ng4; k += kBlockThreads) scene[k] = P.pair_isect[k];
    sv.nN = SPH ? (GEO == kGeoSphLds ? P.nE : P.nN) : 0u;
    sv.sent = reinterpret_cast<const uint4*>(P.sph_lds);
    sv.sid = P.sph_lds_id;
    sv.sbox = P.sph_box;
    sv.nSB = P.nN;
    sv.tnode = P.tri_nodes;
    sv.tsorted = P.tri_sorted;
    sv.tperm = P.tri_perm;
    sv.nTN = P.nTN;
    sv.tri = scene;
    sv.pair = scene;
    sv.node = P.sph_nodes;
    sv.sph = P.sph_isect;
    sv.sph_perm = P.sph_perm;

    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t x = blockIdx.x * kTile + (wave & 1u) * 8u + (lane & 7u);
    const uint32_t j = blockIdx.y * kTile + (wave >> 1) * 8u + (lane >> 3);
    const bool valid = x < (uint32_t)P.W && j < P.row_count;  // every thread stays (barriers)
    const uint32_t y = P.row_start + j * P.row_step;
    const size_t o = (size_t)j * (size_t)P.W + x;
    const uint32_t seed = valid ? P.seeds[(size_t)y * (size_t)P.W + x] : 0u;  // raytrace.metal:37
    float* sum = reinterpret_cast<float*>(lds + kSortLum);
    {
        float4 prev = make_float4(0.0f, 0.0f, 0.0f, 0.0f);   // luminance = 0 (:32)
        if (valid && P.accumulate) prev = P.sum[o];
        sum[tid] = prev.x;
        sum[kBlockThreads + tid] = prev.y;
        sum[2 * kBlockThreads + tid] = prev.z;
    }
    __syncthreads();
    const float fx = (float)x, fy = (float)y, fW = (float)P.W, fH = (float)P.H;
    for (uint32_t n = 0; n < P.spp; ++n) {                       // :34
        PathState s;
        s.i = seed + (P.sample_base + n);
        s.acc = f3{0.0f, 0.0f, 0.0f};
        s.thr = f3{1.0f, 1.0f, 1.0f};
        s.o = ld_f3(P.cam_pos);
        s.d = f3{0.0f, 0.0f, 0.0f};
        if (valid) {
            const float jx = halton_dim<0, SMALL>(s.i), jy = halton_dim<1, SMALL>(s.i);
            const float sx = ((fx + jx) / fW) * 2.0f - 1.0f;
            const float ty = -(((fy + jy) / fH) * 2.0f - 1.0f);
            const float sh = sx * P.halfW, th = ty * P.halfH;
            s.d = normalize((ld_f3(P.cam_u) * sh + ld_f3(P.cam_v) * th) - ld_f3(P.cam_w));
        }
        uint32_t owner = tid;
        bool alive = valid;
        SortedChain<0, B, GEO, SPH, SMALL>::run(P, sv, lds, s, owner, alive);
        __syncthreads();  // sample n's hand-offs land before sample n+1's
    }
    if (!valid) return;
    const f3 lum{sum[tid], sum[kBlockThreads + tid], sum[2 * kBlockThreads + tid]};
    if (P.sum) P.sum[o] = make_float4(lum.x, lum.y, lum.z, (float)P.samples_total);
    if (P.out) {
        const float fs = (float)P.samples_total;                 // :106
        const float r = lum.x / fs, g = lum.y / fs, bl = lum.z / fs;
        store_pixel(P, o, r, g, bl);
    }
}

// rt_math_selfcheck: the shipped sqrt_cr / rcp_cr (rt_math.h) against the
// IEEE sqrtf / division on every float bit pattern b in [lo, lo + n): bad[0]
// counts sqrt mismatches (NaN results compare as NaN), bad[1] reciprocal ones.
__global__ void math_check_kernel(uint32_t lo, uint32_t n, unsigned long long* bad) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const float x = __uint_as_float(lo + i);
        float y = x;
        asm volatile("" : "+v"(y));  // an opaque copy: the references stay the IEEE expansions
        const float s = sqrt_cr(x), sr = sqrtf(y);
        const float r = rcp_cr(x), rr = 1.0f / y;
        const bool sbad = !(__float_as_uint(s) == __float_as_uint(sr) || (s != s && sr != sr));
        const bool rbad = !(__float_as_uint(r) == __float_as_uint(rr) || (r != r && rr != rr));
        if (sbad) atomicAdd(&bad[0], 1ull);
        if (rbad) atomicAdd(&bad[1], 1ull);
    }
}

__global__ void fill_seeds_kernel(uint32_t* seeds, uint64_t key, uint64_t n) {
    for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
         p += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = key + p + 0x9E3779B97F4A7C15ULL;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        z = z ^ (z >> 31);
        seeds[p] = (uint32_t)(z & 0xFFFFFu);
    }
}

// Placement of the gathered row tiles (rt_render_gather / rt_place_tiles): one
// thread per U-byte unit of the frame, consecutive threads along a row, so the
// reads (a tile row) and the writes (a frame row) are both coalesced.  A
// kernel on the caller's stream rather than N strided hipMemcpy2DAsync: a
// device-to-device 2D copy enqueued on the null stream was measured to start
// before the kernels enqueued ahead of it had finished (it read the gather
// buffer's previous contents), and the kernel is one launch whatever N.
// Frames taller than the grid's y extent walk their rows with a grid stride.
template <typename U>
__global__ void place_tiles_kernel(const U* __restrict__ gathered, U* __restrict__ frame, uint32_t row_u,
                                   size_t tile_u, uint32_t H, uint32_t N) {
    for (uint32_t y = blockIdx.y; y < H; y += gridDim.y) {
        const uint32_t k = y % N, j = y / N;
        const U* src = gathered + k * tile_u + (size_t)j * row_u;
        U* dst = frame + (size_t)y * row_u;
        for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < row_u; u += gridDim.x * blockDim.x)
            dst[u] = src[u];
    }
}

hipError_t launch_place_tiles(const void* gathered, void* frame, size_t row_bytes, size_t tile_bytes,
                              uint32_t H, uint32_t N, hipStream_t stream) {
    if (H == 0 || N == 0 || row_bytes == 0) return hipSuccess;
    if (row_bytes % 4 || tile_bytes % 4) return hipErrorInvalidValue;
    const bool wide = row_bytes % 16 == 0 && tile_bytes % 16 == 0 &&
                      reinterpret_cast<uintptr_t>(gathered) % 16 == 0 && reinterpret_cast<uintptr_t>(frame) % 16 == 0;
    const size_t unit = wide ? 16 : 4;
    const uint32_t row_u = (uint32_t)(row_bytes / unit);
    const dim3 grid((row_u + 255u) / 256u, H < 65535u ? H : 65535u);  // grid.y limit: rows by grid stride
    if (wide)
        hipLaunchKernelGGL(place_tiles_kernel<uint4>, grid, dim3(256), 0, stream,
                           static_cast<const uint4*>(gathered), static_cast<uint4*>(frame), row_u,
                           tile_bytes / 16, H, N);
    else
        hipLaunchKernelGGL(place_tiles_kernel<uint32_t>, grid, dim3(256), 0, stream,
                           static_cast<const uint32_t*>(gathered), static_cast<uint32_t*>(frame), row_u,
                           tile_bytes / 4, H, N);
    return hipGetLastError();
}

namespace {

// Lanes per pixel (measured on one GPU's share of the N-GPU weak-scaling frame,
// tools/bench_share.py): 4 for whole frames of ~1 M pixels and more (also +6 % on
// the whole 1080p frame: 4x4-pixel waves, more lanes in flight), 16 below that
// and for interleaved shares, never more than spp.  The LDS sphere-walk kernel
// takes 16 at every size (measured on config 4, the whole 1080p frame: 198.4 ms
// at 16 lanes, 204.8 at 4, 227.6 at 1).
inline int lanes_per_pixel(const KParams& P, int geo) {
    if (P.lanes == 1 || P.lanes == 4 || P.lanes == 16) return P.spp >= P.lanes ? (int)P.lanes : 1;
    const uint64_t px = (uint64_t)P.W * P.row_count;
    // interleaved rows (a rank's share of a multi-GPU frame) take 16 lanes at any
    // size when every lane still gets the Halton tables' 8 rounds (measured,
    // tools/lanes_probe.py: 1080p share of N = 2 20,229 vs 19,922; 4096^2 share
    // of N = 8 19,450 vs 18,824); whole frames of >= 1 M pixels keep 4 (1080p
    // 20,288 vs 20,143; 4096^2 18,505 vs 17,978)
    const bool share16 = P.row_step > 1 && P.spp >= 16u * kHaltonTabMinRounds;
    // the BVH walk kernels (spheres, and since round 6 triangles) take 16 at any
    // size: triangles 100k / 10k / 1M at 1080p x 64 spp 1,176 / 1,234 / 575
    // Msamples/s with 16 lanes vs 1,101 / 1,172 / 514 with 4
    const int want = (px >= 1000000ull && geo != kGeoSphLds && geo != kGeoTriBvh && !share16) ? 4 : 16;
    if (P.spp >= (uint32_t)want) return want;
    return P.spp >= 4 ? 4 : 1;
}

constexpr int kGeoPairSorted = kLayPairSorted;
constexpr int kGeoFreeSph = kLayFreeSph;
constexpr int kGeoFreeTri = kLayFreeTri;
constexpr int kGeoSortSph = kLaySortSph;
constexpr int kGeoSortTri = kLaySortTri;
static_assert(kGeoTriLds == kLayTriLds && kGeoPairLds == kLayPairLds && kGeoTriGlobal == kLayTriGlobal &&
                  kGeoPairSmem == kLayPairSmem && kGeoTriBvh == kLayTriBvh && kGeoPairClu == kLayPairClu &&
                  kGeoSphLds == kLaySphLds,
              "rt_trace.hpp Geo == rt_kernel.hpp KernelLayout");
static_assert(kHaltonTabLdsFloats == kHaltonTabFloats && kSortLdsF4 == kSortF4, "staged_lds_bytes terms");

// The most recent launch of this thread (launch_path_trace copies it out).
thread_local LaunchInfo g_last;

template <int B, int GEO, bool SPH, bool SMALL, int L>
void note_launch(const char* name, const KParams& P, dim3 grid, uint32_t threads, size_t lds) {
    LaunchInfo& I = g_last;
    snprintf(I.kernel, sizeof(I.kernel), "rt::%s<%d, %d, %s, %s, %d>", name, B, GEO,
             SPH ? "true" : "false", SMALL ? "true" : "false", L);
    I.lanes = (uint32_t)L;
    I.tables = halton_tables_on(GEO, SMALL, P.spp, (uint32_t)L) ? 1u : 0u;
    I.small = SMALL ? 1u : 0u;
    I.threads = threads;
    I.grid_x = grid.x;
    I.grid_y = grid.y;
    I.lds = (uint32_t)lds;
}

// Dynamic LDS above 64 KB must be allowed per kernel (the compact sphere BVH).
inline hipError_t allow_lds(const void* kernel, size_t bytes) {
    if (bytes <= 65536) return hipSuccess;
    return hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

template <int B, int GEO, bool SPH, bool SMALL, int L>
hipError_t launch_tl(const KParams& P, size_t lds_bytes, hipStream_t stream) {
    KParams Q = P;
    // wave tile: compact (4x4, 2x2) for whole frames; one row of 64/L pixels
    // when the rows are interleaved (row_step > 1), which keeps a wave's camera
    // rays adjacent in the image (N = 8 share: 10,822 -> 11,211 Msamples/s)
    Q.wave_w = (P.row_step > 1) ? 64u / L : (L == 4 ? 4u : 2u);
    constexpr uint32_t WR = waves_per_row(GEO), WC = waves_per_col(GEO);
    const uint32_t TX = WR * Q.wave_w, TY = WC * ((64u / L) / Q.wave_w);
    const dim3 grid((P.W + TX - 1) / TX, (P.row_count + TY - 1) / TY);
    if (GEO == kGeoSphLds) {
        const hipError_t e = allow_lds((const void*)path_trace_kernel<B, GEO, SPH, SMALL, L>, lds_bytes);
        if (e != hipSuccess) return e;
    }
    const size_t lds = lds_bytes;  // staged_lds_bytes of the layout
    note_launch<B, GEO, SPH, SMALL, L>("path_trace_kernel", Q, grid, block_threads(GEO), lds);
    hipLaunchKernelGGL((path_trace_kernel<B, GEO, SPH, SMALL, L>), grid, dim3(block_threads(GEO)),
                       lds, stream, Q);
    return hipGetLastError();
}

template <int B, int GEO, bool SPH, bool SMALL>
hipError_t launch_t(const KParams& P, size_t lds_bytes, hipStream_t stream) {
    if (SMALL) {
        const int lpp = lanes_per_pixel(P, GEO);
        if (lpp == 16) return launch_tl<B, GEO, SPH, SMALL, 16>(P, lds_bytes, stream);
        if (lpp == 4) return launch_tl<B, GEO, SPH, SMALL, 4>(P, lds_bytes, stream);
    }
    constexpr uint32_t TX = 8u * waves_per_row(GEO), TY = 8u * waves_per_col(GEO);  // 8x8-pixel waves
    const dim3 grid((P.W + TX - 1) / TX, (P.row_count + TY - 1) / TY);
    if (GEO == kGeoSphLds) {
        const hipError_t e = allow_lds((const void*)path_trace_kernel<B, GEO, SPH, SMALL>, lds_bytes);
        if (e != hipSuccess) return e;
    }
    const size_t lds = lds_bytes;  // staged_lds_bytes of the layout
    note_launch<B, GEO, SPH, SMALL, 1>("path_trace_kernel", P, grid, block_threads(GEO), lds);
    hipLaunchKernelGGL((path_trace_kernel<B, GEO, SPH, SMALL>), grid, dim3(block_threads(GEO)),
                       lds, stream, P);
    return hipGetLastError();
}

template <int B, int GEO>
hipError_t launch_g(const KParams& P, size_t lds_bytes, hipStream_t stream) {
    const bool small = P.max_index < kSmallIndexMax;
    if constexpr (GEO == kGeoPairClu)  // triangle-only scenes (launch_path_trace)
        return small ? launch_t<B, GEO, false, true>(P, lds_bytes, stream)
                     : launch_t<B, GEO, false, false>(P, lds_bytes, stream);
    if constexpr (GEO == kGeoSphLds)  // sphere scenes only
        return small ? launch_t<B, GEO, true, true>(P, lds_bytes, stream)
                     : launch_t<B, GEO, true, false>(P, lds_bytes, stream);
    if (P.nS > 0)
        return small ? launch_t<B, GEO, true, true>(P, lds_bytes, stream)
                     : launch_t<B, GEO, true, false>(P, lds_bytes, stream);
    return small ? launch_t<B, GEO, false, true>(P, lds_bytes, stream)
                 : launch_t<B, GEO, false, false>(P, lds_bytes, stream);
}

template <int B, int GEO, bool SPH, bool SMALL>
hipError_t launch_sorted_t(const KParams& P, size_t lds_bytes, hipStream_t stream) {
    const dim3 grid((P.W + kTile - 1) / kTile, (P.row_count + kTile - 1) / kTile);
    note_launch<B, GEO, SPH, SMALL, 1>("path_trace_sorted_kernel", P, grid, kBlockThreads, lds_bytes);
    hipLaunchKernelGGL((path_trace_sorted_kernel<B, GEO, SPH, SMALL>), grid, dim3(kBlockThreads),
                       lds_bytes, stream, P);
    return hipGetLastError();
}

template <int B, int GEO>
hipError_t launch_sorted_g(const KParams& P, size_t lds_bytes, hipStream_t stream) {
    const bool small = P.max_index < kSmallIndexMax;
    const size_t bytes = lds_bytes;  // staged_lds_bytes: path buffers + scene records
    if constexpr (GEO == kGeoSphLds)
        return small ? launch_sorted_t<B, GEO, true, true>(P, bytes, stream)
                     : launch_sorted_t<B, GEO, true, false>(P, bytes, stream);
    if constexpr (GEO == kGeoTriBvh)
        return small ? launch_sorted_t<B, GEO, false, true>(P, bytes, stream)
                     : launch_sorted_t<B, GEO, false, false>(P, bytes, stream);
    if (P.nS > 0)
        return small ? launch_sorted_t<B, GEO, true, true>(P, bytes, stream)
                     : launch_sorted_t<B, GEO, true, false>(P, bytes, stream);
    return small ? launch_sorted_t<B, GEO, false, true>(P, bytes, stream)
                 : launch_sorted_t<B, GEO, false, false>(P, bytes, stream);
}

// The free-running kernel (rt_free.hpp): one pixel per lane, 8x8-pixel waves
// (one row of 64 pixels for interleaved rows), one-wave workgroups.
template <int B, int GEO, bool SMALL>
hipError_t launch_free_t(const KParams& P, size_t lds_bytes, hipStream_t stream) {
    KParams Q = P;
    Q.wave_w = (P.row_step > 1) ? 64u : 8u;
    const uint32_t TY = 64u / Q.wave_w;
    const dim3 grid((P.W + Q.wave_w - 1) / Q.wave_w, (P.row_count + TY - 1) / TY);
    const size_t lds = lds_bytes;  // staged_lds_bytes of the layout
    note_launch<B, GEO, GEO == kGeoSphLds, SMALL, 1>("path_free_kernel", Q, grid, kFreeThreads, lds);
    hipLaunchKernelGGL((path_free_kernel<B, GEO, SMALL>), grid, dim3(kFreeThreads), lds, stream, Q);
    return hipGetLastError();
}

template <int B, int GEO>
hipError_t launch_free(const KParams& P, size_t lds_bytes, hipStream_t stream) {
    if constexpr (B < 1) {
        return hipErrorInvalidValue;
    } else {
        return P.max_index < kSmallIndexMax ? launch_free_t<B, GEO, true>(P, lds_bytes, stream)
                                            : launch_free_t<B, GEO, false>(P, lds_bytes, stream);
    }
}

template <int B>
hipError_t launch_b(const KParams& P, int geo, size_t lds_bytes, hipStream_t stream) {
    if (geo == kGeoFreeSph) return launch_free<B, kGeoSphLds>(P, lds_bytes, stream);
    if (geo == kGeoFreeTri) return launch_free<B, kGeoTriBvh>(P, lds_bytes, stream);
    if (geo == kGeoPairSorted) return launch_sorted_g<B, kGeoPairLds>(P, lds_bytes, stream);
    if (geo == kGeoSortSph) return launch_sorted_g<B, kGeoSphLds>(P, lds_bytes, stream);
    if (geo == kGeoSortTri) return launch_sorted_g<B, kGeoTriBvh>(P, lds_bytes, stream);
    switch (geo) {
        case kGeoPairLds: return launch_g<B, kGeoPairLds>(P, lds_bytes, stream);
        case kGeoPairClu: return launch_g<B, kGeoPairClu>(P, lds_bytes, stream);
        case kGeoSphLds: return launch_g<B, kGeoSphLds>(P, lds_bytes, stream);
        case kGeoPairSmem: return launch_g<B, kGeoPairSmem>(P, lds_bytes, stream);
        case kGeoTriBvh: return launch_g<B, kGeoTriBvh>(P, lds_bytes, stream);
        case kGeoTriLds: return launch_g<B, kGeoTriLds>(P, lds_bytes, stream);
        default: return launch_g<B, kGeoTriGlobal>(P, lds_bytes, stream);
    }
}

}  // namespace

size_t kernel_lds_bytes(uint32_t n_tri, uint32_t n_pairs, uint32_t n_sph, uint32_t n_nodes) {
    (void)n_sph;  // sphere BVH nodes and records stay in global memory (scalar loads)
    (void)n_nodes;
    return n_pairs ? staged_lds_bytes(kLayPairLds, n_tri, n_pairs, 0) : staged_lds_bytes(kLayTriLds, n_tri, 0, 0);
}

KernelChoice choose_kernel(uint32_t nT, uint32_t nP, uint32_t nS, uint32_t nC, uint32_t nTN, bool sph_compact,
                           uint32_t bounces, SceneMem mem, uint32_t walk) {
    auto lds = [&](int lay) { return staged_lds_bytes(lay, nT, nP, nC); };
    const bool pairs = nP > 0 && mem != SceneMem::kLdsSingle;
    int geo = kGeoTriGlobal;
    if (mem != SceneMem::kSmem && lds(pairs ? kGeoPairLds : kGeoTriLds) <= kMaxLdsBytes)
        geo = pairs ? kGeoPairLds : kGeoTriLds;
    if (mem == SceneMem::kPairSmem && nP > 0) geo = kGeoPairSmem;
    // triangle BVH whenever rt_create built one (kTriBvhMinTriangles or no LDS fit),
    // unless another layout is forced
    if (nTN > 0 && (mem == SceneMem::kTriBvh || mem == SceneMem::kAuto)) geo = kGeoTriBvh;
    // the sphere kernel (one-wave workgroups, compact BVH in L2) while its
    // per-workgroup copy of the pair records is small (rt_kernel.hpp)
    if (geo == kGeoPairLds && nS > 0 && sph_compact && mem == SceneMem::kAuto &&
        lds(kGeoSphLds) <= kSphPairLdsMaxBytes)
        geo = kGeoSphLds;
    // box clusters whenever rt_create found some; not with
    // spheres, where the sphere walks dominate and the cluster code's register
    // pressure measured 4.6 % slower than the culled pair loop (config 4)
    if (geo == kGeoPairLds && nC > 0 && nS == 0 && mem == SceneMem::kAuto && lds(kGeoPairClu) <= kMaxLdsBytes)
        geo = kGeoPairClu;
    // Opt-in only: bit-identical, 31% fewer pair tests, but 18% slower on the
    // Cornell 1080p workload (barrier + occupancy cost).
    if (geo == kGeoPairLds && mem == SceneMem::kPairSorted && lds(kGeoPairSorted) <= kMaxLdsBytes)
        geo = kGeoPairSorted;
    // the free-running kernel for BVH scenes (rt_create_options.walk_scheduler)
    if (bounces >= 1 && walk == kWalkFree) {
        if (geo == kGeoSphLds) geo = kGeoFreeSph;
        if (geo == kGeoTriBvh && nS == 0) geo = kGeoFreeTri;
    }
    // octant-sorted paths for BVH scenes (rt_create_options.walk_scheduler)
    if (walk == kWalkSorted) {
        if (geo == kGeoSphLds) geo = kGeoSortSph;
        if (geo == kGeoTriBvh && nS == 0) geo = kGeoSortTri;
    }
    return KernelChoice{geo, lds(geo)};
}

namespace {
hipError_t launch_path_trace_impl(const KParams& P, uint32_t bounces, SceneMem mem,
                                  hipStream_t stream) {
    const KernelChoice kc = choose_kernel(P.nT, P.nP, P.nS, P.nC, P.nTN, P.sph_lds != nullptr, bounces, mem, P.walk);
    const int geo = kc.layout;
    const size_t lds_total = kc.lds_bytes;  // exactly what the layout's staging loops write
#ifdef RT_LDS_UNDERSIZE  // negative control of the RT_LDS_CHECK build: one float4 short
    const size_t lds_req = lds_total >= 16 ? lds_total - 16 : lds_total;
#else
    const size_t lds_req = lds_total;
#endif
#ifdef RT_DEV_ISA  // ISA-inspection builds only (tools/isa.sh): the two headline layouts at B = 3
    if (bounces != 3) return hipErrorInvalidValue;
    if (geo == kGeoFreeSph) return launch_free<3, kGeoSphLds>(P, lds_req, stream);
    if (geo == kGeoFreeTri) return launch_free<3, kGeoTriBvh>(P, lds_req, stream);
    if (geo == kGeoSortSph) return launch_sorted_g<3, kGeoSphLds>(P, lds_req, stream);
    if (geo == kGeoSortTri) return launch_sorted_g<3, kGeoTriBvh>(P, lds_req, stream);
    if (geo == kGeoTriBvh) return launch_g<3, kGeoTriBvh>(P, lds_req, stream);
    return geo == kGeoPairClu ? launch_g<3, kGeoPairClu>(P, lds_req, stream)
                              : launch_g<3, kGeoSphLds>(P, lds_req, stream);
#endif
    switch (bounces) {
        case 0: return launch_b<0>(P, geo, lds_req, stream);
        case 1: return launch_b<1>(P, geo, lds_req, stream);
        case 2: return launch_b<2>(P, geo, lds_req, stream);
        case 3: return launch_b<3>(P, geo, lds_req, stream);
        case 4: return launch_b<4>(P, geo, lds_req, stream);
        default: return hipErrorInvalidValue;
    }
}
}  // namespace

hipError_t launch_path_trace(const KParams& P, uint32_t bounces, SceneMem mem,
                             hipStream_t stream, LaunchInfo* info) {
    const hipError_t e = launch_path_trace_impl(P, bounces, mem, stream);
    if (info) *info = g_last;
    return e;
}


hipError_t lds_check_result(uint32_t* end) {
    *end = 0;
#ifdef RT_LDS_CHECK
    hipError_t e = hipMemcpyFromSymbol(end, HIP_SYMBOL(g_lds_overflow), sizeof(uint32_t));
    if (e != hipSuccess) return e;
    const uint32_t zero = 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_lds_overflow), &zero, sizeof(zero));
#else
    return hipSuccess;
#endif
}

hipError_t read_debug_stats(unsigned long long* out, int n) {
#if defined(RT_FREE_DEBUG)
    // the free kernel's event log (rt_free.hpp), as 64-bit words
    constexpr int kWords = (int)(sizeof(g_free_dbg) / 8);
    if (n > kWords) n = kWords;
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_free_dbg), n * sizeof(unsigned long long));
    if (e != hipSuccess) return e;
    static const uint32_t zero[4] = {0, 0, 0, 0};  // the three slot counters
    return hipMemcpyToSymbol(HIP_SYMBOL(g_free_dbg), zero, sizeof(zero));
#elif defined(RT_STATS)
    if (n > 32) n = 32;
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rt_stats), n * sizeof(unsigned long long));
    if (e != hipSuccess) return e;
    const unsigned long long zero[32] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rt_stats), zero, sizeof(zero));
#else
    (void)out;
    (void)n;
    return hipErrorNotSupported;
#endif
}

hipError_t math_selfcheck(unsigned long long bad[2]) {
    unsigned long long* d = nullptr;
    hipError_t e = hipMalloc((void**)&d, 2 * sizeof(unsigned long long));
    if (e != hipSuccess) return e;
    if ((e = hipMemset(d, 0, 2 * sizeof(unsigned long long))) == hipSuccess) {
        // every float: 2^32 bit patterns in two halves of 2^31
        hipLaunchKernelGGL(math_check_kernel, dim3(16384), dim3(256), 0, 0, 0u, 0x80000000u, d);
        hipLaunchKernelGGL(math_check_kernel, dim3(16384), dim3(256), 0, 0, 0x80000000u, 0x80000000u, d);
        if ((e = hipGetLastError()) == hipSuccess && (e = hipDeviceSynchronize()) == hipSuccess)
            e = hipMemcpy(bad, d, 2 * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    }
    (void)hipFree(d);
    return e;
}

hipError_t launch_fill_seeds(uint32_t* seeds, uint64_t key, uint64_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(fill_seeds_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, seeds,
                       key, n);
    return hipGetLastError();
}

}  // namespace rt

// rt_mis.hip — gfx950 kernel of the MIS integrator: `kernel drawTriangle`
// (Sources/gpuRaytracer/shaders.metal:635-707) with its one-bounce
// three-strategy multiple importance sampling (`recursiveMultiImportanceSampling`,
// :543-625): light-area, cosine-hemisphere and GGX-VNDF samples weighted by the
// power heuristic with beta = 1 (:131-137), next-event estimation at the
// secondary hit (:519-541), GGX/Lambert BRDF (:186-289).
//
// MI355X mapping:
//   * one lane per pixel, wave64 = 8x8 pixel tile, 256-thread workgroups; the
//     triangle records are staged in LDS once per workgroup (shared-edge pair
//     layout, as in rt_kernel.hip) and every query is a closest hit with the
//     wave-level AABB cull (rays of neighbouring pixels share u, so they are
//     coherent);
//   * the MIS sample points u do not depend on the pixel (haltonRandom(i, d),
//     :556,564,584,595,617): the host tabulates them once per launch and the
//     kernel reads them with wave-uniform (scalar) loads;
//   * the tonemap epilogue (:688-706) is fused: one float4 and one uchar4 store.
// Arithmetic follows DESIGN.md §3 / §3.11; oracle/pt_oracle.c (pto_render_mis)
// restates the same operations and the two agree bit for bit.
#include <hip/hip_runtime.h>

#include "rt_kernel.hpp"
#include "rt_trace.hpp"

namespace rt {

namespace {

constexpr float kPiF = 3.14159274f;         // M_PI_F
constexpr float kTwoPiF = 6.28318548f;      // 2.0 * M_PI_F
constexpr float kInvPiF = 0.318309873f;     // 1.0 / M_PI_F (Fd_Lambert, :210-212)

struct MisMat {
    f3 diffuse;
    float metallic, roughness;
};

// IntersectionGPU (:14-20) of a Hit: the normal and the material are read
// from the shading record (staged in LDS) where they are used.
struct MisHit {
    f3 p, din;     // point, ray direction
    uint32_t id;   // triangle
};

__device__ __forceinline__ uint32_t opaque_u32(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}

__device__ __forceinline__ float clamp01(float x) { return fminf(1.0f, fmaxf(0.0f, x)); }

// D_GGX (:193-197): the caller passes roughness as `a`
__device__ __forceinline__ float d_ggx(float NoH, float a) {
    const float a2 = a * a;
    const float f = (NoH * a2 - NoH) * NoH + 1.0f;
    return a2 / ((kPiF * f) * f);
}

// smithG1_GGX (:186-191)
__device__ __forceinline__ float smith_g1(float NoV, float roughness) {
    const float a = roughness * roughness;
    const float a2 = a * a;
    const float NoV2 = NoV * NoV;
    return 2.0f / (1.0f + sqrtf(1.0f + (a2 * (1.0f - NoV2)) / NoV2));
}

// V_SmithGGXCorrelated (:203-208)
__device__ __forceinline__ float v_smith(float NoV, float NoL, float a) {
    const float a2 = a * a;
    const float GGXL = NoV * sqrtf(((-NoL) * a2 + NoL) * NoL + a2);
    const float GGXV = NoL * sqrtf(((-NoV) * a2 + NoV) * NoV + a2);
    return 0.5f / (GGXV + GGXL);
}

// calculateBRDFContribution (:259-289) for view ray direction din, light dir l
__device__ __forceinline__ f3 brdf(f3 din, f3 n, const MisMat& m, f3 l) {
    const f3 v = -normalize(din);
    const f3 h = normalize(v + l);
    const float NoV = fabsf(dot(n, v)) + 1e-5f;
    const float NoL = clamp01(dot(n, l));
    const float NoH = clamp01(dot(n, h));
    const float LoH = clamp01(dot(l, h));
    // f0 = mix(0.04, diffuse, metallic) = 0.04 + (diffuse - 0.04) * metallic
    const f3 f0{0.04f + (m.diffuse.x - 0.04f) * m.metallic, 0.04f + (m.diffuse.y - 0.04f) * m.metallic,
                0.04f + (m.diffuse.z - 0.04f) * m.metallic};
    const float D = d_ggx(NoH, m.roughness);
    const float x = 1.0f - LoH;
    const float x2 = x * x;
    const float p5 = (x2 * x2) * x;  // pow(1 - LoH, 5.0)
    const f3 F{f0.x + (1.0f - f0.x) * p5, f0.y + (1.0f - f0.y) * p5, f0.z + (1.0f - f0.z) * p5};
    const float G = v_smith(NoV, NoL, m.roughness);
    const float DG = D * G;
    const float den = (4.0f * NoV) * NoL + 1e-7f;
    const f3 Fr{(DG * F.x) / den, (DG * F.y) / den, (DG * F.z) / den};
    const f3 Fd = m.diffuse * kInvPiF;
    const float km = 1.0f - m.metallic;
    const f3 kD{(1.0f - F.x) * km, (1.0f - F.y) * km, (1.0f - F.z) * km};
    return (kD * (Fd + Fr)) * NoL;
}

// calculateVNDFPdf (:437-445)
__device__ __forceinline__ float vndf_pdf(f3 V, f3 n, f3 L, float roughness) {
    const f3 h = normalize(V + L);
    const float NoH = fabsf(dot(n, h));
    const float VoH = fabsf(dot(V, h));
    const float NoV = fabsf(dot(n, V));
    const float D = d_ggx(NoH, roughness);
    const float G1 = smith_g1(NoV, roughness);
    return ((D * G1) * VoH) / (4.0f * NoV);
}

// calculateCosineWeightedPdf (:376-380)
__device__ __forceinline__ float cosine_pdf(f3 n, f3 d) { return fmaxf(0.0f, dot(n, d)) / kPiF; }

// calculateSquareLightPdf (:315-326): evaluated at the un-offset hit point
__device__ __forceinline__ float light_pdf(const MisParams& P, f3 p, f3 d) {
    const f3 toL = f3{P.l_center[0], P.l_center[1], P.l_center[2]} - p;
    const float dist = length(toL);
    const float cosT = fmaxf(0.0f, dot(-d, f3{0.0f, -1.0f, 0.0f}));
    return (dist * dist) / (P.l_area * cosT + 1e-6f);
}

// powerHeuristic with beta = 1 (:132-137; pow(x, 1) = x)
__device__ __forceinline__ float power_h(float p1, float p2, float p3, float n) {
    const float a = n * p1;
    const float sum = (a + n * p2) + n * p3;
    return a / (sum + 1e-6f);
}

// cosineWeightedRay direction (:355-374)
__device__ __forceinline__ f3 cosine_dir(f3 n, f3 t, f3 b, float ux, float uy) {
    const float phi = kTwoPiF * ux;
    const float cosT = sqrtf(uy);
    const float sinT = sqrtf(1.0f - uy);
    float sp, cp;
    sincos_pt(phi, &sp, &cp);
    return normalize((t * (cp * sinT) + b * (sp * sinT)) + n * cosT);
}

// vndfRay direction (:382-435); V = -ray direction of the hit
__device__ __forceinline__ f3 vndf_dir(f3 V, f3 n, f3 t, f3 b, float roughness, float ux, float uy) {
    const float alpha = roughness * roughness;
    const f3 Ve = normalize(f3{alpha * dot(V, t), alpha * dot(V, b), dot(V, n)});
    const f3 T1 = normalize(f3{Ve.z, 0.0f, -Ve.x});
    const f3 T2 = cross(Ve, T1);
    const float phi = kTwoPiF * ux;
    const float lenVe = length(Ve);
    const float ctm = lenVe / sqrtf(1.0f + lenVe * lenVe);
    const float ct = ctm + (1.0f - ctm) * uy;
    const float st = sqrtf(1.0f - ct * ct);
    float sp, cp;
    sincos_pt(phi, &sp, &cp);
    const f3 h = normalize((T1 * (cp * st) + T2 * (sp * st)) + Ve * ct);
    const f3 Nh = normalize(f3{alpha * h.x, alpha * h.y, fmaxf(0.0f, h.z)});
    const f3 wH = normalize((t * Nh.x + b * Nh.y) + n * Nh.z);
    const f3 I = -V;
    return I - wH * (2.0f * dot(wH, I));  // reflect(-V, wH)
}

__device__ __forceinline__ MisMat load_mat(const float4* rec) {
    const float4 r1 = rec[1], r2 = rec[2];
    return MisMat{f3{r1.x, r1.y, r1.z}, r1.w, r2.x};
}
// (sv.shade: the shading records, staged in LDS with the scene when it fits)
__device__ __forceinline__ f3 hit_n(const SceneView& sv, const MisHit& x) {
    const float4 r0 = sv.shade[3 * x.id];
    return f3{r0.x, r0.y, r0.z};
}
__device__ __forceinline__ MisMat hit_m(const SceneView& sv, const MisHit& x) {
    return load_mat(sv.shade + 3 * x.id);
}

// SEG (the light queries, tmax = distance to the light sample): with box
// clusters the room is skipped for waves whose segments stay inside it -- a
// hit beyond tmax is no hit, and none of the room's faces can be hit before.
template <int GEO, bool SEG = false>
__device__ __forceinline__ int mis_closest(const SceneView& sv, f3 o, f3 d, float tmax, float* t) {
    *t = tmax;
    if (GEO == kGeoPairClu && SEG) {
        int id = -1;
        cluster_query<false, true>(sv, o, d, 0.001f, t, &id);
        return id;
    }
    return closest_hit<GEO, false, true, 0>(sv, o, d, 0.001f, t);
}

// The primary hit x of the current camera ray: point and ray direction in a
// per-lane LDS stash (slots 0-5, written once per camera ray), re-read where
// they are used -- through an opaque lane index, so the reads are not hoisted
// back into registers across the MIS sample loops (the queries nested in them
// are where the register pressure peaks).
__device__ __forceinline__ uint32_t opaque_lane_slot() { return opaque_u32(threadIdx.x); }
__device__ __forceinline__ MisHit load_x(const SceneView& sv, uint32_t id) {
    const uint32_t k = opaque_lane_slot();
    const float* st = sv.xstash;
    MisHit x;
    x.p = f3{st[k], st[kBlockThreads + k], st[2 * kBlockThreads + k]};
    x.din = f3{st[3 * kBlockThreads + k], st[4 * kBlockThreads + k], st[5 * kBlockThreads + k]};
    x.id = id;
    return x;
}

// s[slot..slot+2] += v in this lane's stash (the running strategy sums; the same
// additions in the same order as a register accumulator)
__device__ __forceinline__ void stash_add(const SceneView& sv, uint32_t slot, f3 v) {
    float* st = sv.xstash;
    const uint32_t k = opaque_lane_slot();
    st[slot * kBlockThreads + k] = st[slot * kBlockThreads + k] + v.x;
    st[(slot + 1) * kBlockThreads + k] = st[(slot + 1) * kBlockThreads + k] + v.y;
    st[(slot + 2) * kBlockThreads + k] = st[(slot + 2) * kBlockThreads + k] + v.z;
}
__device__ __forceinline__ f3 stash_get(const SceneView& sv, uint32_t slot) {
    const uint32_t k = opaque_lane_slot();
    return f3{sv.xstash[slot * kBlockThreads + k], sv.xstash[(slot + 1) * kBlockThreads + k],
              sv.xstash[(slot + 2) * kBlockThreads + k]};
}
__device__ __forceinline__ void stash_set(const SceneView& sv, uint32_t slot, f3 v) {
    const uint32_t k = opaque_lane_slot();
    sv.xstash[slot * kBlockThreads + k] = v.x;
    sv.xstash[(slot + 1) * kBlockThreads + k] = v.y;
    sv.xstash[(slot + 2) * kBlockThreads + k] = v.z;
}

// calculateDirectLightSamplingContribution (:519-541).  POWER: MIS-weighted
// (first hit) or plain (at the secondary hit, samplesPerStrategy = 1).  The
// contribution is formed BEFORE the visibility query (the same operations:
// nothing in it depends on the query), so only it and the query's ray are live
// during the query.
template <int GEO, bool POWER>
__device__ __forceinline__ f3 direct_light(const MisParams& P, const SceneView& sv, const MisHit& x,
                                           float ux, float uy, float nS) {
    const f3 n = hit_n(sv, x);
    const f3 origin = x.p + n * 1e-4f;
    // directSquareLightRay (:291-313)
    const float sx = (ux - 0.5f) * P.l_width;
    const float sy = (uy - 0.5f) * P.l_depth;
    const f3 sp = (f3{P.l_center[0], P.l_center[1], P.l_center[2]} +
                   f3{P.l_tangent[0], P.l_tangent[1], P.l_tangent[2]} * sx) +
                  f3{P.l_bitangent[0], P.l_bitangent[1], P.l_bitangent[2]} * sy;
    const f3 tl = sp - origin;
    const float dist = length(tl);
    const f3 L{tl.x / dist, tl.y / dist, tl.z / dist};
    f3 contrib;
    {
        const float dl_pdf = light_pdf(P, x.p, L);
        const MisMat m = hit_m(sv, x);
        const f3 c = brdf(x.din, n, m, L);
        const f3 Le{P.l_radiance[0], P.l_radiance[1], P.l_radiance[2]};
        if (POWER) {
            const float cos_pdf = cosine_pdf(n, L);
            const float v_pdf = vndf_pdf(-x.din, n, L, m.roughness);
            const float w = power_h(dl_pdf, cos_pdf, v_pdf, nS);
            const f3 a = (c * w) * Le;
            contrib = f3{a.x / dl_pdf, a.y / dl_pdf, a.z / dl_pdf};
        } else {
            const f3 a = c * Le;
            contrib = f3{a.x / dl_pdf, a.y / dl_pdf, a.z / dl_pdf};
        }
    }
    float t;
    const int id = mis_closest<GEO, true>(sv, origin, L, dist, &t);
    if (id < 0 || sv.shade[3 * id].w == 0.0f) return f3{0.0f, 0.0f, 0.0f};  // not HitLight
    return contrib;
}

// Continuation of a cosine or VNDF sample (:576-590, :608-622): the sampled
// ray's closest hit either sees the light (MIS-weighted emission) or a
// surface (next-event estimate there, unweighted).  brdf(x, dir) does not
// depend on the hit: it is formed before the query.
template <int GEO>
__device__ __forceinline__ f3 continue_sample(const MisParams& P, const SceneView& sv,
                                              const MisHit& x, f3 origin, f3 dir, float pdf,
                                              float w, float u2x, float u2y) {
    const f3 c = brdf(x.din, hit_n(sv, x), hit_m(sv, x), dir);
    float t;
    const int id = mis_closest<GEO>(sv, origin, dir, 1000.0f, &t);
    if (id < 0) return f3{0.0f, 0.0f, 0.0f};
    const float4 r0 = sv.shade[3 * id];
    if (r0.w != 0.0f) {  // HitLight
        const f3 a = (c * w) * f3{P.l_radiance[0], P.l_radiance[1], P.l_radiance[2]};
        return f3{a.x / pdf, a.y / pdf, a.z / pdf};
    }
    MisHit y;
    y.p = origin + dir * t;
    y.din = dir;
    y.id = (uint32_t)id;
    const f3 q{c.x / pdf, c.y / pdf, c.z / pdf};
    return q * direct_light<GEO, false>(P, sv, y, u2x, u2y, 1.0f);
}

// recursiveMultiImportanceSampling (:543-625).  x (point, direction) is re-read
// from the lane's LDS stash per sample and the tangent frame of onb() (a
// function of the normal only) is recomputed per sample: the same values, held
// in no register across the nested queries.
template <int GEO>
__device__ __forceinline__ f3 mis_shade_hit(const MisParams& P, const SceneView& sv, uint32_t xid) {
    const uint32_t S = P.S;
    const float nS = (float)S;
    const float4* __restrict__ tab = P.u_tab;
    f3 dl{0.0f, 0.0f, 0.0f}, cs{0.0f, 0.0f, 0.0f}, vn{0.0f, 0.0f, 0.0f};
    for (uint32_t i = 0; i < S; ++i) {  // light sampling (:553-560)
        const float4 u = tab[3 * i];
        dl = dl + direct_light<GEO, true>(P, sv, load_x(sv, xid), u.x, u.y, nS);
    }
    {  // dl waits in the stash through the cosine loop
        float* st = sv.xstash;
        const uint32_t k = threadIdx.x;
        st[9 * kBlockThreads + k] = dl.x;
        st[10 * kBlockThreads + k] = dl.y;
        st[11 * kBlockThreads + k] = dl.z;
    }
    stash_set(sv, 12, f3{0.0f, 0.0f, 0.0f});  // the strategy sum accumulates in the stash
    for (uint32_t i = 0; i < S; ++i) {  // cosine-hemisphere sampling (:562-591)
        const float4 u = tab[3 * i + 1];
        const MisHit x = load_x(sv, xid);
        const f3 n = hit_n(sv, x);
        f3 t, b;
        onb(n, &t, &b);
        const f3 origin = x.p + n * 1e-4f;
        const f3 V = -x.din;
        const f3 dir = cosine_dir(n, t, b, u.x, u.y);
        const float cos_pdf = cosine_pdf(n, dir);
        const float dl_pdf = light_pdf(P, x.p, dir);
        const float v_pdf = vndf_pdf(V, n, dir, hit_m(sv, x).roughness);
        const float w = power_h(cos_pdf, dl_pdf, v_pdf, nS);
        stash_add(sv, 12, continue_sample<GEO>(P, sv, x, origin, dir, cos_pdf, w, u.z, u.w));
    }
    cs = stash_get(sv, 12);
    {  // (directLight + cosine) + vndf (:624), same order; dc waits in the stash
        const uint32_t k0 = opaque_lane_slot();
        const f3 dl2{sv.xstash[9 * kBlockThreads + k0], sv.xstash[10 * kBlockThreads + k0],
                     sv.xstash[11 * kBlockThreads + k0]};
        const f3 dc = dl2 + cs;
        float* st = sv.xstash;
        const uint32_t k = threadIdx.x;
        st[9 * kBlockThreads + k] = dc.x;
        st[10 * kBlockThreads + k] = dc.y;
        st[11 * kBlockThreads + k] = dc.z;
    }
    stash_set(sv, 12, f3{0.0f, 0.0f, 0.0f});  // the strategy sum accumulates in the stash
    for (uint32_t i = 0; i < S; ++i) {  // VNDF sampling (:593-623)
        const float4 u = tab[3 * i + 2];
        const MisHit x = load_x(sv, xid);
        const f3 n = hit_n(sv, x);
        f3 t, b;
        onb(n, &t, &b);
        const f3 origin = x.p + n * 1e-4f;
        const f3 V = -x.din;
        const float rough = hit_m(sv, x).roughness;
        const f3 dir = vndf_dir(V, n, t, b, rough, u.x, u.y);
        const float v_pdf = vndf_pdf(V, n, dir, rough);
        const float cos_pdf = cosine_pdf(n, dir);
        const float dl_pdf = light_pdf(P, x.p, dir);
        const float w = power_h(v_pdf, dl_pdf, cos_pdf, nS);
        stash_add(sv, 12, continue_sample<GEO>(P, sv, x, origin, dir, v_pdf, w, u.z, u.w));
    }
    vn = stash_get(sv, 12);
    const uint32_t k = opaque_lane_slot();
    const f3 dc{sv.xstash[9 * kBlockThreads + k], sv.xstash[10 * kBlockThreads + k],
                sv.xstash[11 * kBlockThreads + k]};
    const f3 sum = dc + vn;
    return f3{sum.x / nS, sum.y / nS, sum.z / nS};
}

}  // namespace

// lanes per pixel: 2 with split launches (17.64 ms per reference frame: three
// rounds of the 6 camera rays, one workgroup per round; 3 lanes 17.89, 1 lane
// 18.02; without the split 3 lanes 18.82 -- round 3: 2 lanes 20.3, 6 lanes
// 19.8, 1 lane 26.1, 4 lanes 25.7)
#ifndef RT_MIS_LANES
#define RT_MIS_LANES 2
#endif
constexpr uint32_t kMisLanes = RT_MIS_LANES;
// A wave holds 64 / ML pixels: an 8 x (8 / ML) tile when ML divides 8, else one
// row of floor(64 / ML) pixels (the lanes past them leave at once); a
// workgroup is 2 x 2 tiles or 1 x 4 rows.
constexpr bool kMisTile = 8u % kMisLanes == 0;
constexpr uint32_t kMisRowPixels = 64u / kMisLanes;
// 7 waves/SIMD: 72 VGPRs without scratch since the primary hit, the pixel sum,
// dl/dc and the running strategy sum wait in the per-lane LDS stash (round 2:
// 120 VGPRs at 4 waves; 6 waves then spilled 54 VGPRs).  DESIGN.md §5
#ifndef RT_MIS_WAVES
#define RT_MIS_WAVES 7
#endif
constexpr int kMisWavesPerEu = RT_MIS_WAVES;
// FREEP: the scene has pairs in no box cluster (P.pair_free != 0).  The
// reference scene has none; with FREEP false their loop is compiled out, which
// also drops the one VGPR its loop-invariant test occupied (8 B of scratch at
// 7 waves/SIMD, round 4).
// The pixel's stored value (:688-706 and textBuffer :705): the sum over its
// camera rays and their count; RGBA8 after exposure, Reinhard, clamp, gamma.
__device__ __forceinline__ void mis_store(const MisParams& P, size_t o, f3 acc) {
    const float nc = (float)P.camera_rays;
    if (P.out) P.out[o] = make_float4(acc.x, acc.y, acc.z, nc);  // textBuffer (:705) + count
    if (P.out8) {
        // :688-706: exposure, Reinhard, clamp, gamma 1/2.2, uchar(c * 255)
        const float e[3] = {(acc.x / nc) * P.exposure, (acc.y / nc) * P.exposure,
                            (acc.z / nc) * P.exposure};
        unsigned char c8[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const float tm = clamp01(e[k] / (e[k] + 1.0f));
            const float g = pow_pt(tm, 1.0f / 2.2f);
            c8[k] = (unsigned char)(g * 255.0f);
        }
        P.out8[o] = make_uchar4(c8[0], c8[1], c8[2], 255);
    }
}

// SPLIT: one workgroup per (tile, round) -- blockIdx.z is the round -- and every
// lane stores its camera ray's result to the records buffer (mis_part_bytes); mis_sum_kernel
// then adds a pixel's rays in order i.  Twice the workgroups of half the length:
// the frame's last workgroups (the tail, when too few are left to fill the GPU)
// end sooner.
template <int GEO, bool FREEP = true, bool SPLIT = false>
__global__ __launch_bounds__(kBlockThreads, kMisWavesPerEu) void mis_kernel(MisParams P) {
    extern __shared__ float4 lds[];
    SceneView sv;
    sv.nT = P.nT;
    sv.nP = P.nP;
    sv.nS = 0;
    sv.nN = 0;
    sv.node = nullptr;
    sv.sph = nullptr;
    sv.sph_perm = nullptr;
    sv.tnode = P.tri_nodes;
    sv.tsorted = P.tri_sorted;
    sv.tperm = P.tri_perm;
    sv.nTN = P.nTN;
    if (GEO == kGeoTriBvh) {
        sv.tri = nullptr;
        sv.pair = nullptr;
    } else if (GEO != kGeoTriGlobal) {
        constexpr bool pairs = GEO == kGeoPairLds || GEO == kGeoPairClu;
        const uint32_t ng4 = pairs ? kPairF4 * sv.nP : 3u * sv.nT;
        const float4* src = pairs ? P.pair_isect : P.tri_isect;
        for (uint32_t k = threadIdx.x; k < ng4; k += kBlockThreads) lds[k] = src[k];
        const uint32_t nc4 = GEO == kGeoPairClu ? kCluF4 * P.nC : 0u;
        if (GEO == kGeoPairClu)  // box clusters after the pair records
            for (uint32_t k = threadIdx.x; k < nc4; k += kBlockThreads) lds[ng4 + k] = P.clusters[k];
        // then the shading records (3 float4 per triangle): read per lane, often
        for (uint32_t k = threadIdx.x; k < 3u * sv.nT; k += kBlockThreads)
            lds[ng4 + nc4 + k] = P.mis_shade[k];
        sv.shade = lds + ng4 + nc4;
        sv.xstash = reinterpret_cast<float*>(lds + ng4 + nc4 + 3u * sv.nT);
        __syncthreads();
        sv.tri = lds;
        sv.pair = lds;
        sv.clu = lds + ng4;
        sv.nC = P.nC;
        sv.pair_free = FREEP ? P.pair_free : 0u;
    } else {
        sv.tri = P.tri_isect;
        sv.pair = nullptr;
    }
    if (GEO == kGeoTriBvh || GEO == kGeoTriGlobal) {
        sv.shade = P.mis_shade;
        sv.xstash = reinterpret_cast<float*>(lds);
    }

    // ML lanes per pixel: lane `sub` traces the camera rays i = r*ML + sub of
    // round r, and the pixel's group leader adds the ML results to the pixel's
    // sum in ray order i (the same additions as one lane per pixel, :652-677).
    // More waves than one lane per pixel, each shorter: the 800x600 frame's
    // 7,500 one-lane waves filled the GPU's wave slots 1.8 times over, the
    // second time only partly.
    // Pixel of a lane; recomputed from an opaque threadIdx where it is used
    // (as in rt_kernel.hip), not held across the camera-ray loop.  A wave is
    // 8 x (8 / ML) pixels (workgroup 2 x 2 waves) or a row of 64 / ML pixels
    // (workgroup 4 rows).
    constexpr uint32_t ML = kMisLanes;
    constexpr uint32_t kWY = kMisTile ? 8u / ML : 1u;
    auto pixel_of = [&](uint32_t tid, uint32_t& x, uint32_t& j) {
        const uint32_t lane = tid & 63u, wave = tid >> 6, pix = lane / ML;
        if (kMisTile) {
            x = blockIdx.x * 16u + (wave & 1u) * 8u + (pix & 7u);
            j = blockIdx.y * (2u * kWY) + (wave >> 1) * kWY + (pix >> 3);
        } else {
            x = blockIdx.x * kMisRowPixels + pix;
            j = blockIdx.y * 4u + wave;
        }
    };
    {
        uint32_t x, j;
        pixel_of(threadIdx.x, x, j);
        if (x >= (uint32_t)P.W || j >= P.row_count) return;  // a pixel's ML lanes leave together
        if (!kMisTile && (threadIdx.x & 63u) >= kMisRowPixels * ML) return;  // lanes past the row
    }
    const f3 cu{P.cam_u[0], P.cam_u[1], P.cam_u[2]}, cv{P.cam_v[0], P.cam_v[1], P.cam_v[2]};
    const f3 cw{P.cam_w[0], P.cam_w[1], P.cam_w[2]};
    const f3 cpos{P.cam_pos[0], P.cam_pos[1], P.cam_pos[2]};
    const float fW = (float)P.W, fH = (float)P.H;
    // the pixel's running sum lives in the lane's stash slots 6-8 between rounds
    // (kept out of the registers the nested MIS queries need)
    {
        float* st = sv.xstash;
        const uint32_t k = threadIdx.x;
        st[6 * kBlockThreads + k] = 0.0f;
        st[7 * kBlockThreads + k] = 0.0f;
        st[8 * kBlockThreads + k] = 0.0f;
    }
    const uint32_t rounds = (P.camera_rays + ML - 1u) / ML;
    const uint32_t r_begin = SPLIT ? blockIdx.z : 0u, r_end = SPLIT ? blockIdx.z + 1u : rounds;
    for (uint32_t r = r_begin; r < r_end; ++r) {  // :652
        const uint32_t tid = opaque_u32(threadIdx.x);
        const uint32_t sub = (tid & 63u) % ML;  // ML need not divide 64
        const uint32_t i = r * ML + sub;
        f3 c{0.0f, 0.0f, 0.0f};
        bool has = false;  // Miss (:665), or a ray past camera_rays: nothing to add
        if (i < P.camera_rays) {
            uint32_t x, j;
            pixel_of(tid, x, j);
            const uint32_t y = P.row_start + j * P.row_step;
            const float fx = (float)x, fy = (float)y;
            // hashRandom(index, i) (:71-85); the 800 is the reference's hard-coded width
            const uint32_t sample_id = (y * 800u + x) * i;
            const float jx = mis_unit(mis_hash(x + y * 800u + sample_id));
            const float jy = mis_unit(mis_hash(y + x * 600u + sample_id + 12345u));
            // generateCameraRay (:214-246)
            const float sx = ((fx + jx) / fW) * 2.0f - 1.0f;
            const float ty = -(((fy + jy) / fH) * 2.0f - 1.0f);
            const float sh = sx * P.halfW, th = ty * P.halfH;
            const f3 d = normalize((cu * sh + cv * th) - cw);
            float t;
            const int id = mis_closest<GEO>(sv, cpos, d, 1000.0f, &t);
            if (id >= 0) {
                const float4 r0 = sv.shade[3 * id];
                has = true;
                if (r0.w != 0.0f) {                         // HitLight (:667-671)
                    c = f3{P.l_radiance[0], P.l_radiance[1], P.l_radiance[2]};
                } else {
                    {  // the primary hit x into this lane's stash
                        const f3 hp = cpos + d * t;
                        float* st = sv.xstash;
                        const uint32_t k = threadIdx.x;
                        st[k] = hp.x;
                        st[kBlockThreads + k] = hp.y;
                        st[2 * kBlockThreads + k] = hp.z;
                        st[3 * kBlockThreads + k] = d.x;
                        st[4 * kBlockThreads + k] = d.y;
                        st[5 * kBlockThreads + k] = d.z;
                    }
                    c = mis_shade_hit<GEO>(P, sv, (uint32_t)id);  // :674-676
                }
            }
        }
        if (SPLIT) {  // mis_sum_kernel adds the records in ray order
            const uint32_t t3 = opaque_u32(threadIdx.x);
            uint32_t x, j;
            pixel_of(t3, x, j);
            const size_t npix = (size_t)P.row_count * (size_t)P.W, px = (size_t)j * (size_t)P.W + x;
            if (r == 0) {
                // record 0: round 0's rays summed in ray order from +0 -- the
                // first ML additions of the pixel's sum (:652-677)
                const int base = (int)((t3 & 63u) - (t3 & 63u) % ML);
                f3 acc{0.0f, 0.0f, 0.0f};
#pragma unroll
                for (uint32_t k = 0; k < ML; ++k) {
                    const f3 ck{__shfl(c.x, base + (int)k), __shfl(c.y, base + (int)k), __shfl(c.z, base + (int)k)};
                    if (__shfl((int)has, base + (int)k) != 0) acc = acc + ck;
                }
                if ((t3 & 63u) % ML == 0) P.part[px] = make_float4(acc.x, acc.y, acc.z, 0.0f);
            } else if (i < P.camera_rays) {
                // record i - ML + 1: this ray's c, which is +0 without a hit --
                // adding it equals skipping it (the sum starts at +0, so it is
                // never -0, and x + (+0) == x for every other x, NaN included)
                P.part[(size_t)(i - ML + 1u) * npix + px] = make_float4(c.x, c.y, c.z, 0.0f);
            }
            continue;
        }
        const uint32_t t2 = opaque_u32(threadIdx.x);
        float* st = sv.xstash;
        f3 acc{st[6 * kBlockThreads + t2], st[7 * kBlockThreads + t2], st[8 * kBlockThreads + t2]};
        if (ML == 1) {
            if (has) acc = acc + c;
        } else {  // in ray order: lane base + k holds ray r*ML + k
            const int base = (int)((t2 & 63u) - (t2 & 63u) % ML);
#pragma unroll
            for (uint32_t k = 0; k < ML; ++k) {
                const f3 ck{__shfl(c.x, base + (int)k), __shfl(c.y, base + (int)k),
                            __shfl(c.z, base + (int)k)};
                const bool hk = __shfl((int)has, base + (int)k) != 0;
                if (hk) acc = acc + ck;  // every lane of the group keeps the same sum
            }
        }
        st[6 * kBlockThreads + t2] = acc.x;
        st[7 * kBlockThreads + t2] = acc.y;
        st[8 * kBlockThreads + t2] = acc.z;
    }
    if (SPLIT) return;
    const uint32_t tl = opaque_u32(threadIdx.x);
    const f3 acc{sv.xstash[6 * kBlockThreads + tl], sv.xstash[7 * kBlockThreads + tl],
                 sv.xstash[8 * kBlockThreads + tl]};
    if ((opaque_u32(threadIdx.x) & 63u) % ML != 0) return;  // the group leader stores the pixel
    uint32_t x, j;
    pixel_of(opaque_u32(threadIdx.x), x, j);
    mis_store(P, (size_t)j * (size_t)P.W + x, acc);
}

// The pixel sums of a SPLIT launch: the camera rays' results added in ray order
// (:652-677, the same additions as the in-kernel sum), then the store.
__global__ void mis_sum_kernel(MisParams P) {
    const uint32_t x = blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
    if (x >= (uint32_t)P.W) return;
    const size_t npix = (size_t)P.row_count * (size_t)P.W, o = (size_t)j * (size_t)P.W + x;
    const float4 r0 = P.part[o];
    f3 acc{r0.x, r0.y, r0.z};  // rays 0 .. ML-1
    for (uint32_t i = kMisLanes; i < P.camera_rays; ++i) {
        const float4 v = P.part[(size_t)(i - kMisLanes + 1u) * npix + o];
        acc = acc + f3{v.x, v.y, v.z};
    }
    mis_store(P, o, acc);
}

constexpr size_t kMisStashBytes = 15u * kBlockThreads * sizeof(float);  // per lane: primary hit, pixel sum, dl/dc, strategy sum

// SPLIT launches (RT_MIS_SPLIT): the records buffer, one float4 per record and
// pixel: record 0 = round 0's rays already summed, then one record per later
// ray -- camera_rays - ML + 1 records (round 5: one per ray, 46 MB at 800x600 x
// 6 rays; now 38.4 MB).  16 B, not 12: a wave's 8-pixel tile rows then write
// whole 128-B lines (three 12-B float planes wrote 32-B row pieces: 51.6 MB of
// HBM writes for 28.8 MB of records, profiles/r6/ab_results.md); 0 (no split)
// when it would exceed kMisPartMax or the split is off.
#ifndef RT_MIS_SPLIT
#define RT_MIS_SPLIT 1
#endif
constexpr size_t kMisPartMax = (size_t)256 << 20;
size_t mis_part_bytes(uint32_t camera_rays, size_t pixels) {
    if (camera_rays <= kMisLanes) return 0u;
    const size_t b = (size_t)(camera_rays - kMisLanes + 1u) * pixels * sizeof(float4);
    return (RT_MIS_SPLIT && camera_rays > kMisLanes && b <= kMisPartMax) ? b : 0u;
}

size_t mis_lds_bytes(uint32_t n_tri, uint32_t n_pairs) {  // scene records + shading records
    return (size_t)((n_pairs ? kPairF4 * n_pairs : 3u * n_tri) + 3u * n_tri) * sizeof(float4);
}

// Dynamic LDS above 64 KB must be allowed per kernel: a scene whose records
// fit the 64 KB of the LDS layouts keeps them with the 15 KB stash on top
// (up to 79 KB per workgroup, fewer workgroups per CU) instead of dropping to
// the global-memory kernel.
template <int GEO, bool FREEP, bool SPLIT>
hipError_t launch_mis_s(const MisParams& P, size_t lds, hipStream_t stream) {
    constexpr uint32_t TX = kMisTile ? 16u : kMisRowPixels, TY = kMisTile ? 2u * (8u / kMisLanes) : 4u;
    const uint32_t rounds = (P.camera_rays + kMisLanes - 1u) / kMisLanes;
    // workgroup: TX x TY pixels (x one round when SPLIT)
    const dim3 grid((P.W + TX - 1) / TX, (P.row_count + TY - 1) / TY, SPLIT ? rounds : 1u);
    if (lds > 65536) {
        const hipError_t e = hipFuncSetAttribute((const void*)mis_kernel<GEO, FREEP, SPLIT>,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((mis_kernel<GEO, FREEP, SPLIT>), grid, dim3(kBlockThreads), lds, stream, P);
    if (SPLIT) {
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(mis_sum_kernel, dim3((P.W + 255) / 256, P.row_count), dim3(256), 0, stream, P);
    }
    return hipGetLastError();
}
template <int GEO, bool FREEP = true>
hipError_t launch_mis_g(const MisParams& P, size_t lds, hipStream_t stream) {
    return P.part ? launch_mis_s<GEO, FREEP, true>(P, lds, stream) : launch_mis_s<GEO, FREEP, false>(P, lds, stream);
}

hipError_t launch_mis(const MisParams& P, SceneMem mem, hipStream_t stream) {
    const bool pairs = mem != SceneMem::kLdsSingle && P.nP > 0;
    const size_t lds = mis_lds_bytes(P.nT, pairs ? P.nP : 0u);
    const bool lds_ok = mem != SceneMem::kSmem && lds <= kMaxLdsBytes;
    const size_t X = kMisStashBytes;
    if (P.nTN > 0 && (mem == SceneMem::kTriBvh || mem == SceneMem::kAuto)) return launch_mis_g<kGeoTriBvh>(P, X, stream);
    if (!lds_ok) return launch_mis_g<kGeoTriGlobal>(P, X, stream);
    const size_t lds_clu = lds + kCluF4 * P.nC * sizeof(float4);
    if (pairs && P.nC > 0 && mem == SceneMem::kAuto && lds_clu <= kMaxLdsBytes)
        return P.pair_free ? launch_mis_g<kGeoPairClu, true>(P, lds_clu + X, stream)
                           : launch_mis_g<kGeoPairClu, false>(P, lds_clu + X, stream);
    if (pairs) return launch_mis_g<kGeoPairLds>(P, lds + X, stream);
    return launch_mis_g<kGeoTriLds>(P, lds + X, stream);
}

}  // namespace rt

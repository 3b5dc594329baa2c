// rt_free.hpp — the free-running path kernel for BVH scenes (sphere scenes
// of config 4, triangle meshes): included by rt_kernel.hip inside namespace rt.
// Opt-in (rt_create_options.walk_scheduler = RT_WALK_FREE): measured slower
// than the lockstep kernels (config 4: 2,808 vs 3,531 Msamples/s; 100k
// triangles 705 vs 844; profiles/r5/ab_results.md), kept because it is
// bit-exact and documents the measurement.
//
// The lockstep kernel (path_trace_kernel) runs each bounce's queries for all
// 64 lanes of a wave together, so a wave walks as long as its LONGEST walk:
// on config 4 a lane's closest-hit walk is 38 steps and its wave's 103 (31 %
// step utilisation).  Here every lane owns ONE pixel and traces
// its spp samples one after another (raytrace.metal:34-104) as its own state
// machine; the wave never waits for one query to finish everywhere:
//   * walk phase: every lane whose query is walking takes BVH steps; a lane
//     that meets a leaf worth testing parks it (tested for all parked lanes
//     together once they are 1/kLeafDen of the walking lanes), a lane whose
//     walk ended waits;
//   * service phase, once at least half the live lanes have finished their
//     query: every such lane runs the shading of raytrace.metal:55-101 up to
//     its NEXT query (shadow any-hit, the next bounce's closest hit, or the
//     next sample's camera ray), then walks again.
// (After Aila & Laine's persistent threads with ray regeneration, inside one
// path tracer's state machine.)  It loses because the lanes of a wave are at
// different queries of different pixels: a node load touches up to 64 cache
// lines where the lockstep kernel's 16-lanes-per-pixel waves share most.
//
// Bit parity: a lane computes exactly the operations of the lockstep kernel
// for its pixel, in the same order -- the same Halton dimensions (the bounce
// index is a run-time value here: the same fixed-digit float loop with the
// base picked per lane, extra digits add +0), the same shading, the same
// (t, id)-ranked queries -- and adds its samples to the pixel sum in sample
// order n = 0, 1, ... (one lane per pixel, no cross-lane sums at all).
//
// Per-lane state: the query (ray, tmin, best, id, walk position, parked leaf)
// in registers; the path's throughput, accumulated colour, pending light term,
// next direction and the pixel sum in a per-lane LDS stash (read and written
// only in the service phase, so they are not live across the walk loop).

// service once >= kFreeParkNum/kFreeParkDen of the live lanes finished their
// query (1/2 measured best of 1/4, 1/3, 1/2, 2/3, 3/4)
#ifndef RT_FREE_PARK_DEN
#define RT_FREE_PARK_DEN 2
#endif
#ifndef RT_FREE_PARK_NUM
#define RT_FREE_PARK_NUM 1
#endif
constexpr int kFreeParkDen = RT_FREE_PARK_DEN, kFreeParkNum = RT_FREE_PARK_NUM;

// stash slots (floats, SoA: slot * 64 + lane)
enum FreeSlot : int {
    kFsThr = 0,       // throughput (3)
    kFsAcc = 3,       // accumulatedColor (3)
    kFsContrib = 6,   // pending light term lc * thr of the shadow query (3)
    kFsDir2 = 9,      // next bounce direction (3)
    kFsLum = 12,      // pixel sum (3)
    kFsSlots = 15,
};

// per-lane phase
enum FreePhase : int {
    kFpClosest = 0,   // walking a closest-hit query
    kFpShadow = 1,    // walking a shadow any-hit query
    kFpDone = 2,      // every sample of the pixel is in its sum
    kFpEnd = 3,       // (service) the sample's path ended
    kFpStartC = 4,    // (service) start a closest-hit query from (o, d)
    kFpStartS = 5,    // (service) start a shadow query from (o, d) up to best
};

// Halton dimension SLOT + 5*b for a run-time bounce b < NB (the SLOT-th
// dimension of sampling.metal's per-bounce layout, raytrace.metal:72-74,
// :93-94), index i < 3^13: halton_small's fixed-digit float loop run with the
// per-lane base; NB-1 selects per constant.  The digit count is the one of
// the smallest base (b = 0); a larger base's extra digits are 0 and add +0.
template <uint32_t SLOT, int NB>
__device__ __forceinline__ float halton_bounce_small(uint32_t i, int b) {
    constexpr int nd = halton_digits(kPrimes[SLOT], kSmallIndexMax);
    float bf = (float)kPrimes[SLOT], c = recip_up(kPrimes[SLOT]), invB = 1.0f / (float)kPrimes[SLOT];
#pragma unroll
    for (int bb = 1; bb < NB; ++bb) {
        const uint32_t base = kPrimes[SLOT + 5 * bb];
        const bool m = b == bb;
        bf = m ? (float)base : bf;
        c = m ? recip_up(base) : c;
        invB = m ? 1.0f / (float)base : invB;
    }
    float x = (float)i;  // exact
    float f = 1.0f;
    float r = 0.0f;
#pragma unroll
    for (int k = 0; k < nd; ++k) {
        f = f * invB;
        const float q = __builtin_floorf(x * c);
        const float digit = __builtin_fmaf(q, -bf, x);  // exact: integers < 2^21
        x = q;
        r = r + f * digit;
    }
    return r;
}

// The reference loop (sampling.metal:107-122) with a run-time base: indices
// past the fixed-digit bound.
template <uint32_t SLOT, int NB>
__device__ __forceinline__ float halton_bounce_generic(uint32_t i, int b) {
    uint32_t base = kPrimes[SLOT];
#pragma unroll
    for (int bb = 1; bb < NB; ++bb) base = (b == bb) ? kPrimes[SLOT + 5 * bb] : base;
    const float invB = 1.0f / (float)base;
    float f = 1.0f, r = 0.0f;
    while (i > 0) {
        f = f * invB;
        r = r + f * (float)(i % base);
        i = i / base;
    }
    return r;
}

template <uint32_t SLOT, int NB, bool SMALL>
__device__ __forceinline__ float halton_bounce(uint32_t i, int b) {
    if constexpr (NB <= 0) {
        return 0.0f;
    } else if constexpr (SMALL) {
        return halton_bounce_small<SLOT, NB>(i, b);
    } else {
        return halton_bounce_generic<SLOT, NB>(i, b);
    }
}

// Event log of a -DRT_FREE_DEBUG diagnostic build (read with rt_debug_stats):
// slots 0/1 record every query start, leaf resolve, query end and sample end
// of the pixels (RT_FREE_DBG_X0, _Y0) and (_X1, _Y1); slot 2 records parked
// leaves whose walk-loop resolve disagrees with the same arithmetic evaluated
// before the branch (RT_FREE_CHECK).  Record = kFreeDbgRec words.
#ifdef RT_FREE_DEBUG
#ifndef RT_FREE_DBG_X0
#define RT_FREE_DBG_X0 18
#define RT_FREE_DBG_Y0 20
#define RT_FREE_DBG_X1 29
#define RT_FREE_DBG_Y1 24
#endif
constexpr int kFreeDbgRec = 12, kFreeDbgMax = 1024;
__device__ uint32_t g_free_dbg[4 + 3 * kFreeDbgMax * kFreeDbgRec];
__device__ __forceinline__ void free_dbg(int slot, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3,
                                         float f4, float f5, float f6, float f7, float f8, float f9,
                                         float f10, float f11) {
    const uint32_t pos = atomicAdd(&g_free_dbg[slot], 1u);
    if (pos >= (uint32_t)kFreeDbgMax) return;
    uint32_t* r = &g_free_dbg[4 + ((uint32_t)slot * kFreeDbgMax + pos) * kFreeDbgRec];
    r[0] = w0; r[1] = w1; r[2] = w2; r[3] = w3;
    r[4] = __float_as_uint(f4); r[5] = __float_as_uint(f5); r[6] = __float_as_uint(f6);
    r[7] = __float_as_uint(f7); r[8] = __float_as_uint(f8); r[9] = __float_as_uint(f9);
    r[10] = __float_as_uint(f10); r[11] = __float_as_uint(f11);
}
#endif

// One-wave workgroups (as the lockstep sphere kernel: a workgroup's wave slots
// are released when its wave ends).
constexpr uint32_t kFreeThreads = 64;
constexpr int kFreeWavesPerEu = 8;

template <int B, int GEO, bool SMALL>
__global__ __launch_bounds__(kFreeThreads, kFreeWavesPerEu) void path_free_kernel(KParams P) {
    static_assert(GEO == kGeoSphLds || GEO == kGeoTriBvh, "free-running kernel: BVH scenes");
    constexpr bool SPH = GEO == kGeoSphLds;
    // parked leaves are tested once they are >= 1/kLeafDen of the walking lanes
    // (the lockstep walks' kSphParkDen / kTriParkDen)
    // (rt_create_options.walk_leaf_den; 1: only when every walker is parked)
    const int kLeafDen = P.walk_leaf_den ? (int)P.walk_leaf_den : (SPH ? kSphParkDen : kTriParkDen);
    extern __shared__ float4 lds[];
    __shared__ uint32_t seed_s[kFreeThreads];
    __shared__ float stash[kFsSlots * kFreeThreads];

    SceneView sv;
    sv.nT = P.nT;
    sv.nP = P.nP;
    sv.nS = SPH ? P.nS : 0u;
    sv.nC = 0;
    sv.htab = nullptr;
    if (SPH) {  // the room's pair records in LDS; the compact sphere BVH stays in L2
        const uint32_t ng4 = kPairF4 * sv.nP;
        RT_LDS_GUARD(16 * (size_t)ng4);
        for (uint32_t k = threadIdx.x; k < ng4; k += kFreeThreads) lds[k] = P.pair_isect[k];
        __syncthreads();
        sv.tri = lds;
        sv.pair = lds;
    }
    sv.sent = reinterpret_cast<const uint4*>(P.sph_lds);
    sv.sid = P.sph_lds_id;
    sv.tnode = P.tri_nodes;
    sv.tsorted = P.tri_sorted;
    sv.tperm = P.tri_perm;
    sv.nTN = P.nTN;
    const uint32_t nLay = SPH ? P.nE : P.nTN;  // entries per octant layout

    // XCD-aware tile order (see path_trace_kernel), one wave = one tile of
    // 8x8 pixels, or one row of 64 pixels when the rows are interleaved
    uint32_t bx, by;
    {
        constexpr uint32_t kXcdRun = 4;
        const uint32_t n = gridDim.x * gridDim.y, full = n / (8u * kXcdRun) * (8u * kXcdRun);
        const uint32_t p = blockIdx.y * gridDim.x + blockIdx.x;
        uint32_t t = p;
        if (p < full) {
            const uint32_t xcd = p % 8u, k = p / 8u;
            t = ((k / kXcdRun) * 8u + xcd) * kXcdRun + k % kXcdRun;
        }
        bx = t % gridDim.x;
        by = t / gridDim.x;
    }
    const uint32_t kWX = P.wave_w, kWY = 64u / kWX;
    auto opaque_tid = []() {
        uint32_t t = threadIdx.x;
        asm volatile("" : "+v"(t));
        return t;
    };
    auto pixel_of = [&](uint32_t t, uint32_t& x, uint32_t& j) {
        x = bx * kWX + t % kWX;
        j = by * kWY + t / kWX;
    };
    auto st_get3 = [&](int slot) {
        const uint32_t t = opaque_tid();
        return f3{stash[slot * 64 + t], stash[(slot + 1) * 64 + t], stash[(slot + 2) * 64 + t]};
    };
    auto st_set3 = [&](int slot, f3 v) {
        const uint32_t t = opaque_tid();
        stash[slot * 64 + t] = v.x;
        stash[(slot + 1) * 64 + t] = v.y;
        stash[(slot + 2) * 64 + t] = v.z;
    };

    int ph = kFpEnd;  // every lane starts by "ending" sample -1
    {
        const uint32_t t = threadIdx.x;
        uint32_t x, j;
        pixel_of(t, x, j);
        const bool valid = x < (uint32_t)P.W && j < P.row_count;
        f3 lum{0.0f, 0.0f, 0.0f};                                        // :32
        if (valid) {
            const uint32_t y = P.row_start + j * P.row_step;
            seed_s[t] = P.seeds[(size_t)y * (size_t)P.W + x] + P.sample_base;  // raytrace.metal:37
            if (P.accumulate) {
                const float4 prev = P.sum[(size_t)j * (size_t)P.W + x];
                lum = f3{prev.x, prev.y, prev.z};
            }
        } else {
            ph = kFpDone;
        }
        st_set3(kFsLum, lum);
        st_set3(kFsAcc, f3{0.0f, 0.0f, 0.0f});
    }

    uint32_t n = 0xFFFFFFFFu;  // current sample (sample -1 "ends" first)
    int b = 0;                 // bounce of the current query
    f3 o{0.0f, 0.0f, 0.0f}, d{0.0f, 0.0f, 1.0f};
    float tmin = 0.001f, best = 0.0f;
    int id = -1;
    uint32_t idx = 0, end = 0;  // walk position (entry index over all layouts)
    constexpr uint32_t kNone = 0xFFFFFFFFu;
    uint32_t leaf = kNone;      // parked leaf (sphere entry / triangle leaf word)
    float pb = 0.0f, pdisc = 0.0f, a = 1.0f;  // sphere roots: b, discriminant, dot(d, d)
    RayBox rb{};
    const f3 cu = ld_f3(P.cam_u), cv = ld_f3(P.cam_v), cw = ld_f3(P.cam_w);
    const float fW = (float)P.W, fH = (float)P.H;
#ifdef RT_FREE_DEBUG
    int dslot = -1;  // this lane's log slot (0/1 for the two watched pixels)
    {
        uint32_t x, j;
        pixel_of(threadIdx.x, x, j);
        const uint32_t y = P.row_start + j * P.row_step;
        if (x == RT_FREE_DBG_X0 && y == RT_FREE_DBG_Y0) dslot = 0;
        if (x == RT_FREE_DBG_X1 && y == RT_FREE_DBG_Y1) dslot = 1;
    }
#define FREE_LOG(...) \
    do {                                 \
        if (dslot >= 0) free_dbg(dslot, __VA_ARGS__); \
    } while (0)
#else
#define FREE_LOG(...) ((void)0)
#endif

    // the expensive part of a parked leaf's test: the IEEE roots of sph_test
    // (shaders_old.metal:108-136) or the leaf's exact triangle tests
    auto resolve_leaf = [&](uint32_t site) {
        (void)site;
        if constexpr (SPH) {
            const float sq = sqrtf(pdisc);
            const float a2 = 2.0f * a;
            float t = (-pb - sq) / a2;
            if (!(t > tmin)) t = (-pb + sq) / a2;
#ifdef RT_FREE_DEBUG
            const float best0 = best;
            const int id0 = id;
#endif
            if (ph == kFpShadow) {
                if (t > tmin && t < best) {
                    id = 0;
                    idx = end;
                }
            } else if (t > tmin && t < 3.0e38f && t <= best) {
                const int s = (int)(sv.nT + sv.sid[leaf]);
                if (t < best || s < id) {
                    best = t;
                    id = s;
                }
            }
            FREE_LOG(2u | (uint32_t)ph << 8 | (uint32_t)b << 16 | site << 24, n, leaf,
                     sv.nT + sv.sid[leaf], pb, pdisc, a, t, best0, __int_as_float(id0), best,
                     __int_as_float(id));
        } else {
            if (ph == kFpShadow) {
                if (tri_leaf_any(sv.tsorted, leaf, o, d, tmin, best)) {
                    id = 0;
                    idx = end;
                }
            } else {
                tri_leaf_closest(sv.tsorted, sv.tperm, leaf, o, d, tmin, best, id);
            }
        }
        leaf = kNone;
    };

#ifdef RT_STATS
    // free-kernel counters (tools/free_stats.py), slots 16 + : [0] waves, [1]
    // service phases, [2] lanes served, [3] live lanes at service, [4] walk
    // steps, [5] lanes stepping, [6] leaf rounds, [7] lanes in leaf rounds,
    // [8] cycles in service, [9] cycles in walk phases, [10] queries started
    // (slots 0-15 are the pair loops' counters)
    RT_STAT(16, 1);
    unsigned long long t_ph = clock64();
#endif
    for (;;) {
        // ---------------- service phase ----------------
#ifdef RT_STATS
        RT_STAT(17, 1);
        RT_STAT(18, __popcll(__ballot(ph <= kFpShadow ? idx >= end : ph == kFpEnd)));
        RT_STAT(19, __popcll(__ballot(ph != kFpDone)));
        {
            const unsigned long long t1 = clock64();
            RT_STAT(25, t1 - t_ph);
            t_ph = t1;
        }
#endif
        // a leaf parked at the end of its walk (the walk phase may stop before
        // the parked leaves reach their round)
        if (leaf != kNone) resolve_leaf(1u);
        const bool fin = ph <= kFpShadow && idx >= end;
        if (fin) FREE_LOG(3u | (uint32_t)ph << 8 | (uint32_t)b << 16, n, idx, end, best, 0.0f, 0.0f, 0.0f,
                          0.0f, 0.0f, 0.0f, __int_as_float(id));
        // (1) a finished shadow query: raytrace.metal:79-89, then the next bounce (:99-100)
        if (fin && ph == kFpShadow) {
            if (id < 0) st_set3(kFsAcc, st_get3(kFsAcc) + st_get3(kFsContrib));
            if (b + 1 < B) {
                d = st_get3(kFsDir2);
                b += 1;
                ph = kFpStartC;
            } else {
                ph = kFpEnd;
            }
        }
        // (2) a finished closest query: raytrace.metal:51-101 up to the shadow ray
        if (fin && ph == kFpClosest) {
            ph = kFpEnd;  // :51-53 miss
            if (id >= 0) {
                f3 N, right, fwd, diffuse;
                bool light;
                f3 emis;
                if (!SPH || (uint32_t)id < sv.nT) {
                    const float4* sh = P.tri_shade + 4 * id;
                    const float4 s0 = sh[0], s1 = sh[1], s2 = sh[2], s3 = sh[3];
                    light = s0.w != 0.0f;
                    emis = f3{s3.x, s3.y, s3.z};
                    N = f3{s0.x, s0.y, s0.z};
                    right = f3{s1.x, s1.y, s1.z};
                    fwd = f3{s2.x, s2.y, s2.z};
                    diffuse = f3{s1.w, s2.w, s3.w};
                } else {
                    const float4* sh = P.sph_shade + 3 * ((uint32_t)id - sv.nT);
                    const float4 s0 = sh[0], s1 = sh[1], S = sh[2];
                    light = s0.w != 0.0f;
                    emis = f3{s1.x, s1.y, s1.z};
                    N = normalize((o + d * best) - f3{S.x, S.y, S.z});
                    shading_frame(N, &right, &fwd);
                    diffuse = f3{s0.x, s0.y, s0.z};
                }
                if (light) {                                       // :55-60 overwrite, stop
                    st_set3(kFsAcc, emis);
                } else {
                    const uint32_t i = seed_s[opaque_tid()] + n;
                    const f3 p = (o + d * best) + N * 1e-3f;       // :67
                    // sampleAreaLight (sampling.metal:198-236), dims 2+5b, 3+5b (:72-74)
                    const float ux = halton_bounce<2, B, SMALL>(i, b) * 2.0f - 1.0f;
                    const float uy = halton_bounce<3, B, SMALL>(i, b) * 2.0f - 1.0f;
                    const f3 lcen = ld_f3(P.light_center);
                    const f3 q = (lcen + f3{0.25f, 0.0f, 0.0f} * ux) + f3{0.0f, 0.0f, 0.25f} * uy;
                    f3 L = q - p;
                    const float dist = length(L);
                    const float inv = 1.0f / fmaxf(dist, 1e-3f);
                    L = L * inv;
                    f3 lc = ld_f3(P.light_color) * (inv * inv);
                    lc = lc * saturate(dot(-L, f3{0.0f, -1.0f, 0.0f}));
                    lc = lc * saturate(dot(N, L));                 // :75
                    const f3 thr = st_get3(kFsThr) * diffuse;      // :76
                    st_set3(kFsThr, thr);
                    const f3 contrib = lc * thr;
                    if (b + 1 < B) {                               // :93-100 (last direction never traced)
                        const float cuu = halton_bounce<4, B - 1, SMALL>(i, b);
                        const float cvv = halton_bounce<5, B - 1, SMALL>(i, b);
                        float sp, cp;
                        sincos_pt(6.28318548f * cuu, &sp, &cp);    // sampling.metal:40-48
                        const float ct = sqrtf(cvv);
                        const float st = sqrtf(1.0f - ct * ct);
                        st_set3(kFsDir2, (right * (st * cp) + N * ct) + fwd * (st * sp));  // sampling.metal:65
                    }
                    o = p;
                    // a zero light term adds +0 to acc whatever the shadow
                    // query says: no query
                    if (contrib.x != 0.0f || contrib.y != 0.0f || contrib.z != 0.0f) {
                        st_set3(kFsContrib, contrib);
                        d = L;
                        best = dist - 1e-3f;                       // :82
                        ph = kFpStartS;
                    } else if (b + 1 < B) {
                        d = st_get3(kFsDir2);
                        b += 1;
                        ph = kFpStartC;
                    }
                }
            }
        }
        // (3) the end of a sample: raytrace.metal:103, then the next sample's camera ray
        if (ph == kFpEnd) {
            if (n != 0xFFFFFFFFu) st_set3(kFsLum, st_get3(kFsLum) + st_get3(kFsAcc));  // :103 in order n
#ifdef RT_FREE_DEBUG
            if (n != 0xFFFFFFFFu) {
                const f3 acc = st_get3(kFsAcc);
                FREE_LOG(4u, n, 0u, 0u, acc.x, acc.y, acc.z, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f);
            }
#endif
            n += 1;
            if (n >= P.spp) {
                ph = kFpDone;
            } else {
                const uint32_t t = opaque_tid();
                const uint32_t i = seed_s[t] + n;
                uint32_t x, j;
                pixel_of(t, x, j);
                const float fx = (float)x, fy = (float)(P.row_start + j * P.row_step);
                const float jx = halton_dim<0, SMALL>(i);                                 // :39-40
                const float jy = halton_dim<1, SMALL>(i);
                // generateCameraRay (sampling.metal:125-157)
                const float sx = ((fx + jx) / fW) * 2.0f - 1.0f;
                const float ty = -(((fy + jy) / fH) * 2.0f - 1.0f);
                const float sh = sx * P.halfW, th = ty * P.halfH;
                d = normalize((cu * sh + cv * th) - cw);
                o = ld_f3(P.cam_pos);
                st_set3(kFsThr, f3{1.0f, 1.0f, 1.0f});
                st_set3(kFsAcc, f3{0.0f, 0.0f, 0.0f});
                b = 0;
                ph = kFpStartC;
            }
        }
        // (4) start a query: the room's pair records (sphere scenes), then the walk
        if (ph >= kFpStartC) {
            const bool shadow = ph == kFpStartS;
            tmin = shadow ? 0.0f : 0.001f;                         // MSL ray default / sampling.metal:154
            id = -1;
            if (!shadow) best = 1000.0f;                           // sampling.metal:155
            if constexpr (SPH) {
                if (shadow) {
                    const f3 e = o + d * best;
                    const f3 lo{fminf(o.x, e.x), fminf(o.y, e.y), fminf(o.z, e.z)};
                    const f3 hi{fmaxf(o.x, e.x), fmaxf(o.y, e.y), fmaxf(o.z, e.z)};
                    if (any_hit<kGeoPairLds, false, false>(sv, o, d, 0.0f, best, lo, hi)) id = 0;
                } else {
                    float t = best;
                    id = closest_hit<kGeoPairLds, false, false, 1>(sv, o, d, 0.001f, &t);
                    best = t;
                }
            }
            a = dot(d, d);
            rb = ray_box(o, d);
            idx = octant(d) * nLay;
            end = idx + nLay;
            if (id >= 0 && shadow) idx = end;                      // occluded by a wall
            ph = shadow ? kFpShadow : kFpClosest;
            FREE_LOG(1u | (uint32_t)ph << 8 | (uint32_t)b << 16, n, idx, end, o.x, o.y, o.z, d.x, d.y, d.z,
                     best, __int_as_float(id));
            RT_STAT(26, __popcll(__ballot(1)));
        }
        const bool live = ph != kFpDone;
#ifdef RT_STATS
        {
            const unsigned long long t1 = clock64();
            RT_STAT(24, t1 - t_ph);
            t_ph = t1;
        }
#endif
        if (__builtin_amdgcn_ballot_w64(live) == 0) break;
        // ---------------- walk phase ----------------
        // Lanes take BVH steps; a lane that meets a leaf worth testing parks it
        // (tested for all parked lanes together once they are 1/kLeafDen of
        // the walking ones, as the lockstep walks do); a lane whose walk ended
        // waits for the service phase, which runs once they are 1/kFreeParkDen
        // of the live lanes.
        const int nlive = __popcll(__builtin_amdgcn_ballot_w64(live));
        for (;;) {
            const bool adv = live && idx < end && leaf == kNone;
            RT_STAT(20, 1);
            RT_STAT(21, __popcll(__ballot(adv)));
            if (adv) {
                if constexpr (SPH) {
                    const uint4 e = sv.sent[idx];
                    if (e.w & 0x80000000u) {
                        idx = lds_node_hit_nf(e, rb, tmin, best) ? idx + 1 : (e.w & 0x7FFFFFFFu);
                    } else {  // sph_test up to the discriminant
                        const f3 oc = o - f3{__uint_as_float(e.x), __uint_as_float(e.y), __uint_as_float(e.z)};
                        const float bq = 2.0f * dot(oc, d);
                        const float cc = dot(oc, oc) - __uint_as_float(e.w);
                        const float disc = bq * bq - (4.0f * a) * cc;
                        if (disc > 0.0f) {
                            leaf = idx;
                            pb = bq;
                            pdisc = disc;
                        }
                        idx = idx + 1;
                    }
                } else {
                    const uint4 e = sv.tnode[idx];
                    const bool inner = (e.w & 0x80000000u) != 0u;
                    if (!lds_node_hit_nf(e, rb, tmin, best)) {
                        idx = inner ? (e.w & 0x7FFFFFFFu) : idx + 1;
                    } else {
                        if (!inner) leaf = e.w;
                        idx = idx + 1;
                    }
                }
            }
            const bool parked = leaf != kNone;
            const int np = __popcll(__builtin_amdgcn_ballot_w64(parked));
            const int nwalk = __popcll(__builtin_amdgcn_ballot_w64(parked || (live && idx < end)));
            if (np > 0 && kLeafDen * np >= nwalk) {
                RT_STAT(22, 1);
                RT_STAT(23, np);
#ifdef RT_FREE_BRANCH
                if (true) {
#ifdef RT_FREE_CHECK
                    // the select form's arithmetic before the branch, compared after it
                    float xb = best;
                    int xi = id;
                    uint32_t xx = idx;
                    float xt = 0.0f;
                    const uint32_t leaf0 = leaf;
                    const float best0 = best;
                    const int id0 = id;
                    if (parked) {
                        const float sq = sqrtf(pdisc);
                        const float a2 = 2.0f * a;
                        float t = (-pb - sq) / a2;
                        const float t2 = (-pb + sq) / a2;
                        t = (t > tmin) ? t : t2;
                        xt = t;
                        const int sidv = (int)(sv.nT + sv.sid[leaf]);
                        if (ph == kFpShadow) {
                            if (t > tmin && t < best) { xi = 0; xx = end; }
                        } else if (t > tmin && t < 3.0e38f && t <= best && (t < best || sidv < id)) {
                            xb = t;
                            xi = sidv;
                        }
                    }
#endif
                    if (parked) resolve_leaf(0u);
#ifdef RT_FREE_CHECK
                    if (parked) atomicAdd(&g_free_dbg[3], 1u);  // resolves checked
                    if (parked && (__float_as_uint(xb) != __float_as_uint(best) || xi != id || xx != idx)) {
                        free_dbg(2, (uint32_t)ph | (uint32_t)b << 8, leaf0, (uint32_t)id0, (uint32_t)xi,
                                 pb, pdisc, a, tmin, best0, xt, best, __int_as_float(id));
                    }
#endif
                } else
#endif
                if constexpr (SPH) {
                    // every lane evaluates the roots, parked lanes keep the
                    // result.  The branch form (RT_FREE_BRANCH: resolve_leaf
                    // under `if (parked)`, as the service phase does) is
                    // bit-exact too (round 6, profiles/r6/free_walk/: the 42
                    // free-scheduler GPU tests, and RT_FREE_CHECK re-evaluated
                    // 43,523 walk-loop resolves of the failing round-5 case in
                    // this form before the branch: 0 disagreements).  Round
                    // 5's 4 wrong values came from an uncommitted intermediate
                    // kernel, not from either form.
                    const float sq = sqrtf(parked ? pdisc : 1.0f);
                    const float a2 = 2.0f * a;
                    float t = (-pb - sq) / a2;
                    const float t2 = (-pb + sq) / a2;
                    t = (t > tmin) ? t : t2;
                    const int sidv = (int)(sv.nT + sv.sid[parked ? leaf : 0u]);
                    const bool sh = ph == kFpShadow;
                    const bool hit_any = sh && t > tmin && t < best;
                    const bool hit_c = !sh && t > tmin && t < 3.0e38f && t <= best && (t < best || sidv < id);
#ifdef RT_FREE_DEBUG
                    const float best0 = best;
                    const int id0 = id;
#endif
                    id = (parked && hit_any) ? 0 : ((parked && hit_c) ? sidv : id);
                    idx = (parked && hit_any) ? end : idx;
                    best = (parked && hit_c) ? t : best;
                    if (parked)
                        FREE_LOG(2u | (uint32_t)ph << 8 | (uint32_t)b << 16 | 2u << 24, n, leaf, (uint32_t)sidv, pb,
                                 pdisc, a, t, best0, __int_as_float(id0), best, __int_as_float(id));
                    leaf = kNone;
                } else {
                    if (parked) resolve_leaf(0u);
                }
            }
            const int nfin = nlive - __popcll(__builtin_amdgcn_ballot_w64(leaf != kNone || (live && idx < end)));
            if (kFreeParkDen * nfin >= kFreeParkNum * nlive) break;
        }
    }

    if (ph != kFpDone || n == 0xFFFFFFFFu) return;  // pixels outside the frame
    const uint32_t t = opaque_tid();
    uint32_t x, j;
    pixel_of(t, x, j);
    const f3 lum = st_get3(kFsLum);
    const size_t o2 = (size_t)j * (size_t)P.W + x;
    if (P.sum) P.sum[o2] = make_float4(lum.x, lum.y, lum.z, (float)P.samples_total);
    if (P.out) {
        const float fs = (float)P.samples_total;                   // :106
        store_pixel(P, o2, lum.x / fs, lum.y / fs, lum.z / fs);
    }
}

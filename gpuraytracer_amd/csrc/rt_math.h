// rt_math.h — fp32 vector math of the path-tracing hot path, written once for
// the gfx950 kernel and for the host-side scene precompute (rt_scene.cpp).
//
// Arithmetic contract: IEEE fp32, round-to-nearest-even, no
// implicit contraction (every TU is compiled with -ffp-contract=off);
// dot/cross use explicit fmaf; division and sqrt are correctly rounded (the
// hipcc default for gfx950; never -ffast-math).  Under this contract the
// device and the host produce bit-identical values, which is what makes the
// GPU-vs-oracle parity bit-exact.
#pragma once

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define RT_HD __host__ __device__ __forceinline__
#else
#define RT_HD inline
#endif

namespace rt {

struct f3 {
    float x, y, z;
};

RT_HD f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
RT_HD f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_HD f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_HD f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
RT_HD f3 operator*(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
RT_HD f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }

// dot(a,b) = fma(a.z,b.z, fma(a.y,b.y, a.x*b.x))
RT_HD float dot(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }
// cross component i = fma(a_j, b_k, -(a_k * b_j))
RT_HD f3 cross(f3 a, f3 b) {
    return f3{fmaf(a.y, b.z, -(a.z * b.y)), fmaf(a.z, b.x, -(a.x * b.z)),
              fmaf(a.x, b.y, -(a.y * b.x))};
}
RT_HD float length(f3 a) { return sqrtf(dot(a, a)); }
// normalize(v) = v * (1 / sqrt(dot(v,v)))
RT_HD f3 normalize(f3 a) { return a * (1.0f / sqrtf(dot(a, a))); }
RT_HD float saturate(float x) { return fminf(fmaxf(x, 0.0f), 1.0f); }

// Halton bases: `constant unsigned int primes[]` (RTrace/sampling.metal:97-104).
#define RT_PRIMES_INIT {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, \
                        41, 43, 47, 53, 59, 61, 67, 71, 73, 79, 83, 89}

// Frame reference vector of alignHemisphereWithNormal (sampling.metal:57).
RT_HD f3 frame_ref() { return f3{0.0072f, 1.0f, 0.0034f}; }

// right = normalize(cross(N, ref)); forward = cross(right, N)   (sampling.metal:51-66)
RT_HD void shading_frame(f3 N, f3* right, f3* fwd) {
    *right = normalize(cross(N, frame_ref()));
    *fwd = cross(*right, N);
}

// Portable sincos for x in [0, 2*pi]: Cody-Waite reduction
// by pi/2 (two fma steps) + minimax polynomials on [-pi/4, pi/4].
RT_HD void sincos_pt(float x, float* s_out, float* c_out) {
    const float k = rintf(x * 0.636619772f);
    float r = fmaf(-k, 1.57079637e+00f, x);
    r = fmaf(-k, -4.37113883e-08f, r);
    const int q = ((int)k) & 3;
    const float r2 = r * r;
    const float s = fmaf(r * r2, fmaf(r2, fmaf(r2, -1.9515295891e-4f, 8.3321608736e-3f),
                                      -1.6666654611e-1f), r);
    const float c = fmaf(r2 * r2, fmaf(r2, fmaf(r2, 2.443315711809948e-5f,
                                                -1.388731625493765e-3f), 4.166664568298827e-2f),
                         fmaf(-0.5f, r2, 1.0f));
    const float ss = (q & 1) ? c : s;
    const float cc = (q & 1) ? s : c;
    *s_out = (q & 2) ? -ss : ss;
    *c_out = ((q + 1) & 2) ? -cc : cc;
}

}  // namespace rt

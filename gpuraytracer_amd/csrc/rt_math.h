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
// Correctly rounded sqrt and reciprocal in fewer instructions
// on the device.  For an argument whose magnitude lies in [2^-100, 2^100) the
// short sequences below equal IEEE sqrtf(x) and 1.0f / x bit for bit -- checked
// on gfx950 for every float of that range (tools/math_probe.hip; the library's
// own rt_math_selfcheck runs the shipped functions over every float, tested in
// tests/test_gpu_parity.py): a hardware rsq + a Goldschmidt/Markstein
// refinement (7 VALU instead of the compiler's 15-instruction IEEE sqrt), and a
// hardware rcp + one fma Newton step (3 instead of ~11 with the div_scale /
// div_fmas / div_fixup sequence).  A wave with any lane outside the range
// (or a negative sqrt argument) takes the IEEE expansions; +-0 keeps its sign
// under sqrt.  The host (and the oracle) use sqrtf and division: the same values.
#ifndef RT_CR_FAST  // 0: the IEEE expansions everywhere (A/B)
#define RT_CR_FAST 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && RT_CR_FAST
__device__ __forceinline__ bool rt_cr_domain(uint32_t b) {  // magnitude bits in [2^-100, 2^100)
    return b - 0x0D800000u < 0x71800000u - 0x0D800000u;
}
__device__ __forceinline__ float sqrt_cr(float x) {
    const bool ok = x == 0.0f || rt_cr_domain(__float_as_uint(x));  // positive x only (sign bit set fails)
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
        const float r = __builtin_amdgcn_rsqf(x);
        float s = x * r, h = 0.5f * r;
        const float e = fmaf(-s, h, 0.5f);
        s = fmaf(s, e, s);
        h = fmaf(h, e, h);
        const float d = fmaf(-s, s, x);
        const float v = fmaf(d, h, s);
        return x == 0.0f ? x : v;
    }
    return sqrtf(x);
}
__device__ __forceinline__ float rcp_cr(float x) {
    if (__builtin_amdgcn_ballot_w64(!rt_cr_domain(__float_as_uint(x) & 0x7FFFFFFFu)) == 0) {
        const float r = __builtin_amdgcn_rcpf(x);
        return fmaf(fmaf(-x, r, 1.0f), r, r);
    }
    return 1.0f / x;
}
#else
RT_HD float sqrt_cr(float x) { return sqrtf(x); }
RT_HD float rcp_cr(float x) { return 1.0f / x; }
#endif
RT_HD float length(f3 a) { return sqrt_cr(dot(a, a)); }
// normalize(v) = v * (1 / sqrt(dot(v,v)))
RT_HD f3 normalize(f3 a) { return a * rcp_cr(sqrt_cr(dot(a, a))); }
// The same values through the IEEE expansions: for kernels where the short
// forms' uniform branch costs registers (the triangle-BVH kernel spilled 20
// more bytes per lane with them)
RT_HD float length_ieee(f3 a) { return sqrtf(dot(a, a)); }
RT_HD f3 normalize_ieee(f3 a) { return a * (1.0f / sqrtf(dot(a, a))); }
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

// ---- MIS integrator helpers (Sources/gpuRaytracer/shaders.metal) ---------

RT_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
RT_HD float u2f(uint32_t x) { return __builtin_bit_cast(float, x); }

// hash (shaders.metal:58-65)
RT_HD uint32_t mis_hash(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// randomFloat (:67-69): float(h) / (float(0xffffffff) + 1) = float(h) * 2^-32, exactly
RT_HD float mis_unit(uint32_t h) { return (float)h * 2.3283064365386963e-10f; }

// buildOrthonormalBasis (:159-172)
RT_HD void onb(f3 n, f3* t, f3* b) {
    const f3 a = fabsf(n.x) > 0.9f ? f3{0.0f, 1.0f, 0.0f} : f3{1.0f, 0.0f, 0.0f};
    *t = normalize(a - n * dot(a, n));
    *b = cross(n, *t);
}

// Portable natural log for normal x > 0 (cephes logf reduction and
// polynomial, Horner steps as explicit fmaf).
RT_HD float log_pt(float x) {
    const uint32_t bx = f2u(x);
    int e = (int)(bx >> 23) - 126;                     // x = m * 2^e, m in [0.5, 1)
    float m = u2f((bx & 0x007FFFFFu) | 0x3F000000u);
    if (m < 0.707106781f) {
        e -= 1;
        m = m + m - 1.0f;
    } else {
        m = m - 1.0f;
    }
    const float z = m * m;
    float y = 7.0376836292e-2f;
    y = fmaf(y, m, -1.1514610310e-1f);
    y = fmaf(y, m, 1.1676998740e-1f);
    y = fmaf(y, m, -1.2420140846e-1f);
    y = fmaf(y, m, 1.4249322787e-1f);
    y = fmaf(y, m, -1.6668057665e-1f);
    y = fmaf(y, m, 2.0000714765e-1f);
    y = fmaf(y, m, -2.4999993993e-1f);
    y = fmaf(y, m, 3.3333331174e-1f);
    y = (y * m) * z;
    const float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(-0.5f, z, y);
    return fmaf(fe, 0.693359375f, m + y);
}

// Portable e^x for x in [-87, 0] (cephes expf; explicit fmaf).
RT_HD float exp_pt(float x) {
    const float z = floorf(x * 1.44269504088896341f + 0.5f);
    float r = fmaf(-z, 0.693359375f, x);
    r = fmaf(-z, -2.12194440e-4f, r);
    float p = 1.9875691500e-4f;
    p = fmaf(p, r, 1.3981999507e-3f);
    p = fmaf(p, r, 8.3334519073e-3f);
    p = fmaf(p, r, 4.1665795894e-2f);
    p = fmaf(p, r, 1.6666665459e-1f);
    p = fmaf(p, r, 5.0000001201e-1f);
    const float y = fmaf(p, r * r, r) + 1.0f;
    return y * u2f((uint32_t)((int)z + 127) << 23);
}

// pow(x, y) for x in [0, 1], y > 0 (the gamma of drawTriangle, :702-703):
// exp(y * log(x)); x <= 2^-100 gives 0 (the true value is < 2^-45).
RT_HD float pow_pt(float x, float y) {
    if (!(x > 7.88860905e-31f)) return 0.0f;
    return exp_pt(y * log_pt(x));
}

// One RGB channel of the reference's image epilogue (RTrace/image.swift:41-60)
// on a value already round-tripped through the rgba16F texture (:35-38):
// x2 exposure, Reinhard, pow(v, 1/2.2), clamp, truncating UInt8.  The pow is
// the portable pow_pt; a NaN (an fp16 inf after Reinhard)
// skips it and clamps to 1, as Swift's min(1.0, NaN) returns 1.0.
RT_HD uint8_t tonemap_channel(float v) {
    v = v * 2.0f;                                   // exposure :41,54
    v = v / (v + 1.0f);                             // Reinhard :55
    if (v == v) v = pow_pt(v, 1.0f / 2.2f);         // gamma :42,56
    v = fmaxf(0.0f, fminf(1.0f, v));                // :59
    return (uint8_t)(v * 255.0f);                   // UInt8(value * 255) :60
}

}  // namespace rt

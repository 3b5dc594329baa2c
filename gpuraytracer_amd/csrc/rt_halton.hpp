// rt_halton.hpp — the Halton radical inverse of the path-tracing kernels
// (RTrace/sampling.metal:97-122), compile-time dimension forms shared by the
// path-tracing kernels.  Every form is bit-identical to the reference loop
// (DESIGN.md §3.3).
#pragma once
#include <hip/hip_runtime.h>

#include "rt_kernel.hpp"

namespace rt {
namespace {

constexpr uint32_t kPrimes[24] = RT_PRIMES_INIT;

// halton(i, D) — sampling.metal:107-122 with a compile-time dimension.
template <uint32_t D>
__device__ __forceinline__ float halton(uint32_t i) {
    static_assert(D < 24, "Halton dimension outside primes[]");
    constexpr uint32_t b = kPrimes[D];
    constexpr float invB = 1.0f / (float)b;
    float f = 1.0f;
    float r = 0.0f;
    while (i > 0) {
        f = f * invB;
        r = r + f * (float)(i % b);
        i = i / b;
    }
    return r;
}

// Digits of every i < imax in base b (compile time).
constexpr int halton_digits(uint32_t b, uint64_t imax) {
    uint64_t cap = 1;
    int n = 0;
    while (cap < imax) {
        cap *= b;
        ++n;
    }
    return n;
}

// Smallest float c >= 1/n.  For every integer x < 2^21 held exactly in a
// float, floor(fl(x * c)) == x / n: c >= 1/n keeps the product at or above the
// quotient q (q is representable), and c's error plus the product's rounding
// (< 2^-22 relative) stay below the 1/x relative gap up to q + 1.  Re-verified
// exhaustively by tests/test_oracle.py::test_halton_float_digits.
constexpr float recip_up(uint32_t n) {
    float c = 1.0f / (float)n;
    if ((double)c * (double)n < 1.0) c = __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, c) + 1u);
    return c;
}

// One digit step on the exact-integer float x < 2^21: returns x / b and sets
// digit = x mod b (also an exact float, i.e. the reference's (float)(i % b)).
// 3 VALU (mul, floor, fma) where a 24-bit magic integer division takes 4
// (mul_u24, mulhi_u24, alignbit, mad_i24) and the digit then needs an int ->
// float conversion: 1080p x 256 spp ran 31.0 -> 29.0 ms.
template <uint32_t b>
__device__ __forceinline__ float digit_step(float x, float& digit) {
    constexpr float c = recip_up(b);  // compile time
    const float q = __builtin_floorf(x * c);
    digit = __builtin_fmaf(q, -(float)b, x);  // exact: integers < 2^21
    return q;
}

// The same radical inverse for i < kSmallIndexMax = 3^13 (every reference
// seed is < 2^20, renderer.swift:100, so up to 545k samples per pixel; 3^13
// rather than 2^21 drops the top digit of bases 3, 5 and 11, which a
// 2^21 bound would need): the loop runs a fixed digit count, fully unrolled, so
// f = invB^k folds to compile-time constants and no loop control remains.  The
// extra iterations past i's last digit add f*0 = +0 to r >= 0: bit-identical.
// Digits come from float reciprocal multiplies (exact, see recip_up).  Base 2
// is exact in fp32 at every step (sums of distinct powers of two spanning
// <= 21 bits), so it equals the bit-reversed index: 3 instructions instead of
// 21 digit steps.
constexpr uint32_t kSmallIndexMax = 1594323;  // 3^13
constexpr int kSmallIndexBits = 21;           // base-2 bit-reversal width
static_assert(kSmallIndexMax <= (1u << kSmallIndexBits), "float digit steps need x < 2^21");
template <uint32_t D>
__device__ __forceinline__ float halton_small(uint32_t i) {
    constexpr uint32_t b = kPrimes[D];
    if constexpr (b == 2) {
        return (float)(__builtin_bitreverse32(i) >> (32 - kSmallIndexBits)) *
               (1.0f / (float)(1u << kSmallIndexBits));
    } else {
        constexpr int nd = halton_digits(b, kSmallIndexMax);
        constexpr float invB = 1.0f / (float)b;
        float x = (float)i;  // exact
        float f = 1.0f;
        float r = 0.0f;
#pragma unroll
        for (int k = 0; k < nd; ++k) {
            f = f * invB;
            float digit;
            x = digit_step<b>(x, digit);
            r = r + f * digit;
        }
        return r;
    }
}

// ---- low-digit tables --------------------------------------
// The reference adds the digits lowest first, so after the k lowest digits its
// running sum depends only on i mod b^k.  A workgroup fills T_D[v] (v < b^k,
// the loop's r after k digit steps of v; digits past v's own add +0) in LDS
// with the same fp32 operations, and halton_tab continues from T_D[i mod b^k]
// with the remaining digits of i / b^k: the same sum, bit for bit.  k per
// dimension fits the tables in ~18 KB of LDS (the camera jitter and bounces
// 0-1; 24 of the 73 digit steps of a 3-bounce sample).
// i / b^k and i mod b^k come from one float digit step with n = b^k (< 2^23).
constexpr int kTabDigits[24] = {0, 6, 4, 3, 2, 2, 0, 2, 2, 2, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
constexpr uint32_t ipow(uint32_t b, int k) { return k == 0 ? 1u : b * ipow(b, k - 1); }
constexpr uint32_t tab_size(int D) { return kTabDigits[D] ? ipow(kPrimes[D], kTabDigits[D]) : 0u; }
constexpr uint32_t tab_offset(int D) { return D == 0 ? 0u : tab_offset(D - 1) + tab_size(D - 1); }
constexpr uint32_t kHaltonTabFloats = tab_offset(24);
// f = invB^k as the reference's loop forms it (f = f * invB, k times)
constexpr float f_after(uint32_t b, int k) {
    float f = 1.0f;
    for (int j = 0; j < k; ++j) f = f * (1.0f / (float)b);
    return f;
}

template <uint32_t D>
__device__ __forceinline__ void fill_halton_table(float* tab, uint32_t tid, uint32_t nthreads) {
    constexpr uint32_t b = kPrimes[D];
    constexpr int k = kTabDigits[D];
    constexpr float invB = 1.0f / (float)b;
    constexpr uint32_t off = tab_offset(D), size = tab_size(D);  // compile time
    for (uint32_t v0 = tid; v0 < size; v0 += nthreads) {
        uint32_t v = v0;
        float f = 1.0f;
        float r = 0.0f;
#pragma unroll
        for (int j = 0; j < k; ++j) {
            f = f * invB;
            r = r + f * (float)(v % b);
            v = v / b;
        }
        tab[off + v0] = r;
    }
}

// All tables; every thread of the workgroup calls it (then a barrier).
__device__ __forceinline__ void fill_halton_tables(float* tab, uint32_t tid, uint32_t nthreads) {
    fill_halton_table<1>(tab, tid, nthreads);
    fill_halton_table<2>(tab, tid, nthreads);
    fill_halton_table<3>(tab, tid, nthreads);
    fill_halton_table<4>(tab, tid, nthreads);
    fill_halton_table<5>(tab, tid, nthreads);
    fill_halton_table<7>(tab, tid, nthreads);
    fill_halton_table<8>(tab, tid, nthreads);
    fill_halton_table<9>(tab, tid, nthreads);
    fill_halton_table<10>(tab, tid, nthreads);
    static_assert(kHaltonTabFloats == 729 + 625 + 343 + 121 + 169 + 361 + 529 + 841 + 961,
                  "table list");
}

// halton_small<D> for i < kSmallIndexMax starting from the low-digit table.
template <uint32_t D>
__device__ __forceinline__ float halton_tab(uint32_t i, const float* tab) {
    constexpr uint32_t b = kPrimes[D];
    constexpr int k = kTabDigits[D];
    constexpr int nd = halton_digits(b, kSmallIndexMax);
    constexpr float invB = 1.0f / (float)b;
    constexpr uint32_t bk = ipow(b, k), off = tab_offset(D);
    static_assert(k > 0 && k < nd, "dimension without a table");
    float low;
    float x = digit_step<bk>((float)i, low);  // i / b^k and i mod b^k, exact
    float r = tab[off + (uint32_t)low];
    constexpr float fk = f_after(b, k);  // compile time (a run-time call needs a stack)
    float f = fk;
#pragma unroll
    for (int j = k; j < nd; ++j) {
        f = f * invB;
        float digit;
        x = digit_step<b>(x, digit);
        r = r + f * digit;
    }
    return r;
}

// TAB: the kernel may stage the low-digit tables (SMALL indices only); tab is
// null (wave-uniform) when this launch has too few samples per lane to pay for
// filling them.
template <uint32_t D, bool SMALL, bool TAB = false>
__device__ __forceinline__ float halton_dim(uint32_t i, const float* tab = nullptr) {
    if constexpr (TAB && SMALL && kTabDigits[D] > 0)
        if (tab != nullptr) return halton_tab<D>(i, tab);
    if (SMALL) return halton_small<D>(i);
    return halton<D>(i);
}

}  // namespace
}  // namespace rt

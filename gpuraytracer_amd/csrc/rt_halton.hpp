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

// Digits of i < 2^bits in base b (compile time).
constexpr int halton_digits(uint32_t b, int bits) {
    uint64_t cap = 1;
    int n = 0;
    while (cap < (1ull << bits)) {
        cap *= b;
        ++n;
    }
    return n;
}

// 24-bit integer multiplies (full rate; the 32-bit v_mul_lo/hi_u32 are not).
extern "C" __device__ uint32_t rt_mul_u24(uint32_t, uint32_t) __asm("llvm.amdgcn.mul.u24");
extern "C" __device__ uint32_t rt_mulhi_u24(uint32_t, uint32_t) __asm("llvm.amdgcn.mulhi.u24");
extern "C" __device__ int32_t rt_mul_i24(int32_t, int32_t) __asm("llvm.amdgcn.mul.i24");

// q = floor(i / b) = (i * M) >> S for every i < 2^21 with M < 2^24, per base
// primes[d].  Found by exhaustive search and re-verified exhaustively by
// tests/test_oracle.py::test_halton_small_magic_table (parses this table).
constexpr uint32_t kMagicM[24] = {524288, 699051, 838861, 1198373, 762601, 2581111, 1973791,
                                  1766023, 1458889, 2314099, 2164803, 3627507, 818401, 48771,
                                  2855697, 1266205, 2274877, 2200291, 1001625, 1890391, 3677199,
                                  1698959, 3234163, 1508065};
constexpr uint32_t kMagicS[24] = {20, 21, 22, 23, 23, 25, 25, 25, 25, 26, 26, 27,
                                  25, 21, 27, 26, 27, 27, 26, 27, 28, 27, 28, 27};

// The same radical inverse for i < 2^21 (every reference seed is < 2^20,
// renderer.swift:100): the loop runs a fixed digit count, fully unrolled, so
// f = invB^k folds to compile-time constants and no loop control remains.  The
// extra iterations past i's last digit add f*0 = +0 to r >= 0: bit-identical.
// Digits come from 24-bit magic multiplies (exact, see kMagicM).  Base 2 is
// exact in fp32 at every step (sums of distinct powers of two spanning <= 21
// bits), so it equals the bit-reversed index: 3 instructions instead of 21
// digit steps.
constexpr int kSmallIndexBits = 21;
template <uint32_t D>
__device__ __forceinline__ float halton_small(uint32_t i) {
#ifdef RT_TIMING_NO_HALTON  // timing-only experiment (share of the Halton digits), NOT exact
    return (float)((i * (2654435761u + 2u * D)) >> 8) * (1.0f / 16777216.0f);
#endif
    constexpr uint32_t b = kPrimes[D];
    if constexpr (b == 2) {
        return (float)(__builtin_bitreverse32(i) >> (32 - kSmallIndexBits)) *
               (1.0f / (float)(1u << kSmallIndexBits));
    } else {
        constexpr int nd = halton_digits(b, kSmallIndexBits);
        constexpr float invB = 1.0f / (float)b;
        constexpr uint32_t M = kMagicM[D], S = kMagicS[D];
        float f = 1.0f;
        float r = 0.0f;
#pragma unroll
        for (int k = 0; k < nd; ++k) {
            f = f * invB;
            const uint32_t q = __builtin_amdgcn_alignbit(rt_mulhi_u24(i, M), rt_mul_u24(i, M), S);
            const uint32_t digit = (uint32_t)((int32_t)i + rt_mul_i24((int32_t)q, -(int32_t)b));
            r = r + f * (float)digit;
            i = q;
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
constexpr int kTabDigits[24] = {0, 6, 4, 3, 2, 2, 0, 2, 2, 2, 2, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
// q = floor(i / b^k) = (i * M) >> S for every i < 2^21 (exhaustively verified
// by tests/test_oracle.py::test_halton_table_magic, which parses this table)
constexpr uint32_t kTabM[24] = {0, 1472897, 1717987, 782611, 2218475, 198547, 0, 2974355, 1014879,
                                2553489, 2234635, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
constexpr uint32_t kTabS[24] = {0, 30, 30, 28, 28, 25, 0, 30, 29,
                                31, 31, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
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

// halton_small<D> for i < 2^21 starting from the low-digit table.
template <uint32_t D>
__device__ __forceinline__ float halton_tab(uint32_t i, const float* tab) {
    constexpr uint32_t b = kPrimes[D];
    constexpr int k = kTabDigits[D];
    constexpr int nd = halton_digits(b, kSmallIndexBits);
    constexpr float invB = 1.0f / (float)b;
    constexpr uint32_t bk = ipow(b, k), TM = kTabM[D], TS = kTabS[D], off = tab_offset(D);
    static_assert(k > 0 && k < nd, "dimension without a table");
    uint32_t q;
    if constexpr (TS >= 32)
        q = rt_mulhi_u24(i, TM) >> (TS - 32);
    else
        q = __builtin_amdgcn_alignbit(rt_mulhi_u24(i, TM), rt_mul_u24(i, TM), TS);
    const uint32_t low = (uint32_t)((int32_t)i + rt_mul_i24((int32_t)q, -(int32_t)bk));
    float r = tab[off + low];
    constexpr float fk = f_after(b, k);  // compile time (a run-time call needs a stack)
    float f = fk;
    constexpr uint32_t M = kMagicM[D], S = kMagicS[D];
    i = q;
#pragma unroll
    for (int j = k; j < nd; ++j) {
        f = f * invB;
        const uint32_t q2 = __builtin_amdgcn_alignbit(rt_mulhi_u24(i, M), rt_mul_u24(i, M), S);
        const uint32_t digit = (uint32_t)((int32_t)i + rt_mul_i24((int32_t)q2, -(int32_t)b));
        r = r + f * (float)digit;
        i = q2;
    }
    return r;
}

// TAB: the kernel may stage the low-digit tables (SMALL indices only); tab is
// null (wave-uniform) when this launch has too few samples per lane to pay for
// filling them.
template <uint32_t D, bool SMALL, bool TAB = false>
__device__ __forceinline__ float halton_dim(uint32_t i, const float* tab = nullptr) {
#ifndef RT_TIMING_NO_HALTON
    if constexpr (TAB && SMALL && kTabDigits[D] > 0)
        if (tab != nullptr) return halton_tab<D>(i, tab);
#endif
    if (SMALL) return halton_small<D>(i);
    return halton<D>(i);
}

}  // namespace
}  // namespace rt

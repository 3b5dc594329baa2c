// rt_halton.hpp — the Halton radical inverse of the path-tracing kernels
// (RTrace/sampling.metal:97-122), compile-time dimension forms shared by
// rt_kernel.hip and rt_stream.hip.  Every form is bit-identical to the
// reference loop.
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

template <uint32_t D, bool SMALL>
__device__ __forceinline__ float halton_dim(uint32_t i) {
    if (SMALL) return halton_small<D>(i);
    return halton<D>(i);
}

}  // namespace
}  // namespace rt

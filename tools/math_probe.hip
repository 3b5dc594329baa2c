// Exhaustive check of short correctly-rounded fp32 sqrt / reciprocal
// sequences against the compiler's IEEE sqrtf and 1.0f / x on gfx950
// (both sides of the parity contract use correctly rounded
// sqrt and division).  Every float of the tested ranges is run once.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/math_probe.hip -o tools/math_probe
//   tools/math_probe > math_probe.json
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>

// S2: the hardware sqrt, then the +-1 ulp correction of the compiler's IEEE
// expansion, without its input scaling and class checks (valid where x is a
// positive normal float well inside the exponent range)
__device__ __forceinline__ float sqrt_s2(float x) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = fmaf(-sm, s, x), rp = fmaf(-sp, s, x);
    float r = (rm <= 0.0f) ? sm : s;
    r = (rp > 0.0f) ? sp : r;
    return r;
}
// S1: rsq + Goldschmidt / Markstein refinement
__device__ __forceinline__ float sqrt_s1(float x) {
    const float r = __builtin_amdgcn_rsqf(x);
    float s = x * r, h = 0.5f * r;
    const float e = fmaf(-s, h, 0.5f);
    s = fmaf(s, e, s);
    h = fmaf(h, e, h);
    const float d = fmaf(-s, s, x);
    return fmaf(d, h, s);
}
// R1: hardware reciprocal + one Newton-Raphson step in fma form
__device__ __forceinline__ float rcp_r1(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = fmaf(-x, r, 1.0f);
    return fmaf(e, r, r);
}
// R2: two steps
__device__ __forceinline__ float rcp_r2(float x) {
    float r = __builtin_amdgcn_rcpf(x);
    float e = fmaf(-x, r, 1.0f);
    r = fmaf(e, r, r);
    e = fmaf(-x, r, 1.0f);
    return fmaf(e, r, r);
}

// counts[k] = mismatches of candidate k; first[k] = the first mismatching input bits
__global__ void probe(uint32_t lo, uint32_t n, unsigned long long* counts, uint32_t* first) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t b = lo + i;
        const float x = __uint_as_float(b);
        volatile float vx = x;  // keep the IEEE references from folding into the candidates
        const float ref_s = sqrtf(vx);
        const float ref_r = 1.0f / vx;
        const uint32_t got[4] = {__float_as_uint(sqrt_s1(x)), __float_as_uint(sqrt_s2(x)),
                                 __float_as_uint(rcp_r1(x)), __float_as_uint(rcp_r2(x))};
        const uint32_t want[4] = {__float_as_uint(ref_s), __float_as_uint(ref_s), __float_as_uint(ref_r),
                                  __float_as_uint(ref_r)};
        for (int k = 0; k < 4; ++k)
            if (got[k] != want[k]) {
                atomicAdd(&counts[k], 1ull);
                atomicMin(&first[k], b);
            }
    }
}

int main() {
    // ranges (bit patterns, positive floats): [2^-100, 2^100) and all positive
    // normals [2^-126, 2^128); the reciprocal also for the negative range
    struct R {
        const char* name;
        uint32_t lo, hi;
    } ranges[] = {{"pos_2^-100_2^100", 0x0D800000u, 0x71800000u},
                  {"pos_normal", 0x00800000u, 0x7F800000u},
                  {"neg_2^-100_2^100", 0x8D800000u, 0xF1800000u}};
    unsigned long long* dc;
    uint32_t* df;
    (void)hipMalloc(&dc, 4 * sizeof(unsigned long long));
    (void)hipMalloc(&df, 4 * sizeof(uint32_t));
    printf("{");
    for (int q = 0; q < 3; ++q) {
        const unsigned long long zero[4] = {0, 0, 0, 0};
        const uint32_t ff[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        (void)hipMemcpy(dc, zero, sizeof(zero), hipMemcpyHostToDevice);
        (void)hipMemcpy(df, ff, sizeof(ff), hipMemcpyHostToDevice);
        const uint32_t n = ranges[q].hi - ranges[q].lo;
        hipLaunchKernelGGL(probe, dim3(8192), dim3(256), 0, 0, ranges[q].lo, n, dc, df);
        if (hipDeviceSynchronize() != hipSuccess) return 1;
        unsigned long long c[4];
        uint32_t f[4];
        (void)hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
        (void)hipMemcpy(f, df, sizeof(f), hipMemcpyDeviceToHost);
        printf("%s\"%s\": {\"floats\": %u, \"sqrt_rsq_markstein\": [%llu, \"0x%08x\"], \"sqrt_hw_fixup\": [%llu, \"0x%08x\"], "
               "\"rcp_1nr\": [%llu, \"0x%08x\"], \"rcp_2nr\": [%llu, \"0x%08x\"]}",
               q ? ", " : "", ranges[q].name, n, c[0], f[0], c[1], f[1], c[2], f[2], c[3], f[3]);
    }
    printf("}\n");
    return 0;
}

// Vector-memory pipeline probe (tools/td_probe.sh): what one per-lane load
// instruction costs the TA/TD of a CU as a function of the active lanes, the
// lanes that share a cache line and the bytes per lane -- the question behind
// the BVH walks' TD-bound profile.  Every lane runs a
// dependent chain of loads from a buffer of random words (each address
// depends on the previous load), like a walk's entry loads.
//   td_probe <mode> <active_lanes> <lanes_per_line> <buffer_MB> [iters]
// mode: 4 = global_load_dwordx4, 1 = global_load_dword.  lanes_per_line
// lanes (consecutive) read consecutive 16-B (4-B) chunks of one 128-B line.
// Prints one JSON line: ms, loads per wave, ns per dependent load.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ uint32_t mix(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352dU;
    x ^= x >> 15;
    x *= 0x846ca68bU;
    x ^= x >> 16;
    return x;
}

template <int MODE>
__global__ __launch_bounds__(256, 8) void probe(const uint32_t* __restrict__ buf, uint32_t line_mask,
                                                uint32_t active, uint32_t lpl, uint32_t iters,
                                                uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t group = lane / lpl, sub = lane % lpl;
    uint32_t line = mix(wave * 64u + group) & line_mask;  // 128-B line index, same for a group
    uint32_t acc = 0;
    if (lane < active) {
        for (uint32_t k = 0; k < iters; ++k) {
            uint32_t v;
            if (MODE == 4) {
                const uint4 q = reinterpret_cast<const uint4*>(buf)[(size_t)line * 8u + (sub & 7u)];
                v = q.x ^ q.y ^ q.z ^ q.w;
            } else {
                v = buf[(size_t)line * 32u + (sub & 31u)];
            }
            acc += v;
            // the next line depends on this load (never 0xFFFFFFFF in the buffer)
            line = (mix(line + k) + (v == 0xFFFFFFFFu ? 1u : 0u)) & line_mask;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;  // keep the chain
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: td_probe <4|1> <active_lanes> <lanes_per_line> <buffer_MB> [iters]\n");
        return 2;
    }
    const int mode = atoi(argv[1]);
    const uint32_t active = (uint32_t)atoi(argv[2]), lpl = (uint32_t)atoi(argv[3]);
    const uint32_t mb = (uint32_t)atoi(argv[4]);
    const uint32_t iters = argc > 5 ? (uint32_t)atoi(argv[5]) : 2000u;
    if ((mode != 1 && mode != 4) || active < 1 || active > 64 || lpl < 1 || lpl > 64 || mb < 1 || mb > 1024 ||
        (mb & (mb - 1)) != 0) {
        fprintf(stderr, "bad arguments\n");
        return 2;
    }
    const size_t bytes = (size_t)mb << 20;
    const uint32_t lines = (uint32_t)(bytes / 128u);
    std::vector<uint32_t> h(bytes / 4);
    uint32_t s = 12345u;
    for (auto& w : h) {
        s = s * 1664525u + 1013904223u;
        w = s == 0xFFFFFFFFu ? 0u : s;
    }
    uint32_t *d = nullptr, *o = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
    if (hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) return 1;
    const dim3 grid(2048), block(256);  // 8,192 waves: 8 per SIMD on 256 CUs
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
        (void)hipEventRecord(e0, 0);
        if (mode == 4)
            hipLaunchKernelGGL(probe<4>, grid, block, 0, 0, d, lines - 1u, active, lpl, iters, o);
        else
            hipLaunchKernelGGL(probe<1>, grid, block, 0, 0, d, lines - 1u, active, lpl, iters, o);
        (void)hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) return 1;
        float ms = 0.0f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep > 0 && ms < best) best = ms;
    }
    const double waves = 2048.0 * 4.0;
    printf("{\"mode\": %d, \"active\": %u, \"lanes_per_line\": %u, \"buffer_mb\": %u, \"iters\": %u, "
           "\"ms\": %.4f, \"wave_loads\": %.0f, \"ns_per_dependent_load\": %.2f, "
           "\"G_lane_loads_per_s\": %.2f}\n",
           mode, active, lpl, mb, iters, best, waves * iters, best * 1e6 / iters,
           waves * iters * active / (best * 1e-3) / 1e9);
    (void)hipFree(d);
    (void)hipFree(o);
    return 0;
}

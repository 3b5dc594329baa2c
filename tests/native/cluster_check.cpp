// CPU check of the container shrink of the box clusters (rt_scene.cpp
// build_clusters), linked against librtpt.so (the scene
// compiler) and oracle/liboracle.so (the reference triangle test): for the
// Cornell room of both Cornell scenes, random segments [o, o + d*tmax] whose
// ends pass the kernel's container test (rt_trace.hpp cluster_candidates<SEG>:
// both ends strictly inside the stored shrunk box on every axis, e computed in
// the kernel's float order) must have no accepted hit (t in (0.001, tmax)) on
// any triangle of the container -- half of them with an end pulled to within a
// few ulps of a shrunk plane, where the rounding matters.
//   cluster_check <mis 0|1> <seed> [widen]   (exit 0 and "ok" on success; a
//   positive `widen` grows the stored box by that much, a negative control that
//   must fail)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "rt_scene.hpp"
#include "../../oracle/pt_oracle.h"

#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            printf("FAIL: " __VA_ARGS__);               \
            printf("\n");                               \
            return 1;                                   \
        }                                               \
    } while (0)

int main(int argc, char** argv) {
    const bool mis = argc > 1 && atoi(argv[1]) != 0;
    const unsigned seed = argc > 2 ? (unsigned)atoi(argv[2]) : 1u;
    const float widen = argc > 3 ? (float)atof(argv[3]) : 0.0f;
    CameraGPU cam;
    MaterialGPU mats[64];
    rt_float3 verts[192];
    SquareLightGPU light;
    uint32_t nt = 0;
    CHECK((mis ? pto_cornell_box_mis : pto_cornell_box)(64, 48, &cam, mats, verts, &light, &nt) == 0,
          "scene");
    rt::CompiledScene cs;
    const char* err = nullptr;
    CHECK(rt::compile_scene(cam, mats, verts, nt, light, nullptr, 0, &cs, &err), "compile: %s", err);
    const size_t rec = 28;
    const size_t nc = cs.clusters.size() / rec;
    int containers = 0;
    std::mt19937 g(seed);
    std::uniform_real_distribution<float> U(0.0f, 1.0f);
    for (size_t c = 0; c < nc; ++c) {
        const float* r = cs.clusters.data() + c * rec;
        uint32_t flags;
        memcpy(&flags, &r[15], 4);
        if (!(flags & 8u)) continue;
        ++containers;
        float lo[3], hi[3];
        for (int a = 0; a < 3; ++a) {
            lo[a] = r[4 * a] - widen;
            hi[a] = r[4 * a + 1] + widen;
            CHECK(lo[a] < hi[a], "cluster %zu axis %d: empty shrunk box", c, a);
        }
        uint32_t all;
        memcpy(&all, &r[22], 4);
        std::vector<int> tris;
        for (int k = 0; k < 32; ++k)
            if ((all >> k) & 1u) {
                tris.push_back(2 * k);
                tris.push_back(2 * k + 1);
            }
        CHECK(!tris.empty(), "container without faces");
        long tested = 0;
        for (int it = 0; it < 200000; ++it) {
            float o[3], e[3], d[3];
            for (int a = 0; a < 3; ++a) {
                o[a] = lo[a] + (hi[a] - lo[a]) * U(g);
                e[a] = lo[a] + (hi[a] - lo[a]) * U(g);
            }
            if (it & 1) {  // pull one end onto a shrunk plane, a few ulps either side
                float* p = (it & 2) ? o : e;
                const int a = (int)(g() % 3u);
                float v = (g() & 1u) ? lo[a] : hi[a];
                const int steps = (int)(g() % 9u) - 4;
                for (int s = 0; s < abs(steps); ++s) v = nextafterf(v, steps > 0 ? INFINITY : -INFINITY);
                p[a] = v;
            }
            float len2 = 0.0f;
            for (int a = 0; a < 3; ++a) {
                d[a] = e[a] - o[a];
                len2 += d[a] * d[a];
            }
            if (!(len2 > 1e-12f)) continue;
            const float inv = 1.0f / sqrtf(len2);
            for (int a = 0; a < 3; ++a) d[a] *= inv;
            const float tmax = sqrtf(len2) * (0.5f + U(g));  // shorter or longer than o -> e
            // the kernel's e = o + d * tmax (no contraction) and its test
            bool inside = true;
            for (int a = 0; a < 3; ++a) {
                const volatile float dt = d[a] * tmax;
                const float ek = o[a] + dt;
                inside = inside && o[a] > lo[a] && o[a] < hi[a] && ek > lo[a] && ek < hi[a];
            }
            if (!inside) continue;
            ++tested;
            for (int t : tris) {
                float vv[3][3];
                for (int j = 0; j < 3; ++j) {
                    vv[j][0] = verts[3 * t + j].x;
                    vv[j][1] = verts[3 * t + j].y;
                    vv[j][2] = verts[3 * t + j].z;
                }
                float th;
                CHECK(!pto_ray_triangle(o, d, vv[0], vv[1], vv[2], 0.001f, tmax, &th),
                      "segment inside the shrunk box hits triangle %d at t=%g (tmax %g)", t, th, tmax);
            }
        }
        CHECK(tested > 1000, "too few segments passed the container test (%ld)", tested);
    }
    CHECK(containers == 1, "expected one container (the room), got %d", containers);
    printf("ok\n");
    return 0;
}

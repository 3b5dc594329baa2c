// CPU check of the host triangle-BVH build (rt_scene.cpp build_tri_sah), linked
// against librtpt.so: layout structure, conservative fp16 boxes, and a
// stackless closest-hit walk of every octant layout equal to brute force.
//   tri_bvh_check <n> <seed> <dup> [leaf_max] [trav_cost]   (exit 0 and "ok" on success)
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "rt_scene.hpp"

using rt::TriIsect;

static float half_to_float(uint16_t h) {
    const uint32_t s = (h >> 15) & 1u, e = (h >> 10) & 31u, m = h & 1023u;
    float v;
    if (e == 0) v = ldexpf((float)m, -24);
    else if (e == 31) v = m ? NAN : INFINITY;
    else v = ldexpf((float)(m | 1024u), (int)e - 25);
    return s ? -v : v;
}

struct Box { double lo[3], hi[3]; };

// near/far entries: in the layout of octant `oct` the lo slot of axis a holds
// the plane a ray of that octant enters through (hi when bit a is set)
static Box entry_box(const uint32_t* w, uint32_t oct) {
    const uint16_t h[6] = {(uint16_t)(w[0] & 0xFFFF), (uint16_t)(w[0] >> 16), (uint16_t)(w[1] & 0xFFFF),
                           (uint16_t)(w[1] >> 16), (uint16_t)(w[2] & 0xFFFF), (uint16_t)(w[2] >> 16)};
    Box b;
    for (int a = 0; a < 3; ++a) {
        const bool neg = (oct >> a) & 1u;
        b.lo[a] = half_to_float(h[neg ? 3 + a : a]);
        b.hi[a] = half_to_float(h[neg ? a : 3 + a]);
    }
    return b;
}

static void tri_verts(const TriIsect& t, double v[3][3]) {
    for (int a = 0; a < 3; ++a) {
        v[0][a] = t.q[a];
        v[1][a] = (double)(t.q[a] + t.q[3 + a]);  // v0 + e1 as the build's fp32 add
        v[2][a] = (double)(t.q[a] + t.q[6 + a]);
    }
}

// double-precision ray/triangle (Moeller-Trumbore); the walk and the brute
// force use the same test, so only the walk's coverage is checked here
static bool hit(const TriIsect& T, const double o[3], const double d[3], double tmax, double* t) {
    double v[3][3];
    tri_verts(T, v);
    double e1[3], e2[3], p[3], s[3], q[3];
    for (int a = 0; a < 3; ++a) { e1[a] = v[1][a] - v[0][a]; e2[a] = v[2][a] - v[0][a]; s[a] = o[a] - v[0][a]; }
    p[0] = d[1] * e2[2] - d[2] * e2[1]; p[1] = d[2] * e2[0] - d[0] * e2[2]; p[2] = d[0] * e2[1] - d[1] * e2[0];
    const double det = e1[0] * p[0] + e1[1] * p[1] + e1[2] * p[2];
    if (fabs(det) < 1e-300) return false;
    const double u = (s[0] * p[0] + s[1] * p[1] + s[2] * p[2]) / det;
    if (u < 0 || u > 1) return false;
    q[0] = s[1] * e1[2] - s[2] * e1[1]; q[1] = s[2] * e1[0] - s[0] * e1[2]; q[2] = s[0] * e1[1] - s[1] * e1[0];
    const double vv = (d[0] * q[0] + d[1] * q[1] + d[2] * q[2]) / det;
    if (vv < 0 || u + vv > 1) return false;
    const double tt = (e2[0] * q[0] + e2[1] * q[1] + e2[2] * q[2]) / det;
    if (!(tt > 1e-3 && tt < tmax)) return false;
    *t = tt;
    return true;
}

static bool box_hit(const Box& b, const double o[3], const double d[3], double tmax) {
    double t0 = 1e-3, t1 = tmax;
    for (int a = 0; a < 3; ++a) {
        if (d[a] == 0.0) {
            if (o[a] < b.lo[a] || o[a] > b.hi[a]) return false;
            continue;
        }
        double ta = (b.lo[a] - o[a]) / d[a], tb = (b.hi[a] - o[a]) / d[a];
        if (ta > tb) { const double x = ta; ta = tb; tb = x; }
        t0 = ta > t0 ? ta : t0;
        t1 = tb < t1 ? tb : t1;
    }
    return t0 <= t1 * (1 + 1e-12) + 1e-12;
}

#define CHECK(c, ...) do { if (!(c)) { printf(__VA_ARGS__); printf("\n"); return 1; } } while (0)

int main(int argc, char** argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 2000;
    const unsigned seed = argc > 2 ? (unsigned)atoi(argv[2]) : 1u;
    const bool dup = argc > 3 && atoi(argv[3]) != 0;
    const uint32_t leaf_max = argc > 4 ? (uint32_t)atoi(argv[4]) : rt::kTriLeafMax;
    const double trav_cost = argc > 5 ? atof(argv[5]) : 1.0;
    std::mt19937 g(seed);
    std::uniform_real_distribution<float> U(-2.3f, 2.3f), E(-0.25f, 0.25f);
    std::vector<TriIsect> tri(n);
    for (int k = 0; k < n; ++k) {
        TriIsect& r = tri[k];
        if (dup && (k & 1)) { r = tri[k - 1]; continue; }  // exact duplicates: ties at equal t
        for (int a = 0; a < 3; ++a) { r.q[a] = U(g); r.q[3 + a] = E(g); r.q[6 + a] = E(g); }
        r.q[9] = r.q[4] * r.q[8] - r.q[5] * r.q[7];
        r.q[10] = r.q[5] * r.q[6] - r.q[3] * r.q[8];
        r.q[11] = r.q[3] * r.q[7] - r.q[4] * r.q[6];
    }
    const float margin = 1e-4f;
    std::vector<uint32_t> nodes, perm;
    std::vector<TriIsect> sorted;
    CHECK(rt::build_tri_sah(tri, margin, &nodes, &sorted, &perm, leaf_max, trav_cost), "build failed");
    CHECK(nodes.size() % 32 == 0, "node array size %zu", nodes.size());
    const uint32_t total = (uint32_t)(nodes.size() / 32);
    // perm is a permutation, sorted follows it
    std::vector<int> seen(n, 0);
    for (int k = 0; k < n; ++k) {
        CHECK(perm[k] < (uint32_t)n && !seen[perm[k]]++, "perm not a permutation at %d", k);
        CHECK(!memcmp(&sorted[k], &tri[perm[k]], sizeof(TriIsect)), "sorted[%d] != tri[perm]", k);
    }
    for (uint32_t oct = 0; oct < 8; ++oct) {
        const uint32_t* L = nodes.data() + (size_t)oct * total * 4;
        std::vector<int> cover(n, 0);
        for (uint32_t i = 0; i < total; ++i) {
            const uint32_t* w = L + 4 * (size_t)i;
            const Box b = entry_box(w, oct);
            for (int a = 0; a < 3; ++a) CHECK(b.lo[a] <= b.hi[a], "oct %u entry %u: near/far order", oct, i);
            if (w[3] & 0x80000000u) {
                const uint32_t esc = (w[3] & 0x7FFFFFFFu) - oct * total;
                CHECK(esc > i + 1 && esc <= total, "oct %u entry %u: escape %u", oct, i, esc);
                // the box holds every entry of its subtree [i+1, esc)
                for (uint32_t j = i + 1; j < esc; ++j) {
                    const Box c = entry_box(L + 4 * (size_t)j, oct);
                    for (int a = 0; a < 3; ++a)
                        CHECK(b.lo[a] <= c.lo[a] && c.hi[a] <= b.hi[a], "oct %u: entry %u box not inside %u", oct, j, i);
                }
            } else {
                const uint32_t first = w[3] & 0xFFFFFFu, cnt = (w[3] >> 24) + 1u;
                CHECK(first + cnt <= (uint32_t)n, "oct %u entry %u: leaf range", oct, i);
                for (uint32_t k = first; k < first + cnt; ++k) {
                    ++cover[k];
                    double v[3][3];
                    tri_verts(sorted[k], v);
                    for (int p = 0; p < 3; ++p)
                        for (int a = 0; a < 3; ++a)
                            CHECK(b.lo[a] <= v[p][a] - margin * 0.99 && v[p][a] + margin * 0.99 <= b.hi[a],
                                  "oct %u leaf %u: triangle %u outside its padded box", oct, i, k);
                }
            }
        }
        for (int k = 0; k < n; ++k) CHECK(cover[k] == 1, "oct %u: triangle %d in %d leaves", oct, k, cover[k]);
    }
    // stackless closest-hit walks == brute force on random rays
    std::uniform_real_distribution<double> R(-1.0, 1.0);
    int hits = 0;
    for (int r = 0; r < 4000; ++r) {
        double o[3] = {2.4 * R(g), 2.4 * R(g), 2.4 * R(g)}, d[3] = {R(g), R(g), R(g)};
        if (r % 7 == 0) d[r % 3] = 0.0;  // axis-parallel components
        double bt = 1000.0;
        int bid = -1;
        for (int k = 0; k < n; ++k) {
            double t;
            if (hit(tri[k], o, d, 1000.0, &t) && (t < bt || (t == bt && k < bid))) { bt = t; bid = k; }
        }
        const uint32_t oct = (d[0] < 0 || (d[0] == 0 && signbit(d[0]))) | ((d[1] < 0) << 1) | ((d[2] < 0) << 2);
        const uint32_t* L = nodes.data() + (size_t)oct * total * 4;
        double wt = 1000.0;
        int wid = -1;
        for (uint32_t i = 0; i < total;) {
            const uint32_t* w = L + 4 * (size_t)i;
            const bool inner = (w[3] & 0x80000000u) != 0;
            if (!box_hit(entry_box(w, oct), o, d, wt)) {
                i = inner ? (w[3] & 0x7FFFFFFFu) - oct * total : i + 1;
                continue;
            }
            if (!inner) {
                const uint32_t first = w[3] & 0xFFFFFFu, cnt = (w[3] >> 24) + 1u;
                for (uint32_t k = first; k < first + cnt; ++k) {
                    double t;
                    const int id = (int)perm[k];
                    if (hit(sorted[k], o, d, 1000.0, &t) && t <= wt && (t < wt || id < wid || wid < 0)) { wt = t; wid = id; }
                }
            }
            ++i;
        }
        CHECK(wid == bid && (bid < 0 || wt == bt), "ray %d: walk (%d, %.9g) != brute force (%d, %.9g)", r, wid, wt, bid, bt);
        hits += bid >= 0;
    }
    CHECK(hits > 400, "too few hits (%d) to mean anything", hits);
    printf("ok %u nodes/layout, %d of 4000 rays hit\n", total, hits);
    return 0;
}

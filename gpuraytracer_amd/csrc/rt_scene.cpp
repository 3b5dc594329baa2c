// rt_scene.cpp — host scene model, builders and record precompute.
// Compiled with -ffp-contract=off (see rt_math.h).
#include "rt_scene.hpp"

#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <system_error>
#include <thread>

#include "../../include/rtpt.h"
#include "rt_kernel.hpp"

namespace rt {

namespace {

// Swift's Float.pi is rounded toward zero (0x40490FDA), unlike M_PI_F.
constexpr float kSwiftPi = 3.14159250f;

f3 from_abi(const rt_float3& v) { return f3{v.x, v.y, v.z}; }

Material make_material(float r, float g, float b, float metallic, float roughness,
                       f3 emissive = f3{0.0f, 0.0f, 0.0f}) {
    Material m;
    m.diffuse[0] = r; m.diffuse[1] = g; m.diffuse[2] = b; m.diffuse[3] = 1.0f;
    m.metallic = metallic;
    m.roughness = roughness;
    m.emissive[0] = emissive.x; m.emissive[1] = emissive.y; m.emissive[2] = emissive.z;
    return m;
}

// createRotatedBoxVertices (scene.swift:177-210): simd_float4x4 with columns
// (c,0,s,0),(0,1,0,0),(-s,0,c,0),(0,0,0,1) applied to (x,y,z,1), then + center.
void rotated_box(f3 center, float width, float height, float depth, float rot_y, f3 out[8]) {
    const float hw = width / 2, hh = height / 2, hd = depth / 2;
    const f3 base[8] = {{-hw, -hh, -hd}, {hw, -hh, -hd}, {hw, hh, -hd}, {-hw, hh, -hd},
                        {-hw, -hh, hd},  {hw, -hh, hd},  {hw, hh, hd},  {-hw, hh, hd}};
    // Evaluate cos/sin at run time through the C library (like the oracle), so
    // no compiler constant-folds them with a differently rounded routine.
    volatile float angle = rot_y;
    const float c = cosf(angle), s = sinf(angle);
    for (int k = 0; k < 8; ++k) {
        const f3 b = base[k];
        const float rx = c * b.x + (-s) * b.z;
        const float rz = s * b.x + c * b.z;
        out[k] = f3{rx + center.x, b.y + center.y, rz + center.z};
    }
}

// createBoxTriangles (scene.swift:212-240)
void box_triangles(const f3 v[8], const Material& m, std::vector<Triangle>* tris) {
    static const int faces[12][3] = {{0, 2, 1}, {0, 3, 2}, {4, 5, 6}, {4, 6, 7},
                                     {0, 4, 7}, {0, 7, 3}, {1, 6, 5}, {1, 2, 6},
                                     {0, 5, 4}, {0, 1, 5}, {3, 6, 2}, {3, 7, 6}};
    for (const auto& f : faces) tris->push_back(Triangle{{v[f[0]], v[f[1]], v[f[2]]}, m});
}

// PCG32 (O'Neill) — generator of the config-4 sphere field.
struct Pcg32 {
    uint64_t state = 0, inc = 0;
    Pcg32(uint64_t initstate, uint64_t initseq) {
        inc = (initseq << 1u) | 1u;
        next();
        state += initstate;
        next();
    }
    uint32_t next() {
        const uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        const uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        const uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((-rot) & 31u));
    }
    float uniform(float lo, float hi) {
        return lo + (hi - lo) * ((float)(next() >> 8) * 5.9604645e-08f);
    }
};

}  // namespace

rt_float3 to_abi(f3 v) {
    rt_float3 r;
    memset(&r, 0, sizeof(r));
    r.x = v.x; r.y = v.y; r.z = v.z;
    return r;
}

f3 SquareLight::emitted_luminance() const {  // scene.swift:257-270
    const float flux = luminous_efficacy * watts;
    const float area = width * depth;
    const float exitance = flux / area;
    const float lum = exitance / kSwiftPi;
    return f3{material.diffuse[0], material.diffuse[1], material.diffuse[2]} * lum;
}

std::vector<Triangle> create_cornell_box_scene() {
    std::vector<Triangle> t;
    const float half = 5.0f / 2.0f;
    const Material red = make_material(0.9f, 0.0f, 0.0f, 0.05f, 0.3f);
    const Material green = make_material(0.0f, 0.7f, 0.0f, 0.05f, 0.8f);
    const Material white = make_material(0.9f, 0.9f, 0.9f, 0.05f, 0.8f);
    const Material box = make_material(0.9f, 0.9f, 0.9f, 0.05f, 0.3f);
    const float h = half;
    // back (:81-90), left/red (:93-102), right/green (:105-114),
    // floor (:117-126), ceiling (:129-138)
    t.push_back({{{-h, -h, -h}, {h, h, -h}, {-h, h, -h}}, white});
    t.push_back({{{-h, -h, -h}, {h, -h, -h}, {h, h, -h}}, white});
    t.push_back({{{-h, -h, -h}, {-h, h, h}, {-h, -h, h}}, red});
    t.push_back({{{-h, -h, -h}, {-h, h, -h}, {-h, h, h}}, red});
    t.push_back({{{h, -h, -h}, {h, h, h}, {h, h, -h}}, green});
    t.push_back({{{h, -h, -h}, {h, -h, h}, {h, h, h}}, green});
    t.push_back({{{-h, -h, -h}, {h, -h, h}, {h, -h, -h}}, white});
    t.push_back({{{-h, -h, -h}, {-h, -h, h}, {h, -h, h}}, white});
    t.push_back({{{-h, h, -h}, {h, h, h}, {-h, h, h}}, white});
    t.push_back({{{-h, h, -h}, {h, h, -h}, {h, h, h}}, white});
    f3 v[8];
    const float tall_h = 2.8f;  // :141-155
    rotated_box(f3{-1.0f, -half + tall_h / 2 - 0.05f, -1.5f}, 1.2f, tall_h, 1.2f,
                kSwiftPi / 2.4f, v);
    box_triangles(v, box, &t);
    const float short_h = 1.2f;  // :158-172
    rotated_box(f3{0.7f, -half + short_h / 2 - 0.05f, 1.2f}, 1.2f, short_h, 1.2f,
                -kSwiftPi / 2.5f, v);
    box_triangles(v, box, &t);
    return t;
}

static Scene cornell_box(int32_t width, int32_t height, float light_size) {
    Scene s;
    s.camera.position = f3{0, 0, 9};
    s.camera.direction = normalize(f3{0, 0, -2.5f} - f3{0, 0, 9});
    s.camera.up = f3{0, 1, 0};
    s.camera.resolution[0] = width;
    s.camera.resolution[1] = height;
    s.camera.horizontal_fov = kSwiftPi / 4.0f;
    s.camera.ev100 = 5.0f;

    const float half = 5.0f / 2.0f;
    const float light_w = light_size, light_d = light_size;
    const float light_y = half - 0.01f;
    const f3 lc{0, light_y, 0};
    const float hw = light_w / 2, hd = light_d / 2;
    const f3 v0{lc.x - hw, light_y, lc.z - hd}, v1{lc.x + hw, light_y, lc.z - hd};
    const f3 v2{lc.x + hw, light_y, lc.z + hd}, v3{lc.x - hw, light_y, lc.z + hd};
    const Material light_m = make_material(1.0f, 0.95f, 0.9f, 0.0f, 0.0f, f3{1.0f, 1.0f, 1.0f});
    s.light.center = lc;
    s.light.vertices[0] = v0; s.light.vertices[1] = v1;
    s.light.vertices[2] = v2; s.light.vertices[3] = v3;
    s.light.material = light_m;
    s.light.luminous_efficacy = 100.0f;
    s.light.watts = 12.0f;
    s.light.width = light_w;
    s.light.depth = light_d;

    s.triangles = create_cornell_box_scene();
    s.triangles.push_back(Triangle{{v0, v1, v2}, light_m});  // :58-59
    s.triangles.push_back(Triangle{{v0, v2, v3}, light_m});
    return s;
}

Scene init_cornell_box(int32_t width, int32_t height) { return cornell_box(width, height, 1.0f); }

Scene init_cornell_box_mis(int32_t width, int32_t height) { return cornell_box(width, height, 1.5f); }

Scene init_random_spheres(int32_t width, int32_t height, uint32_t n, uint64_t seed) {
    Scene s = init_cornell_box(width, height);
    std::vector<Triangle> kept;
    for (size_t k = 0; k < s.triangles.size(); ++k)
        if (k < 10 || k >= 34) kept.push_back(s.triangles[k]);  // walls + light
    s.triangles = kept;
    Pcg32 rng(seed, 54u);
    for (uint32_t i = 0; i < n; ++i) {
        Sphere sp;
        const float cx = rng.uniform(-2.3f, 2.3f);
        const float cy = rng.uniform(-2.3f, 2.2f);
        const float cz = rng.uniform(-2.3f, 2.3f);
        const float r = rng.uniform(0.05f, 0.20f);
        const float ar = rng.uniform(0.1f, 0.9f);
        const float ag = rng.uniform(0.1f, 0.9f);
        const float ab = rng.uniform(0.1f, 0.9f);
        sp.center = f3{cx, cy, cz};
        sp.radius = r;
        sp.material = make_material(ar, ag, ab, 0.0f, 1.0f);
        s.spheres.push_back(sp);
    }
    return s;
}

MaterialGPU convert_material(const Material& m) {
    MaterialGPU g;
    memset(&g, 0, sizeof(g));
    g.diffuse.x = m.diffuse[0]; g.diffuse.y = m.diffuse[1];
    g.diffuse.z = m.diffuse[2]; g.diffuse.w = m.diffuse[3];
    g.metallic = m.metallic;
    g.roughness = m.roughness;
    g.emissive = to_abi(f3{m.emissive[0], m.emissive[1], m.emissive[2]});
    return g;
}

SquareLightGPU convert_square_light(const SquareLight& l) {
    SquareLightGPU g;
    memset(&g, 0, sizeof(g));
    g.center = to_abi(l.center);
    g.color.x = l.material.diffuse[0]; g.color.y = l.material.diffuse[1];   // color = diffuse
    g.color.z = l.material.diffuse[2]; g.color.w = l.material.diffuse[3];   // (:36)
    g.emittedRadiance = to_abi(l.emitted_luminance());
    g.width = l.width;
    g.depth = l.depth;
    return g;
}

CameraGPU convert_camera(const Camera& c) {
    CameraGPU g;
    memset(&g, 0, sizeof(g));
    g.position = to_abi(c.position);
    g.direction = to_abi(c.direction);
    g.up = to_abi(c.up);
    g.resolution.x = c.resolution[0];
    g.resolution.y = c.resolution[1];
    g.horizontalFov = c.horizontal_fov;
    g.ev100 = c.ev100;
    return g;
}

SphereGPU convert_sphere(const Sphere& s) {
    SphereGPU g;
    memset(&g, 0, sizeof(g));
    g.center = to_abi(s.center);
    g.material = convert_material(s.material);
    g.radius = s.radius;
    return g;
}

uint32_t seed_splitmix(uint64_t key, uint64_t p) {
    uint64_t z = key + p + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z = z ^ (z >> 31);
    return (uint32_t)(z & 0xFFFFFu);
}

static bool same_bits(const float* a, const float* b, int n) {
    return memcmp(a, b, sizeof(float) * (size_t)n) == 0;
}

// Conservative culling margin: far above the fp32 rounding of the triangle
// test at the scene's scale (~1e-6 relative), far below the 1e-3 surface
// offset of raytrace.metal:67.
static float culling_margin(const rt_float3* verts, uint32_t n_tri, const SphereGPU* sph = nullptr,
                            uint32_t n_sph = 0) {
    float ext = 2.5f;
    for (uint32_t k = 0; k < 3 * n_tri; ++k)
        ext = fmaxf(ext, fmaxf(fabsf(verts[k].x), fmaxf(fabsf(verts[k].y), fabsf(verts[k].z))));
    for (uint32_t k = 0; k < n_sph; ++k)
        ext = fmaxf(ext, fmaxf(fabsf(sph[k].center.x), fmaxf(fabsf(sph[k].center.y),
                                                              fabsf(sph[k].center.z))) +
                             fabsf(sph[k].radius));
    return 4e-5f * ext;
}

// BVH over the spheres (median split of the centroids on the longest axis,
// one sphere per leaf by default), emitted as 8 depth-first layouts, one per ray-direction
// octant: at every inner node the child on the near side of the split for that
// octant comes first, so a closest-hit walk meets near spheres early and culls
// more.  Only speed depends on the tree and the order: the kernel skips a node
// only when no sphere inside can beat the current closest hit, and ties are
// resolved by sphere id, so the result is that of testing every sphere in id
// order.
struct BvhBuild {
    struct Node {
        float lo[3], hi[3];
        int axis;                 // split axis (inner nodes)
        uint32_t left, right;     // children (inner nodes)
        uint32_t first, count;    // sphere range (leaves), count 0 for inner nodes
    };
    const SphereGPU* sph;
    float margin;
    uint32_t leaf_max = 1;  // measured best for config 4 (sphere_leaf_max sweep 1..8)
    bool sah = true;        // SAH splits (false: median of the longest axis)
    std::vector<uint32_t> ids;
    std::vector<Node> tree;

    void grow(uint32_t id, float lo[3], float hi[3]) const {
        const SphereGPU& s = sph[id];
        const float c[3] = {s.center.x, s.center.y, s.center.z};
        const float r = fabsf(s.radius);
        for (int a = 0; a < 3; ++a) {
            lo[a] = fminf(lo[a], c[a] - r);
            hi[a] = fmaxf(hi[a], c[a] + r);
        }
    }
    static double area(const float lo[3], const float hi[3]) {
        const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
        return x * y + y * z + z * x;
    }

    void bounds(uint32_t b, uint32_t e, float lo[3], float hi[3], bool centroids) const {
        for (int a = 0; a < 3; ++a) {
            lo[a] = INFINITY;
            hi[a] = -INFINITY;
        }
        for (uint32_t k = b; k < e; ++k) {
            const SphereGPU& s = sph[ids[k]];
            const float c[3] = {s.center.x, s.center.y, s.center.z};
            const float r = centroids ? 0.0f : fabsf(s.radius);
            for (int a = 0; a < 3; ++a) {
                lo[a] = fminf(lo[a], c[a] - r);
                hi[a] = fmaxf(hi[a], c[a] + r);
            }
        }
    }

    uint32_t build(uint32_t b, uint32_t e) {
        const uint32_t me = (uint32_t)tree.size();
        tree.push_back(Node{});
        float lo[3], hi[3];
        bounds(b, e, lo, hi, false);
        for (int a = 0; a < 3; ++a) {
            tree[me].lo[a] = lo[a] - margin;
            tree[me].hi[a] = hi[a] + margin;
        }
        if (e - b <= leaf_max) {
            tree[me].first = b;
            tree[me].count = e - b;
            return me;
        }
        float clo[3], chi[3];
        bounds(b, e, clo, chi, true);
        int axis = 0;
        for (int a = 1; a < 3; ++a)
            if (chi[a] - clo[a] > chi[axis] - clo[axis]) axis = a;
        uint32_t mid = b + (e - b) / 2;
        auto by_axis = [&](int ax) {
            return [this, ax](uint32_t x, uint32_t y) {
                const float cx[3] = {sph[x].center.x, sph[x].center.y, sph[x].center.z};
                const float cy[3] = {sph[y].center.x, sph[y].center.y, sph[y].center.z};
                return cx[ax] < cy[ax] || (cx[ax] == cy[ax] && x < y);
            };
        };
        if (sah) {
            // exact SAH sweep over the centroid order of every axis:
            // cost(split) = area(left) * n_left + area(right) * n_right
            double best_cost = INFINITY;
            int best_axis = axis;
            uint32_t best_mid = mid;
            const uint32_t n = e - b;
            std::vector<double> right_area(n);
            for (int a = 0; a < 3; ++a) {
                std::sort(ids.begin() + b, ids.begin() + e, by_axis(a));
                float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
                for (uint32_t k = e; k-- > b + 1;) {  // right part = [k, e)
                    grow(ids[k], lo, hi);
                    right_area[k - b] = area(lo, hi);
                }
                for (int q = 0; q < 3; ++q) {
                    lo[q] = INFINITY;
                    hi[q] = -INFINITY;
                }
                for (uint32_t k = b + 1; k < e; ++k) {  // left part = [b, k)
                    grow(ids[k - 1], lo, hi);
                    const double c = area(lo, hi) * (k - b) + right_area[k - b] * (e - k);
                    if (c < best_cost) {
                        best_cost = c;
                        best_axis = a;
                        best_mid = k;
                    }
                }
            }
            axis = best_axis;
            mid = best_mid;
        }
        std::nth_element(ids.begin() + b, ids.begin() + mid, ids.begin() + e, by_axis(axis));
        const uint32_t l = build(b, mid);
        const uint32_t r = build(mid, e);
        tree[me].axis = axis;
        tree[me].left = l;
        tree[me].right = r;
        tree[me].count = 0;
        return me;
    }

    // Depth-first emission for octant `oct` (bit a set: direction component a < 0).
    void emit(uint32_t t, int oct, std::vector<BvhNode>* out) const {
        const Node& n = tree[t];
        const uint32_t me = (uint32_t)out->size();
        out->push_back(BvhNode{});
        for (int a = 0; a < 3; ++a) {
            (*out)[me].lo[a] = n.lo[a];
            (*out)[me].hi[a] = n.hi[a];
        }
        if (n.count) {
            (*out)[me].leaf = (n.count << 24) | n.first;
        } else {
            const bool neg = (oct >> n.axis) & 1;  // moving toward lower coordinates
            emit(neg ? n.right : n.left, oct, out);
            emit(neg ? n.left : n.right, oct, out);
            (*out)[me].leaf = 0;
        }
        (*out)[me].escape = (uint32_t)out->size();
    }
};

// fp16 bits of x rounded toward -inf (dir < 0) or +inf (dir > 0)
static uint16_t half_dir(float x, int dir) {
    const _Float16 h = (_Float16)x;  // round to nearest even
    uint16_t b;
    memcpy(&b, &h, 2);
    const float back = (float)h;
    const bool neg = (b & 0x8000u) != 0, zero = (b & 0x7FFFu) == 0;
    if (dir < 0 && back > x) b = zero ? 0x8001u : (neg ? b + 1 : b - 1);
    if (dir > 0 && back < x) b = zero ? 0x0001u : (neg ? b - 1 : b + 1);
    return b;
}

// The leaf-box layout (CompiledScene::sph_box): one entry per node of every
// octant layout, escapes = node indices over all layouts.
static void build_sphere_box(CompiledScene* out) {
    out->sph_box.clear();
    const uint32_t nn = out->sph_layout_nodes;
    if (nn == 0 || out->sph_isect.size() >= (1u << 24)) return;
    std::vector<uint32_t> ent;
    ent.reserve((size_t)8 * nn * 4);
    for (int oct = 0; oct < 8; ++oct) {
        const BvhNode* L = out->sph_nodes.data() + (size_t)oct * nn;
        const uint32_t lay_base = (uint32_t)oct * nn;
        for (uint32_t i = 0; i < nn; ++i) {
            const BvhNode& n = L[i];
            uint16_t h[6];
            for (int a = 0; a < 3; ++a) {
                if (!isfinite(n.lo[a]) || !isfinite(n.hi[a])) return;
                h[a] = half_dir(n.lo[a], -1);
                h[3 + a] = half_dir(n.hi[a], +1);
                if ((oct >> a) & 1) std::swap(h[a], h[3 + a]);  // near/far, as build_sphere_lds
            }
            uint32_t w;
            if (n.leaf == 0) {
                if (n.escape > nn) return;
                w = (lay_base + n.escape) | 0x80000000u;
            } else {
                const uint32_t first = n.leaf & 0xFFFFFFu, cnt = n.leaf >> 24;
                if (cnt == 0 || cnt > 128 || n.escape != i + 1) return;
                w = first | (cnt - 1u) << 24;
            }
            const uint32_t q[4] = {h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16,
                                   h[4] | (uint32_t)h[5] << 16, w};
            ent.insert(ent.end(), q, q + 4);
        }
    }
    out->sph_box.swap(ent);
}

static void build_sphere_lds(CompiledScene* out) {
    out->sph_lds.clear();
    out->sph_lds_id.clear();
    out->sph_lds_entries = 0;
    const uint32_t nn = out->sph_layout_nodes;
    if (nn == 0 || out->sph_isect.size() > 0xFFFFu) return;
    // A leaf of c spheres becomes c consecutive sphere entries (each one's
    // escape is the next entry): the parent's box already bounds them.  Entry
    // index of every node = prefix sum of the entries of the nodes before it.
    std::vector<uint32_t> pos(nn + 1);
    {
        const BvhNode* L = out->sph_nodes.data();
        uint32_t k = 0;
        for (uint32_t i = 0; i < nn; ++i) {
            pos[i] = k;
            k += L[i].leaf == 0 ? 1u : (L[i].leaf >> 24);
        }
        pos[nn] = k;
    }
    const uint32_t ne = pos[nn];  // the same in every layout (a permutation of the same nodes)
    if (ne > 0x7FFFu) return;
    std::vector<uint32_t> ent;
    std::vector<uint16_t> ids;
    for (int li = 0; li < 8; ++li) {  // one layout per direction octant
        const int oct = li;
        // escapes are entry indices of the concatenated layouts (layout li
        // starts at li * ne), so a walk's position alone names its layout
        const uint32_t lay_base = (uint32_t)li * ne;
        const BvhNode* L = out->sph_nodes.data() + (size_t)oct * nn;
        uint32_t k = 0;  // running entry index of this layout
        std::vector<uint32_t> lpos(nn + 1);
        for (uint32_t i = 0; i < nn; ++i) {
            lpos[i] = k;
            k += L[i].leaf == 0 ? 1u : (L[i].leaf >> 24);
        }
        lpos[nn] = k;
        for (uint32_t i = 0; i < nn; ++i) {
            const BvhNode& n = L[i];
            if (n.leaf == 0) {
                uint16_t h[6];
                for (int a = 0; a < 3; ++a) {
                    if (!isfinite(n.lo[a]) || !isfinite(n.hi[a])) return;
                    h[a] = half_dir(n.lo[a], -1);
                    h[3 + a] = half_dir(n.hi[a], +1);
                    // near/far boxes: in the layout of octant `oct` the box plane a ray
                    // of that octant enters through (hi when component a is negative)
                    // takes the lo slot, so the walk's slab test needs no min/max pairs
                    if ((oct >> a) & 1) std::swap(h[a], h[3 + a]);
                }
                if (n.escape > nn) return;
                const uint32_t w[4] = {h[0] | (uint32_t)h[1] << 16, h[2] | (uint32_t)h[3] << 16,
                                       h[4] | (uint32_t)h[5] << 16, (lay_base + lpos[n.escape]) | 0x80000000u};
                ent.insert(ent.end(), w, w + 4);
                ids.push_back(0);
            } else {
                if (n.escape != i + 1) return;  // a leaf's escape is the next node
                const uint32_t first = n.leaf & 0xFFFFFFu, cnt = n.leaf >> 24;
                for (uint32_t j = first; j < first + cnt; ++j) {
                    uint32_t w[4];
                    memcpy(w, out->sph_isect[j].q, 16);
                    if (w[3] & 0x80000000u) return;  // r*r is never negative
                    ent.insert(ent.end(), w, w + 4);
                    ids.push_back((uint16_t)out->sph_perm[j]);
                }
            }
        }
        if (k != ne) return;
    }
    // set together, only once every check passed: a nonzero count always
    // comes with its entries
    out->sph_lds.swap(ent);
    out->sph_lds_id.swap(ids);
    out->sph_lds_entries = ne;
}

static void build_sphere_bvh(CompiledScene* out, const SphereGPU* spheres, uint32_t n,
                             float margin, const BuildOptions& opt) {
    out->sph_isect.clear();
    out->sph_box.clear();
    out->sph_perm.clear();
    out->sph_nodes.clear();
    out->sph_layout_nodes = 0;
    if (n == 0) return;
    BvhBuild bb;
    bb.sph = spheres;
    bb.margin = margin;
    bb.sah = opt.sphere_sah;
    if (opt.sphere_leaf_max >= 1 && opt.sphere_leaf_max <= 255) bb.leaf_max = opt.sphere_leaf_max;
    bb.ids.resize(n);
    for (uint32_t k = 0; k < n; ++k) bb.ids[k] = k;
    bb.build(0, n);
    const uint32_t nn = (uint32_t)bb.tree.size();
    for (int oct = 0; oct < 8; ++oct) {
        std::vector<BvhNode> layout;
        layout.reserve(nn);
        bb.emit(0, oct, &layout);
        out->sph_nodes.insert(out->sph_nodes.end(), layout.begin(), layout.end());
    }
    out->sph_layout_nodes = nn;
    out->sph_perm = bb.ids;
    out->sph_isect.resize(n);
    for (uint32_t k = 0; k < n; ++k) {
        const SphereGPU& sp = spheres[bb.ids[k]];
        const float r2 = sp.radius * sp.radius;
        const float q[4] = {sp.center.x, sp.center.y, sp.center.z, r2};
        memcpy(out->sph_isect[k].q, q, sizeof(q));
    }
    build_sphere_lds(out);
    build_sphere_box(out);
}

// Triangle BVH built on the host with binned SAH:
// 32 centroid bins per axis, cost area(left) * n_left + area(right) * n_right,
// leaves of up to kTriLeafMax triangles where the SAH prefers them, every box
// padded by the culling margin.  Emitted in
// the compact layout the triangle walks read (rt_trace.hpp tri_cbvh_*): 8
// depth-first layouts, one per ray-direction octant, near child first along
// the node's split axis; 16 B per node: the fp16 box rounded outward, then
// escape | 2^31 (an entry index over all 8 layouts) for an inner node or, for
// a leaf, its first leaf-order triangle | (count - 1) << 24.  Only speed
// depends on the tree.
bool build_tri_sah(const std::vector<TriIsect>& tri, float margin, std::vector<uint32_t>* nodes,
                   std::vector<TriIsect>* sorted, std::vector<uint32_t>* perm, uint32_t leaf_max,
                   double trav_cost) {
    const uint32_t n = (uint32_t)tri.size();
    if (n == 0 || n >= (1u << 24)) return false;
    leaf_max = std::min(128u, std::max(1u, leaf_max));  // speed only
    if (!(trav_cost > 0.0)) trav_cost = 1.0;
    std::vector<float> bl(3 * (size_t)n), bh(3 * (size_t)n), cen(3 * (size_t)n);
    for (uint32_t k = 0; k < n; ++k) {
        const float* q = tri[k].q;  // v0 0..2, e1 3..5, e2 6..8 (as refit_kernel sees the triangle)
        for (int a = 0; a < 3; ++a) {
            const float v0 = q[a], v1 = q[a] + q[3 + a], v2 = q[a] + q[6 + a];
            bl[3 * k + a] = fminf(v0, fminf(v1, v2));
            bh[3 * k + a] = fmaxf(v0, fmaxf(v1, v2));
            cen[3 * k + a] = 0.5f * (bl[3 * k + a] + bh[3 * k + a]);
        }
    }
    struct Node {
        float lo[3], hi[3];
        int axis;
        uint32_t left, right, first, count;
    };
    std::vector<Node> tree;
    tree.reserve(2 * (size_t)n);
    std::vector<uint32_t> ids(n);
    for (uint32_t k = 0; k < n; ++k) ids[k] = k;
    constexpr int kBins = 32;
    auto area = [](const float* lo, const float* hi) {
        const double x = (double)hi[0] - lo[0], y = (double)hi[1] - lo[1], z = (double)hi[2] - lo[2];
        return x * y + y * z + z * x;
    };
    // iterative build (deep trees must not exhaust the host stack)
    struct Job { uint32_t node, b, e; };
    std::vector<Job> jobs;
    tree.push_back(Node{});
    jobs.push_back({0, 0, n});
    while (!jobs.empty()) {
        const Job J = jobs.back();
        jobs.pop_back();
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        float clo[3] = {INFINITY, INFINITY, INFINITY}, chi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (uint32_t k = J.b; k < J.e; ++k) {
            const uint32_t t = ids[k];
            for (int a = 0; a < 3; ++a) {
                lo[a] = fminf(lo[a], bl[3 * t + a]);
                hi[a] = fmaxf(hi[a], bh[3 * t + a]);
                clo[a] = fminf(clo[a], cen[3 * t + a]);
                chi[a] = fmaxf(chi[a], cen[3 * t + a]);
            }
        }
        Node& N = tree[J.node];
        for (int a = 0; a < 3; ++a) {
            N.lo[a] = lo[a] - margin;
            N.hi[a] = hi[a] + margin;
        }
        N.axis = 0;
        if (J.e - J.b == 1) {
            N.first = J.b;
            N.count = 1;
            continue;
        }
        N.count = 0;
        const uint32_t nb = J.e - J.b;
        // binned SAH over the centroid bounds of every axis
        double best = INFINITY;
        int best_axis = -1, best_bin = 0;
        for (int a = 0; a < 3; ++a) {
            const float ext = chi[a] - clo[a];
            if (!(ext > 0.0f)) continue;
            const float scale = (float)kBins / ext;
            float blo[kBins][3], bhi[kBins][3];
            uint32_t cnt[kBins] = {0};
            for (int i = 0; i < kBins; ++i)
                for (int q = 0; q < 3; ++q) {
                    blo[i][q] = INFINITY;
                    bhi[i][q] = -INFINITY;
                }
            for (uint32_t k = J.b; k < J.e; ++k) {
                const uint32_t t = ids[k];
                const int bi = std::min(kBins - 1, (int)((cen[3 * t + a] - clo[a]) * scale));
                ++cnt[bi];
                for (int q = 0; q < 3; ++q) {
                    blo[bi][q] = fminf(blo[bi][q], bl[3 * t + q]);
                    bhi[bi][q] = fmaxf(bhi[bi][q], bh[3 * t + q]);
                }
            }
            double right_area[kBins];
            uint32_t right_cnt[kBins];
            float rlo[3] = {INFINITY, INFINITY, INFINITY}, rhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t rc = 0;
            for (int i = kBins - 1; i >= 1; --i) {  // right part = bins [i, kBins)
                rc += cnt[i];
                for (int q = 0; q < 3; ++q) {
                    rlo[q] = fminf(rlo[q], blo[i][q]);
                    rhi[q] = fmaxf(rhi[q], bhi[i][q]);
                }
                right_area[i] = rc ? area(rlo, rhi) : 0.0;
                right_cnt[i] = rc;
            }
            float llo[3] = {INFINITY, INFINITY, INFINITY}, lhi[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t lc = 0;
            for (int i = 1; i < kBins; ++i) {  // left part = bins [0, i)
                lc += cnt[i - 1];
                for (int q = 0; q < 3; ++q) {
                    llo[q] = fminf(llo[q], blo[i - 1][q]);
                    lhi[q] = fmaxf(lhi[q], bhi[i - 1][q]);
                }
                if (lc == 0 || right_cnt[i] == 0) continue;
                const double c = area(llo, lhi) * lc + right_area[i] * right_cnt[i];
                if (c < best) {
                    best = c;
                    best_axis = a;
                    best_bin = i;
                }
            }
        }
        // a leaf of up to leaf_max triangles when testing them all costs less
        // than the split (SAH, a box step costing trav_cost triangle tests)
        if (nb <= leaf_max) {
            const float* lo0 = N.lo;  // padded box: only ratios matter
            const double split = best_axis >= 0 ? trav_cost + best / area(lo0, N.hi) : INFINITY;
            if ((double)nb <= split) {
                N.first = J.b;
                N.count = nb;
                continue;
            }
        }
        uint32_t mid;
        if (best_axis >= 0) {
            const int a = best_axis;
            const float scale = (float)kBins / (chi[a] - clo[a]);
            const float c0 = clo[a];
            auto it = std::partition(ids.begin() + J.b, ids.begin() + J.e, [&](uint32_t t) {
                return std::min(kBins - 1, (int)((cen[3 * t + a] - c0) * scale)) < best_bin;
            });
            mid = (uint32_t)(it - ids.begin());
            N.axis = a;
        } else {  // every centroid in one point: split by index
            mid = J.b + (J.e - J.b) / 2;
            int a = 0;
            for (int q = 1; q < 3; ++q)
                if (hi[q] - lo[q] > hi[a] - lo[a]) a = q;
            N.axis = a;
        }
        if (mid == J.b || mid == J.e) mid = J.b + (J.e - J.b) / 2;
        const uint32_t l = (uint32_t)tree.size();
        tree.push_back(Node{});
        const uint32_t r = (uint32_t)tree.size();
        tree.push_back(Node{});
        tree[J.node].left = l;
        tree[J.node].right = r;
        jobs.push_back({r, mid, J.e});
        jobs.push_back({l, J.b, mid});
    }
    const uint32_t total = (uint32_t)tree.size();  // 2n - 1
    // subtree entry counts (one entry per node)
    std::vector<uint32_t> size(total, 1u);
    for (uint32_t i = total; i-- > 0;)  // children are created after their parent
        if (!tree[i].count) size[i] = 1u + size[tree[i].left] + size[tree[i].right];
    nodes->assign((size_t)8 * total * 4, 0u);
    auto emit_layout = [&](uint32_t oct) {
        uint32_t* L = nodes->data() + (size_t)oct * total * 4;
        // explicit-stack preorder: (node, entry index)
        std::vector<std::pair<uint32_t, uint32_t>> st;
        st.push_back({0u, 0u});
        while (!st.empty()) {
            const auto [v, idx] = st.back();
            st.pop_back();
            const Node& N = tree[v];
            uint16_t h[6];
            for (int a = 0; a < 3; ++a) {
                h[a] = half_dir(N.lo[a], -1);
                h[3 + a] = half_dir(N.hi[a], +1);
                // near/far boxes as in the sphere layouts: the plane a ray of this
                // octant enters through takes the lo slot (rt_trace.hpp lds_node_hit_nf)
                if ((oct >> a) & 1u) std::swap(h[a], h[3 + a]);
            }
            uint32_t* w = L + 4 * (size_t)idx;
            w[0] = h[0] | (uint32_t)h[1] << 16;
            w[1] = h[2] | (uint32_t)h[3] << 16;
            w[2] = h[4] | (uint32_t)h[5] << 16;
            if (N.count) {
                w[3] = N.first | (N.count - 1u) << 24;  // leaf: first leaf-order triangle, count - 1
            } else {
                w[3] = (oct * total + idx + size[v]) | 0x80000000u;
                const bool neg = (oct >> N.axis) & 1u;  // moving toward lower coordinates
                const uint32_t near = neg ? N.right : N.left, far = neg ? N.left : N.right;
                st.push_back({far, idx + 1 + size[near]});
                st.push_back({near, idx + 1});
            }
        }
    };
    {  // the 8 layouts are independent: one host thread each; a layout whose
        // thread cannot be started (thread limits) is written on this thread
        std::vector<std::thread> th;
        bool started[8] = {true, false, false, false, false, false, false, false};
        for (uint32_t oct = 1; oct < 8; ++oct) {
            try {
                th.emplace_back(emit_layout, oct);
                started[oct] = true;
            } catch (const std::system_error&) {
            }
        }
        emit_layout(0);
        for (uint32_t oct = 1; oct < 8; ++oct)
            if (!started[oct]) emit_layout(oct);
        for (auto& t : th) t.join();
    }
    sorted->resize(n);
    perm->resize(n);
    for (uint32_t k = 0; k < n; ++k) {
        (*sorted)[k] = tri[ids[k]];
        (*perm)[k] = ids[k];
    }
    return true;
}

// Pair layout: triangles (2k, 2k+1) with the same v0 and one common edge
// vector S (bitwise, as computed above).  All-or-nothing, so the kernel keeps
// testing primitives in id order.
static void build_pairs(CompiledScene* out, const rt_float3* verts, float margin) {
    out->pair_isect.clear();
    const size_t n = out->tri_isect.size();
    if (n == 0 || (n & 1)) return;
    std::vector<PairIsect> pairs(n / 2);
    for (size_t k = 0; k < n / 2; ++k) {
        const float* A = out->tri_isect[2 * k].q;      // v0 0..2, e1 3..5, e2 6..8, n 9..11
        const float* B = out->tri_isect[2 * k + 1].q;
        if (!same_bits(A, B, 3)) return;
        const float *S, *eA, *eB;
        uint32_t m;
        if (same_bits(A + 3, B + 6, 3)) {         // A.e1 == B.e2
            S = A + 3; eA = A + 6; eB = B + 3; m = 0u;
        } else if (same_bits(A + 6, B + 3, 3)) {  // A.e2 == B.e1
            S = A + 6; eA = A + 3; eB = B + 6; m = 0x80000000u;
        } else {
            return;
        }
        float mf;
        memcpy(&mf, &m, 4);
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (size_t v = 6 * k; v < 6 * k + 6; ++v) {
            const float c[3] = {verts[v].x, verts[v].y, verts[v].z};
            for (int a = 0; a < 3; ++a) {
                lo[a] = fminf(lo[a], c[a]);
                hi[a] = fmaxf(hi[a], c[a]);
            }
        }
        for (int a = 0; a < 3; ++a) {
            lo[a] -= margin;
            hi[a] += margin;
        }
        const float q[28] = {A[0],  A[1],  A[2],  S[0],  S[1],  S[2],  eA[0], eA[1], eA[2], A[9],
                             A[10], A[11], eB[0], eB[1], eB[2], B[9],  B[10], B[11], mf,    0.0f,
                             lo[0], lo[1], lo[2], hi[0], hi[1], hi[2], 0.0f,  0.0f};
        memcpy(pairs[k].q, q, sizeof(q));
    }
    out->pair_isect.swap(pairs);
}

// ---- box clusters ----------------------------------------
// A run of consecutive pair records (quads) whose quads all lie on the faces of
// one oriented box: the Cornell room (5 walls, open front), each rotated box
// (6 faces), a lone rectangle (the light: a flat box).  The kernel slab-tests a
// ray against the padded box and runs the exact pair test only on the faces
// whose plane the ray can cross inside the box; an accepted hit point lies
// within the culling margin of its quad, hence inside the padded box and within
// the margin of its face plane, so no accepted triangle is skipped.
namespace {
struct D3 {
    double x, y, z;
};
D3 d3(const rt_float3& v) { return D3{v.x, v.y, v.z}; }
D3 sub(D3 a, D3 b) { return D3{a.x - b.x, a.y - b.y, a.z - b.z}; }
double ddot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
D3 dcross(D3 a, D3 b) { return D3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
D3 dscale(D3 a, double s) { return D3{a.x * s, a.y * s, a.z * s}; }
bool dnormalize(D3* a) {
    const double l = sqrt(ddot(*a, *a));
    if (!(l > 0.0) || !isfinite(l)) return false;
    *a = dscale(*a, 1.0 / l);
    return true;
}

struct BoxFit {
    D3 u[3];
    double lo[3], hi[3];
    int slot_pair[6];
};

// Quads [k0, k1) of the pair list: do they lie on the faces of one box?
bool fit_box(const rt_float3* verts, uint32_t k0, uint32_t k1, double tol, BoxFit* f) {
    auto vtx = [&](uint32_t k, int i) { return d3(verts[6 * k + i]); };  // both triangles' corners
    auto normal = [&](uint32_t k, D3* n) {
        *n = dcross(sub(vtx(k, 1), vtx(k, 0)), sub(vtx(k, 2), vtx(k, 0)));
        return dnormalize(n);
    };
    D3 n0;
    if (!normal(k0, &n0)) return false;
    f->u[0] = n0;
    bool have1 = false;
    for (uint32_t k = k0 + 1; k < k1 && !have1; ++k) {
        D3 n;
        if (!normal(k, &n)) return false;
        const double c = ddot(n, n0);
        if (fabs(c) > 1.0 - 1e-9) continue;
        if (fabs(c) > 1e-6) return false;  // faces of a box are parallel or perpendicular
        f->u[1] = sub(n, dscale(n0, c));
        if (!dnormalize(&f->u[1])) return false;
        have1 = true;
    }
    if (!have1) {  // flat (one plane): frame from the first quad's edge
        D3 e = sub(vtx(k0, 1), vtx(k0, 0));
        e = sub(e, dscale(n0, ddot(e, n0)));
        if (!dnormalize(&e)) return false;
        f->u[1] = e;
    }
    f->u[2] = dcross(f->u[0], f->u[1]);
    if (!dnormalize(&f->u[2])) return false;
    for (int a = 0; a < 3; ++a) {
        f->lo[a] = INFINITY;
        f->hi[a] = -INFINITY;
    }
    for (uint32_t k = k0; k < k1; ++k)
        for (int i = 0; i < 6; ++i)
            for (int a = 0; a < 3; ++a) {
                const double p = ddot(f->u[a], vtx(k, i));
                f->lo[a] = fmin(f->lo[a], p);
                f->hi[a] = fmax(f->hi[a], p);
            }
    for (int s = 0; s < 6; ++s) f->slot_pair[s] = -1;
    for (uint32_t k = k0; k < k1; ++k) {
        D3 n;
        if (!normal(k, &n)) return false;
        int axis = -1;
        for (int a = 0; a < 3; ++a)
            if (fabs(ddot(n, f->u[a])) > 1.0 - 1e-9) axis = a;
        if (axis < 0) return false;
        // all four corners on the low or on the high face plane of that axis
        int side = -1;
        for (int sd = 0; sd < 2 && side < 0; ++sd) {
            const double plane = sd ? f->hi[axis] : f->lo[axis];
            bool on = true;
            for (int i = 0; i < 6; ++i) on = on && fabs(ddot(f->u[axis], vtx(k, i)) - plane) <= tol;
            if (on) side = sd;
        }
        if (side < 0) return false;
        int slot = 2 * axis + side;
        if (f->slot_pair[slot] >= 0) {
            // a flat box has lo == hi: both slots name the same plane
            if (f->hi[axis] - f->lo[axis] <= tol && f->slot_pair[slot ^ 1] < 0) slot ^= 1;
            else return false;
        }
        f->slot_pair[slot] = (int)k;
    }
    return true;
}
}  // namespace

static void build_clusters(CompiledScene* out, const rt_float3* verts, uint32_t n_tri,
                           float margin, double cam_ext) {
    out->clusters.clear();
    out->pair_free_mask = 0;
    const uint32_t np = (uint32_t)out->pair_isect.size();
    if (np == 0 || np > 31) return;
    double ext = 0.0;
    for (uint32_t k = 0; k < 3 * n_tri; ++k)
        ext = fmax(ext, fmax(fabs(verts[k].x), fmax(fabs(verts[k].y), fabs(verts[k].z))));
    // corners must sit on their face plane within tol (fp32 vertices of a
    // rotated box are planar to ~1e-7 of the scene scale)
    const double tol = 1e-5 * fmax(1.0, ext);
    // Along a face's normal an accepted hit point is off the face plane only by
    // the rounding of t (~1e-7 of the distance travelled) and the planarity
    // tol; across a face it can be off by the bary rounding: the culling margin.
    const double tol_n = tol + 1e-5 * fmax(ext, cam_ext);
    uint32_t free_mask = 0;
    std::vector<float> cl;
    for (uint32_t k0 = 0; k0 < np;) {
        BoxFit best, f;
        uint32_t k1 = k0;
        while (k1 < np && fit_box(verts, k0, k1 + 1, tol, &f)) {
            best = f;
            ++k1;
        }
        if (k1 == k0) {  // this quad is not a rectangle face of any box
            free_mask |= 1u << k0;
            ++k0;
            continue;
        }
        // Axes that are world axes move to that position with a + sign, so the
        // kernel reuses the ray's own reciprocals for them (flags bit a).
        {
            BoxFit cf = best;
            int pos[3] = {-1, -1, -1};
            bool used[3] = {false, false, false};
            for (int a = 0; a < 3; ++a) {
                const double c[3] = {best.u[a].x, best.u[a].y, best.u[a].z};
                for (int j = 0; j < 3; ++j)
                    if (fabs(c[j]) == 1.0 && !used[j]) {
                        pos[a] = j;
                        used[j] = true;
                    }
            }
            for (int a = 0; a < 3; ++a)
                for (int j = 0; j < 3 && pos[a] < 0; ++j)
                    if (!used[j]) {
                        pos[a] = j;
                        used[j] = true;
                    }
            for (int a = 0; a < 3; ++a) {
                const int j = pos[a];
                const double c[3] = {best.u[a].x, best.u[a].y, best.u[a].z};
                const bool flip = c[j] == -1.0;
                cf.u[j] = flip ? dscale(best.u[a], -1.0) : best.u[a];
                cf.lo[j] = flip ? -best.hi[a] : best.lo[a];
                cf.hi[j] = flip ? -best.lo[a] : best.hi[a];
                cf.slot_pair[2 * j] = best.slot_pair[2 * a + (flip ? 1 : 0)];
                cf.slot_pair[2 * j + 1] = best.slot_pair[2 * a + (flip ? 0 : 1)];
            }
            best = cf;
        }
        uint32_t flags = 0;
        for (int a = 0; a < 3; ++a) {
            const double c[3] = {best.u[a].x, best.u[a].y, best.u[a].z};
            if (c[a] == 1.0) flags |= 1u << a;
        }
        // container (bit 3): world-aligned with room inside (the kernel skips
        // it for shadow segments that stay inside, rt_trace.hpp)
        bool roomy = flags == 7u;
        for (int a = 0; a < 3; ++a) roomy = roomy && best.hi[a] - best.lo[a] > 1e-3 * fmax(1.0, ext);
        if (roomy) flags |= 8u;
        // single face (bit 4): the kernel takes it whenever the padded box is hit
        int nfaces = 0;
        uint32_t all_faces = 0;
        for (int sl = 0; sl < 6; ++sl)
            if (best.slot_pair[sl] >= 0) {
                ++nfaces;
                all_faces |= 1u << best.slot_pair[sl];
            }
        if (nfaces == 1) flags |= 16u;
        // padding per axis: tol_n, plus the margin if some face lies across it
        double pad[3];
        for (int a = 0; a < 3; ++a) {
            bool across = false;
            for (int sl = 0; sl < 6; ++sl) across = across || (best.slot_pair[sl] >= 0 && sl / 2 != a);
            pad[a] = tol_n + (across ? (double)margin : 0.0);
        }
        auto bits = [](uint32_t v) {
            float f;
            memcpy(&f, &v, 4);
            return f;
        };
        for (int a = 0; a < 3; ++a) {
            const float lo_f = (float)(best.lo[a] - pad[a]), hi_f = (float)(best.hi[a] + pad[a]);
            if (flags & 8u) {
                // A container's axes are world axes, so the kernel reads no axis
                // vector: (x, y) hold the box shrunk past each face plane by
                // tol_seg (rt_trace.hpp, cluster_candidates<SEG>: a segment that
                // stays that far inside cannot have an accepted hit on a face).
                // The face triangles lie within tol of the plane; an exact
                // crossing outside (0, tmax) shows up inside it only through the
                // rounding of t, a few 2^-24 of the distance to the plane
                // (< 2 ext): 1e-6 of the scene extent covers it 10x over.  Then a
                // 2^-20 relative slack on the bounds and on the largest
                // |coordinate| inside the box for the rounding of the bound and
                // of e = o + d*tmax (a segment end outside the box fails the
                // test anyway, one inside it has |e| <= M).
                const double tol_seg = tol + 1e-6 * fmax(ext, cam_ext);
                const float kSlack = 9.5367431640625e-07f;  // 2^-20
                const float M = fmaxf(fabsf(lo_f), fabsf(hi_f));
                const float in_lo = (float)(best.lo[a] + tol_seg) + kSlack * (fabsf(lo_f) + M);
                const float in_hi = (float)(best.hi[a] - tol_seg) - kSlack * (fabsf(hi_f) + M);
                cl.push_back(in_lo);
                cl.push_back(in_hi);
                cl.push_back(0.0f);
            } else {
                cl.push_back((float)best.u[a].x);
                cl.push_back((float)best.u[a].y);
                cl.push_back((float)best.u[a].z);
            }
            cl.push_back(lo_f);
        }
        cl.push_back((float)(best.hi[0] + pad[0]));
        cl.push_back((float)(best.hi[1] + pad[1]));
        cl.push_back((float)(best.hi[2] + pad[2]));
        cl.push_back(bits(flags));
        for (int sl = 0; sl < 6; ++sl)  // pair bit of each face slot (2*axis + side)
            cl.push_back(bits(best.slot_pair[sl] < 0 ? 0u : 1u << best.slot_pair[sl]));
        cl.push_back(bits(all_faces));
        cl.push_back(0.0f);
        // face-plane half width factor per axis: the face plane lies pad inside
        // the padded slab, an accepted hit within tol_n of it
        for (int a = 0; a < 3; ++a) cl.push_back((float)(pad[a] + tol_n));
        cl.push_back(0.0f);
        k0 = k1;
    }
    // single-face clusters last: the kernel's main cluster loop stops at the
    // first one and a lean loop slab-tests the rest (rt_trace.hpp)
    std::vector<float> multi, single;
    const size_t rec = 28;  // floats per cluster record (rt_kernel.hpp kCluF4 = 7 float4)
    for (size_t c = 0; c < cl.size() / rec; ++c) {
        uint32_t flags;
        memcpy(&flags, &cl[c * rec + 15], 4);
        std::vector<float>& dst = (flags & 16u) ? single : multi;
        dst.insert(dst.end(), cl.begin() + c * rec, cl.begin() + (c + 1) * rec);
    }
    multi.insert(multi.end(), single.begin(), single.end());
    out->clusters.swap(multi);
    out->pair_free_mask = free_mask;
    out->clu_oct.clear();
    for (size_t c = 0; c < out->clusters.size() / rec; ++c) {
        const float* r = &out->clusters[c * rec];
        uint32_t flags;
        memcpy(&flags, &r[15], 4);
        for (uint32_t oct = 0; oct < 8; ++oct) {
            float m[6];
            for (int s = 0; s < 6; ++s) m[s] = r[16 + s];
            for (int a = 0; a < 3; ++a)
                if ((flags >> a & 1u) && (oct >> a & 1u)) std::swap(m[2 * a], m[2 * a + 1]);
            out->clu_oct.insert(out->clu_oct.end(), m, m + 6);
            out->clu_oct.push_back(r[22]);  // all faces
            out->clu_oct.push_back(0.0f);
        }
    }
}

static bool finite3(const rt_float3& v) {
    return isfinite(v.x) && isfinite(v.y) && isfinite(v.z);
}

bool compile_scene(const CameraGPU& cam, const MaterialGPU* mats, const rt_float3* verts,
                   uint32_t n_tri, const SquareLightGPU& light, const SphereGPU* spheres,
                   uint32_t n_sph, CompiledScene* out, const char** err, const BuildOptions& opt) {
    if (cam.resolution.x <= 0 || cam.resolution.y <= 0) {
        *err = "camera resolution must be positive";
        return false;
    }
    if (cam.resolution.x / cam.resolution.y == 0) {
        // aspectRatio = float(res.x / res.y) (sampling.metal:132) would be 0 and
        // halfHeight infinite: every ray NaN.  Reject instead of rendering NaNs.
        *err = "camera resolution.x < resolution.y gives aspectRatio 0 (integer division)";
        return false;
    }
    if (n_tri && (!mats || !verts)) {
        *err = "materials/vertices must be non-null when n_triangles > 0";
        return false;
    }
    if (n_sph && !spheres) {
        *err = "spheres must be non-null when n_spheres > 0";
        return false;
    }
    if (!finite3(cam.position) || !finite3(cam.direction) || !finite3(cam.up)) {
        *err = "camera vectors must be finite";
        return false;
    }
    CamConst& c = out->cam;
    c.W = cam.resolution.x;
    c.H = cam.resolution.y;
    const float aspect = (float)(cam.resolution.x / cam.resolution.y);  // :132
    c.halfW = tanf(cam.horizontalFov / 2.0f);                            // :133
    c.halfH = c.halfW / aspect;                                          // :134
    const f3 w = -normalize(from_abi(cam.direction));                    // :137
    const f3 u = normalize(cross(from_abi(cam.up), w));                  // :138
    const f3 v = normalize(cross(w, u));                                 // :139
    const f3 p = from_abi(cam.position);
    c.pos[0] = p.x; c.pos[1] = p.y; c.pos[2] = p.z;
    c.u[0] = u.x; c.u[1] = u.y; c.u[2] = u.z;
    c.v[0] = v.x; c.v[1] = v.y; c.v[2] = v.z;
    c.w[0] = w.x; c.w[1] = w.y; c.w[2] = w.z;

    out->light.center[0] = light.center.x;
    out->light.center[1] = light.center.y;
    out->light.center[2] = light.center.z;
    out->light.color[0] = light.color.x;  // squareLights[0].color.xyz (raytrace.metal:22)
    out->light.color[1] = light.color.y;
    out->light.color[2] = light.color.z;

    out->tri_isect.resize(n_tri);
    out->tri_shade.resize(n_tri);
    for (uint32_t k = 0; k < n_tri; ++k) {
        const f3 a = from_abi(verts[3 * k]), b = from_abi(verts[3 * k + 1]),
                 cc = from_abi(verts[3 * k + 2]);
        const f3 e1 = b - a, e2 = cc - a;        // sampling.metal:23-24
        const f3 n = cross(e1, e2);
        const f3 N = normalize(n);               // sampling.metal:25
        f3 right, fwd;
        shading_frame(N, &right, &fwd);
        const f3 em = from_abi(mats[k].emissive);
        const float light_flag = (length(em) > 0.0f) ? 1.0f : 0.0f;  // raytrace.metal:57
        const float q[12] = {a.x, a.y, a.z, e1.x, e1.y, e1.z, e2.x, e2.y, e2.z, n.x, n.y, n.z};
        memcpy(out->tri_isect[k].q, q, sizeof(q));
        const float s[16] = {N.x, N.y, N.z, light_flag,
                             right.x, right.y, right.z, mats[k].diffuse.x,
                             fwd.x, fwd.y, fwd.z, mats[k].diffuse.y,
                             em.x, em.y, em.z, mats[k].diffuse.z};
        memcpy(out->tri_shade[k].s, s, sizeof(s));
    }
    // one margin for every culling box: scene and camera scale
    const float margin = fmaxf(culling_margin(verts, n_tri, spheres, n_sph),
                               4e-5f * fmaxf(fabsf(cam.position.x),
                                             fmaxf(fabsf(cam.position.y), fabsf(cam.position.z))));
    build_pairs(out, verts, margin);
    build_clusters(out, verts, n_tri, margin,
                   fmax(fabs(cam.position.x), fmax(fabs(cam.position.y), fabs(cam.position.z))));
    out->margin = margin;
    for (int a = 0; a < 3; ++a) {
        out->tri_lo[a] = INFINITY;
        out->tri_hi[a] = -INFINITY;
    }
    for (uint32_t k = 0; k < 3 * n_tri; ++k) {
        const float c[3] = {verts[k].x, verts[k].y, verts[k].z};
        for (int a = 0; a < 3; ++a) {
            out->tri_lo[a] = fminf(out->tri_lo[a], c[a]);
            out->tri_hi[a] = fmaxf(out->tri_hi[a], c[a]);
        }
    }
    out->sph_shade.resize(n_sph);
    build_sphere_bvh(out, spheres, n_sph, margin, opt);
    for (uint32_t k = 0; k < n_sph; ++k) {
        const SphereGPU& sp = spheres[k];
        const f3 em = from_abi(sp.material.emissive);
        const float light_flag = (length(em) > 0.0f) ? 1.0f : 0.0f;
        const float s[12] = {sp.material.diffuse.x, sp.material.diffuse.y, sp.material.diffuse.z,
                             light_flag, em.x, em.y, em.z, 0.0f,
                             sp.center.x, sp.center.y, sp.center.z, sp.radius * sp.radius};
        memcpy(out->sph_shade[k].s, s, sizeof(s));
    }
    // MIS integrator records (Sources/gpuRaytracer/shaders.metal)
    out->mis_shade.resize(n_tri);
    for (uint32_t k = 0; k < n_tri; ++k) {
        const float* ts = out->tri_shade[k].s;  // (N.xyz, light) first
        const float s[12] = {ts[0], ts[1], ts[2], ts[3],
                             mats[k].diffuse.x, mats[k].diffuse.y, mats[k].diffuse.z, mats[k].metallic,
                             mats[k].roughness, 0.0f, 0.0f, 0.0f};
        memcpy(out->mis_shade[k].s, s, sizeof(s));
    }
    MisLightConst& ml = out->mis_light;
    f3 t, b;
    onb(f3{0.0f, -1.0f, 0.0f}, &t, &b);  // directSquareLightRay (:292-293)
    const float c3[3] = {light.center.x, light.center.y, light.center.z};
    const float t3[3] = {t.x, t.y, t.z}, b3[3] = {b.x, b.y, b.z};
    const float r3[3] = {light.emittedRadiance.x, light.emittedRadiance.y, light.emittedRadiance.z};
    memcpy(ml.center, c3, sizeof(c3));
    memcpy(ml.tangent, t3, sizeof(t3));
    memcpy(ml.bitangent, b3, sizeof(b3));
    memcpy(ml.radiance, r3, sizeof(r3));
    ml.width = light.width;
    ml.depth = light.depth;
    ml.area = light.width * light.depth;  // calculateSquareLightPdf (:323)
    {
        volatile float ev = cam.ev100;     // run-time libm (never constant folded)
        ml.exposure = 1.0f / (1.2f * powf(2.0f, ev));
    }
    return true;
}

}  // namespace rt

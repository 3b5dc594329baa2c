// rt_scene.hpp — host-side scene model and the device record layout.
//
// Host mirror of the reference's scene/marshalling layer:
//   RTrace/scene.swift        (Scene, initCornellBox, createCornellBoxScene, ...)
//   RTrace/computeShader.swift (convertMaterial/convertSquareLight/convertCameras)
// plus the "compile" step that replaces the Metal BVH build
// (computeShader.swift:45-97): per-primitive records precomputed once with the
// contract arithmetic of rt_math.h and staged into LDS by the kernel.
#pragma once

#include <stdint.h>
#include <vector>

#include "rt_math.h"
#include "../../include/rt_types.h"

namespace rt {

// ---- device record layout (all float4-aligned) -------------
// Triangle intersection record, 3 x float4 = 48 B, staged in LDS:
//   q0 = (v0.x, v0.y, v0.z, e1.x)  q1 = (e1.y, e1.z, e2.x, e2.y)
//   q2 = (e2.z, n.x, n.y, n.z)      n = cross(e1, e2) (unnormalized)
struct TriIsect {
    float q[12];
};
// Shared-edge triangle pair (2k, 2k+1), 7 x float4 = 112 B, staged in LDS:
//   r0 = (v0.xyz, S.x)  r1 = (S.yz, eA.xy)  r2 = (eA.z, nA.xyz)
//   r3 = (eB.xyz, nB.x) r4 = (nB.yz, m, 0)   (see rt_kernel.hip pair_dots)
//   r5 = (lo.xyz, hi.x) r6 = (hi.yz, 0, 0)   AABB of both triangles, padded by
//   the culling margin
struct PairIsect {
    float q[28];
};
// Triangle shading record, 4 x float4 = 64 B, read from global on a hit:
//   s0 = (N.xyz, light)  s1 = (right.xyz, diffuse.r)
//   s2 = (fwd.xyz, diffuse.g)  s3 = (emissive.xyz, diffuse.b)
struct TriShade {
    float s[16];
};
// Sphere intersection record, 16 B, in BVH leaf order (read from global memory): (c.xyz, r*r)
struct SphIsect {
    float q[4];
};
// Sphere BVH node, 2 x float4 = 32 B, nodes in depth-first order (stackless
// traversal): n0 = (lo.xyz, escape), n1 = (hi.xyz, leaf); escape = index of
// the node after this subtree; leaf = count << 24 | first (count 0: internal
// node whose first child is the next node).  Boxes are padded by the culling
// margin.  Eight layouts (one per ray-direction octant,
// near child first) of the same tree are stored back to back.
struct BvhNode {
    float lo[3];
    uint32_t escape;
    float hi[3];
    uint32_t leaf;
};
// Sphere shading record by sphere id, 48 B: (diffuse.rgb, light),
// (emissive.rgb, 0), (c.xyz, r*r)
struct SphShade {
    float s[12];
};

// Camera constants of generateCameraRay (sampling.metal:125-157), computed
// once per scene instead of once per sample (same contract ops).
struct CamConst {
    float pos[3], u[3], v[3], w[3];
    float halfW, halfH;
    int32_t W, H;
};

struct LightConst {
    float center[3], color[3];
};

// Square light as the MIS integrator uses it (Sources/gpuRaytracer/
// shaders.metal:291-326): basis of the hard-coded normal (0,-1,0), size and
// emittedRadiance.  Computed once per scene with the contract ops.
struct MisLightConst {
    float center[3], tangent[3], bitangent[3], radiance[3];
    float width, depth, area;
    float exposure;  // cameraExposure (shaders.metal:145-150), host libm powf
};

// Per-triangle record of the MIS integrator, 48 B:
// (N.xyz, light), (diffuse.rgb, metallic), (roughness, 0, 0, 0)
struct MisShade {
    float s[12];
};

struct CompiledScene {
    CamConst cam;
    LightConst light;
    std::vector<TriIsect> tri_isect;
    std::vector<TriShade> tri_shade;
    std::vector<PairIsect> pair_isect;  // empty unless every (2k, 2k+1) shares v0 + an edge
    std::vector<SphIsect> sph_isect;    // in BVH leaf order
    std::vector<uint32_t> sph_perm;     // leaf-order index -> sphere id (shading, ties)
    std::vector<BvhNode> sph_nodes;     // 8 octant layouts of sph_layout_nodes nodes each
    uint32_t sph_layout_nodes = 0;
    uint32_t sph_lds_entries = 0;       // entries per layout of sph_lds (a leaf of c spheres: c)
    std::vector<SphShade> sph_shade;    // by sphere id
    // Compact sphere BVH: one layout per direction octant,
    // 16 B per entry: inner node = fp16 near/far box (lo rounded down, hi up;
    // the plane a ray of the layout's octant enters through in the first
    // slot) + (escape | 0x80000000); leaf (one sphere) = (c.xyz, r*r) fp32,
    // its sphere id in sph_lds_id.  Empty when the tree does not qualify.
    std::vector<uint32_t> sph_lds;      // 8 layouts x sph_lds_entries x 4 words
    std::vector<uint16_t> sph_lds_id;   // 8 layouts x sph_lds_entries
    // The same tree with LEAF BOXES (round 6): one 16-B entry per node in the
    // same near/far fp16 form, inner nodes as above, a leaf node = its padded
    // box + (first leaf-order sphere | (count - 1) << 24); the spheres stay in
    // sph_isect (leaf order).  Every step of a walk is then the same box test.
    std::vector<uint32_t> sph_box;      // 8 layouts x sph_layout_nodes x 4 words
    // Box clusters over the pair records: 28 floats each,
    // (u0.xyz, lo0) (u1.xyz, lo1) (u2.xyz, lo2) (hi0, hi1, hi2, flags)
    // (m0, m1, m2, m3) (m4, m5, all, 0) (w0, w1, w2, 0): an oriented box (padded
    // extents) whose faces hold consecutive pair records; m_s = bit of the pair
    // on face slot s = 2*axis + side (0: none), all = their union; flags bit a
    // = axis a is world axis a (+), bit 3 = container, bit 4 = single face;
    // w_a = face-plane half width factor of axis a.
    std::vector<float> clusters;
    // Per cluster and ray-direction octant (8 floats, cluster-major): the face
    // masks m0..m5 with the two faces of every world axis swapped when the
    // octant's bit for that axis is set (the ray enters through the high face),
    // then all, 0 -- the path-trace kernel's cluster test reads the entry /
    // exit masks of world axes without a per-lane select (rt_trace.hpp).
    std::vector<float> clu_oct;
    uint32_t pair_free_mask = 0;        // pairs in no cluster (tested by every lane)
    float tri_lo[3], tri_hi[3];         // bounds of the triangle vertices (BVH build)
    float margin = 0.0f;                // culling margin
    MisLightConst mis_light;
    std::vector<MisShade> mis_shade;    // by triangle id
};

constexpr uint32_t kTriLeafMax = 1;  // triangles per leaf of the host SAH build (default)
// Host binned-SAH triangle BVH in the compact 8-octant layout (rt_scene.cpp):
// nodes = 8 layouts x (nodes per layout) entries of 4 words, sorted = records in leaf order,
// perm = leaf order -> triangle id.  leaf_max: triangles per leaf at most (1..128),
// trav_cost: cost of a box step in triangle tests (SAH leaf rule).  False for
// n == 0 or n >= 2^24.
bool build_tri_sah(const std::vector<TriIsect>& tri, float margin, std::vector<uint32_t>* nodes,
                   std::vector<TriIsect>* sorted, std::vector<uint32_t>* perm,
                   uint32_t leaf_max = kTriLeafMax, double trav_cost = 1.0);

// Speed-only choices of the host builds (rt_create_options, include/rtpt.h):
// none of them changes a rendered value.
struct BuildOptions {
    bool sphere_sah = true;        // exact SAH sweeps (false: median split of the longest axis)
    uint32_t sphere_leaf_max = 1;  // spheres per leaf (measured best for config 4)
};

// Validates and precomputes; returns false with *err set on bad input.
bool compile_scene(const CameraGPU& cam, const MaterialGPU* mats, const rt_float3* verts,
                   uint32_t n_tri, const SquareLightGPU& light, const SphereGPU* spheres,
                   uint32_t n_sph, CompiledScene* out, const char** err,
                   const BuildOptions& opt = BuildOptions());

// ---- scene builders (scene.swift) ------------------------------------------
struct Material {  // scene.swift:277-282
    float diffuse[4];
    float metallic, roughness;
    float emissive[3];
};

struct Triangle {  // scene.swift:242-245
    f3 vertices[3];
    Material material;
};

struct SquareLight {  // scene.swift:248-271
    f3 center;
    f3 vertices[4];
    Material material;
    float luminous_efficacy, watts;  // LightType.bulb
    float width, depth;
    f3 emitted_luminance() const;
};

struct Sphere {  // scene.swift:284-288
    f3 center;
    Material material;
    float radius;
};

struct Camera {  // scene.swift:290-301
    f3 position, direction, up;
    int32_t resolution[2];
    float horizontal_fov;
    float ev100;
};

struct Scene {  // scene.swift:8-12 (+ spheres for config 4)
    Camera camera;
    SquareLight light;
    std::vector<Triangle> triangles;
    std::vector<Sphere> spheres;
};

Scene init_cornell_box(int32_t width, int32_t height);                  // scene.swift:14-62
// Sources/gpuRaytracer/main.swift:21-67: the same room with a 1.5 x 1.5 light
Scene init_cornell_box_mis(int32_t width, int32_t height);
std::vector<Triangle> create_cornell_box_scene();                       // scene.swift:64-175
Scene init_random_spheres(int32_t width, int32_t height, uint32_t n, uint64_t seed);

// computeShader.swift conversions
MaterialGPU convert_material(const Material& m);                        // :13-20
SquareLightGPU convert_square_light(const SquareLight& l);              // :33-41
CameraGPU convert_camera(const Camera& c);                              // :242-253
SphereGPU convert_sphere(const Sphere& s);                              // :232-240
rt_float3 to_abi(f3 v);

// splitmix64(key + p) mod 2^20 (replaces arc4random, renderer.swift:99-101)
uint32_t seed_splitmix(uint64_t key, uint64_t p);

}  // namespace rt

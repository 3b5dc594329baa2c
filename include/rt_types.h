/*
 * rt_types.h — the boundary ABI structs of the path-tracing hot path.
 *
 * These restate the layout of the reference's shared Swift/Metal header
 * `RTrace/shaderTypes.h:13-62` (Apple `simd_float3` = 16 B / 16-B aligned,
 * `simd_float4` = 16 B, `simd_int2` = 8 B) as plain C structs, so a Swift
 * `Renderer` (or any FFI caller) can hand the very same arrays it built for the
 * Metal argument table (`RTrace/renderer.swift:49-72`) to the C-ABI in
 * `rtpt.h`.  Every size and offset is pinned by static asserts below
 * (SURVEY.md Appendix C).
 *
 * Plain C99/C11 + C++; used by the HIP library, the C++ host, and the CPU
 * oracle (which only reads the layout).
 */
#ifndef RT_TYPES_H
#define RT_TYPES_H

#include <stdint.h>
#include <stddef.h>

#if defined(__cplusplus)
#define RT_ALIGN(n) alignas(n)
#else
#define RT_ALIGN(n) _Alignas(n)
#endif

/* simd_float3: 12 B of payload padded to 16 B, 16-B aligned. */
typedef struct rt_float3 {
    RT_ALIGN(16) float x;
    float y, z, _pad;
} rt_float3;

/* simd_float4 */
typedef struct rt_float4 {
    RT_ALIGN(16) float x;
    float y, z, w;
} rt_float4;

/* simd_int2 */
typedef struct rt_int2 {
    RT_ALIGN(8) int32_t x;
    int32_t y;
} rt_int2;

/* shaderTypes.h:13-18 */
typedef struct MaterialGPU {
    rt_float4 diffuse;
    float metallic;
    float roughness;
    rt_float3 emissive;
} MaterialGPU;

/* shaderTypes.h:20-23 (not read by pathTrace; kept for ABI completeness) */
typedef struct TriangleGPU {
    rt_float3 vertices[3];
    MaterialGPU material;
} TriangleGPU;

/* shaderTypes.h:25-29 (used by the sphere primitive, config 4) */
typedef struct SphereGPU {
    rt_float3 center;
    MaterialGPU material;
    float radius;
} SphereGPU;

/* shaderTypes.h:31-38 */
typedef struct CameraGPU {
    rt_float3 position;
    rt_float3 direction;
    rt_float3 up;
    rt_int2 resolution;
    float horizontalFov;
    float ev100;
} CameraGPU;

/* shaderTypes.h:56-62 */
typedef struct SquareLightGPU {
    rt_float3 center;
    rt_float4 color;
    rt_float3 emittedRadiance;
    float width;
    float depth;
} SquareLightGPU;

#if defined(__cplusplus)
#define RT_STATIC_ASSERT(c, m) static_assert(c, m)
#define RT_ALIGNOF(t) alignof(t)
#else
#define RT_STATIC_ASSERT(c, m) _Static_assert(c, m)
#define RT_ALIGNOF(t) _Alignof(t)
#endif

RT_STATIC_ASSERT(sizeof(rt_float3) == 16 && RT_ALIGNOF(rt_float3) == 16, "simd_float3 layout");
RT_STATIC_ASSERT(sizeof(rt_float4) == 16, "simd_float4 layout");
RT_STATIC_ASSERT(sizeof(rt_int2) == 8 && RT_ALIGNOF(rt_int2) == 8, "simd_int2 layout");
RT_STATIC_ASSERT(sizeof(MaterialGPU) == 48, "MaterialGPU size");
RT_STATIC_ASSERT(offsetof(MaterialGPU, metallic) == 16, "MaterialGPU.metallic");
RT_STATIC_ASSERT(offsetof(MaterialGPU, roughness) == 20, "MaterialGPU.roughness");
RT_STATIC_ASSERT(offsetof(MaterialGPU, emissive) == 32, "MaterialGPU.emissive");
RT_STATIC_ASSERT(sizeof(TriangleGPU) == 96, "TriangleGPU size");
RT_STATIC_ASSERT(offsetof(TriangleGPU, material) == 48, "TriangleGPU.material");
RT_STATIC_ASSERT(sizeof(SphereGPU) == 80, "SphereGPU size");
RT_STATIC_ASSERT(offsetof(SphereGPU, material) == 16, "SphereGPU.material");
RT_STATIC_ASSERT(offsetof(SphereGPU, radius) == 64, "SphereGPU.radius");
RT_STATIC_ASSERT(sizeof(CameraGPU) == 64, "CameraGPU size");
RT_STATIC_ASSERT(offsetof(CameraGPU, direction) == 16, "CameraGPU.direction");
RT_STATIC_ASSERT(offsetof(CameraGPU, up) == 32, "CameraGPU.up");
RT_STATIC_ASSERT(offsetof(CameraGPU, resolution) == 48, "CameraGPU.resolution");
RT_STATIC_ASSERT(offsetof(CameraGPU, horizontalFov) == 56, "CameraGPU.horizontalFov");
RT_STATIC_ASSERT(offsetof(CameraGPU, ev100) == 60, "CameraGPU.ev100");
RT_STATIC_ASSERT(sizeof(SquareLightGPU) == 64, "SquareLightGPU size");
RT_STATIC_ASSERT(offsetof(SquareLightGPU, color) == 16, "SquareLightGPU.color");
RT_STATIC_ASSERT(offsetof(SquareLightGPU, emittedRadiance) == 32, "SquareLightGPU.emittedRadiance");
RT_STATIC_ASSERT(offsetof(SquareLightGPU, width) == 48, "SquareLightGPU.width");
RT_STATIC_ASSERT(offsetof(SquareLightGPU, depth) == 52, "SquareLightGPU.depth");

#endif /* RT_TYPES_H */

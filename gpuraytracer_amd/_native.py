"""ctypes binding of librtpt.so (the C-ABI declared in include/rtpt.h).

The ABI structs mirror ``RTrace/shaderTypes.h`` (see include/rt_types.h):
Apple ``simd_float3`` is 16 bytes with 16-byte alignment, so the padding that
the C compiler inserts is spelled out explicitly here and every size is
asserted against the C header's static asserts.
"""
from __future__ import annotations

import ctypes
import os

ABI_VERSION = 7
_HERE = os.path.dirname(os.path.abspath(__file__))
# RTPT_LIB overrides the in-tree library (A/B builds of the kernel).
library_path = os.environ.get("RTPT_LIB") or os.path.join(_HERE, "librtpt.so")


class float3(ctypes.Structure):
    """simd_float3: x, y, z + 4 bytes of padding (16 B)."""

    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float),
                ("_pad", ctypes.c_float)]

    def __iter__(self):
        return iter((self.x, self.y, self.z))


class float4(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("z", ctypes.c_float),
                ("w", ctypes.c_float)]


class int2(ctypes.Structure):
    _fields_ = [("x", ctypes.c_int32), ("y", ctypes.c_int32)]


class MaterialGPU(ctypes.Structure):  # shaderTypes.h:13-18
    _fields_ = [("diffuse", float4), ("metallic", ctypes.c_float),
                ("roughness", ctypes.c_float), ("_pad", ctypes.c_float * 2),
                ("emissive", float3)]


class SphereGPU(ctypes.Structure):  # shaderTypes.h:25-29
    _fields_ = [("center", float3), ("material", MaterialGPU), ("radius", ctypes.c_float),
                ("_pad", ctypes.c_float * 3)]


class CameraGPU(ctypes.Structure):  # shaderTypes.h:31-38
    _fields_ = [("position", float3), ("direction", float3), ("up", float3),
                ("resolution", int2), ("horizontalFov", ctypes.c_float),
                ("ev100", ctypes.c_float)]


class SquareLightGPU(ctypes.Structure):  # shaderTypes.h:56-62
    _fields_ = [("center", float3), ("color", float4), ("emittedRadiance", float3),
                ("width", ctypes.c_float), ("depth", ctypes.c_float),
                ("_pad", ctypes.c_float * 2)]


for _t, _n in ((float3, 16), (MaterialGPU, 48), (SphereGPU, 80), (CameraGPU, 64),
               (SquareLightGPU, 64)):
    assert ctypes.sizeof(_t) == _n, (_t.__name__, ctypes.sizeof(_t))
assert MaterialGPU.emissive.offset == 32 and SphereGPU.radius.offset == 64
assert CameraGPU.resolution.offset == 48 and CameraGPU.horizontalFov.offset == 56
assert SquareLightGPU.width.offset == 48


class SceneDesc(ctypes.Structure):  # rt_scene_desc
    _fields_ = [("camera", ctypes.POINTER(CameraGPU)),
                ("materials", ctypes.POINTER(MaterialGPU)),
                ("square_lights", ctypes.POINTER(SquareLightGPU)),
                ("n_square_lights", ctypes.c_uint32),
                ("vertices", ctypes.POINTER(float3)),
                ("n_triangles", ctypes.c_uint32),
                ("spheres", ctypes.POINTER(SphereGPU)),
                ("n_spheres", ctypes.c_uint32),
                ("device", ctypes.c_int32)]


class RenderParamsC(ctypes.Structure):  # rt_render_params
    _fields_ = [(n, ctypes.c_uint32) for n in
                ("spp", "bounces", "sample_base", "row_start", "row_step", "row_count",
                 "accumulate", "flags")]


class SceneInfo(ctypes.Structure):  # rt_scene_info
    _fields_ = [(n, ctypes.c_uint32) for n in
                ("n_triangles", "n_triangle_pairs", "n_spheres", "lds_bytes",
                 "n_sphere_nodes", "n_triangle_bvh_nodes", "n_box_clusters", "pair_free_mask",
                 "sphere_kernel_lds_bytes", "kernel_layout", "kernel_lds_bytes")]


class CreateOptions(ctypes.Structure):  # rt_create_options
    _fields_ = [("scene_layout", ctypes.c_uint32), ("lanes_per_pixel", ctypes.c_uint32),
                ("tri_bvh_build", ctypes.c_uint32), ("tri_leaf_max", ctypes.c_uint32),
                ("tri_leaf_cost", ctypes.c_float), ("sphere_leaf_max", ctypes.c_uint32),
                ("sphere_median", ctypes.c_uint32), ("walk_scheduler", ctypes.c_uint32),
                ("walk_leaf_den", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 7)]


assert ctypes.sizeof(CreateOptions) == 64

# rt_scene_layout / rt_tri_bvh_build / rt_walk_scheduler (include/rtpt.h)
LAYOUTS = {"auto": 0, "pairs": 1, "single": 2, "global": 3, "smem": 3, "pairsmem": 4, "sorted": 5, "bvh": 6}
TRI_BUILDS = {"default": 0, "host": 1, "lbvh": 2, "gpusah": 3}
WALKS = {"auto": 0, "lockstep": 1, "free": 2, "sorted": 3}

RT_OK = 0
RT_OUT_DEVICE, RT_OUT_FP16, RT_OUT_NONE, RT_KEEP_SUM, RT_OUT_RGBA8 = 0x1, 0x2, 0x4, 0x8, 0x10
RT_MAX_BOUNCES = 4
RT_COMM_ID_BYTES = 128
STATUS = {0: "RT_OK", 1: "RT_ERR_INVALID_ARG", 2: "RT_ERR_NO_DEVICE", 3: "RT_ERR_OUT_OF_MEMORY",
          4: "RT_ERR_LAUNCH", 5: "RT_ERR_STATE", 6: "RT_ERR_COMM"}

class LaunchInfo(ctypes.Structure):  # rt_launch_info
    _fields_ = [("kernel", ctypes.c_char * 96)] + [(n, ctypes.c_uint32) for n in
                ("lanes_per_pixel", "halton_tables", "small_index", "block_threads", "grid_x",
                 "grid_y", "lds_bytes")]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["kernel"] = self.kernel.decode()
        return d


class BuildStats(ctypes.Structure):  # rt_build_stats
    _fields_ = [("tri_bvh_build", ctypes.c_uint32), ("tri_bvh_nodes", ctypes.c_uint32),
                ("tri_bvh_build_ms", ctypes.c_float), ("scene_compile_ms", ctypes.c_float),
                ("tri_bvh_temp_kib", ctypes.c_uint32)]


class TileLayout(ctypes.Structure):  # rt_tile_layout_info
    _fields_ = [("rows", ctypes.c_uint32), ("rows_max", ctypes.c_uint32),
                ("row_bytes", ctypes.c_uint64), ("tile_bytes", ctypes.c_uint64)]


class MisParamsC(ctypes.Structure):  # rt_mis_params
    _fields_ = [(n, ctypes.c_uint32) for n in
                ("camera_rays", "mis_samples", "row_start", "row_step", "row_count", "flags")]


# Every entry point of include/rtpt.h: name -> (restype, argtypes)
_P = ctypes.c_void_p
SIGNATURES = {
    "rt_create": (ctypes.c_int, [ctypes.POINTER(SceneDesc), ctypes.POINTER(_P)]),
    "rt_create_ex": (ctypes.c_int, [ctypes.POINTER(SceneDesc), ctypes.POINTER(CreateOptions),
                                    ctypes.POINTER(_P)]),
    "rt_create_options_default": (None, [ctypes.POINTER(CreateOptions)]),
    "rt_set_seeds": (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_int32]),
    "rt_fill_seeds": (ctypes.c_int, [_P, ctypes.c_uint64]),
    "rt_render": (ctypes.c_int, [_P, ctypes.POINTER(RenderParamsC), _P]),
    "rt_render_async": (ctypes.c_int, [_P, ctypes.POINTER(RenderParamsC), _P, _P]),
    "rt_last_kernel_ms": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_float)]),
    "rt_destroy": (ctypes.c_int, [_P]),
    "rt_last_launch": (ctypes.c_int, [_P, ctypes.POINTER(LaunchInfo)]),
    "rt_build_info": (ctypes.c_int, [_P, ctypes.POINTER(BuildStats)]),
    "rt_math_selfcheck": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)]),
    "rt_comm_unique_id": (ctypes.c_int, [_P]),
    "rt_comm_init": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, _P]),
    "rt_render_gather": (ctypes.c_int, [_P, ctypes.POINTER(RenderParamsC), _P, _P]),
    "rt_comm_info": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    "rt_tile_layout": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                      ctypes.c_uint32, ctypes.POINTER(TileLayout)]),
    "rt_place_tiles": (ctypes.c_int, [_P, _P, ctypes.c_int32, ctypes.c_uint32, _P, _P]),
    "rt_place_tiles_host": (ctypes.c_int, [_P, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_uint32, _P]),
    "rt_build_sha": (ctypes.c_char_p, []),
    "rt_debug_stats": (ctypes.c_int, [_P, _P, ctypes.c_int]),
    "rt_last_error": (ctypes.c_char_p, [_P]),
    "rt_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "rt_abi_version": (ctypes.c_int, []),
    "rt_seed_splitmix": (None, [ctypes.c_uint64, _P, ctypes.c_size_t]),
    "rt_scene_cornell_box": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32,
                                            ctypes.POINTER(CameraGPU),
                                            ctypes.POINTER(MaterialGPU),
                                            ctypes.POINTER(float3),
                                            ctypes.POINTER(SquareLightGPU),
                                            ctypes.POINTER(ctypes.c_uint32)]),
    "rt_scene_random_spheres": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32,
                                               ctypes.c_uint64, ctypes.POINTER(CameraGPU),
                                               ctypes.POINTER(MaterialGPU),
                                               ctypes.POINTER(float3),
                                               ctypes.POINTER(SquareLightGPU),
                                               ctypes.POINTER(ctypes.c_uint32),
                                               ctypes.POINTER(SphereGPU)]),
    "rt_render_mis": (ctypes.c_int, [_P, ctypes.POINTER(MisParamsC), _P, _P]),
    "rt_scene_cornell_box_mis": (ctypes.c_int, [ctypes.c_int32, ctypes.c_int32,
                                                ctypes.POINTER(CameraGPU),
                                                ctypes.POINTER(MaterialGPU),
                                                ctypes.POINTER(float3),
                                                ctypes.POINTER(SquareLightGPU),
                                                ctypes.POINTER(ctypes.c_uint32)]),
    "rt_tonemap_rgba8": (None, [_P, ctypes.c_size_t, _P]),
    "rt_scene_describe": (ctypes.c_int, [ctypes.POINTER(SceneDesc), ctypes.POINTER(SceneInfo)]),
    "rt_scene_describe_ex": (ctypes.c_int, [ctypes.POINTER(SceneDesc), ctypes.POINTER(CreateOptions),
                                            ctypes.POINTER(SceneInfo)]),
}


class RtError(RuntimeError):
    """A non-RT_OK status from librtpt.so, with rt_last_error()'s message."""

    def __init__(self, status: int, message: str):
        super().__init__(f"{STATUS.get(status, status)}: {message}")
        self.status = status


def _preload_hip_runtime():
    """Make this process use ONE HIP runtime.

    torch-ROCm ships its own libamdhip64 (SONAME libamdhip64.so.7, NEEDED as
    "libamdhip64.so").  If librtpt.so pulled in /opt/rocm's copy first, torch
    would later map a second runtime and fail to see the GPU ("No HIP GPUs are
    available").  Preloading torch's copy (without importing torch) makes
    librtpt.so's NEEDED libamdhip64.so.7 resolve to it and torch reuse it, so
    device pointers, streams and events are shared.  Without torch the system
    runtime is used.  RTPT_SYSTEM_HIP=1 opts out.
    """
    if os.environ.get("RTPT_SYSTEM_HIP") == "1":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.submodule_search_locations:
        return
    for d in spec.submodule_search_locations:
        cand = os.path.join(d, "lib", "libamdhip64.so")
        if os.path.exists(cand):
            ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
            return


def _load():
    if not os.path.exists(library_path):
        raise ImportError(
            f"{library_path} is missing: build the HIP extension first "
            "(`make` or `python -c 'import __graft_entry__ as g; g.build()'`). "
            "There is no CPU fallback.")
    _preload_hip_runtime()
    handle = ctypes.CDLL(library_path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    if handle.rt_abi_version() != ABI_VERSION:
        raise ImportError(f"librtpt.so ABI {handle.rt_abi_version()} != {ABI_VERSION}")
    if not os.environ.get("RTPT_LIB"):  # A/B builds (RTPT_LIB) are checked by their maker
        from .srchash import have_sources, kernel_source_sha
        built = handle.rt_build_sha().decode()
        if not have_sources() or built == "unknown":
            # installed without its sources, or built outside the Makefile:
            # nothing to compare against
            import warnings
            warnings.warn(f"{library_path}: source hash not checked (library hash {built!r}, "
                          f"sources {'present' if have_sources() else 'absent'})")
        elif built != kernel_source_sha():
            raise ImportError(f"{library_path} was built from other sources (hash {built}, "
                              f"tree {kernel_source_sha()}): rebuild it with `make`")
    return handle


lib = _load()


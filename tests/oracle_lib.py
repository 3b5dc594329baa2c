"""ctypes access to the CPU oracle (oracle/liboracle.so) — test-side only."""
import ctypes
import os

import numpy as np

from gpuraytracer_amd import CameraGPU, MaterialGPU, SphereGPU, SquareLightGPU, float3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# RTPT_ORACLE_LIB: the sanitizer build (make asan-test, tests/run_sanitized.py)
_lib = ctypes.CDLL(os.environ.get("RTPT_ORACLE_LIB") or os.path.join(ROOT, "oracle", "liboracle.so"))
_lib.pto_halton.restype = ctypes.c_float
_lib.pto_halton.argtypes = [ctypes.c_uint32, ctypes.c_uint32]
_lib.pto_last_tests.restype = ctypes.c_uint64
_lib.pto_seed_splitmix.argtypes = [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t]
_lib.pto_render.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_void_p, ctypes.c_uint32,
                            ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [ctypes.c_void_p] * 3 + [ctypes.c_int]
lib = _lib


def _p(x):
    if x is None:
        return None
    if isinstance(x, np.ndarray):
        return x.ctypes.data_as(ctypes.c_void_p)
    return ctypes.cast(ctypes.pointer(x) if isinstance(x, ctypes.Structure) else x, ctypes.c_void_p)


def halton(i, d):
    return _lib.pto_halton(i, d)


def render(scene, seeds, spp, bounces=3, sample_base=0, row_start=0, row_step=1, row_count=0,
           sum_in=None, want_sum=False, threads=None):
    """Oracle render of a gpuraytracer_amd.Scene; returns out (and sum)."""
    H, W = scene.height, scene.width
    rows = row_count or (H - 1 - row_start) // row_step + 1
    out = np.zeros((rows, W, 4), np.float32)
    s_out = np.zeros((rows, W, 4), np.float32) if want_sum else None
    sd = np.ascontiguousarray(seeds, dtype=np.uint32)
    threads = threads or min(8, os.cpu_count() or 1)
    r = _lib.pto_render(_p(scene.camera), _p(scene.materials), _p(scene.light), _p(scene.vertices),
                        scene.n_triangles, _p(scene.spheres), scene.n_spheres, _p(sd), spp, bounces,
                        sample_base, row_start, row_step, row_count,
                        _p(None if sum_in is None else np.ascontiguousarray(sum_in, np.float32)),
                        _p(s_out), _p(out), threads)
    assert r == 0, "oracle rejected the input"
    return (out, s_out) if want_sum else out


_lib.pto_primary_ids.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_void_p]


def primary_ids(scene):
    """Closest-hit primitive id of every pixel's camera ray through the pixel
    centre (-1: miss), (H, W) int32 -- pto_primary_ids."""
    ids = np.empty((scene.height, scene.width), np.int32)
    r = _lib.pto_primary_ids(_p(scene.camera), _p(scene.materials), _p(scene.light),
                             _p(scene.vertices), scene.n_triangles, _p(ids))
    assert r == 0
    return ids


def cornell_box(width, height):
    cam, light = CameraGPU(), SquareLightGPU()
    mats, verts, n = (MaterialGPU * 36)(), (float3 * 108)(), ctypes.c_uint32()
    assert _lib.pto_cornell_box(width, height, ctypes.byref(cam), mats, verts, ctypes.byref(light),
                                ctypes.byref(n)) == 0
    return cam, mats, verts, light, n.value


def random_spheres(width, height, n_spheres, seed=42):
    cam, light = CameraGPU(), SquareLightGPU()
    mats, verts, n = (MaterialGPU * 12)(), (float3 * 36)(), ctypes.c_uint32()
    sph = (SphereGPU * max(1, n_spheres))()
    assert _lib.pto_random_spheres(width, height, n_spheres, ctypes.c_uint64(seed),
                                   ctypes.byref(cam), mats, verts, ctypes.byref(light),
                                   ctypes.byref(n), sph) == 0
    return cam, mats, verts, light, n.value, sph


def seeds(width, height, key=0x5EED00000000):
    out = np.empty(width * height, np.uint32)
    _lib.pto_seed_splitmix(key, out.ctypes.data_as(ctypes.c_void_p), out.size)
    return out.reshape(height, width)


def tonemap(rgba32f):
    a = np.ascontiguousarray(rgba32f, np.float32)
    out = np.empty(a.shape[:-1] + (4,), np.uint8)
    _lib.pto_tonemap_rgba8(a.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(a.size // 4),
                           out.ctypes.data_as(ctypes.c_void_p))
    return out


_lib.pto_pow.restype = ctypes.c_float
_lib.pto_pow.argtypes = [ctypes.c_float, ctypes.c_float]
_lib.pto_render_mis.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] * 6 + \
    [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]


def cornell_box_mis(width, height):
    cam, light = CameraGPU(), SquareLightGPU()
    mats, verts, n = (MaterialGPU * 36)(), (float3 * 108)(), ctypes.c_uint32()
    assert _lib.pto_cornell_box_mis(width, height, ctypes.byref(cam), mats, verts,
                                    ctypes.byref(light), ctypes.byref(n)) == 0
    return cam, mats, verts, light, n.value


def render_mis(scene, camera_rays=6, mis_samples=300, row_start=0, row_step=1, row_count=0,
               threads=None):
    """Oracle MIS render (pto_render_mis); returns (sum float32, rgba8)."""
    H, W = scene.height, scene.width
    rows = row_count or (H - 1 - row_start) // row_step + 1
    out = np.zeros((rows, W, 4), np.float32)
    out8 = np.zeros((rows, W, 4), np.uint8)
    threads = threads or min(8, os.cpu_count() or 1)
    r = _lib.pto_render_mis(_p(scene.camera), _p(scene.materials), _p(scene.light),
                            _p(scene.vertices), scene.n_triangles, camera_rays, mis_samples,
                            row_start, row_step, row_count, _p(out), _p(out8), threads)
    assert r == 0, "oracle rejected the input"
    return out, out8

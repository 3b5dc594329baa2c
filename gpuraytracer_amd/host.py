"""Host-side mirror of the reference's Swift Scene/Renderer API.

``Scene``     <- RTrace/scene.swift (``initCornellBox``, scene.swift:14-62) and
                 RTrace/computeShader.swift conversions (convertCameras, ...).
``Renderer``  <- RTrace/renderer.swift: ``__init__`` = ``Renderer.init()``
                 (:29-115: upload scene, seed texture), ``draw()`` =
                 ``Renderer.draw()`` (:117-146: dispatch + wait + read back).

Everything executes in librtpt.so (C++ host + gfx950 kernel); this module
only marshals arrays through ctypes.  Failures raise :class:`RtError` (the
reference ``fatalError``s).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, fields

import numpy as np

from ._native import (LAYOUTS, RT_COMM_ID_BYTES, RT_KEEP_SUM, RT_OK, RT_OUT_DEVICE, RT_OUT_FP16,
                      RT_OUT_NONE, RT_OUT_RGBA8, TRI_BUILDS, WALKS,
                      BuildStats, CameraGPU, CreateOptions, LaunchInfo, MaterialGPU, MisParamsC, RenderParamsC,
                      RtError, SceneDesc, SceneInfo, SphereGPU, SquareLightGPU, TileLayout, float3,
                      lib)

DEFAULT_SEED_KEY = 0x5EED00000000


def _check(status: int, ctx=None):
    if status != RT_OK:
        raise RtError(status, lib.rt_last_error(ctx).decode())


def seed_splitmix(width: int, height: int, key: int = DEFAULT_SEED_KEY) -> np.ndarray:
    """seed[p] = splitmix64(key + p) mod 2^20 — the deterministic stand-in for
    ``arc4random() % (1024*1024)`` (renderer.swift:99-101)."""
    n = int(width) * int(height)
    out = np.empty(n, dtype=np.uint32)
    lib.rt_seed_splitmix(ctypes.c_uint64(key), out.ctypes.data_as(ctypes.c_void_p), n)
    return out.reshape(height, width)


def tonemap_rgba8(rgba32f: np.ndarray) -> np.ndarray:
    """image.swift:35-65 epilogue: fp16 round trip, x2 exposure, Reinhard,
    gamma 1/2.2, truncating UInt8 (alpha 255)."""
    a = np.ascontiguousarray(rgba32f, dtype=np.float32)
    n = a.size // 4
    out = np.empty(a.shape[:-1] + (4,), dtype=np.uint8)
    lib.rt_tonemap_rgba8(a.ctypes.data_as(ctypes.c_void_p), n,
                         out.ctypes.data_as(ctypes.c_void_p))
    return out


def comm_unique_id() -> bytes:
    """rt_comm_unique_id: the RCCL communicator id rank 0 hands to every rank."""
    buf = (ctypes.c_uint8 * RT_COMM_ID_BYTES)()
    _check(lib.rt_comm_unique_id(buf))
    return bytes(buf)


def _pixel_flags(fp16: bool = False, rgba8: bool = False) -> int:
    return (RT_OUT_FP16 if fp16 else 0) | (RT_OUT_RGBA8 if rgba8 else 0)


def tile_layout(width: int, height: int, world: int, rank: int, fp16: bool = False,
                rgba8: bool = False) -> dict:
    """rt_tile_layout: rank's rows of the rt_render_gather partition (y = rank +
    j*world) and the padded tile every rank sends (rows_max, tile_bytes)."""
    t = TileLayout()
    _check(lib.rt_tile_layout(width, height, world, rank, _pixel_flags(fp16, rgba8), ctypes.byref(t)))
    return {k: getattr(t, k) for k, _ in TileLayout._fields_}


def place_tiles_host(gathered: np.ndarray, width: int, height: int, world: int) -> np.ndarray:
    """rt_place_tiles_host: ``gathered`` = ``world`` padded tiles back to back
    (uint8/uint16/float32 RGBA pixels, any shape with 4 channels last); returns
    the (height, width, 4) frame rank 0 of rt_render_gather would assemble."""
    g = np.ascontiguousarray(gathered)
    fp16, rgba8 = g.dtype == np.uint16, g.dtype == np.uint8
    if g.dtype not in (np.float32, np.uint16, np.uint8):
        raise ValueError("gathered pixels must be float32, uint16 (fp16 bits) or uint8")
    lay = tile_layout(width, height, world, 0, fp16, rgba8)
    if g.nbytes != world * lay["tile_bytes"]:
        raise ValueError(f"gathered holds {g.nbytes} bytes, expected {world} x {lay['tile_bytes']}")
    frame = np.empty((height, width, 4), g.dtype)
    _check(lib.rt_place_tiles_host(g.ctypes.data_as(ctypes.c_void_p), width, height, world,
                                   _pixel_flags(fp16, rgba8), frame.ctypes.data_as(ctypes.c_void_p)))
    return frame


@dataclass
class Options:
    """rt_create_options (include/rtpt.h): per-context, speed-only choices --
    none changes a rendered value.  Defaults are the library's measured best.
    ``layout`` in ``LAYOUTS`` (auto, pairs, single, global, pairsmem, sorted,
    bvh), ``tri_build`` in ``TRI_BUILDS`` (default, host, lbvh, gpusah),
    ``walk`` in ``WALKS`` (auto, lockstep, free, sorted);
    ``walk_leaf_den`` the free scheduler's leaf-round threshold (0 = default)."""

    layout: str = "auto"
    lanes: int = 0
    tri_build: str = "default"
    tri_leaf_max: int = 0
    tri_leaf_cost: float = 0.0
    sphere_leaf_max: int = 0
    sphere_median: bool = False
    walk: str = "auto"
    walk_leaf_den: int = 0

    def c(self) -> CreateOptions:
        o = CreateOptions()
        o.scene_layout = LAYOUTS[self.layout]
        o.lanes_per_pixel = self.lanes
        o.tri_bvh_build = TRI_BUILDS[self.tri_build]
        o.tri_leaf_max = self.tri_leaf_max
        o.tri_leaf_cost = self.tri_leaf_cost
        o.sphere_leaf_max = self.sphere_leaf_max
        o.sphere_median = 1 if self.sphere_median else 0
        o.walk_scheduler = WALKS[self.walk]
        o.walk_leaf_den = self.walk_leaf_den
        return o

    # tools and the bench take their A/B knobs from the environment; the
    # library itself reads none (a stray variable cannot change a context)
    _ENV = {"layout": "RTPT_SCENE_MEM", "lanes": "RTPT_LANES", "tri_build": "RTPT_TRI_BUILD",
            "tri_leaf_max": "RTPT_TRI_LEAF", "tri_leaf_cost": "RTPT_TRI_CT",
            "sphere_leaf_max": "RTPT_BVH_LEAF", "walk": "RTPT_WALK"}

    @classmethod
    def from_env(cls, env=None) -> "Options":
        """Options from RTPT_* variables (bench.py / tools only)."""
        env = os.environ if env is None else env
        o = cls()
        for f in fields(cls):
            v = env.get(cls._ENV.get(f.name, ""))
            if v:
                setattr(o, f.name, type(getattr(o, f.name))(v) if f.type != "str" else v)
        if env.get("RTPT_BVH_SAH") == "0":
            o.sphere_median = True
        return o


class Scene:
    """The shaderTypes.h arrays of one scene (what Renderer.init uploads)."""

    def __init__(self, camera: CameraGPU, materials, vertices, light: SquareLightGPU,
                 spheres=None):
        self.camera = camera
        self.materials = materials            # (MaterialGPU * n_tri)
        self.vertices = vertices              # (float3 * 3n_tri), 16-B stride
        self.light = light
        self.spheres = spheres                # (SphereGPU * n_sph) or None

    @property
    def n_triangles(self) -> int:
        return len(self.materials)

    @property
    def n_spheres(self) -> int:
        return 0 if self.spheres is None else len(self.spheres)

    @property
    def width(self) -> int:
        return int(self.camera.resolution.x)

    @property
    def height(self) -> int:
        return int(self.camera.resolution.y)

    @classmethod
    def cornell_box(cls, width: int = 800, height: int = 600) -> "Scene":
        """initCornellBox() (scene.swift:14-62), resolution overridden."""
        cam, light = CameraGPU(), SquareLightGPU()
        mats = (MaterialGPU * 36)()
        verts = (float3 * 108)()
        n = ctypes.c_uint32()
        _check(lib.rt_scene_cornell_box(width, height, ctypes.byref(cam), mats, verts,
                                        ctypes.byref(light), ctypes.byref(n)))
        assert n.value == 36
        return cls(cam, mats, verts, light)

    @classmethod
    def cornell_box_mis(cls, width: int = 800, height: int = 600) -> "Scene":
        """The SwiftPM build's scene (Sources/gpuRaytracer/main.swift:21-67):
        the same room with a 1.5 x 1.5 light."""
        cam, light = CameraGPU(), SquareLightGPU()
        mats = (MaterialGPU * 36)()
        verts = (float3 * 108)()
        n = ctypes.c_uint32()
        _check(lib.rt_scene_cornell_box_mis(width, height, ctypes.byref(cam), mats, verts,
                                            ctypes.byref(light), ctypes.byref(n)))
        assert n.value == 36
        return cls(cam, mats, verts, light)

    @classmethod
    def random_spheres(cls, width: int = 1920, height: int = 1080, n_spheres: int = 1000,
                       seed: int = 42) -> "Scene":
        """Config-4 scene: Cornell walls + light + PCG32(seed) spheres."""
        cam, light = CameraGPU(), SquareLightGPU()
        mats = (MaterialGPU * 12)()
        verts = (float3 * 36)()
        sph = (SphereGPU * max(n_spheres, 1))()
        n = ctypes.c_uint32()
        _check(lib.rt_scene_random_spheres(width, height, n_spheres, ctypes.c_uint64(seed),
                                           ctypes.byref(cam), mats, verts, ctypes.byref(light),
                                           ctypes.byref(n), sph))
        return cls(cam, mats, verts, light, sph if n_spheres else None)

    @classmethod
    def random_triangles(cls, width: int = 1920, height: int = 1080, n: int = 100_000,
                         seed: int = 7, size: float = 0.25) -> "Scene":
        """Stress scene for the triangle BVH: the Cornell room (ids 0-35, light
        34-35) plus ``n`` random small triangles (ids 36..) inside it, diffuse
        albedo in [0.1, 0.9] (numpy PCG64 ``seed``)."""
        base = cls.cornell_box(width, height)
        rng = np.random.default_rng(seed)
        mats = (MaterialGPU * (36 + n))()
        verts = (float3 * (3 * (36 + n)))()
        ctypes.memmove(ctypes.addressof(mats), ctypes.addressof(base.materials), 36 * 48)
        ctypes.memmove(ctypes.addressof(verts), ctypes.addressof(base.vertices), 108 * 16)
        c = rng.uniform(-2.3, 2.3, size=(n, 1, 3)).astype(np.float32)
        e = rng.uniform(-size, size, size=(n, 2, 3)).astype(np.float32)
        tri = np.concatenate([c, c + e], axis=1).reshape(-1, 3)          # v0, v0+a, v0+b
        vv = np.frombuffer(verts, np.float32).reshape(-1, 4)
        vv[108:, :3] = tri
        mm = np.frombuffer(mats, np.float32).reshape(-1, 12)
        mm[36:, 0:3] = rng.uniform(0.1, 0.9, size=(n, 3)).astype(np.float32)
        mm[36:, 3] = 1.0
        mm[36:, 5] = 0.5
        return cls(base.camera, mats, verts, base.light)

    @classmethod
    def random_boxes(cls, width: int = 1920, height: int = 1080, n_boxes: int = 4,
                     seed: int = 3) -> "Scene":
        """Box-cluster stress scene: the Cornell room (walls = ids 0-9) plus
        ``n_boxes`` randomly rotated boxes (12 triangles each, one shared-edge
        pair per face) and the light rectangle last (numpy PCG64 ``seed``)."""
        base = cls.cornell_box(width, height)
        rng = np.random.default_rng(seed)
        n = 10 + 12 * n_boxes + 2
        mats = (MaterialGPU * n)()
        verts = (float3 * (3 * n))()
        ctypes.memmove(ctypes.addressof(mats), ctypes.addressof(base.materials), 10 * 48)
        ctypes.memmove(ctypes.addressof(verts), ctypes.addressof(base.vertices), 30 * 16)
        vv = np.frombuffer(verts, np.float32).reshape(-1, 4)
        mm = np.frombuffer(mats, np.float32).reshape(-1, 12)
        for b in range(n_boxes):
            c = rng.uniform(-1.8, 1.8, 3)
            h = rng.uniform(0.15, 0.7, 3)
            R, _ = np.linalg.qr(rng.normal(size=(3, 3)))
            col = rng.uniform(0.1, 0.9, 3)
            for f in range(6):
                a, s = f // 2, (1.0 if f % 2 else -1.0)
                i, j = (a + 1) % 3, (a + 2) % 3
                P = [c + s * h[a] * R[a] + u * h[i] * R[i] + v * h[j] * R[j]
                     for u, v in ((-1, -1), (1, -1), (1, 1), (-1, 1))]
                for t, tri in enumerate(((P[0], P[1], P[2]), (P[0], P[2], P[3]))):
                    k = 10 + 12 * b + 2 * f + t
                    vv[3 * k:3 * k + 3, :3] = np.array(tri, np.float32)
                    mm[k, 0:3] = col
                    mm[k, 3] = 1.0
                    mm[k, 5] = 0.5
        ctypes.memmove(ctypes.addressof(mats) + (n - 2) * 48, ctypes.addressof(base.materials) + 34 * 48, 96)
        ctypes.memmove(ctypes.addressof(verts) + 3 * (n - 2) * 16,
                       ctypes.addressof(base.vertices) + 3 * 34 * 16, 96)
        return cls(base.camera, mats, verts, base.light)

    def describe(self, options: Options | None = None) -> dict:
        """Device layout rt_create would choose (rt_scene_describe_ex).  It
        describes the lockstep kernels: with ``walk`` free or sorted a BVH
        scene runs another kernel (``Renderer.last_launch()`` names it and its
        LDS bytes)."""
        info = SceneInfo()
        opt = None if options is None else ctypes.byref(options.c())
        _check(lib.rt_scene_describe_ex(ctypes.byref(self.desc()), opt, ctypes.byref(info)))
        return {k: getattr(info, k) for k, _ in SceneInfo._fields_}

    def desc(self, device: int = 0) -> SceneDesc:
        d = SceneDesc()
        d.camera = ctypes.pointer(self.camera)
        d.materials = ctypes.cast(self.materials, ctypes.POINTER(MaterialGPU))
        d.square_lights = ctypes.pointer(self.light)
        d.n_square_lights = 1
        d.vertices = ctypes.cast(self.vertices, ctypes.POINTER(float3))
        d.n_triangles = self.n_triangles
        if self.spheres is not None:
            d.spheres = ctypes.cast(self.spheres, ctypes.POINTER(SphereGPU))
            d.n_spheres = self.n_spheres
        d.device = device
        return d


@dataclass
class RenderParams:
    """rt_render_params (include/rtpt.h)."""

    spp: int = 400          # raytrace.metal:24
    bounces: int = 3        # raytrace.metal:25
    sample_base: int = 0
    row_start: int = 0
    row_step: int = 1
    row_count: int = 0      # 0 = every row from row_start with row_step
    accumulate: bool = False
    keep_sum: bool = False
    fp16: bool = False
    rgba8: bool = False     # the fused image.swift:35-65 epilogue (RT_OUT_RGBA8)

    def c(self, flags: int = 0) -> RenderParamsC:
        p = RenderParamsC()
        p.spp, p.bounces, p.sample_base = self.spp, self.bounces, self.sample_base
        p.row_start, p.row_step, p.row_count = self.row_start, self.row_step, self.row_count
        p.accumulate = 1 if self.accumulate else 0
        p.flags = (flags | (RT_KEEP_SUM if self.keep_sum else 0) | (RT_OUT_FP16 if self.fp16 else 0)
                   | (RT_OUT_RGBA8 if self.rgba8 else 0))
        return p

    def rows(self, height: int) -> int:
        if self.row_count:
            return self.row_count
        step = self.row_step or 1
        return (height - 1 - self.row_start) // step + 1


@dataclass
class MisParams:
    """rt_mis_params (include/rtpt.h): kernel drawTriangle of the SwiftPM build."""

    camera_rays: int = 6    # cameraRaysPerPixel, Sources/gpuRaytracer/shaders.metal:644
    mis_samples: int = 300  # misSamples, :648
    row_start: int = 0
    row_step: int = 1
    row_count: int = 0

    def c(self, flags: int = 0) -> MisParamsC:
        p = MisParamsC()
        p.camera_rays, p.mis_samples = self.camera_rays, self.mis_samples
        p.row_start, p.row_step, p.row_count = self.row_start, self.row_step, self.row_count
        p.flags = flags
        return p

    def rows(self, height: int) -> int:
        return RenderParams(row_start=self.row_start, row_step=self.row_step,
                            row_count=self.row_count).rows(height)


class Renderer:
    """renderer.swift's Renderer on the MI355X C-ABI."""

    def __init__(self, scene: Scene, device: int = 0, seeds=None,
                 seed_key: int = DEFAULT_SEED_KEY, options: Options | None = None):
        self.scene = scene
        self.device = device
        self.options = options or Options()
        ctx = ctypes.c_void_p()
        _check(lib.rt_create_ex(ctypes.byref(scene.desc(device)), ctypes.byref(self.options.c()),
                                ctypes.byref(ctx)))
        self._ctx = ctx
        if seeds is not None:
            s = np.ascontiguousarray(seeds, dtype=np.uint32)
            if s.size != scene.width * scene.height:
                raise ValueError("seed texture must have width*height entries")
            _check(lib.rt_set_seeds(ctx, s.ctypes.data_as(ctypes.c_void_p), scene.width,
                                    scene.height), ctx)
        else:
            _check(lib.rt_fill_seeds(ctx, ctypes.c_uint64(seed_key)), ctx)

    def close(self):
        if getattr(self, "_ctx", None):
            lib.rt_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        self.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_seeds(self, seeds):
        s = np.ascontiguousarray(seeds, dtype=np.uint32)
        _check(lib.rt_set_seeds(self._ctx, s.ctypes.data_as(ctypes.c_void_p), self.scene.width,
                                self.scene.height), self._ctx)

    def render(self, params: RenderParams | None = None, out=None, stream=None):
        """Render into host memory (returns (rows, W, 4) float32, uint16 bits
        for fp16, uint8 for rgba8), or into a device tensor ``out`` (anything with
        ``data_ptr()``) enqueued on ``stream`` (a raw hipStream_t int / torch
        stream; default torch's current stream) without a host sync."""
        p = params or RenderParams()
        if out is None:
            rows = p.rows(self.scene.height)
            dt = np.uint8 if p.rgba8 else np.uint16 if p.fp16 else np.float32
            img = np.empty((rows, self.scene.width, 4), dtype=dt)
            _check(lib.rt_render(self._ctx, ctypes.byref(p.c()),
                                 img.ctypes.data_as(ctypes.c_void_p)), self._ctx)
            return img
        if stream is None:
            import torch  # plumbing only: the stream the caller's events see
            stream = torch.cuda.current_stream().cuda_stream
        elif hasattr(stream, "cuda_stream"):
            stream = stream.cuda_stream
        ptr = out if isinstance(out, int) else out.data_ptr()
        _check(lib.rt_render_async(self._ctx, ctypes.byref(p.c(RT_OUT_DEVICE)),
                                   ctypes.c_void_p(ptr), ctypes.c_void_p(stream)), self._ctx)
        return out

    def render_progressive(self, params: RenderParams, batch_spp: int, out, stream=None,
                           gather: bool = False):
        """Progressive accumulation: ``params.spp`` samples as
        launches of ``batch_spp`` samples into the context's running fp32 sums
        (``RT_KEEP_SUM`` / ``accumulate`` with ``sample_base`` advancing), all
        enqueued on ``stream``; the last launch writes the averaged frame to the
        device tensor ``out``.  Bit-identical to one launch of ``params.spp``.
        ``gather``: every launch goes through rt_render_gather (this rank's rows
        of the communicator's partition), the last one gathers the frame into
        ``out`` on rank 0 -- one RCCL gather per frame."""
        if stream is None:
            import torch
            stream = torch.cuda.current_stream().cuda_stream
        elif hasattr(stream, "cuda_stream"):
            stream = stream.cuda_stream
        total, done = params.spp, 0
        ptr = out if (out is None or isinstance(out, int)) else out.data_ptr()
        while done < total:
            n = min(batch_spp, total - done)
            last = done + n == total
            p = RenderParams(spp=n, bounces=params.bounces, sample_base=params.sample_base + done,
                             row_start=params.row_start, row_step=params.row_step,
                             row_count=params.row_count, accumulate=done > 0, keep_sum=True,
                             fp16=params.fp16, rgba8=params.rgba8)
            flags = RT_OUT_DEVICE if last else (RT_OUT_DEVICE | RT_OUT_NONE)
            fn = lib.rt_render_gather if gather else lib.rt_render_async
            _check(fn(self._ctx, ctypes.byref(p.c(flags)), ctypes.c_void_p(ptr if last else None),
                      ctypes.c_void_p(stream)), self._ctx)
            done += n
        return out

    def accumulate(self, params: RenderParams):
        """Add samples to the context's running sums only (no image output)."""
        _check(lib.rt_render(self._ctx, ctypes.byref(params.c(RT_OUT_NONE | RT_KEEP_SUM)), None),
               self._ctx)

    def draw(self, spp: int = 400, bounces: int = 3) -> np.ndarray:
        """Renderer.draw(): the whole frame, synchronously; (H, W, 4) float32."""
        return self.render(RenderParams(spp=spp, bounces=bounces))

    def render_mis(self, params: MisParams | None = None, out=None, out8=None):
        """MIS integrator (rt_render_mis).  Host: returns (sum, rgba8) with
        sum (rows, W, 4) float32 = (radiance summed over camera rays, camera
        rays) and rgba8 (rows, W, 4) uint8.  Device: pass tensors ``out`` and/or
        ``out8`` (anything with ``data_ptr()``); the call is synchronous."""
        p = params or MisParams()
        if out is None and out8 is None:
            rows = p.rows(self.scene.height)
            img = np.empty((rows, self.scene.width, 4), dtype=np.float32)
            img8 = np.empty((rows, self.scene.width, 4), dtype=np.uint8)
            _check(lib.rt_render_mis(self._ctx, ctypes.byref(p.c()),
                                     img.ctypes.data_as(ctypes.c_void_p),
                                     img8.ctypes.data_as(ctypes.c_void_p)), self._ctx)
            return img, img8
        ptr = lambda t: None if t is None else ctypes.c_void_p(t if isinstance(t, int) else t.data_ptr())  # noqa: E731
        _check(lib.rt_render_mis(self._ctx, ctypes.byref(p.c(RT_OUT_DEVICE)), ptr(out), ptr(out8)),
               self._ctx)
        return out, out8

    def comm_init(self, rank: int, world: int, comm_id: bytes):
        """rt_comm_init: join the world-rank RCCL communicator (collective)."""
        if len(comm_id) != RT_COMM_ID_BYTES:
            raise ValueError("comm_id must be the 128 bytes of rt_comm_unique_id()")
        buf = (ctypes.c_uint8 * RT_COMM_ID_BYTES).from_buffer_copy(comm_id)
        _check(lib.rt_comm_init(self._ctx, rank, world, buf), self._ctx)
        self.rank, self.world = rank, world

    def render_gather(self, params: RenderParams | None = None, out=None, stream=None):
        """rt_render_gather (collective): this rank renders rows y = rank (mod
        world), the tiles are gathered over RCCL into the frame on rank 0.
        Host: returns the (H, W, 4) frame on rank 0 (None elsewhere).  Device:
        ``out`` (rank 0; anything with ``data_ptr()``) is filled on ``stream``
        without a host sync."""
        p = params or RenderParams()
        if out is None:
            frame = None
            if getattr(self, "rank", 0) == 0 and not (p.c().flags & RT_OUT_NONE):
                dt = np.uint8 if p.rgba8 else np.uint16 if p.fp16 else np.float32
                frame = np.empty((self.scene.height, self.scene.width, 4), dtype=dt)
            ptr = None if frame is None else frame.ctypes.data_as(ctypes.c_void_p)
            _check(lib.rt_render_gather(self._ctx, ctypes.byref(p.c()), ptr, None), self._ctx)
            return frame
        if stream is None:
            import torch
            stream = torch.cuda.current_stream().cuda_stream
        elif hasattr(stream, "cuda_stream"):
            stream = stream.cuda_stream
        ptr = out if isinstance(out, int) else out.data_ptr()
        _check(lib.rt_render_gather(self._ctx, ctypes.byref(p.c(RT_OUT_DEVICE)), ctypes.c_void_p(ptr),
                                    ctypes.c_void_p(stream)), self._ctx)
        return out

    def comm_info(self) -> tuple[int, int]:
        """rt_comm_info: (ranks in the communicator, this rank) as RCCL reports them."""
        n, r = ctypes.c_int32(), ctypes.c_int32()
        _check(lib.rt_comm_info(self._ctx, ctypes.byref(n), ctypes.byref(r)), self._ctx)
        return n.value, r.value

    def place_tiles(self, gathered, world: int, out=None, fp16: bool = False, rgba8: bool = False,
                    stream=None):
        """rt_place_tiles: rank 0's placement step of rt_render_gather on a device
        buffer ``gathered`` (``world`` padded tiles back to back), ordered on
        ``stream`` (default: torch's current stream).  Returns the host frame
        (blocking), or fills the device tensor ``out`` without a host sync."""
        gp = gathered if isinstance(gathered, int) else gathered.data_ptr()
        flags = _pixel_flags(fp16, rgba8)
        if stream is None:
            import torch
            stream = torch.cuda.current_stream().cuda_stream
        elif hasattr(stream, "cuda_stream"):
            stream = stream.cuda_stream
        if out is None:  # host frame: ordered on `stream` too, then the call blocks
            dt = np.uint8 if rgba8 else np.uint16 if fp16 else np.float32
            frame = np.empty((self.scene.height, self.scene.width, 4), dt)
            _check(lib.rt_place_tiles(self._ctx, ctypes.c_void_p(gp), world, flags,
                                      frame.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(stream)),
                   self._ctx)
            return frame
        ptr = out if isinstance(out, int) else out.data_ptr()
        _check(lib.rt_place_tiles(self._ctx, ctypes.c_void_p(gp), world, flags | RT_OUT_DEVICE,
                                  ctypes.c_void_p(ptr), ctypes.c_void_p(stream)), self._ctx)
        return out

    def last_launch(self) -> dict:
        """The kernel instantiation and launch shape of the last render
        (rt_last_launch): kernel name as rocprofv3 reports it, lanes per
        pixel, whether the LDS Halton tables were filled, grid, LDS bytes."""
        info = LaunchInfo()
        _check(lib.rt_last_launch(self._ctx, ctypes.byref(info)), self._ctx)
        return info.as_dict()

    def build_info(self) -> dict:
        """rt_build_info: which triangle-BVH build ran (0 none, 1 host SAH, 2 GPU
        LBVH, 3 GPU SAH), its nodes per layout and the build / scene-compile
        wall times in ms."""
        b = BuildStats()
        _check(lib.rt_build_info(self._ctx, ctypes.byref(b)), self._ctx)
        return {k: getattr(b, k) for k, _ in BuildStats._fields_}

    def last_kernel_ms(self) -> float:
        ms = ctypes.c_float()
        _check(lib.rt_last_kernel_ms(self._ctx, ctypes.byref(ms)), self._ctx)
        return float(ms.value)

"""GPU parity: the gfx950 kernel through the C-ABI against the oracle.

Bar: bit-exact (the arithmetic contract of DESIGN.md §3 makes GPU == CPU
oracle exactly); the reported tolerance check (1e-5 relative, north_star) is
asserted as well so a failure message shows both.
All tests here call librtpt.so (the HIP path); nothing falls back to the CPU.
"""
import os

import numpy as np
import pytest

import oracle_lib
from gpuraytracer_amd import (CameraGPU, MaterialGPU, Options, RenderParams, Renderer, RtError, Scene,
                              SphereGPU, SquareLightGPU, float3, seed_splitmix)

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
REL_TOL = 1e-5  # north_star: "within 1e-5 relative"


def assert_parity(gpu, ref, what=""):
    gpu = np.asarray(gpu, np.float32)
    ref = np.asarray(ref, np.float32)
    assert gpu.shape == ref.shape, (gpu.shape, ref.shape)
    diff = gpu.view(np.uint32) != ref.view(np.uint32)
    if diff.any():
        rel = np.abs(gpu - ref) / np.maximum(np.abs(ref), 1e-30)
        idx = np.argwhere(diff)[:8].tolist()
        raise AssertionError(f"{what}: {int(diff.sum())} values differ (max rel {rel.max():.3g}) "
                             f"first at {idx}; within {REL_TOL}: {bool((rel <= REL_TOL).all())}")


def load_fixture(name):
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    cam = CameraGPU.from_buffer_copy(g["camera"].tobytes())
    light = SquareLightGPU.from_buffer_copy(g["light"].tobytes())
    mats = (MaterialGPU * (len(g["materials"]) // 48)).from_buffer_copy(g["materials"].tobytes())
    verts = (float3 * (len(g["vertices"]) // 16)).from_buffer_copy(g["vertices"].tobytes())
    sph = None
    if "spheres" in g:
        sph = (SphereGPU * (len(g["spheres"]) // 80)).from_buffer_copy(g["spheres"].tobytes())
    spp, bounces, base = (int(v) for v in g["params"])
    return Scene(cam, mats, verts, light, sph), g["seeds"], spp, bounces, base, g["out"]


@pytest.mark.parametrize("name", ["cornell_16x16_s4_b3", "cornell_128x128_s1_b3",
                                  "cornell_24x13_s3_b4_u32seeds", "spheres60_16x16_s2_b3"])
def test_golden_fixtures_bit_exact(name):
    scene, seeds, spp, bounces, base, expect = load_fixture(name)
    with Renderer(scene, seeds=seeds) as r:
        out = r.render(RenderParams(spp=spp, bounces=bounces, sample_base=base))
    assert_parity(out, expect, name)


@pytest.mark.parametrize("bounces", [0, 1, 2, 3, 4])
def test_cornell_vs_oracle_all_bounce_counts(bounces):
    s = Scene.cornell_box(72, 40)  # not a multiple of the 16x16 workgroup tile
    sd = seed_splitmix(72, 40, key=1234)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=5, bounces=bounces))
    assert_parity(out, oracle_lib.render(s, sd, 5, bounces), f"bounces={bounces}")


@pytest.mark.parametrize("top", [3 ** 13 - 1, 3 ** 13])
def test_halton_index_bound_edges(top):
    """Largest Halton index 3^13 - 1 (the fixed-digit kernels, kSmallIndexMax in
    rt_halton.hpp: 13 base-3 digits) and 3^13 (the generic loop), with indices
    spread over the base-3/5/11 top digits; both bit-exact vs the oracle."""
    spp = 8
    W, H = 40, 24
    rng = np.random.default_rng(top)
    sd = rng.integers(top - spp + 1 - 400000, top - spp + 2, (H, W), dtype=np.int64)
    sd[3, 7] = top - spp + 1  # max index = top
    sd = sd.astype(np.uint32)
    s = Scene.cornell_box(W, H)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=spp, bounces=3))
    assert_parity(out, oracle_lib.render(s, sd, spp, 3), f"top={top}")


def test_reference_default_800x600_rows_vs_oracle():
    """The reference's own configuration (800x600, 400 spp, 3 bounces,
    raytrace.metal:24-25 / scene.swift:18) — checked on a band of rows."""
    s = Scene.cornell_box(800, 600)
    with Renderer(s) as r:
        out = r.render(RenderParams(spp=400, bounces=3, row_start=297, row_count=3))
    sd = seed_splitmix(800, 600)
    assert_parity(out, oracle_lib.render(s, sd, 400, 3, row_start=297, row_count=3), "800x600x400")


def test_spheres_1000_vs_oracle():
    s = Scene.random_spheres(48, 32, 1000, seed=42)
    sd = seed_splitmix(48, 32)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=2, bounces=3))
    assert_parity(out, oracle_lib.render(s, sd, 2, 3), "spheres1000")


@pytest.mark.parametrize("leaf", ["2", "3", "8"])
def test_sphere_bvh_multi_sphere_leaves(leaf):
    # sphere_leaf_max > 1: leaves hold several spheres (the default is one per leaf)
    s = Scene.random_spheres(40, 24, 700, seed=5)
    sd = seed_splitmix(40, 24)
    with Renderer(s, seeds=sd, options=Options(sphere_leaf_max=int(leaf))) as r:
        out = r.render(RenderParams(spp=2, bounces=3))
    assert_parity(out, oracle_lib.render(s, sd, 2, 3), "leaf" + leaf)


def test_duplicate_spheres_tie_to_lower_id():
    # exact duplicates (same centre and radius, different albedo) hit at the same t:
    # the BVH walks must return the lower sphere id, as the id-ordered scan does
    s = Scene.random_spheres(40, 24, 300, seed=11)
    n = s.n_spheres
    for k in range(0, n - 1, 2):
        s.spheres[k + 1].center = s.spheres[k].center
        s.spheres[k + 1].radius = s.spheres[k].radius
        s.spheres[k + 1].material.diffuse.x = 0.05 + 0.9 * ((k * 37) % 17) / 17.0
    sd = seed_splitmix(40, 24)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=2, bounces=3))
    assert_parity(out, oracle_lib.render(s, sd, 2, 3), "duplicates")


@pytest.mark.parametrize("layout", ["auto", "pairs"])
def test_sphere_bvh_lds_and_global_walks_bit_exact(layout):
    """auto: the compact fp16 sphere BVH (8 octant layouts, near/far boxes,
    per-lane walks); pairs: the 32-B-node BVH read with scalar loads in the
    pair-record kernel.  Both are the oracle."""
    s = Scene.random_spheres(40, 24, 700, seed=13)
    sd = seed_splitmix(40, 24, key=13)
    with Renderer(s, seeds=sd, options=Options(layout=layout)) as r:
        out = r.render(RenderParams(spp=3, bounces=3))
    assert_parity(out, oracle_lib.render(s, sd, 3, 3), f"spheres700-{layout}")


def test_sphere_bvh_lds_fp16_boxes_far_spheres():
    """Spheres out to |x| ~ 7000 (fp16 box corners 4 units apart, rounded
    outward): the LDS walk must still return the brute-force hits."""
    s = Scene.random_spheres(40, 24, 200, seed=17)
    for k in range(0, 200, 2):  # every other sphere far away and large
        sp = s.spheres[k]
        sp.center.x, sp.center.y, sp.center.z = (sp.center.x * 2900.0, sp.center.y * 2900.0,
                                                 -abs(sp.center.z) * 2900.0 - 50.0)
        sp.radius = sp.radius * 2900.0
    assert s.describe()["sphere_kernel_lds_bytes"] > 0
    sd = seed_splitmix(40, 24, key=17)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=2, bounces=3))
    assert_parity(out, oracle_lib.render(s, sd, 2, 3), "far spheres")


def test_large_sphere_scene_bvh():
    # 5000 spheres: deep BVH (2047 nodes), ties and leaves far beyond the 1000-sphere case
    s = Scene.random_spheres(24, 16, 5000, seed=9)
    sd = seed_splitmix(24, 16)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=1, bounces=2))
    assert_parity(out, oracle_lib.render(s, sd, 1, 2), "spheres5000")


def test_row_tiles_equal_full_frame():
    s = Scene.cornell_box(64, 48)
    with Renderer(s) as r:
        full = r.render(RenderParams(spp=3))
        for start, step in [(0, 2), (1, 2), (3, 8), (47, 1)]:
            tile = r.render(RenderParams(spp=3, row_start=start, row_step=step))
            assert_parity(tile, full[start::step], f"tile {start}/{step}")


def test_progressive_batches_equal_single_shot():
    s = Scene.cornell_box(40, 24)
    with Renderer(s) as r:
        single = r.render(RenderParams(spp=10))
        r.accumulate(RenderParams(spp=3, keep_sum=True))
        r.accumulate(RenderParams(spp=4, sample_base=3, accumulate=True))
        last = r.render(RenderParams(spp=3, sample_base=7, accumulate=True))
    assert_parity(last, single, "progressive")


def test_fp16_output_matches_rounded_oracle():
    s = Scene.cornell_box(32, 16)
    with Renderer(s) as r:
        h = r.render(RenderParams(spp=4, fp16=True))
        f = r.render(RenderParams(spp=4))
    ref = f.astype(np.float16).view(np.uint16)  # IEEE round-to-nearest-even
    assert np.array_equal(h, ref)


def test_device_output_async_matches_host():
    import torch
    s = Scene.cornell_box(48, 32)
    with Renderer(s) as r:
        host = r.render(RenderParams(spp=2))
        dev = torch.empty((32, 48, 4), dtype=torch.float32, device="cuda:0")
        r.render(RenderParams(spp=2), out=dev)
        torch.cuda.synchronize()
        assert r.last_kernel_ms() > 0
    assert_parity(dev.cpu().numpy(), host, "device out")


def test_full_size_1080p_properties():
    """Config-2 frame size: batching is exact, a row band matches the oracle,
    the image is finite with alpha 1 and black outside the open box front."""
    s = Scene.cornell_box(1920, 1080)
    with Renderer(s) as r:
        one = r.render(RenderParams(spp=4))
        r.accumulate(RenderParams(spp=1, keep_sum=True))
        two = r.render(RenderParams(spp=3, sample_base=1, accumulate=True))
    assert_parity(two, one, "1080p batched")
    assert np.isfinite(one).all() and np.all(one[..., 3] == 1.0)
    assert np.all(one[:, :8, :3] == 0.0)  # left edge sees past the room (black)
    sd = seed_splitmix(1920, 1080)
    band = oracle_lib.render(s, sd, 4, 3, row_start=539, row_count=2)
    assert_parity(one[539:541], band, "1080p rows 539-540")


def test_full_frame_1080p_bit_exact_vs_oracle():
    """The headline workload's frame (config 2 geometry, 1920x1080, 3 bounces)
    at 8 spp, every pixel against the C oracle (~17 M samples on 16 host
    threads): box clusters and 4 lanes per pixel at full size.  8 spp is 2
    rounds per lane, below kHaltonTabMinRounds: the Halton tables are OFF here;
    the timed configuration with the tables on is checked by
    test_gpu_configs.py::test_headline_instantiation_*."""
    s = Scene.cornell_box(1920, 1080)
    sd = seed_splitmix(1920, 1080)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=8, bounces=3))
    ref = oracle_lib.render(s, sd, 8, 3, threads=16)
    assert_parity(out, ref, "1080p x 8 spp full frame")


def test_spheres_frame_bit_exact_vs_oracle():
    """Config-4 scene (1000 spheres, LDS SAH BVH) on a 240x135 frame x 8 spp."""
    s = Scene.random_spheres(240, 135, 1000, seed=42)
    sd = seed_splitmix(240, 135)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=8, bounces=3))
    ref = oracle_lib.render(s, sd, 8, 3, threads=16)
    assert_parity(out, ref, "spheres 240x135 x 8 spp")


def test_spheres_16_lanes_frame_and_rows_bit_exact_vs_oracle():
    """The config-4 launch shape: the LDS sphere-walk kernel takes 16 lanes per
    pixel whenever spp >= 16 (rt_kernel.hip lanes_per_pixel), whole frame and
    interleaved rows (one GPU's share of a multi-GPU frame)."""
    s = Scene.random_spheres(64, 40, 1000, seed=42)
    sd = seed_splitmix(64, 40)
    with Renderer(s, seeds=sd) as r:
        full = r.render(RenderParams(spp=20, bounces=3))
        assert r.last_launch()["lanes_per_pixel"] == 16
        assert "<3, 7, true, true, 16>" in r.last_launch()["kernel"]
        tile = r.render(RenderParams(spp=20, bounces=3, row_start=3, row_step=8))
    ref = oracle_lib.render(s, sd, 20, 3, threads=16)
    assert_parity(full, ref, "spheres 64x40 x 20 spp, 16 lanes")
    assert_parity(tile, ref[3::8], "spheres rows 3::8, 16 lanes")


def test_mixed_scene_sphere_kernel_and_pair_fallback_bit_exact():
    """Cornell box (36 triangles, both boxes) + 300 spheres: the one-wave sphere
    kernel; with 37 more quads (55 pairs, over the 6 KB per-workgroup budget) the
    pair kernel with the 32-B-node sphere walks.  Both are the oracle."""
    from test_abi import _with_quads
    base = Scene.cornell_box(48, 32)
    sph = Scene.random_spheres(48, 32, 300, seed=21).spheres
    sd = seed_splitmix(48, 32, key=21)
    for n_quads, sphere_kernel in ((0, True), (36, True), (37, False)):
        if n_quads:
            mats, verts = _with_quads(base, n_quads)
            s = Scene(base.camera, mats, verts, base.light, sph)
        else:
            s = Scene(base.camera, base.materials, base.vertices, base.light, sph)
        with Renderer(s, seeds=sd) as r:
            out = r.render(RenderParams(spp=3, bounces=3))
            k = r.last_launch()["kernel"]
        assert (k.startswith("rt::path_trace_kernel<3, 7,") or k.startswith("rt::path_trace_kernel<3, 8,")) == sphere_kernel, k
        assert_parity(out, oracle_lib.render(s, sd, 3, 3), f"mixed +{n_quads} quads")


def test_errors_are_status_codes():
    s = Scene.cornell_box(16, 8)
    with Renderer(s) as r:
        with pytest.raises(RtError) as e:
            r.render(RenderParams(spp=1, bounces=5))
        assert e.value.status == 1
        with pytest.raises(RtError) as e:
            r.render(RenderParams(spp=1, accumulate=True, sample_base=4))
        assert e.value.status == 5
        with pytest.raises(RtError):
            r.render(RenderParams(spp=1, row_start=8))
        out = r.render(RenderParams(spp=1))  # context still usable
        assert out.shape == (8, 16, 4)


@pytest.mark.parametrize("layout", ["single", "smem", "sorted", "pairsmem", "bvh", "pairs"])
def test_alternate_scene_layouts_bit_exact(layout):
    """The single-triangle LDS layout, the global (scalar-load) layout and the
    octant-sorted path kernel give the same bits as the default pair kernel
    and the oracle."""
    s = Scene.cornell_box(56, 40)
    sd = seed_splitmix(56, 40, key=99)
    with Renderer(s, seeds=sd, options=Options(layout=layout)) as r:
        out = r.render(RenderParams(spp=3, bounces=3))
    assert_parity(out, oracle_lib.render(s, sd, 3, 3), layout)


def random_quad_scene(w, h, n_quads, seed, twist=0.0):
    """Cornell camera/light + random planar-ish quads as shared-edge pairs:
    stresses the pair layout and the conservative segment culling.  twist > 0
    lifts the 4th corner of every other quad off its plane (such a quad is in
    no box cluster: every lane tests it)."""
    base = Scene.cornell_box(w, h)
    rng = np.random.default_rng(seed)
    n = 2 * n_quads + 2
    mats = (MaterialGPU * n)()
    verts = (float3 * (3 * n))()
    for q in range(n_quads):
        c = rng.uniform(-2.2, 2.2, 3)
        a, b = rng.normal(size=3), rng.normal(size=3)
        a *= rng.uniform(0.05, 1.5) / np.linalg.norm(a)
        b *= rng.uniform(0.05, 1.5) / np.linalg.norm(b)
        P = [c, c + a, c + a + b, c + b]
        if twist and q % 2:
            P[3] = P[3] + twist * np.cross(a, b) / np.linalg.norm(np.cross(a, b))
        for t, tri in enumerate([(P[0], P[1], P[2]), (P[0], P[2], P[3])]):
            k = 2 * q + t
            for v in range(3):
                verts[3 * k + v].x, verts[3 * k + v].y, verts[3 * k + v].z = (float(x) for x in tri[v])
            col = rng.uniform(0.1, 0.9, 3)
            mats[k].diffuse.x, mats[k].diffuse.y, mats[k].diffuse.z, mats[k].diffuse.w = (*col, 1.0)
    for t in range(2):  # keep the emissive light pair (ids 34, 35 of the Cornell scene)
        k = 2 * n_quads + t
        mats[k] = base.materials[34 + t]
        for v in range(3):
            verts[3 * k + v] = base.vertices[3 * (34 + t) + v]
    return Scene(base.camera, mats, verts, base.light)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_random_quads_pair_layout_and_culling_bit_exact(seed):
    s = random_quad_scene(48, 32, 25, seed)
    assert s.describe()["n_triangle_pairs"] == 26
    sd = seed_splitmix(48, 32, key=seed)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=16, bounces=4))
    assert_parity(out, oracle_lib.render(s, sd, 16, 4), f"quads seed {seed}")


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_random_rotated_boxes_clusters_bit_exact(seed):
    """Box clusters on 4 randomly rotated boxes in the room:
    the per-lane slab test + candidate faces must give the brute-force bits."""
    s = Scene.random_boxes(48, 32, 4, seed=seed)
    assert s.describe()["n_box_clusters"] == 6
    sd = seed_splitmix(48, 32, key=100 + seed)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=4, bounces=4))
    assert_parity(out, oracle_lib.render(s, sd, 4, 4), f"boxes{seed}")


@pytest.mark.parametrize("seed", [4, 5])
def test_twisted_quads_free_pairs_and_clusters_bit_exact(seed):
    """Non-planar quads fall out of the box clusters (tested by every lane),
    planar ones form flat clusters: both kinds in one query."""
    s = random_quad_scene(48, 32, 20, seed, twist=0.2)
    info = s.describe()
    assert info["pair_free_mask"] != 0 and info["n_box_clusters"] > 0
    sd = seed_splitmix(48, 32, key=seed)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=4, bounces=4))
    assert_parity(out, oracle_lib.render(s, sd, 4, 4), f"twisted{seed}")


def test_render_progressive_async_equals_single_shot():
    import torch
    s = Scene.cornell_box(48, 32)
    with Renderer(s) as r:
        one = r.render(RenderParams(spp=10, bounces=3))
        d = torch.empty((32, 48, 4), dtype=torch.float32, device="cuda")
        r.render_progressive(RenderParams(spp=10, bounces=3), 4, out=d)
        torch.cuda.synchronize()
        tiles = torch.empty((11, 48, 4), dtype=torch.float32, device="cuda")
        r.render_progressive(RenderParams(spp=10, bounces=3, row_start=1, row_step=3), 3,
                             out=tiles)
        torch.cuda.synchronize()
    assert_parity(d.cpu().numpy(), one, "progressive")
    assert_parity(tiles.cpu().numpy(), one[1::3], "progressive tiles")


def triangle_soup(w, h, n, seed, dup=False):
    """Cornell room + n random small triangles (ids 36..): beyond the LDS layouts,
    so rt_create builds the triangle BVH on the GPU (rt_lbvh.hip)."""
    base = Scene.cornell_box(w, h)
    rng = np.random.default_rng(seed)
    mats = (MaterialGPU * (36 + n))()
    verts = (float3 * (3 * (36 + n)))()
    ctypes_memmove(mats, base.materials, 36 * 48)
    ctypes_memmove(verts, base.vertices, 108 * 16)
    c = rng.uniform(-2.3, 2.3, size=(n, 3)).astype(np.float32)
    if dup:  # every odd triangle repeats the previous one (ties at equal t)
        c[1::2] = c[0::2][: len(c[1::2])]
    for k in range(n):
        e = rng.uniform(-0.25, 0.25, size=(2, 3)).astype(np.float32)
        if dup and k % 2 == 1:
            pv = [verts[3 * (36 + k - 1) + j] for j in range(3)]
            for j in range(3):
                verts[3 * (36 + k) + j].x, verts[3 * (36 + k) + j].y, verts[3 * (36 + k) + j].z = pv[j].x, pv[j].y, pv[j].z
        else:
            for j, p in enumerate((c[k], c[k] + e[0], c[k] + e[1])):
                verts[3 * (36 + k) + j].x, verts[3 * (36 + k) + j].y, verts[3 * (36 + k) + j].z = (float(v) for v in p)
        m = mats[36 + k]
        m.diffuse.x, m.diffuse.y, m.diffuse.z = (float(v) for v in rng.uniform(0.1, 0.9, 3))
        m.diffuse.w = 1.0
        m.roughness = 0.5
    return Scene(base.camera, mats, verts, base.light)


def ctypes_memmove(dst, src, n):
    import ctypes
    ctypes.memmove(ctypes.addressof(dst), ctypes.addressof(src), n)


TRI_BUILD_OPTIONS = {
    "host": Options(tri_build="host"),
    "lbvh": Options(tri_build="lbvh"),
    # leaves of up to 4 triangles (word first | (count - 1) << 24): the count > 1
    # loops of tri_leaf_closest / tri_leaf_any in the packet and parked-leaf walks
    "host_leaf4": Options(tri_build="host", tri_leaf_max=4, tri_leaf_cost=2.0),
    "gpusah": Options(tri_build="gpusah"),
    "gpusah_leaf4": Options(tri_build="gpusah", tri_leaf_max=4, tri_leaf_cost=2.0),
}
BUILD_CODE = {"host": 1, "lbvh": 2, "gpusah": 3}


@pytest.mark.parametrize("build", list(TRI_BUILD_OPTIONS))
@pytest.mark.parametrize("n,dup", [(3000, False), (2500, True)])
def test_triangle_bvh_gpu_build_bit_exact(n, dup, build):
    """Every triangle-BVH build -- the host binned-SAH tree, the GPU Morton
    LBVH (rt_lbvh.hip), the GPU binned SAH (rt_gsah.hip) and multi-triangle
    leaves -- in the same compact layout, against the oracle."""
    s = triangle_soup(40, 24, n, seed=n, dup=dup)
    assert s.describe()["lds_bytes"] == 0  # does not fit LDS: the BVH path
    sd = seed_splitmix(40, 24)
    with Renderer(s, seeds=sd, options=TRI_BUILD_OPTIONS[build]) as r:
        out = r.render(RenderParams(spp=2, bounces=3))
        info = r.build_info()
    assert info["tri_bvh_build"] == BUILD_CODE[build.split("_")[0]], info
    total = 2 * (n + 36) - 1
    assert (info["tri_bvh_nodes"] == total) if "leaf4" not in build else (info["tri_bvh_nodes"] < total), info
    assert_parity(out, oracle_lib.render(s, sd, 2, 3), f"soup{n}")


def test_gpu_sah_1m_triangles_bounded_temporaries():
    """1M triangles: the GPU SAH build gives bin slots (2,688 B) only to nodes
    that can split, at most 65,536 at a time (the deep levels run in batches),
    so its peak temporary device memory stays ~0.5 GB (round 5: one slot per
    node of a level, doubling: 2.7-5.4 GB).  The batched build is the host
    SAH's tree: same node count, and the frames rendered on both trees agree
    bit for bit (each walk returns the brute-force (t, id) answer)."""
    n = 1_000_000
    s = Scene.random_triangles(64, 48, n)
    sd = seed_splitmix(64, 48)
    p = RenderParams(spp=2, bounces=3)
    with Renderer(s, seeds=sd, options=Options(tri_build="gpusah")) as r:
        info = r.build_info()
        gpu = r.render(p)
    with Renderer(s, seeds=sd, options=Options(tri_build="host")) as r:
        host_info = r.build_info()
        host = r.render(p)
    assert info["tri_bvh_build"] == 3 and host_info["tri_bvh_build"] == 1, (info, host_info)
    assert info["tri_bvh_nodes"] == host_info["tri_bvh_nodes"] == 2 * (n + 36) - 1, (info, host_info)
    assert 0 < info["tri_bvh_temp_kib"] * 1024 < 600e6, info
    assert host_info["tri_bvh_temp_kib"] == 0
    assert np.array_equal(gpu.view(np.uint32), host.view(np.uint32))


@pytest.mark.parametrize("build", ["gpusah", "host"])
def test_triangle_bvh_coincident_centroids(build):
    """600 copies of one small triangle (every centroid in one point: the SAH
    builds split such a node by index) plus the room: bit-exact, ties to the
    lower id, and the GPU build reports 2n - 1 nodes."""
    base = Scene.cornell_box(40, 24)
    n = 36 + 600
    mats = (MaterialGPU * n)()
    verts = (float3 * (3 * n))()
    ctypes_memmove(mats, base.materials, 36 * 48)
    ctypes_memmove(verts, base.vertices, 108 * 16)
    for k in range(36, n):
        for j, p in enumerate(((0.1, -0.5, 0.2), (0.35, -0.45, 0.25), (0.15, -0.2, 0.1))):
            verts[3 * k + j].x, verts[3 * k + j].y, verts[3 * k + j].z = p
        m = mats[k]
        m.diffuse.x, m.diffuse.y, m.diffuse.z, m.diffuse.w = 0.2 + 0.6 * (k % 7) / 7.0, 0.5, 0.5, 1.0
    s = Scene(base.camera, mats, verts, base.light)
    sd = seed_splitmix(40, 24)
    with Renderer(s, seeds=sd, options=Options(tri_build=build)) as r:
        out = r.render(RenderParams(spp=3, bounces=3))
        info = r.build_info()
    assert info["tri_bvh_nodes"] == 2 * n - 1, info
    assert_parity(out, oracle_lib.render(s, sd, 3, 3), f"coincident {build}")


def test_triangle_bvh_forced_on_cornell_and_mis(monkeypatch):
    s = Scene.cornell_box(64, 48)
    sd = seed_splitmix(64, 48)
    with Renderer(s, seeds=sd, options=Options(layout="bvh")) as r:
        out = r.render(RenderParams(spp=3, bounces=4))
    assert_parity(out, oracle_lib.render(s, sd, 3, 4), "bvh cornell")
    from gpuraytracer_amd import MisParams
    m = Scene.cornell_box_mis(40, 24)
    with Renderer(m, options=Options(layout="bvh")) as r:
        got, got8 = r.render_mis(MisParams(camera_rays=2, mis_samples=12))
    ref, ref8 = oracle_lib.render_mis(m, 2, 12)
    assert_parity(got, ref, "bvh mis")
    assert np.array_equal(got8, ref8)


@pytest.mark.parametrize("lanes", ["1", "4", "16", "auto"])
def test_lanes_per_pixel_and_interleaved_rows_bit_exact(lanes):
    # 1, 4 or 16 lanes per pixel (samples shuffled back into sample order) and
    # one-row wave tiles for interleaved rows all give the oracle's sums
    s = Scene.cornell_box(56, 40)
    sd = seed_splitmix(56, 40)
    with Renderer(s, seeds=sd, options=Options(lanes=0 if lanes == "auto" else int(lanes))) as r:
        full = r.render(RenderParams(spp=19, bounces=3))
        tile = r.render(RenderParams(spp=19, bounces=3, row_start=2, row_step=5))
    ref = oracle_lib.render(s, sd, 19, 3)
    assert_parity(full, ref, "lanes" + lanes)
    assert_parity(tile, ref[2::5], "tile lanes" + lanes)


@pytest.mark.parametrize("mem", [None, "bvh", "spheres"])
def test_zero_light_terms_black_materials_bit_exact(mem):
    """Lanes whose light term is exactly 0 skip their shadow query (DESIGN.md
    §3.14): black boxes and a black wall make whole paths carry a zero
    throughput (every later light term is 0), and the ceiling and the light's
    back side give zero terms on lit materials.  Box clusters, the triangle BVH
    (bounce 0 on wave packets, which keep the query) and the sphere kernel
    (half the spheres black)."""
    s = Scene.cornell_box(48, 32)
    mats = s.materials
    for k in list(range(0, 2)) + list(range(10, 34)):  # a wall and both boxes
        mats[k].diffuse.x = mats[k].diffuse.y = mats[k].diffuse.z = 0.0
    sph = None
    if mem == "spheres":
        sph = Scene.random_spheres(48, 32, 300, seed=5).spheres
        for k in range(0, 300, 2):
            m = sph[k].material
            m.diffuse.x = m.diffuse.y = m.diffuse.z = 0.0
    scene = Scene(s.camera, mats, s.vertices, s.light, sph)
    sd = seed_splitmix(48, 32, key=9)
    with Renderer(scene, seeds=sd, options=Options(layout="bvh" if mem == "bvh" else "auto")) as r:
        out = r.render(RenderParams(spp=4, bounces=3))
    assert_parity(out, oracle_lib.render(scene, sd, 4, 3), f"black materials {mem}")
    assert np.isfinite(out).all()


@pytest.mark.parametrize("case", range(13))
def test_launch_lds_equals_staged_bytes_per_layout(case):
    """Every kernel layout: the launch requests exactly the dynamic LDS
    rt_scene_describe_ex reports (staged_lds_bytes: what its staging loops
    write) and renders bit-exact.  tests/test_abi.py restates the bytes per
    layout on the CPU; an -DRT_LDS_CHECK build also checks them inside the
    kernels against the dispatch's LDS."""
    from test_abi import LAYOUT_CASES, layout_scene
    name, opt, layout, lds = LAYOUT_CASES[case]
    s = layout_scene(name)
    assert s.describe(Options(**opt))["kernel_lds_bytes"] == lds
    sd = seed_splitmix(48, 32)
    with Renderer(s, seeds=sd, options=Options(**opt)) as r:
        out = r.render(RenderParams(spp=2, bounces=3))
        info = r.last_launch()
    assert info["lds_bytes"] == lds, (info, layout)
    assert_parity(out, oracle_lib.render(s, sd, 2, 3), f"layout {layout}")


def test_short_sqrt_and_reciprocal_equal_ieee_on_every_float():
    """The kernels' sqrt_cr / rcp_cr (rt_math.h: a hardware rsq / rcp plus a
    refinement, taken when every lane's argument is in [2^-100, 2^100)) equal the
    IEEE sqrtf and 1/x -- the oracle's arithmetic -- on all 2^32 float bit
    patterns (NaN results compare as NaN)."""
    import ctypes
    from gpuraytracer_amd import lib
    bad = (ctypes.c_uint64 * 2)()
    assert lib.rt_math_selfcheck(bad) == 0
    assert list(bad) == [0, 0], list(bad)


@pytest.mark.parametrize("comp", ["x", "y", "z"])
def test_light_center_signed_zero(comp):
    """shade() drops the zero terms of the light sample point (0*ux, 0*uy)
    unless the light centre has a -0 y or z (the host's light_plain flag): a
    centre component of -0 (the literal form for y, z; the short form for x)
    and of +0 stay bit-exact vs the oracle."""
    s = Scene.cornell_box(40, 24)
    for val in (-0.0, 0.0):
        setattr(s.light.center, comp, val)
        sd = seed_splitmix(40, 24, key=3)
        with Renderer(s, seeds=sd) as r:
            out = r.render(RenderParams(spp=4, bounces=3))
        assert_parity(out, oracle_lib.render(s, sd, 4, 3), f"light centre {comp}={val}")

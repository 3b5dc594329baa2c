"""CPU: the oracle against known answers, the independent numpy restatement,
the committed golden fixtures, and the reference's own PNG geometry."""
import ctypes
import json
import math
import os

import numpy as np
import pytest

import oracle_lib
from gpuraytracer_amd import Scene, seed_splitmix

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
L = oracle_lib.lib
F3 = ctypes.c_float * 3


def f3(*v):
    return F3(*v)


# ---- halton (sampling.metal:107-122) ---------------------------------------
@pytest.mark.parametrize("i,d,expect", [
    (0, 0, 0.0), (1, 0, 0.5), (2, 0, 0.25), (3, 0, 0.75), (4, 0, 0.125),
    (1, 1, np.float32(1 / 3)), (2, 1, np.float32(2 / 3)),
    (3, 1, np.float32(1 / 3) * np.float32(1 / 3)),  # f = invB*invB rounded in fp32
    (1, 2, np.float32(0.2)),
])
def test_halton_known_answers(i, d, expect):
    assert np.float32(oracle_lib.halton(i, d)) == np.float32(expect)


def test_halton_base2_is_bit_reversal():
    # for base 2 every partial sum is exact: radical inverse == bitreverse(i) / 2^32
    for i in [1, 5, 123457, 2**20 - 1, 2**23 + 11]:
        rev = int(f"{i:032b}"[::-1], 2)
        assert np.float32(oracle_lib.halton(i, 0)) == np.float32(rev / 2.0**32)


def test_halton_loop_order_matches_numpy():
    import pt_oracle_np as P
    i = np.array([0, 1, 7, 999, 2**20 - 1, 2**20 + 399, 2**31 + 5, 2**32 - 1], np.uint32)
    for d in range(24):
        c = np.array([oracle_lib.halton(int(v), d) for v in i], np.float32)
        assert np.array_equal(c.view(np.uint32), P.halton(i, d).view(np.uint32)), d


# ---- portable sincos ---------------------------------------------------------
def test_sincos_accuracy_and_quadrants():
    s, c = ctypes.c_float(), ctypes.c_float()
    xs = np.linspace(0, 2 * np.pi, 20001, dtype=np.float32)
    err = 0.0
    for x in xs[::7]:
        L.pto_sincos(ctypes.c_float(x), ctypes.byref(s), ctypes.byref(c))
        err = max(err, abs(s.value - math.sin(float(x))), abs(c.value - math.cos(float(x))))
    assert err < 4e-7
    L.pto_sincos(ctypes.c_float(0.0), ctypes.byref(s), ctypes.byref(c))
    assert (s.value, c.value) == (0.0, 1.0)


def test_sincos_matches_numpy_restatement():
    import pt_oracle_np as P
    xs = (np.random.default_rng(1).random(4000) * np.float32(6.28318548)).astype(np.float32)
    sn, cn = P.sincos(xs)
    s, c = ctypes.c_float(), ctypes.c_float()
    for k, x in enumerate(xs):
        L.pto_sincos(ctypes.c_float(x), ctypes.byref(s), ctypes.byref(c))
        assert np.float32(s.value) == sn[k] and np.float32(c.value) == cn[k]


# ---- ray / primitive tests ---------------------------------------------------
def tri(o, d, v0, v1, v2, tmin=0.001, tmax=1000.0):
    t = ctypes.c_float()
    L.pto_ray_triangle.restype = ctypes.c_int
    L.pto_ray_triangle.argtypes = [F3, F3, F3, F3, F3, ctypes.c_float, ctypes.c_float,
                                   ctypes.POINTER(ctypes.c_float)]
    hit = L.pto_ray_triangle(f3(*o), f3(*d), f3(*v0), f3(*v1), f3(*v2), tmin, tmax, ctypes.byref(t))
    return hit, t.value


def test_ray_triangle_hit_miss_and_both_faces():
    v0, v1, v2 = (0, 0, 0), (1, 0, 0), (0, 1, 0)
    hit, t = tri((0.25, 0.25, 5), (0, 0, -1), v0, v1, v2)
    assert hit and t == 5.0
    hit, t = tri((0.25, 0.25, -5), (0, 0, 1), v0, v1, v2)   # back face: no culling
    assert hit and t == 5.0
    assert not tri((0.8, 0.8, 5), (0, 0, -1), v0, v1, v2)[0]  # outside u+v<=1
    assert not tri((0.25, 0.25, 5), (1, 0, 0), v0, v1, v2)[0]  # parallel: det == 0
    assert not tri((0.25, 0.25, 5), (0, 0, 1), v0, v1, v2)[0]  # behind origin
    assert not tri((0.25, 0.25, 5), (0, 0, -1), v0, v1, v2, tmax=5.0)[0]  # t < tmax strict
    hit, _ = tri((0.0, 0.0, 5), (0, 0, -1), v0, v1, v2)      # vertex: edges inclusive
    assert hit


def sph(o, d, c, r, tmin=0.001, tmax=1000.0):
    t = ctypes.c_float()
    L.pto_ray_sphere.restype = ctypes.c_int
    L.pto_ray_sphere.argtypes = [F3, F3, F3, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                 ctypes.POINTER(ctypes.c_float)]
    return L.pto_ray_sphere(f3(*o), f3(*d), f3(*c), r, tmin, tmax, ctypes.byref(t)), t.value


def test_ray_sphere_front_inside_behind_tangent():
    hit, t = sph((0, 0, 5), (0, 0, -1), (0, 0, 0), 1.0)
    assert hit and t == 4.0
    hit, t = sph((0, 0, 0), (0, 0, -1), (0, 0, 0), 1.0)       # inside: far root (corrected rule)
    assert hit and t == 1.0
    assert not sph((0, 0, 5), (0, 0, 1), (0, 0, 0), 1.0)[0]    # sphere behind the ray
    assert not sph((1, 0, 5), (0, 0, -1), (0, 0, 0), 1.0)[0]   # tangent: disc == 0 is a miss
    hit, t = sph((0, 0, 5), (0, 0, -2), (0, 0, 0), 1.0)       # un-normalised direction
    assert hit and t == 2.0


# ---- camera / light / cosine sample ----------------------------------------------
def test_camera_center_and_corner_rays():
    cam, *_ = oracle_lib.cornell_box(800, 600)
    d = F3()
    L.pto_camera_ray.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_float,
                                 ctypes.c_float, F3]
    L.pto_camera_ray(ctypes.byref(cam), 400, 300, 0.0, 0.0, d)
    assert list(d) == [0.0, 0.0, -1.0]                          # basis u=(1,0,0) v=(0,1,0) w=(0,0,1)
    L.pto_camera_ray(ctypes.byref(cam), 0, 0, 0.0, 0.0, d)
    hw = np.float32(math.tan(np.float32(np.float32(3.1415925) / 4) / 2))
    # aspect = float(800/600) = 1 (integer division, sampling.metal:132) -> halfH == halfW
    v = np.array([-hw, hw, -1.0]) / np.linalg.norm([-hw, hw, -1.0])
    assert np.allclose(list(d), v, atol=1e-6)


def test_area_light_directly_below():
    _, _, _, light, _ = oracle_lib.cornell_box(8, 8)
    ldir, col, dist = F3(), F3(), ctypes.c_float()
    L.pto_sample_area_light.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_float, F3, F3,
                                        ctypes.POINTER(ctypes.c_float), F3]
    L.pto_sample_area_light(ctypes.byref(light), 0.5, 0.5, f3(0, 0.49, 0), ldir, ctypes.byref(dist), col)
    assert list(ldir) == [0.0, 1.0, 0.0] and np.float32(dist.value) == np.float32(2.0)
    # color = (1, .95, .9) / dist^2 * cos(0) (sampling.metal:226-233)
    assert np.allclose(list(col), np.array([1.0, 0.95, 0.9]) / 4.0, rtol=1e-6)


def test_cosine_sample_pole_is_normal():
    d = F3()
    L.pto_cosine_direction.argtypes = [ctypes.c_float, ctypes.c_float, F3, F3]
    for n in [(0, 1, 0), (1, 0, 0), (0, 0, -1)]:
        L.pto_cosine_direction(0.0, 1.0, f3(*n), d)
        assert np.allclose(list(d), n, atol=1e-7)


# ---- scene builders ---------------------------------------------------------------
def test_cornell_scene_matches_appendix_b():
    cam, mats, verts, light, n = oracle_lib.cornell_box(800, 600)
    assert n == 36
    v = np.frombuffer(bytes(verts), np.float32).reshape(108, 4)[:, :3]
    m = np.frombuffer(bytes(mats), np.float32).reshape(36, 12)
    assert np.array_equal(v[0:3], [[-2.5, -2.5, -2.5], [2.5, 2.5, -2.5], [-2.5, 2.5, -2.5]])
    ly = np.float32(2.5) - np.float32(0.01)  # lightY = half - 0.01 in Float (scene.swift:25)
    assert np.array_equal(v[102:105], np.array([[-0.5, ly, -0.5], [0.5, ly, -0.5], [0.5, ly, 0.5]],
                                               np.float32))
    assert np.allclose(m[2, :3], [0.9, 0, 0]) and np.allclose(m[4, :3], [0, 0.7, 0])   # red/green
    assert np.array_equal(m[34, 8:11], [1, 1, 1]) and np.all(m[:34, 8:11] == 0)          # emissive
    assert light.center.y == ly and light.color.y == np.float32(0.95)
    assert cam.resolution.x == 800 and cam.horizontalFov == np.float32(3.1415925) / 4
    # boxes inside the room in x/z; their bottoms sit 0.05 below the floor
    # (centre y = -half + h/2 - 0.05, scene.swift:144,160)
    assert np.abs(v[30:102][:, [0, 2]]).max() <= 2.5
    assert np.float32(v[30:66, 1].min()) == np.float32(-2.55)


def test_product_scene_builder_equals_oracle():
    for w, h in [(800, 600), (1920, 1080), (17, 9)]:
        s = Scene.cornell_box(w, h)
        cam, mats, verts, light, n = oracle_lib.cornell_box(w, h)
        assert bytes(s.camera) == bytes(cam)
        assert bytes(s.materials) == bytes(mats)
        assert bytes(s.vertices) == bytes(verts)
        assert bytes(s.light) == bytes(light)
    s = Scene.random_spheres(64, 32, 1000, seed=42)
    cam, mats, verts, light, n, sph_ = oracle_lib.random_spheres(64, 32, 1000, seed=42)
    assert n == 12 and bytes(s.vertices) == bytes(verts) and bytes(s.spheres) == bytes(sph_)
    r = np.frombuffer(bytes(sph_), np.float32).reshape(1000, 20)
    assert r[:, 16].min() >= 0.05 and r[:, 16].max() <= 0.2
    assert r[:, 0].min() >= -2.3 and r[:, 1].max() <= 2.2


def test_seed_function_matches_product_and_range():
    from gpuraytracer_amd import seed_splitmix
    a = oracle_lib.seeds(37, 11)
    b = seed_splitmix(37, 11)
    assert np.array_equal(a, b) and a.max() < 2**20 and len(np.unique(a)) > 390


# ---- renders ----------------------------------------------------------------------
def test_oracle_equals_numpy_restatement_8x8():
    import pt_oracle_np as P
    s = Scene.cornell_box(8, 8)
    sd = oracle_lib.seeds(8, 8)
    for bounces in (1, 2, 3, 4):
        out = oracle_lib.render(s, sd, 2, bounces)
        sc = P.Scene(s.camera, s.materials, s.light, s.vertices)
        ref = P.render(sc, sd, 2, bounces)
        assert np.array_equal(out.view(np.uint32), ref.view(np.uint32)), bounces


@pytest.mark.parametrize("name", ["cornell_16x16_s4_b3", "cornell_128x128_s1_b3",
                                  "cornell_24x13_s3_b4_u32seeds", "spheres60_16x16_s2_b3"])
def test_oracle_reproduces_golden(name):
    from gpuraytracer_amd import CameraGPU, MaterialGPU, SphereGPU, SquareLightGPU, float3
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    cam = CameraGPU.from_buffer_copy(g["camera"].tobytes())
    light = SquareLightGPU.from_buffer_copy(g["light"].tobytes())
    mats = (MaterialGPU * (len(g["materials"]) // 48)).from_buffer_copy(g["materials"].tobytes())
    verts = (float3 * (len(g["vertices"]) // 16)).from_buffer_copy(g["vertices"].tobytes())
    sph_ = None
    if "spheres" in g:
        sph_ = (SphereGPU * (len(g["spheres"]) // 80)).from_buffer_copy(g["spheres"].tobytes())
    s = Scene(cam, mats, verts, light, sph_)
    spp, bounces, base = (int(v) for v in g["params"])
    out = oracle_lib.render(s, g["seeds"], spp, bounces, sample_base=base)
    assert np.array_equal(out.view(np.uint32), g["out"].view(np.uint32))


def test_batched_equals_single_shot_and_rows():
    s = Scene.cornell_box(20, 12)
    sd = oracle_lib.seeds(20, 12)
    full = oracle_lib.render(s, sd, 6, 3)
    _, s1 = oracle_lib.render(s, sd, 2, 3, want_sum=True)
    _, s2 = oracle_lib.render(s, sd, 3, 3, sample_base=2, sum_in=s1, want_sum=True)
    out3 = oracle_lib.render(s, sd, 1, 3, sample_base=5, sum_in=s2)
    assert np.array_equal(out3.view(np.uint32), full.view(np.uint32))
    tile = oracle_lib.render(s, sd, 6, 3, row_start=1, row_step=3)
    assert np.array_equal(tile.view(np.uint32), full[1::3].view(np.uint32))


def test_light_footprint_matches_reference_png():
    """example.png (reference, README.md:1) is an earlier revision, but its
    light footprint pins the camera + light geometry of the live scene."""
    fp = json.load(open(os.path.join(GOLDEN, "footprint.json")))
    W, H = fp["width"], fp["height"]
    s = Scene.cornell_box(W, H)
    sd = oracle_lib.seeds(W, H)
    y0, y1 = fp["rows"]
    x0, x1 = fp["cols"]
    band = oracle_lib.render(s, sd, 1, 1, row_start=y0 - 6, row_count=(y1 - y0) + 13)
    lit = np.all(band[..., :3] == 1.0, axis=-1)  # emissive (1,1,1) overwrite on a light hit
    ys, xs = np.nonzero(lit)
    ys = ys + y0 - 6
    assert abs(int(ys.min()) - y0) <= 2 and abs(int(ys.max()) - y1) <= 2
    assert abs(int(xs.min()) - x0) <= 3 and abs(int(xs.max()) - x1) <= 3
    corner = oracle_lib.render(s, sd, 1, 3, row_count=1)[0, 0]
    assert np.all(corner[:3] == 0.0) and fp["corner_rgb"] == [0, 0, 0]


def test_tonemap_matches_image_swift():
    from gpuraytracer_amd import tonemap_rgba8
    x = np.random.default_rng(3).random((64, 4), dtype=np.float32) * 3
    x[0, :3] = [0.0, 1.0, 70000.0]  # fp16 overflow -> inf -> 1.0 -> 255
    a, b = tonemap_rgba8(x), oracle_lib.tonemap(x)
    assert np.array_equal(a, b)
    assert list(a[0]) == [0, 212, 255, 255]  # 1.0 -> (2/3)^(1/2.2)*255 = 212


def test_halton_float_digits():
    """rt_halton.hpp digit_step: with c = the smallest float >= 1/n (recip_up),
    q = floor(fl(x * c)) and digit = fma(q, -n, x) in fp32 are x / n and x mod n
    for every integer x < 2^21, for all 24 Halton bases and the low-digit table
    moduli b^k (kTabDigits, parsed from the header)."""
    import re
    src = open(os.path.join(os.path.dirname(GOLDEN), "..", "gpuraytracer_amd", "csrc",
                            "rt_halton.hpp")).read()
    K = [int(v) for v in re.search(r"kTabDigits\[24\] = \{([^}]*)\}", src).group(1).split(",")]
    primes = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61, 67, 71, 73,
              79, 83, 89]
    i = np.arange(1 << 21, dtype=np.int64)
    x = i.astype(np.float32)
    for d, b in enumerate(primes):
        for n in [b] + ([b ** K[d]] if K[d] else []):
            assert n < (1 << 23)
            c = np.float32(1) / np.float32(n)
            if float(c) * n < 1.0:  # exact in double: 24-bit x 23-bit
                c = np.nextafter(c, np.float32(2))
            q = np.floor(x * c)  # float32 product, rounded once
            digit = (x.astype(np.float64) - q.astype(np.float64) * n).astype(np.float32)  # fma: exact
            assert np.array_equal(q.astype(np.int64), i // n), (b, n)
            assert np.array_equal(digit.astype(np.int64), i % n), (b, n)


def test_halton_low_digit_split_is_the_reference_sum():
    """rt_halton.hpp halton_tab, emulated operation for operation in numpy
    float32 for every dimension with a table (kTabDigits parsed from the
    header): the table T[v] (fill_halton_table: k reference steps of v),
    i / b^k and i mod b^k by one float digit step with n = b^k, then the fixed
    nd = digits(b, 3^13) float digit steps (f from f_after(b, k)).  Equals the
    reference loop (sampling.metal:107-122, variable length) bit for bit on a
    stride of [0, 3^13) and its top index 3^13 - 1."""
    import re
    f32 = np.float32
    src = open(os.path.join(os.path.dirname(GOLDEN), "..", "gpuraytracer_amd", "csrc",
                            "rt_halton.hpp")).read()
    K = [int(v) for v in re.search(r"kTabDigits\[24\] = \{([^}]*)\}", src).group(1).split(",")]
    small_max = int(re.search(r"constexpr uint32_t kSmallIndexMax = (\d+);", src).group(1))
    assert small_max == 3 ** 13
    primes = [2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37, 41, 43, 47, 53, 59, 61, 67, 71, 73,
              79, 83, 89]

    def recip_up(n):
        c = f32(1) / f32(n)
        return np.nextafter(c, f32(2)) if float(c) * n < 1.0 else c

    def digit_step(x, n):  # q = floor(x * c), digit = fma(q, -n, x): exact integers
        q = np.floor(x * recip_up(n)).astype(f32)
        return q, (x.astype(np.float64) - q.astype(np.float64) * n).astype(f32)

    i = np.unique(np.concatenate([np.arange(0, small_max, 97), [small_max - 1],
                                  np.random.default_rng(5).integers(0, small_max, 20000)]))
    dims = [d for d in range(24) if K[d] > 0]
    assert dims == [1, 2, 3, 4, 5, 7, 8, 9, 10]
    for d in dims:
        b, k = primes[d], K[d]
        inv = f32(1) / f32(b)
        nd, cap = 0, 1
        while cap < small_max:
            cap *= b
            nd += 1
        # reference loop, variable length (lanes stop when i reaches 0)
        ref, f, v = np.zeros(i.shape, f32), f32(1), i.copy()
        while (v > 0).any():
            f = f32(f * inv)
            live = v > 0
            ref = np.where(live, (ref + (f * (v % b).astype(f32)).astype(f32)).astype(f32), ref)
            v //= b
        # the table: T[v] after k steps of v
        tv = np.arange(b ** k, dtype=np.int64)
        tab, f = np.zeros(tv.shape, f32), f32(1)
        for _ in range(k):
            f = f32(f * inv)
            tab = (tab + (f * (tv % b).astype(f32)).astype(f32)).astype(f32)
            tv //= b
        # halton_tab
        x, low = digit_step(i.astype(f32), b ** k)
        r = tab[low.astype(np.int64)]
        f = f32(1)
        for _ in range(k):
            f = f32(f * inv)  # f_after(b, k)
        for _ in range(k, nd):
            f = f32(f * inv)
            x, dig = digit_step(x, b)
            r = (r + (f * dig).astype(f32)).astype(f32)
        assert np.array_equal(r.view(np.uint32), ref.view(np.uint32)), (d, b)


# ---- MIS integrator (Sources/gpuRaytracer/shaders.metal) ----------------------------
def test_mis_scene_builder_equals_oracle_and_main_swift():
    s = Scene.cornell_box_mis(800, 600)
    cam, mats, verts, light, n = oracle_lib.cornell_box_mis(800, 600)
    assert n == 36
    for a, b in ((s.camera, cam), (s.materials, mats), (s.vertices, verts), (s.light, light)):
        assert bytes(a) == bytes(b)
    # main.swift:27-28,49-59: 1.5 x 1.5 light; emittedLuminance = diffuse * 1200 / 2.25 / Float.pi
    assert light.width == 1.5 and light.depth == 1.5
    lum = np.float32(np.float32(1200.0) / np.float32(2.25)) / np.float32(3.1415925)
    assert light.emittedRadiance.x == np.float32(1.0) * lum
    assert light.emittedRadiance.y == np.float32(0.95) * lum
    v = np.frombuffer(bytes(verts), np.float32).reshape(-1, 4)
    assert np.array_equal(v[102:108, [0, 2]].min(0), [-0.75, -0.75])
    # the room and boxes are RTrace's
    assert np.array_equal(v[:102], np.frombuffer(bytes(Scene.cornell_box(800, 600).vertices),
                                                 np.float32).reshape(-1, 4)[:102])


def test_pow_contract_accuracy():
    xs = np.concatenate([np.geomspace(1e-30, 1.0, 4000, dtype=np.float32),
                         np.linspace(0, 1, 4001, dtype=np.float32)])
    y = np.float32(1.0) / np.float32(2.2)
    got = np.array([oracle_lib.lib.pto_pow(float(x), float(y)) for x in xs], np.float32)
    ref = np.power(xs.astype(np.float64), float(y))
    ok = xs > 7.88860905e-31
    rel = np.abs(got[ok] - ref[ok]) / ref[ok]
    # exp(y log x): error ~ |y log x| * 2^-24, i.e. a few ulp where a byte of
    # gamma output is decided (x >= 1e-3) and < 4e-6 relative down to 1e-30
    assert rel.max() < 4e-6, rel.max()
    assert rel[xs[ok] >= 1e-3].max() < 6e-7
    assert np.all(got[~ok] == 0) and oracle_lib.lib.pto_pow(1.0, float(y)) == 1.0
    import pt_oracle_mis_np as M
    assert np.array_equal(M.pow_pt(xs, y).view(np.uint32), got.view(np.uint32))


@pytest.mark.parametrize("w,h,rays,samples", [(8, 6, 2, 6), (7, 5, 1, 9)])
def test_mis_oracle_equals_numpy_restatement(w, h, rays, samples):
    import pt_oracle_mis_np as M
    s = Scene.cornell_box_mis(w, h)
    out, out8 = oracle_lib.render_mis(s, rays, samples)
    sc = M.Scene(s.camera, s.materials, s.light, s.vertices)
    ref, ref8 = M.render_mis(sc, rays, samples)
    assert np.array_equal(out.view(np.uint32), ref.view(np.uint32))
    assert np.array_equal(out8, ref8)


def test_mis_oracle_reproduces_golden():
    from gpuraytracer_amd import CameraGPU, MaterialGPU, SquareLightGPU, float3
    g = np.load(os.path.join(GOLDEN, "mis_16x12_c2_m12.npz"))
    s = Scene(CameraGPU.from_buffer_copy(g["camera"].tobytes()),
              (MaterialGPU * 36).from_buffer_copy(g["materials"].tobytes()),
              (float3 * 108).from_buffer_copy(g["vertices"].tobytes()),
              SquareLightGPU.from_buffer_copy(g["light"].tobytes()))
    rays, samples = (int(v) for v in g["params"])
    out, out8 = oracle_lib.render_mis(s, rays, samples)
    assert np.array_equal(out.view(np.uint32), g["out"].view(np.uint32))
    assert np.array_equal(out8, g["out8"])


def test_mis_light_pixels_known_answer():
    # a pixel whose camera rays all hit the light sums emittedRadiance camera_rays
    # times (shaders.metal:667-671) and tonemaps to a fixed byte (:688-706)
    s = Scene.cornell_box_mis(80, 60)
    out, out8 = oracle_lib.render_mis(s, 6, 3, row_start=8, row_count=6)
    Le = np.array([s.light.emittedRadiance.x, s.light.emittedRadiance.y,
                   s.light.emittedRadiance.z], np.float32)
    six = np.zeros(3, np.float32)
    for _ in range(6):
        six = six + Le
    lit = np.all(out[..., :3] == six, axis=-1)
    ys, xs = np.nonzero(lit)
    assert lit.sum() >= 8 and 30 <= xs.min() and xs.max() <= 49  # centred light patch
    import pt_oracle_mis_np as M
    e = (six / np.float32(6)) * (np.float32(1) / (np.float32(1.2) * np.float32(32.0)))
    tm = np.minimum(np.float32(1), np.maximum(np.float32(0), e / (e + np.float32(1))))
    expect = (M.pow_pt(tm, np.float32(1) / np.float32(2.2)) * np.float32(255)).astype(np.uint8)
    assert np.all(out8[lit][:, :3] == expect) and np.all(out8[..., 3] == 255)
    assert np.all(out[..., 3] == 6)


def test_geometry_matches_reference_example_png():
    """The live scene as the oracle's camera sees it (primary-hit ids through
    the pixel centres, 800x600 = scene.swift:18) against the geometry measured
    from the reference's example.png (tests/golden/make_example_masks.py):
    colour classes (open front = black, red wall, green wall, light) and every
    luminance step the image shows along 54 rows and 74 columns -- the walls'
    floor/ceiling lines, both boxes' silhouettes and creases, the light's rim.
    Pins geometry only: the PNG is an earlier revision, its radiance is not a
    fixture (parity of radiance stays unpinned)."""
    g = np.load(os.path.join(GOLDEN, "example_png_geometry.npz"))
    ids = oracle_lib.primary_ids(Scene.cornell_box(800, 600))
    ocls = np.full(ids.shape, 4, np.uint8)
    ocls[ids < 0] = 0
    ocls[(ids == 2) | (ids == 3)] = 1      # red wall (scene.swift:93-102)
    ocls[(ids == 4) | (ids == 5)] = 2      # green wall (:105-114)
    ocls[(ids == 34) | (ids == 35)] = 3    # the light (:58-59)
    cls = g["cls"]
    assert (ocls == cls).mean() >= 0.99
    # IoU bars: the light is a 113 x 22 px patch, whose one-pixel rim alone is
    # ~11 % of its area (measured 0.953); the large regions agree to >= 0.97
    for c, name, bar in [(0, "open front", 0.97), (1, "red wall", 0.97),
                         (2, "green wall", 0.97), (3, "light", 0.95)]:
        a, b = cls == c, ocls == c
        iou = (a & b).sum() / (a | b).sum()
        assert iou >= bar, f"{name}: IoU {iou:.4f}"
    face = np.where(ids < 0, -1, ids // 2)  # a quad's two triangles form one face
    floor = 3                               # ids 6-7 (:117-126)
    unmatched, on_floor, offs = [], 0, []
    # a step measured on line L at position p was smoothed over lines L-4..L+4
    # (the 9-px filter across the line): it matches a face boundary along any
    # of those lines within +-3 px of p
    for (line, pos), axis in [(e, 0) for e in g["row_edges"]] + [(e, 1) for e in g["col_edges"]]:
        best = None
        for ln in range(max(0, line - 4), min(face.shape[axis] if axis else face.shape[0], line + 5)):
            prof = face[ln] if axis == 0 else face[:, ln]
            near = [abs(k - pos) for k in range(max(1, pos - 3), min(len(prof), pos + 4))
                    if prof[k] != prof[k - 1]]
            if near and (best is None or min(near) < best):
                best = min(near)
        if best is not None:
            offs.append(best)
        else:
            unmatched.append((axis, int(line), int(pos)))
            on_floor += int((face[line, pos] if axis == 0 else face[pos, line]) == floor)
    n = len(g["row_edges"]) + len(g["col_edges"])
    # every step the image shows is a face boundary of the live scene within
    # +-3 px, except the floor's shadow edges (lighting, not geometry)
    assert on_floor == len(unmatched), [u for u in unmatched]
    assert len(unmatched) <= 0.1 * n, len(unmatched)
    assert np.median(offs) <= 1 and len(offs) >= 0.9 * n
    # both boxes' silhouettes are among the matched steps (scene.swift:141-172)
    for lo, hi in [(10, 22), (22, 34)]:
        box = (ids >= lo) & (ids < hi)
        ys, xs = np.nonzero(box)
        edges_on_box = [(y, x) for y, x in g["row_edges"]
                        if box[y].any() and min(abs(x - xs[ys == y].min()), abs(x - 1 - xs[ys == y].max())) <= 3]
        assert edges_on_box, f"no image edge on the silhouette of box ids {lo}-{hi - 1}"


def test_radiance_vs_reference_example_png():
    """What the reference's one rendered artefact says about RADIANCE.

    The oracle renders the live scene (800x600 x 64 spp, the reference's
    resolution, scene.swift:18), tonemapped by image.swift:35-65, and its mean
    colour over each surface (primary-hit ids, eroded 4 px) is compared with
    the same surfaces of example.png (tests/golden/example_png_regions.json,
    made by tests/golden/make_example_regions.py).

    * White/grey surfaces agree within +-5 levels per channel: the NEE radiance
      scale is right -- light.color (computeShader.swift:36) with the inverse
      square falloff of sampleAreaLight (sampling.metal:198-236), not
      emittedRadiance (~380x larger).
    * The PNG's red and green walls have exactly zero off-channels, the
      oracle's do not: the live integrator's light-hit overwrite
      `accumulatedColor = emissive` (raytrace.metal:59, no throughput) puts
      white into every wall path that bounces into the light, so the PNG
      cannot come from the live kernel (an earlier revision; its light pixels
      also differ: 234 vs 212).  Radiance parity is therefore structurally
      unpinnable from any reference artefact."""
    import sys as _sys
    _sys.path.insert(0, GOLDEN)
    from make_example_regions import region_masks
    fx = json.load(open(os.path.join(GOLDEN, "example_png_regions.json")))["regions"]
    s = Scene.cornell_box(800, 600)
    img8 = oracle_lib.tonemap(oracle_lib.render(s, seed_splitmix(800, 600), 64, 3))
    rgb = img8[..., :3].astype(np.float64)
    got = {k: rgb[m].mean(axis=0) for k, m in region_masks(oracle_lib.primary_ids(s)).items()}
    for k in ("back_wall", "floor", "ceiling", "tall_box", "short_box"):
        assert fx[k]["pixels"] > 10000
        d = np.abs(got[k] - np.array(fx[k]["mean_rgb"]))
        assert d.max() <= 5.0, (k, got[k].round(1).tolist(), fx[k]["mean_rgb"])
    for k, ch in (("red_wall", 0), ("green_wall", 1)):
        png = np.array(fx[k]["mean_rgb"])
        off = [c for c in range(3) if c != ch]
        assert png[ch] > 60 and np.all(png[off] == 0.0), (k, png)        # pure colour in the PNG
        assert abs(got[k][ch] - png[ch]) <= 5.0                            # its own channel agrees
        assert np.all(got[k][off] > 20.0), (k, got[k].round(1).tolist())  # white from the overwrite
    assert fx["light"]["mean_rgb"] == [234.0, 233.0, 232.0]
    assert np.all(got["light"] == 212.0)  # emissive (1,1,1) through image.swift's tonemap

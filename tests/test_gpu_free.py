"""GPU: the two alternative walk schedulers for BVH scenes, bit for bit against
the oracle -- the free-running path kernel (rt_free.hpp, walk_scheduler =
free: every lane traces its own pixel's samples as a state machine, lanes
whose walk ended park and are served together) and the octant-sorted path
kernel (walk_scheduler = sorted: between bounces a workgroup's paths are
counting-sorted by direction octant, finished paths dropped): sphere scenes (bounces 1-4, multi-sphere leaves, exact duplicate
spheres, indices past the fixed-digit Halton bound, progressive batches,
interleaved rows, fp16 / RGBA8 stores) and triangle meshes (host SAH and GPU
LBVH trees, duplicate triangles), plus the config-4 frame at its bench size."""
import numpy as np
import pytest

import oracle_lib
from gpuraytracer_amd import Options, RenderParams, Renderer, Scene, seed_splitmix
from test_gpu_parity import assert_parity, triangle_soup

pytestmark = pytest.mark.gpu
KERNEL = {"free": "rt::path_free_kernel<", "sorted": "rt::path_trace_sorted_kernel<"}


@pytest.fixture(params=["free", "sorted"])
def walk(request):
    return request.param


def render_free(scene, seeds, params, walk, **opt):
    with Renderer(scene, seeds=seeds, options=Options(walk=walk, **opt)) as r:
        out = r.render(params)
        info = r.last_launch()
    assert info["kernel"].startswith(KERNEL[walk]), info
    return out


@pytest.mark.parametrize("bounces", [1, 2, 3, 4])
def test_free_spheres_bounce_counts(bounces, walk):
    s = Scene.random_spheres(40, 24, 700, seed=13)
    sd = seed_splitmix(40, 24, key=13)
    out = render_free(s, sd, RenderParams(spp=3, bounces=bounces), walk)
    assert_parity(out, oracle_lib.render(s, sd, 3, bounces), f"free spheres b{bounces}")


def test_free_spheres_1000_more_samples(walk):
    s = Scene.random_spheres(48, 32, 1000, seed=42)
    sd = seed_splitmix(48, 32)
    out = render_free(s, sd, RenderParams(spp=9, bounces=3), walk)
    assert_parity(out, oracle_lib.render(s, sd, 9, 3), "free spheres1000")


@pytest.mark.parametrize("den", [1, 64])
@pytest.mark.parametrize("kind", ["spheres", "triangles"])
def test_free_leaf_rounds_at_both_sites(kind, den):
    """The free scheduler resolves a parked leaf in two places: in the walk
    loop's leaf rounds and, for leaves still parked when the walk phase stops,
    at the top of the service phase.  walk_leaf_den = 1 holds the leaf rounds
    until every walker is parked, so most leaves reach the service site;
    64 runs a round for almost every parked leaf.  Both bit-exact."""
    if kind == "spheres":
        s = Scene.random_spheres(48, 32, 1000, seed=42)
    else:
        s = triangle_soup(48, 32, 3000, seed=3000, dup=True)
    sd = seed_splitmix(48, 32)
    out = render_free(s, sd, RenderParams(spp=9, bounces=3), "free", walk_leaf_den=den)
    assert_parity(out, oracle_lib.render(s, sd, 9, 3), f"free {kind} leaf den {den}")


@pytest.mark.parametrize("leaf", [3, 8])
def test_free_spheres_multi_sphere_leaves(leaf, walk):
    s = Scene.random_spheres(40, 24, 700, seed=5)
    sd = seed_splitmix(40, 24)
    out = render_free(s, sd, RenderParams(spp=2, bounces=3), walk, sphere_leaf_max=leaf)
    assert_parity(out, oracle_lib.render(s, sd, 2, 3), f"free leaf{leaf}")


def test_free_duplicate_spheres_tie_to_lower_id(walk):
    s = Scene.random_spheres(40, 24, 300, seed=11)
    for k in range(0, s.n_spheres - 1, 2):
        s.spheres[k + 1].center = s.spheres[k].center
        s.spheres[k + 1].radius = s.spheres[k].radius
        s.spheres[k + 1].material.diffuse.x = 0.05 + 0.9 * ((k * 37) % 17) / 17.0
    sd = seed_splitmix(40, 24)
    out = render_free(s, sd, RenderParams(spp=2, bounces=3), walk)
    assert_parity(out, oracle_lib.render(s, sd, 2, 3), "free duplicates")


@pytest.mark.parametrize("top", [3 ** 13 - 1, 3 ** 13 + 40])
def test_free_halton_index_bound(top, walk):
    """The largest index 3^13 - 1 (fixed-digit loop with the per-lane base) and
    indices past it (the reference loop with a run-time base)."""
    W, H, spp = 24, 16, 5
    rng = np.random.default_rng(top)
    sd = rng.integers(top - spp + 1 - 300000, top - spp + 2, (H, W), dtype=np.int64)
    sd[3, 7] = top - spp + 1
    sd = sd.astype(np.uint32)
    s = Scene.random_spheres(W, H, 400, seed=3)
    out = render_free(s, sd, RenderParams(spp=spp, bounces=3), walk)
    assert_parity(out, oracle_lib.render(s, sd, spp, 3), f"free index {top}")


def test_free_progressive_rows_and_stores(walk):
    s = Scene.random_spheres(40, 30, 500, seed=7)
    sd = seed_splitmix(40, 30, key=7)
    ref = oracle_lib.render(s, sd, 10, 3)
    with Renderer(s, seeds=sd, options=Options(walk=walk)) as r:
        r.render(RenderParams(spp=4, bounces=3, keep_sum=True))
        got = r.render(RenderParams(spp=6, bounces=3, sample_base=4, accumulate=True, keep_sum=True))
        assert r.last_launch()["kernel"].startswith(KERNEL[walk])
        tile = r.render(RenderParams(spp=10, bounces=3, row_start=1, row_step=4))
        h16 = r.render(RenderParams(spp=10, bounces=3, fp16=True))
        u8 = r.render(RenderParams(spp=10, bounces=3, rgba8=True))
    assert_parity(got, ref, "free progressive")
    assert_parity(tile, ref[1::4], "free interleaved rows")
    assert np.array_equal(h16, ref.astype(np.float16).view(np.uint16))
    assert np.array_equal(u8, oracle_lib.tonemap(ref))


@pytest.mark.parametrize("build", ["host", "lbvh", "gpusah"])
@pytest.mark.parametrize("n,dup", [(3000, False), (2500, True)])
def test_free_triangle_bvh(n, dup, build, walk):
    s = triangle_soup(40, 24, n, seed=n, dup=dup)
    sd = seed_splitmix(40, 24)
    out = render_free(s, sd, RenderParams(spp=3, bounces=3), walk, tri_build=build)
    assert_parity(out, oracle_lib.render(s, sd, 3, 3), f"free soup{n} {build}")


def test_free_triangle_bvh_forced_on_cornell(walk):
    s = Scene.cornell_box(48, 32)
    sd = seed_splitmix(48, 32)
    out = render_free(s, sd, RenderParams(spp=5, bounces=4), walk, layout="bvh")
    assert_parity(out, oracle_lib.render(s, sd, 5, 4), "free bvh cornell")


def test_free_c4_frame_1080p_256spp_bands(walk):
    """Config 4 at its bench size through the free-running kernel: the whole
    1920x1080 frame at 256 spp in one launch, three 4-row bands against the
    brute-force oracle bit for bit, the whole frame finite."""
    W, H = 1920, 1080
    s = Scene.random_spheres(W, H, 1000, seed=42)
    sd = seed_splitmix(W, H)
    frame = render_free(s, sd, RenderParams(spp=256, bounces=3), walk)
    assert np.isfinite(frame).all() and np.all(frame[..., 3] == 1.0)
    for start in (100, 540, 900):
        ref = oracle_lib.render(s, sd, 256, 3, row_start=start, row_count=4, threads=16)
        assert_parity(frame[start:start + 4], ref, f"free C4 rows {start}+4")

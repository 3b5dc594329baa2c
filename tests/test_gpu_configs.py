"""GPU parity of the exact configurations the bench times, and of the
multi-GPU configs' per-rank work, on one MI355X through the C-ABI.

* The headline launch (BASELINE config 2, 1920x1080 x 256 spp, 3 bounces)
  runs ``rt::path_trace_kernel<3, 6, false, true, 4>`` with the LDS Halton
  low-digit tables filled (4 lanes per pixel, 64 rounds per lane >=
  kHaltonTabMinRounds = 8).  ``rt_last_launch`` names the instantiation, and
  these tests assert they ran that same one against the C oracle.
* C3 (4096x4096 x 1024 spp over 8 GPUs) and C5 (8192x8192 x 4096 spp,
  progressive, over 8 GPUs): one rank's interleaved share (rows k, k+8, ...)
  rendered on this GPU, bands checked bit-exact against the oracle and the
  whole share checked through size-independent properties.
* The fused RGBA8 epilogue (RTrace/image.swift:35-65) against the oracle's
  tonemap, byte for byte.
"""
import numpy as np
import pytest

import oracle_lib
from gpuraytracer_amd import Options, RenderParams, Renderer, Scene, seed_splitmix
from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu

TIMED_KERNEL = "rt::path_trace_kernel<3, 6, false, true, 4>"  # what bench.py times (config 2)


def _timed(r):
    info = r.last_launch()
    assert info["kernel"] == TIMED_KERNEL, info
    assert info["lanes_per_pixel"] == 4 and info["halton_tables"] == 1, info
    return info


def test_headline_instantiation_full_frame_32spp_vs_oracle():
    """The whole 1080p frame at 32 spp: auto lanes pick L = 4 (>= 1 M pixels),
    8 rounds per lane, so the LDS Halton tables are on -- the timed kernel,
    every pixel against the oracle (66 M samples, ~3 s on 16 host threads)."""
    s = Scene.cornell_box(1920, 1080)
    sd = seed_splitmix(1920, 1080)
    with Renderer(s, seeds=sd) as r:
        out = r.render(RenderParams(spp=32, bounces=3))
        info = _timed(r)
        assert (info["grid_x"], info["grid_y"]) == (240, 135)
    assert_parity(out, oracle_lib.render(s, sd, 32, 3, threads=16), "1080p x 32 spp")


@pytest.mark.parametrize("rows", [(0, 3), (361, 4), (539, 2), (1076, 4)])
def test_headline_instantiation_256spp_row_bands_vs_oracle(rows):
    """Full-width 1080p bands at the bench's 256 spp with 4 lanes per pixel
    forced (a small launch alone would pick 16): 64 rounds per lane, tables
    on, the same instantiation as the timed whole-frame launch."""
    start, count = rows
    s = Scene.cornell_box(1920, 1080)
    sd = seed_splitmix(1920, 1080)
    with Renderer(s, seeds=sd, options=Options(lanes=4)) as r:
        out = r.render(RenderParams(spp=256, bounces=3, row_start=start, row_count=count))
        _timed(r)
    ref = oracle_lib.render(s, sd, 256, 3, row_start=start, row_count=count, threads=16)
    assert_parity(out, ref, f"1080p rows {start}+{count} x 256 spp")


@pytest.mark.parametrize("lanes,spp", [(4, 32), (16, 128)])
@pytest.mark.parametrize("top", [3 ** 13 - 1, 3 ** 13])
def test_halton_index_bound_edges_with_tables(top, lanes, spp):
    """The fixed-digit boundary (largest index 3^13 - 1: the table kernel with
    halton_tab's continuation T_D[i mod b^k] + digits of i / b^k, at >= 8
    rounds per lane with L = 4 and L = 16; 3^13: the generic loop)."""
    W, H = 40, 24
    rng = np.random.default_rng(top + lanes)
    sd = rng.integers(top - spp + 1 - 400000, top - spp + 2, (H, W), dtype=np.int64)
    sd[5, 9] = top - spp + 1  # max index = top
    sd = sd.astype(np.uint32)
    s = Scene.cornell_box(W, H)
    with Renderer(s, seeds=sd, options=Options(lanes=lanes)) as r:
        out = r.render(RenderParams(spp=spp, bounces=3))
        info = r.last_launch()
    small = top < 3 ** 13
    assert info["small_index"] == int(small)
    # the generic-loop kernel (index >= 3^13) runs one lane per pixel, no tables
    assert info["lanes_per_pixel"] == (lanes if small else 1), info
    assert info["halton_tables"] == int(small), info
    assert_parity(out, oracle_lib.render(s, sd, spp, 3), f"top={top} L={lanes}")


@pytest.mark.parametrize("rank", [0, 5])
def test_c3_rank_share_4096(rank):
    """Config 3: rank k of 8 renders rows k, k+8, ... of the 4096x4096 frame
    at 1024 spp (2.1 G samples).  Two rows of the share bit-exact vs the
    oracle; the share is finite with alpha 1; rows are the global ones."""
    W = H = 4096
    s = Scene.cornell_box(W, H)
    sd = seed_splitmix(W, H)
    with Renderer(s, seeds=sd) as r:
        share = r.render(RenderParams(spp=1024, bounces=3, row_start=rank, row_step=8))
        info = r.last_launch()
    assert share.shape == (512, W, 4)
    # interleaved share: 16 lanes per pixel (64 rounds per lane, tables on)
    assert info["lanes_per_pixel"] == 16 and info["halton_tables"] == 1, info
    assert np.isfinite(share).all() and np.all(share[..., 3] == 1.0)
    j = 255  # share row j = image row rank + 8 j (mid-frame: boxes, walls)
    ref = oracle_lib.render(s, sd, 1024, 3, row_start=rank + 8 * j, row_step=8, row_count=2,
                            threads=16)
    assert_parity(share[j:j + 2], ref, f"C3 rank {rank} rows")


def test_c5_rank_share_8192_progressive():
    """Config 5: rank 3 of 8 on the 8192x8192 frame (1024 rows x 8192),
    progressive batches of 64 spp into the running fp32 sum.  The whole share
    batched (2 x 64) equals one 128-spp launch bit for bit; a band at 256 spp
    (4 batches) matches the oracle."""
    W = H = 8192
    s = Scene.cornell_box(W, H)
    sd = seed_splitmix(W, H)
    rank = 3
    with Renderer(s, seeds=sd) as r:
        single = r.render(RenderParams(spp=128, row_start=rank, row_step=8))
        r.accumulate(RenderParams(spp=64, row_start=rank, row_step=8, keep_sum=True))
        batched = r.render(RenderParams(spp=64, sample_base=64, row_start=rank, row_step=8,
                                        accumulate=True))
        assert_parity(batched, single, "C5 share batched vs single")
        assert np.isfinite(single).all() and np.all(single[..., 3] == 1.0)
        del single, batched
        j0 = 500
        band = RenderParams(row_start=rank + 8 * j0, row_step=8, row_count=2)
        for b in range(4):
            p = RenderParams(spp=64, sample_base=64 * b, row_start=band.row_start, row_step=8,
                             row_count=2, accumulate=b > 0, keep_sum=True)
            last = r.render(p) if b == 3 else r.accumulate(p)
    ref = oracle_lib.render(s, sd, 256, 3, row_start=rank + 8 * j0, row_step=8, row_count=2,
                            threads=16)
    assert_parity(last, ref, "C5 band 256 spp progressive")


def test_progressive_from_nonzero_sample_base():
    """A running sum may start at any sample index: samples [5, 12) in two
    batches equal one launch of samples [5, 12) (divisor 7 both ways)."""
    s = Scene.cornell_box(40, 24)
    with Renderer(s) as r:
        single = r.render(RenderParams(spp=7, sample_base=5))
        r.accumulate(RenderParams(spp=3, sample_base=5, keep_sum=True))
        both = r.render(RenderParams(spp=4, sample_base=8, accumulate=True))
    assert_parity(both, single, "progressive from 5")
    sd = seed_splitmix(40, 24)
    assert_parity(single, oracle_lib.render(s, sd, 7, 3, sample_base=5), "base 5 vs oracle")


@pytest.mark.parametrize("size,spp", [((64, 48), 8), ((1920, 1080), 32)])
def test_rgba8_epilogue_matches_oracle_tonemap(size, spp):
    """RT_OUT_RGBA8: the image.swift:35-65 epilogue fused into the kernel's
    store equals the oracle render tonemapped by the oracle, byte for byte."""
    W, H = size
    s = Scene.cornell_box(W, H)
    sd = seed_splitmix(W, H)
    with Renderer(s, seeds=sd) as r:
        img8 = r.render(RenderParams(spp=spp, rgba8=True))
        f32 = r.render(RenderParams(spp=spp))
    assert img8.dtype == np.uint8 and img8.shape == (H, W, 4)
    ref = oracle_lib.tonemap(oracle_lib.render(s, sd, spp, 3, threads=16))
    assert np.array_equal(oracle_lib.tonemap(f32), ref)
    bad = np.argwhere(img8 != ref)
    assert bad.size == 0, f"{len(bad)} bytes differ, first at {bad[:4].tolist()}"
    assert np.all(img8[..., 3] == 255)


def test_rgba8_device_output_progressive():
    """RGBA8 as the last launch of a progressive render into device memory."""
    import torch
    s = Scene.cornell_box(96, 64)
    with Renderer(s) as r:
        dev = torch.empty((64, 96, 4), dtype=torch.uint8, device="cuda:0")
        r.render_progressive(RenderParams(spp=12, rgba8=True), 4, out=dev)
        torch.cuda.synchronize()
        ref = oracle_lib.tonemap(r.render(RenderParams(spp=12)))
    assert np.array_equal(dev.cpu().numpy(), ref)


C4_KERNEL = "rt::path_trace_kernel<3, 7, true, true, 16>"  # what bench.py --scene spheres times
C4_BLOCK = 64                  # one wave of 2x2 pixels per workgroup (rt_kernel.hpp RT_SPH_BLOCK)
C4_GRID = (1920 // 2, 1080 // 2)


def test_c4_timed_launch_1080p_256spp_bands_vs_oracle():
    """Config 4 exactly as the bench times it: the whole 1920x1080 frame of the
    1000-sphere scene at 256 spp in ONE launch (16 lanes per pixel, 16 rounds
    per lane, C4_BLOCK-thread workgroups walking the 8-layout leaf-box BVH in
    L2, grid C4_GRID).  Three 4-row bands of that frame (top, middle, lower
    third) are compared with the brute-force oracle bit for bit (5.9 M
    samples on the host); the whole frame is finite with alpha 1."""
    W, H = 1920, 1080
    s = Scene.random_spheres(W, H, 1000, seed=42)
    sd = seed_splitmix(W, H)
    with Renderer(s, seeds=sd) as r:
        frame = r.render(RenderParams(spp=256, bounces=3))
        info = r.last_launch()
    assert info["kernel"] == C4_KERNEL, info
    assert info["lanes_per_pixel"] == 16 and info["block_threads"] == C4_BLOCK, info
    assert (info["grid_x"], info["grid_y"]) == C4_GRID, info
    assert info["lds_bytes"] == s.describe()["sphere_kernel_lds_bytes"], info
    assert np.isfinite(frame).all() and np.all(frame[..., 3] == 1.0)
    for start in (100, 540, 900):
        ref = oracle_lib.render(s, sd, 256, 3, row_start=start, row_count=4, threads=16)
        assert_parity(frame[start:start + 4], ref, f"C4 rows {start}+4 x 256 spp")


def test_triangle_bvh_whole_1080p_frame_rows_vs_oracle():
    """The triangle-BVH kernel as the triangle benches run it: a whole 1920x1080
    frame of the room + 10k random triangles (GPU SAH build, 16 lanes per pixel,
    select-form steps checked every 4) at 16 spp in one launch; a row of the
    middle and one of the lower third against the brute-force oracle bit for bit."""
    W, H = 1920, 1080
    s = Scene.random_triangles(W, H, 10_000)
    sd = seed_splitmix(W, H)
    with Renderer(s, seeds=sd) as r:
        frame = r.render(RenderParams(spp=16, bounces=3))
        info = r.last_launch()
    assert info["kernel"] == "rt::path_trace_kernel<3, 5, false, true, 16>", info
    assert np.isfinite(frame).all() and np.all(frame[..., 3] == 1.0)
    for start, n in ((540, 1), (800, 1)):
        ref = oracle_lib.render(s, sd, 16, 3, row_start=start, row_count=n, threads=16)
        assert_parity(frame[start:start + n], ref, f"10k triangles rows {start}+{n}")

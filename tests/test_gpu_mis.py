"""GPU parity of the MIS integrator (rt_render_mis, gpuraytracer_amd/csrc/rt_mis.hip)
against the C oracle (pto_render_mis), itself pinned by the numpy restatement
(oracle/pt_oracle_mis_np.py) and the golden fixture.  Bar: bit-exact for the
float sums and the RGBA8 bytes.  Every call goes through librtpt.so.
"""
import os

import numpy as np
import pytest

import oracle_lib
from gpuraytracer_amd import (CameraGPU, MaterialGPU, MisParams, Options, Renderer, RtError, Scene,
                              SquareLightGPU, float3)

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def assert_same(gpu, ref, what):
    g, r = np.asarray(gpu), np.asarray(ref)
    assert g.shape == r.shape, (g.shape, r.shape)
    if g.dtype == np.float32:
        gb, rb = g.view(np.uint32), r.view(np.uint32)
        nan = np.isnan(g) & np.isnan(r)  # NaN payloads differ between x86 and gfx950
        diff = (gb != rb) & ~nan
    else:
        diff = g != r
    if diff.any():
        idx = np.argwhere(diff)[:6].tolist()
        raise AssertionError(f"{what}: {int(diff.sum())} values differ, first at {idx}: "
                             f"gpu {g[tuple(np.argwhere(diff)[0])]} ref {r[tuple(np.argwhere(diff)[0])]}")


def test_mis_golden_fixture_bit_exact():
    g = np.load(os.path.join(GOLDEN, "mis_16x12_c2_m12.npz"))
    s = Scene(CameraGPU.from_buffer_copy(g["camera"].tobytes()),
              (MaterialGPU * 36).from_buffer_copy(g["materials"].tobytes()),
              (float3 * 108).from_buffer_copy(g["vertices"].tobytes()),
              SquareLightGPU.from_buffer_copy(g["light"].tobytes()))
    rays, samples = (int(v) for v in g["params"])
    with Renderer(s) as r:
        out, out8 = r.render_mis(MisParams(camera_rays=rays, mis_samples=samples))
    assert_same(out, g["out"], "sum")
    assert_same(out8, g["out8"], "rgba8")


@pytest.mark.parametrize("rays,samples", [(1, 3), (2, 30), (3, 31), (5, 12), (7, 9)])
def test_mis_vs_oracle(rays, samples):
    s = Scene.cornell_box_mis(72, 40)  # not a multiple of the 16x16 tile
    with Renderer(s) as r:
        out, out8 = r.render_mis(MisParams(camera_rays=rays, mis_samples=samples))
    ref, ref8 = oracle_lib.render_mis(s, rays, samples)
    assert_same(out, ref, "sum")
    assert_same(out8, ref8, "rgba8")


def test_mis_reference_parameters_800x600_rows():
    # drawTriangle's own configuration: 800x600, 6 camera rays, 300 MIS samples
    s = Scene.cornell_box_mis(800, 600)
    p = MisParams(camera_rays=6, mis_samples=300, row_start=37, row_step=113)
    with Renderer(s) as r:
        out, out8 = r.render_mis(p)
    ref, ref8 = oracle_lib.render_mis(s, 6, 300, row_start=37, row_step=113)
    assert out.shape == (5, 800, 4)
    assert_same(out, ref, "sum")
    assert_same(out8, ref8, "rgba8")


def test_mis_row_tiles_equal_full_frame_and_rtrace_scene():
    s = Scene.cornell_box(48, 32)  # the RTrace scene works too (1 x 1 light)
    with Renderer(s) as r:
        full, full8 = r.render_mis(MisParams(camera_rays=2, mis_samples=9))
        tile, tile8 = r.render_mis(MisParams(camera_rays=2, mis_samples=9, row_start=1,
                                             row_step=3))
    assert_same(tile, full[1::3], "tile")
    assert_same(tile8, full8[1::3], "tile8")
    ref, ref8 = oracle_lib.render_mis(s, 2, 9)
    assert_same(full, ref, "sum")


def test_mis_frame_without_split_equals_split_rows():
    """A frame whose per-ray buffer would pass 1 GB (rt_mis.hip kMisPartMax) runs
    without the split: the kernel adds the rounds of camera rays itself (2 rounds
    of 2 lanes here).  Rows of that frame equal the same rows rendered through the
    split launch (per-ray buffer + ordered sum kernel) and the oracle."""
    W = H = 4800
    rays = 3
    assert W * H * rays * 16 > (1 << 30)
    s = Scene.cornell_box_mis(W, H)
    p_rows = MisParams(camera_rays=rays, mis_samples=3, row_start=7, row_step=997)
    with Renderer(s) as r:
        full, full8 = r.render_mis(MisParams(camera_rays=rays, mis_samples=3))
        rows, rows8 = r.render_mis(p_rows)
    assert_same(full[7::997], rows, "frame rows vs split rows")
    assert_same(full8[7::997], rows8, "frame rows vs split rows (rgba8)")
    ref, ref8 = oracle_lib.render_mis(s, rays, 3, row_start=7, row_step=997)
    assert_same(rows, ref, "split rows vs oracle")
    assert_same(rows8, ref8, "split rows vs oracle (rgba8)")


def test_mis_device_outputs_match_host():
    import torch
    s = Scene.cornell_box_mis(40, 24)
    p = MisParams(camera_rays=2, mis_samples=12)
    with Renderer(s) as r:
        host, host8 = r.render_mis(p)
        d = torch.empty((24, 40, 4), dtype=torch.float32, device="cuda")
        d8 = torch.empty((24, 40, 4), dtype=torch.uint8, device="cuda")
        r.render_mis(p, out=d, out8=d8)
        only8 = torch.zeros_like(d8)
        r.render_mis(p, out8=only8)
    assert_same(d.cpu().numpy(), host, "device sum")
    assert_same(d8.cpu().numpy(), host8, "device rgba8")
    assert_same(only8.cpu().numpy(), host8, "rgba8 only")


@pytest.mark.parametrize("layout", ["single", "smem", "pairs"])
def test_mis_scene_layouts_bit_exact(layout):
    s = Scene.cornell_box_mis(40, 24)
    with Renderer(s, options=Options(layout=layout)) as r:
        out, out8 = r.render_mis(MisParams(camera_rays=2, mis_samples=12))
    ref, ref8 = oracle_lib.render_mis(s, 2, 12)
    assert_same(out, ref, layout)
    assert_same(out8, ref8, layout)


def test_mis_lds_layout_above_64k_with_the_stash_bit_exact():
    """A forced single-record LDS layout whose records (96 B per triangle:
    intersection + shading) take 57.6 KB: with the 15 KB stash on top the
    workgroup asks for 72.6 KB of dynamic LDS (hipFuncSetAttribute above
    64 KB, rt_mis.hip launch_mis_g) instead of falling back to global memory."""
    s = Scene.random_triangles(40, 24, 564, seed=3)  # 600 triangles
    assert 49 * 1024 < 96 * 600 <= 64 * 1024
    with Renderer(s, options=Options(layout="single")) as r:
        out, out8 = r.render_mis(MisParams(camera_rays=2, mis_samples=9))
    ref, ref8 = oracle_lib.render_mis(s, 2, 9)
    assert_same(out, ref, "single 600")
    assert_same(out8, ref8, "single 600")


def test_mis_box_clusters_rotated_boxes_bit_exact():
    """MIS queries through the box clusters on randomly rotated boxes."""
    s = Scene.random_boxes(40, 24, 4, seed=5)
    assert s.describe()["n_box_clusters"] == 6
    with Renderer(s) as r:
        out, out8 = r.render_mis(MisParams(camera_rays=2, mis_samples=9))
    ref, ref8 = oracle_lib.render_mis(s, 2, 9)
    assert_same(out, ref, "boxes")
    assert_same(out8, ref8, "boxes")


def test_mis_errors_are_status_codes():
    s = Scene.cornell_box_mis(16, 8)
    with Renderer(s) as r:
        for bad in (MisParams(camera_rays=0), MisParams(mis_samples=2), MisParams(row_start=8)):
            with pytest.raises(RtError):
                r.render_mis(bad)
    with Renderer(Scene.random_spheres(16, 8, 10)) as r:
        with pytest.raises(RtError, match="triangle scenes only"):
            r.render_mis(MisParams(camera_rays=1, mis_samples=3))

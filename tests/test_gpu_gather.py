"""GPU: the multi-GPU entry points of the C-ABI (rt_comm_unique_id,
rt_comm_init, rt_render_gather) on this one MI355X.

RCCL refuses two ranks on one device, so a one-GPU box runs a world of 1:
the same code path as rank 0 of N (tile render into the context's staging,
ncclGather over the communicator, strided placement of the rows), checked
bit-exact against rt_render and the oracle.  N > 1 runs in the driver's
8-GPU scaling bench (bench.py --gpus N); its row partition and reassembly are
covered on the CPU by tests/test_multirank.py.
"""
import numpy as np
import pytest

import oracle_lib
from gpuraytracer_amd import RenderParams, Renderer, RtError, Scene, comm_unique_id, seed_splitmix
from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu


def test_gather_world_of_one_equals_render_and_oracle():
    s = Scene.cornell_box(72, 40)
    sd = seed_splitmix(72, 40)
    with Renderer(s, seeds=sd) as r:
        with pytest.raises(RtError) as e:
            r.render_gather(RenderParams(spp=4))
        assert e.value.status == 5  # RT_ERR_STATE: no communicator yet
        r.comm_init(0, 1, comm_unique_id())
        with pytest.raises(RtError) as e:
            r.comm_init(0, 1, comm_unique_id())
        assert e.value.status == 5
        with pytest.raises(RtError) as e:
            r.render_gather(RenderParams(spp=4, row_step=2))
        assert e.value.status == 1  # the communicator owns the partition
        g = r.render_gather(RenderParams(spp=4))
        one = r.render(RenderParams(spp=4))
        g8 = r.render_gather(RenderParams(spp=4, rgba8=True))
        g16 = r.render_gather(RenderParams(spp=4, fp16=True))
    assert_parity(g, one, "gather vs render")
    assert_parity(g, oracle_lib.render(s, sd, 4, 3), "gather vs oracle")
    assert np.array_equal(g8, oracle_lib.tonemap(g))
    assert np.array_equal(g16, g.astype(np.float16).view(np.uint16))


def test_gather_device_output_and_progressive():
    import torch
    s = Scene.cornell_box(64, 48)
    with Renderer(s) as r:
        r.comm_init(0, 1, comm_unique_id())
        dev = torch.empty((48, 64, 4), dtype=torch.float32, device="cuda:0")
        r.render_gather(RenderParams(spp=6), out=dev)
        prog = torch.empty_like(dev)
        r.render_progressive(RenderParams(spp=6), 2, out=prog, gather=True)
        torch.cuda.synchronize()
        ref = r.render(RenderParams(spp=6))
    assert_parity(dev.cpu().numpy(), ref, "device gather")
    assert_parity(prog.cpu().numpy(), ref, "progressive gather")


def _render_tiles(r, s, world, spp, fp16, rgba8, stream):
    """Every rank's tile of the rt_render_gather partition rendered on this one
    GPU into ONE buffer laid out as ncclGather delivers it to rank 0: `world`
    padded tiles back to back (rt_tile_layout); padding and the tiles of ranks
    without rows keep a 0xAB fill, so a wrong offset or stride shows."""
    import ctypes
    import torch
    from gpuraytracer_amd import tile_layout
    lay = [tile_layout(s.width, s.height, world, k, fp16, rgba8) for k in range(world)]
    tb = lay[0]["tile_bytes"]
    gathered = torch.full((world * tb,), 0xAB, dtype=torch.uint8, device="cuda:0")
    for k in range(world):
        assert lay[k]["tile_bytes"] == tb and lay[k]["rows_max"] == lay[0]["rows_max"]
        if lay[k]["rows"] == 0:
            continue
        p = RenderParams(spp=spp, row_start=k, row_step=world, row_count=lay[k]["rows"], fp16=fp16,
                         rgba8=rgba8)
        r.render(p, out=gathered.data_ptr() + k * tb, stream=stream)
    return gathered


@pytest.mark.parametrize("H", [1080, 17, 5])
def test_place_tiles_n_ranks_equals_single_frame(H):
    """The N > 1 placement of rt_render_gather (rt_place_tiles, the code rank 0
    runs after its ncclGather) for N = 2, 3, 8, 16 -- H mod N != 0 and N > H
    included -- in all three pixel formats, into host and device frames: every
    frame is bit-identical to one rt_render of the whole frame."""
    import torch
    W, spp = (1920 if H == 1080 else 40), 2  # W >= H: the reference's integer aspect
    s = Scene.cornell_box(W, H)
    with Renderer(s) as r:
        # torch's current (null) stream, and a side stream at H = 17: the tile
        # renders and the placement are ordered on the caller's stream
        stream = torch.cuda.Stream() if H == 17 else torch.cuda.current_stream()
        for fp16, rgba8 in ((False, False), (True, False), (False, True)):
            ref = r.render(RenderParams(spp=spp, fp16=fp16, rgba8=rgba8))
            for world in (2, 3, 8, 16):
                g = _render_tiles(r, s, world, spp, fp16, rgba8, stream)
                dt = torch.uint8 if rgba8 else torch.int16 if fp16 else torch.float32
                dev = torch.empty((H, W, 4), dtype=dt, device="cuda:0")
                r.place_tiles(g, world, out=dev, fp16=fp16, rgba8=rgba8, stream=stream)
                host = r.place_tiles(g, world, fp16=fp16, rgba8=rgba8, stream=stream)
                torch.cuda.synchronize()
                d = dev.cpu().numpy().view(ref.dtype)
                tag = f"H={H} N={world} fp16={fp16} rgba8={rgba8}"
                assert np.array_equal(host.view(np.uint8), ref.view(np.uint8)), tag + " host frame"
                assert np.array_equal(d.view(np.uint8), ref.view(np.uint8)), tag + " device frame"


def test_comm_info_reports_rccl_world():
    s = Scene.cornell_box(16, 8)
    with Renderer(s) as r:
        with pytest.raises(RtError) as e:
            r.comm_info()
        assert e.value.status == 5
        r.comm_init(0, 1, comm_unique_id())
        assert r.comm_info() == (1, 0)


def test_gather_calls_on_two_streams_in_a_row():
    """Two device-output gathers on different streams without a host sync in
    between: the second waits for the first's reads of the context's tile
    buffers (ev_tiles), so both frames are right."""
    import torch
    s = Scene.cornell_box(48, 32)
    with Renderer(s) as r:
        r.comm_init(0, 1, comm_unique_id())
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        a = torch.empty((32, 48, 4), dtype=torch.float32, device="cuda:0")
        b = torch.empty_like(a)
        r.render_gather(RenderParams(spp=8), out=a, stream=s1)
        r.render_gather(RenderParams(spp=3), out=b, stream=s2)
        torch.cuda.synchronize()
        ra, rb = r.render(RenderParams(spp=8)), r.render(RenderParams(spp=3))
    assert_parity(a.cpu().numpy(), ra, "first gather")
    assert_parity(b.cpu().numpy(), rb, "second gather")

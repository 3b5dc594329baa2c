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

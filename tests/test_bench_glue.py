"""CPU: bench.py's multi-rank glue (world 2 and 3, gloo) with the GPU
touchpoints replaced by a CPU stand-in (``FakeBackend``): rank bookkeeping,
the communicator-id broadcast, the barriers, the max over ranks, the
``comm_ranks`` report, the weak-scaling value and rank 0's placement proof
(``gather_check``: rows of every rank re-rendered locally, bit for bit).

The stand-in renders each rank's interleaved rows with the CPU oracle and
gathers the padded tiles over gloo into rank 0, which places them with the
product's placement code (``rt_place_tiles_host``) -- what rt_render_gather
does on the GPU with ncclGather and rt_place_tiles.  A stand-in that swaps two
ranks' tiles must make the placement proof fail.
"""
import io
import json
import os
import socket
import sys
import time
from contextlib import redirect_stdout

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class FakeEvent:
    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class FakeRenderer:
    swap_tiles = False  # fault injection: rank 0 places rank 1's tile as its own

    def __init__(self, scene):
        from gpuraytracer_amd import seed_splitmix
        self.scene = scene
        self.seeds = seed_splitmix(scene.width, scene.height)
        self.rank, self.world = 0, 1

    def comm_init(self, rank, world, comm_id):
        assert isinstance(comm_id, bytes) and len(comm_id) == 128
        self.rank, self.world = rank, world

    def comm_info(self):
        return self.world, self.rank

    def _rows(self, params, start, step, count):
        import oracle_lib
        return oracle_lib.render(self.scene, self.seeds, params.spp, params.bounces,
                                 row_start=start, row_step=step, row_count=count, threads=2)

    def render(self, params, out=None, stream=None):
        img = self._rows(params, params.row_start, params.row_step, params.row_count)
        if out is None:
            return img
        out.copy_(torch.from_numpy(img))
        return out

    def render_gather(self, params, out=None, stream=None):
        import torch.distributed as dist
        from gpuraytracer_amd import place_tiles_host, tile_layout
        W, H = self.scene.width, self.scene.height
        lay = tile_layout(W, H, self.world, self.rank)
        tile = torch.zeros((lay["rows_max"], W, 4), dtype=torch.float32)
        if lay["rows"]:
            tile[:lay["rows"]] = torch.from_numpy(self._rows(params, self.rank, self.world, lay["rows"]))
        got = [torch.zeros_like(tile) for _ in range(self.world)] if self.rank == 0 else None
        dist.gather(tile, got, dst=0)
        if self.rank == 0:
            if self.swap_tiles:
                got[0], got[1] = got[1], got[0]
            out.copy_(torch.from_numpy(place_tiles_host(torch.stack(got).numpy(), W, H, self.world)))
        return out

    def render_progressive(self, params, batch_spp, out, stream=None, gather=False):
        return self.render_gather(params, out) if gather else self.render(params, out)

    def last_launch(self):
        return {"kernel": "fake"}

    def last_kernel_ms(self):
        return 1.0

    def close(self):
        pass


class FakeBackend:
    def __init__(self, local):
        self.local = local

    def renderer(self, scene):
        return FakeRenderer(scene)

    def comm_unique_id(self):
        return os.urandom(128)

    def empty_frame(self, H, W):
        return torch.empty((H, W, 4), dtype=torch.float32)

    def stream(self):
        return None

    def event(self):
        return FakeEvent()

    def synchronize(self):
        pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, argv, swap, result_path):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    FakeRenderer.swap_tiles = swap
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.main(argv, backend_factory=FakeBackend)
    if rank == 0:
        with open(result_path, "w") as f:
            f.write(buf.getvalue())


def _run(world, tmp_path, swap=False, H=17):
    W, spp, steps = 24, 2, 2
    argv = ["--gpus", str(world), "--width", str(W), "--height", str(H), "--spp", str(spp),
            "--steps", str(steps), "--warmup", "1", "--cpu-baseline", "off"]
    out = str(tmp_path / "line.json")
    mp.spawn(_worker, args=(world, _free_port(), argv, swap, out), nprocs=world, join=True)
    lines = [ln for ln in open(out).read().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, "rank 0 prints exactly one JSON line"
    return json.loads(lines[0]), W, H, spp, steps


@pytest.mark.parametrize("world", [2, 3])
def test_bench_multirank_line(world, tmp_path):
    rec, W, H, spp, steps = _run(world, tmp_path)
    assert rec["n_gpus"] == world and rec["comm_ranks"] == world and rec["comm_ranks_consistent"]
    assert rec["scaling"] == "weak" and rec["config"]["spp_frame"] == spp * world
    assert rec["gather_check"]["rows"] == sorted(set(range(world)) | {H - 1})
    assert rec["gather_check"]["bit_exact_vs_local_render"] is True
    assert rec["frame_ok"] is True
    # whole-job throughput: all ranks' samples over the max-over-ranks time
    want = W * H * spp * world / (rec["ms_per_step"] * 1e-3) / 1e6
    assert abs(rec["value"] - want) <= 0.01 * want + 1e-3
    assert rec["roofline"]["kernel_ms_basis"].startswith("the render launch")
    # the gather's share of a step (step - render launch, max over ranks) next to
    # the render times, so an N > 1 record separates imbalance from the collective
    # (the stand-in's render "launch" is a constant 1 ms, so only the bound holds here)
    assert isinstance(rec["gather_ms"], float)
    assert rec["gather_ms"] <= rec["step_ms_max_rank"] + 1e-6
    assert rec["kernel_ms_min_rank"] <= rec["kernel_ms_max_rank"]
    assert rec["gather_ms_basis"].startswith("step - render")
    assert rec["cpu_baseline"] is None


def test_bench_placement_proof_catches_misplaced_tiles(tmp_path):
    rec, *_ = _run(2, tmp_path, swap=True)
    assert rec["gather_check"]["bit_exact_vs_local_render"] is False


def test_spawn_ranks_refuses_more_ranks_than_gpus():
    sys.path.insert(0, ROOT)
    import bench
    with pytest.raises(SystemExit) as e:
        bench.spawn_ranks(4, ["--gpus", "4"], count_gpus=lambda: 1)
    assert "only 1 GPU" in str(e.value)

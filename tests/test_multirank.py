"""CPU: the N>1 path of bench.py — interleaved row tiles + one gather — with the
gloo backend (world_size 2 and 3), the oracle standing in for each rank's GPU.
The assembled frame must equal the single-rank frame bit-for-bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gpuraytracer_amd.tiles import assemble, rank_rows, tile_rows_max


def test_rank_rows_cover_frame_exactly_once():
    for H in (1, 7, 13, 1080):
        for N in (1, 2, 3, 4, 8):
            seen = []
            for k in range(N):
                start, step, count = rank_rows(H, N, k)
                seen += [start + j * step for j in range(count)]
                assert count <= tile_rows_max(H, N)
            assert sorted(seen) == list(range(H))


def test_assemble_numpy_roundtrip():
    H, W, N = 13, 5, 4
    frame = np.random.default_rng(0).random((H, W, 4), dtype=np.float32)
    rmax = tile_rows_max(H, N)
    tiles = []
    for k in range(N):
        t = np.full((rmax, W, 4), np.nan, np.float32)
        _, _, count = rank_rows(H, N, k)
        t[:count] = frame[k::N]
        tiles.append(t)
    assert np.array_equal(assemble(tiles, H), frame)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, W, H, spp, result_path):
    import torch
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_lib
    from gpuraytracer_amd import Scene, seed_splitmix

    scene = Scene.cornell_box(W, H)
    seeds = seed_splitmix(W, H)
    start, step, count = rank_rows(H, world, rank)
    rmax = tile_rows_max(H, world)
    tile = torch.zeros((rmax, W, 4), dtype=torch.float32)
    if count:  # a rank past the last row renders nothing (row_count 0 means "all rows")
        tile[:count] = torch.from_numpy(
            oracle_lib.render(scene, seeds, spp * world, 3, row_start=start, row_step=step,
                              row_count=count, threads=2))
    gathered = [torch.zeros_like(tile) for _ in range(world)] if rank == 0 else None
    dist.gather(tile, gathered, dst=0)
    if rank == 0:
        np.save(result_path, assemble(gathered, H).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 17), (3, 17), (3, 2)])
def test_gloo_gather_equals_single_rank_frame(world, H, tmp_path):
    """(3, 2): more ranks than rows -- rank 2 owns no row and still joins the
    gather with an empty (padded) tile."""
    import oracle_lib
    from gpuraytracer_amd import Scene, seed_splitmix

    W, spp = 24, 2
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), W, H, spp, out), nprocs=world, join=True)
    frame = np.load(out)
    ref = oracle_lib.render(Scene.cornell_box(W, H), seed_splitmix(W, H), spp * world, 3)
    assert np.array_equal(frame.view(np.uint32), ref.view(np.uint32))

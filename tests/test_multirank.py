"""CPU: the N>1 path of bench.py — interleaved row tiles + one gather — with the
gloo backend (world_size 2 and 3), the oracle standing in for each rank's GPU.
The assembled frame must equal the single-rank frame bit-for-bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from gpuraytracer_amd import place_tiles_host, tile_layout
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


@pytest.mark.parametrize("H", [1, 2, 5, 17, 1080])
def test_c_abi_tile_layout_matches_partition(H):
    """rt_tile_layout (the arithmetic rt_render_gather and its placement use)
    against the Python partition, N in {1, 2, 3, 8, 16}, N > H included."""
    W = 7
    for N in (1, 2, 3, 8, 16):
        for k in range(N):
            for fp16, rgba8, px in ((False, False, 16), (True, False, 8), (False, True, 4)):
                lay = tile_layout(W, H, N, k, fp16, rgba8)
                _, _, count = rank_rows(H, N, k)
                assert lay["rows"] == count, (H, N, k)
                assert lay["rows_max"] == tile_rows_max(H, N)
                assert lay["row_bytes"] == W * px
                assert lay["tile_bytes"] == tile_rows_max(H, N) * W * px


@pytest.mark.parametrize("H", [1, 2, 5, 17, 1080])
def test_c_abi_place_tiles_host_roundtrip(H):
    """rt_place_tiles_host (rank 0's placement after the gather, host form):
    the frame cut into padded interleaved tiles, the padding filled with junk,
    comes back bit-identical for N in {1, 2, 3, 8, 16} in all pixel formats."""
    W = 6
    rng = np.random.default_rng(H)
    for dt in (np.float32, np.uint16, np.uint8):
        frame = rng.integers(0, 255, size=(H, W, 4)).astype(dt)
        for N in (1, 2, 3, 8, 16):
            rmax = tile_rows_max(H, N)
            tiles = np.full((N, rmax, W, 4), 0xAB, dt)
            for k in range(N):
                _, _, count = rank_rows(H, N, k)
                tiles[k, :count] = frame[k::N]
            out = place_tiles_host(tiles, W, H, N)
            assert np.array_equal(out, frame), (dt, N)
    with pytest.raises(ValueError):
        place_tiles_host(np.zeros((3, 2), np.float32), W, H, 2)


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
    if rank == 0:  # the product's placement code (rt_place_tiles_host)
        np.save(result_path, place_tiles_host(torch.stack(gathered).numpy(), W, H, world))
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

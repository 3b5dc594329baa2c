"""Row-tile partition of a frame across ranks and its reassembly.

Each pixel depends only on the scene, its seed and (x, y, n),
so ranks render disjoint rows with the GLOBAL y and the frame is assembled by
one gather.  Rows are interleaved (rank k renders y = k, k+N, k+2N, ...): the
cheap rows (camera sees past the open box front, top/bottom) and the expensive
ones are spread evenly over the ranks, which is what keeps weak scaling flat.
"""
from __future__ import annotations

import numpy as np


def rank_rows(height: int, world: int, rank: int) -> tuple[int, int, int]:
    """(row_start, row_step, row_count) of ``rank``'s interleaved tile.

    row_count is 0 for a rank past the last row (more ranks than rows); such a
    rank must skip its render -- RenderParams reads row_count 0 as "every row"
    -- and join the gather with an empty tile (rt_render_gather does this)."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    count = (height - 1 - rank) // world + 1 if rank < height else 0
    return rank, world, count


def tile_rows_max(height: int, world: int) -> int:
    """Rows of the largest tile (gather buffers are padded to it)."""
    return (height + world - 1) // world


def assemble(tiles, height: int):
    """Interleave gathered (padded) tiles back into an (H, W, C) frame.

    ``tiles``: sequence of N arrays/tensors of shape (rows_max, W, C)."""
    world = len(tiles)
    first = tiles[0]
    is_np = isinstance(first, np.ndarray)
    if is_np:
        frame = np.empty((height,) + tuple(first.shape[1:]), first.dtype)
    else:
        import torch
        frame = torch.empty((height,) + tuple(first.shape[1:]), dtype=first.dtype,
                            device=first.device)
    for k, t in enumerate(tiles):
        _, _, count = rank_rows(height, world, k)
        frame[k::world] = t[:count]
    return frame

#!/usr/bin/env python3
"""Exploration: what one GPU's N = 8 share costs, by row mapping and lanes per pixel.
Prints Msamples/s for the full frame (N = 1), the interleaved share (rows k mod 8),
and contiguous blocks of the same row count, at 4 and 16 lanes per pixel."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime)
from gpuraytracer_amd import RenderParams, Options, Renderer, Scene  # noqa: E402

W, H, SPP = 1920, 1080, 256
res = {}


def t(r, p, rows):
    r.render(p)
    ms = []
    for _ in range(3):
        r.render(p)
        ms.append(r.last_kernel_ms())
    k = min(ms)
    return round(W * rows * p.spp / (k * 1e-3) / 1e6, 1), round(k, 3), r.last_launch()["kernel"]


for lanes in ("4", "16"):
    os.environ["RTPT_LANES"] = lanes
    with Renderer(Scene.cornell_box(W, H), options=Options.from_env()) as r:
        res[f"full_L{lanes}"] = t(r, RenderParams(spp=SPP), H)
        for k in (0, 4):
            res[f"interleaved8_rank{k}_L{lanes}"] = t(
                r, RenderParams(spp=SPP * 8, row_start=k, row_step=8, row_count=135), 135)
        for start in (0, 472, 945):
            res[f"block135_at{start}_L{lanes}"] = t(
                r, RenderParams(spp=SPP * 8, row_start=start, row_step=1, row_count=135), 135)
        res[f"interleaved2_rank0_L{lanes}"] = t(
            r, RenderParams(spp=SPP * 2, row_start=0, row_step=2, row_count=540), 540)
for k, v in res.items():
    print(k, v)
print(json.dumps(res))

#!/usr/bin/env python3
"""Lanes per pixel (RTPT_LANES=4 vs 16) on whole frames and on interleaved
per-GPU shares of the multi-GPU configs (speed only; results are identical)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime)
from gpuraytracer_amd import RenderParams, Options, Renderer, Scene  # noqa: E402

CASES = [  # (W, H, row_step, spp)
    (1920, 1080, 1, 256), (1920, 1080, 2, 512), (1920, 1080, 8, 2048),
    (4096, 4096, 8, 128), (4096, 4096, 1, 32),
]
for lanes in ("4", "16"):
    os.environ["RTPT_LANES"] = lanes
    for W, H, n, spp in CASES:
        with Renderer(Scene.cornell_box(W, H), options=Options.from_env()) as r:
            p = RenderParams(spp=spp, row_start=0, row_step=n, row_count=(H + n - 1) // n)
            r.render(p)
            ms = []
            for _ in range(3):
                r.render(p)
                ms.append(r.last_kernel_ms())
            print(f"L={lanes} {W}x{H} step {n} spp {spp}:",
                  round(W * p.row_count * p.spp / (min(ms) * 1e-3) / 1e6, 1), flush=True)

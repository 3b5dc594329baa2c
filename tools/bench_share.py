#!/usr/bin/env python3
"""One GPU's share of the N-GPU weak-scaling bench (rows y = k (mod N) at 256*N spp),
timed on one GPU: shows how per-GPU throughput depends on N (pixel parallelism)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401  (one HIP runtime)
from gpuraytracer_amd import RenderParams, Options, Renderer, Scene  # noqa: E402
from gpuraytracer_amd.tiles import rank_rows  # noqa: E402

W, H, SPP = 1920, 1080, 256
res = {}
with Renderer(Scene.cornell_box(W, H), options=Options.from_env()) as r:
    for n in (1, 2, 4, 8):
        start, step, rows = rank_rows(H, n, 0)
        p = RenderParams(spp=SPP * n, bounces=3, row_start=start, row_step=step, row_count=rows)
        r.render(p)
        ms = []
        for _ in range(3):
            r.render(p)
            ms.append(r.last_kernel_ms())
        k = min(ms)
        res[n] = {"rows": rows, "spp": SPP * n, "kernel_ms": round(k, 3),
                  "msamples_per_s": round(W * rows * SPP * n / (k * 1e-3) / 1e6, 1)}
print(json.dumps(res))

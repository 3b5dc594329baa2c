#!/usr/bin/env python3
"""Run one render with a -DRT_STATS build (RTPT_LIB=variants/librtpt_stats.so)
and print the per-query culling / divergence counters of rt_kernel.hip."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (one HIP runtime)
from gpuraytracer_amd import RenderParams, Renderer, Scene, lib  # noqa: E402

W, H, SPP = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
with Renderer(Scene.cornell_box(W, H)) as r:
    r.render(RenderParams(spp=SPP, bounces=3))
    st = (ctypes.c_uint64 * 16)()
    assert lib.rt_debug_stats(r._ctx, st, 16) == 0, lib.rt_last_error(r._ctx)
names = ["camera", "bounce", "shadow"]
samples = W * H * SPP
out = {}
for q, n in enumerate(names):
    visits, tested, lanes, divs = st[4 * q:4 * q + 4]
    out[n] = {"pair_visits_per_wave_query": None, "visited": visits, "tested": tested,
              "tested_frac": tested / max(visits, 1), "lane_util": lanes / max(64 * tested, 1),
              "div_blocks_per_tested": divs / max(tested, 1),
              "tested_per_sample": tested * 64 / samples}
q, rounds, rl, ql = st[12:16]
out["clusters"] = {"queries_per_wave": q, "rounds_per_query": rounds / max(q, 1),
                   "lanes_per_round": rl / max(rounds, 1), "lanes_per_query": ql / max(q, 1),
                   "candidate_tests_per_sample": rl / samples}
print(json.dumps(out, indent=1))

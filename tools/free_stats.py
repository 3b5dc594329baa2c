#!/usr/bin/env python3
"""Counters of the free-running kernel (rt_free.hpp) from a -DRT_STATS build
(RTPT_LIB=abvar/librtpt_stats.so):  tools/free_stats.py spheres|triangles [W H SPP]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (one HIP runtime)
from gpuraytracer_amd import Options, RenderParams, Renderer, Scene, lib  # noqa: E402

a = sys.argv[1:]
kind = a[0] if a else "spheres"
W, H, SPP = (int(a[1]), int(a[2]), int(a[3])) if len(a) >= 4 else (480, 270, 16)
scene = (Scene.random_spheres(W, H, 1000, seed=42) if kind == "spheres"
         else Scene.random_triangles(W, H, 100_000))
with Renderer(scene, options=Options(walk="free")) as r:
    r.render(RenderParams(spp=SPP, bounces=3))
    st0 = (ctypes.c_uint64 * 32)()
    assert lib.rt_debug_stats(r._ctx, st0, 32) == 0, lib.rt_last_error(r._ctx)
    st = list(st0)[16:]
    kernel = r.last_launch()["kernel"]
waves = max(st[0], 1)
samples = W * H * SPP
out = {
    "kernel": kernel,
    "services_per_wave": st[1] / waves,
    "lanes_served_per_service": st[2] / max(st[1], 1),
    "live_lanes_per_service": st[3] / max(st[1], 1),
    "walk_steps_per_wave": st[4] / waves,
    "step_lane_util": st[5] / max(64 * st[4], 1),
    "leaf_rounds_per_wave": st[6] / waves,
    "lanes_per_leaf_round": st[7] / max(st[6], 1),
    "service_cycle_share": st[8] / max(st[8] + st[9], 1),
    "cycles_per_wave": (st[8] + st[9]) / waves,
    "queries_per_sample": st[10] / samples,
    "walk_steps_per_query_lane": st[5] / max(st[10], 1),
    "cycles_per_walk_step": st[9] / max(st[4], 1),
    "cycles_per_service": st[8] / max(st[1], 1),
}
print(json.dumps(out, indent=1))

#!/usr/bin/env python3
"""Per-lane BVH walk counters of a -DRT_STATS build (RTPT_LIB=abvar/librtpt_stats.so)
on the config-4 scene, or on the random-triangle scene with a 5th argument:
  tools/sphere_stats.py [W H SPP [N [triangles]]]
(sphere_walk and tri_cbvh_walk share the slots; a triangle scene has no spheres)"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401,E402  (one HIP runtime)
from gpuraytracer_amd import RenderParams, Options, Renderer, Scene, lib  # noqa: E402

a = sys.argv[1:]
W, H, SPP = (int(a[0]), int(a[1]), int(a[2])) if len(a) >= 3 else (480, 270, 16)
TRI = len(a) >= 5 and a[4] == "triangles"
NS = int(a[3]) if len(a) >= 4 else (100000 if TRI else 1000)
scene = Scene.random_triangles(W, H, NS, seed=7) if TRI else Scene.random_spheres(W, H, NS, seed=42)
with Renderer(scene, options=Options.from_env()) as r:
    r.render(RenderParams(spp=SPP, bounces=3))
    st = (ctypes.c_uint64 * 32)()
    assert lib.rt_debug_stats(r._ctx, st, 32) == 0, lib.rt_last_error(r._ctx)
samples = W * H * SPP
out = {}
for name, b in (("closest", 16), ("any", 24)):
    walks, lanes, steps, step_lanes, leaf_lanes, rounds, parked = st[b:b + 7]
    out[name] = {
        "walks_per_sample": walks * 64 / samples,
        "lanes_per_walk": lanes / max(walks, 1),
        "steps_per_walk": steps / max(walks, 1),
        "step_lane_util": step_lanes / max(64 * steps, 1),
        "lane_steps_per_lane_walk": step_lanes / max(lanes, 1),
        "root_rounds_per_walk": rounds / max(walks, 1),
        "split_rounds_per_walk": leaf_lanes / max(walks, 1),  # slot +4: split rounds (RT_SPH_SPLIT)
        "parked_per_round": parked / max(rounds, 1),
        "roots_per_lane_walk": parked / max(lanes, 1),
    }
out["packet"] = {"walks_per_sample": st[23] * 64 / samples,
                 "iters_per_walk": st[31] / max(st[23], 1)}
print(json.dumps(out, indent=1))

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
from gpuraytracer_amd import RenderParams, Options, Renderer, Scene, lib  # noqa: E402

W, H, SPP = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
with Renderer(Scene.cornell_box(W, H), options=Options.from_env()) as r:
    r.render(RenderParams(spp=SPP, bounces=3))
    info = r.last_launch()
    st = (ctypes.c_uint64 * 32)()
    assert lib.rt_debug_stats(r._ctx, st, 32) == 0, lib.rt_last_error(r._ctx)
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
# lane-slot accounting (shader-clock cycles per wave, slots 16-25): where a
# wave's lanes sit idle because their path already ended (miss / light hit at
# an earlier bounce) vs. the cycles of live lanes
round_cyc, n_rounds = st[24], st[25]
bounce = []
idle_dead = 0.0
for b in range(4):
    cyc, cyc_live = st[16 + b], st[20 + b]
    if not cyc:
        continue
    live = cyc_live / cyc / 64.0          # cycle-weighted live fraction at bounce entry
    # lanes dead before bounce b idle for its whole duration
    idle_dead += cyc * (1.0 - live)
    bounce.append({"bounce": b, "cycles_share_of_rounds": cyc / max(round_cyc, 1),
                   "live_lane_frac_at_entry": live})
out["lane_slots"] = {
    "kernel": info["kernel"], "lanes_per_pixel": info["lanes_per_pixel"],
    "rounds_per_wave": n_rounds, "bounces": bounce,
    # share of all round cycles x 64 lanes lost to lanes whose path had ended
    "ended_path_idle_frac": idle_dead / max(round_cyc, 1),
    "note": "remaining lane-slot loss (PMC lane util 1 - SQ_THREAD_CYCLES_VALU/"
            "(64*SQ_ACTIVE_INST_VALU)) minus ended_path_idle_frac = divergence inside the "
            "queries (candidate rounds) and shading branches"}
print(json.dumps(out, indent=1))

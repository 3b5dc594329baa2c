#!/usr/bin/env python3
"""Event log of the free-running kernel (rt_free.hpp) from a -DRT_FREE_DEBUG
build (RTPT_LIB=abvar/librtpt_<v>.so), for test_free_spheres_1000_more_samples:
renders 48x32 x 9 spp on 1000 spheres with walk=free, lists the pixels that
differ from the oracle, then replays the watched pixels' queries:
per sample, the kernel's accumulatedColor against pto_trace_sample; per query,
the kernel's (best, id) against a brute-force id-ordered scan of the spheres
(pto_ray_sphere, strict <); every leaf resolve; and slot 2, the parked leaves
whose walk-loop resolve disagreed with the select-form arithmetic (RT_FREE_CHECK).

    tools/free_debug.py [out.json]"""
import ctypes
import json
import os
import struct
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: F401,E402  (one HIP runtime)
import oracle_lib  # noqa: E402
from gpuraytracer_amd import Options, RenderParams, Renderer, Scene, lib, seed_splitmix  # noqa: E402

W, H, SPP, B = 48, 32, 9, 3
REC, MAX = 12, 1024
WATCH = [(18, 20), (29, 24)]

scene = Scene.random_spheres(W, H, 1000, seed=42)
seeds = seed_splitmix(W, H)
nwords = (4 + 3 * MAX * REC) // 2
with Renderer(scene, seeds=seeds, options=Options(walk="free")) as r:
    st = (ctypes.c_uint64 * nwords)()
    lib.rt_debug_stats(r._ctx, st, nwords)  # clear
    out = r.render(RenderParams(spp=SPP, bounces=B))
    kernel = r.last_launch()["kernel"]
    logged = lib.rt_debug_stats(r._ctx, st, nwords) == 0  # false: not a debug build
raw = np.frombuffer(bytes(st), dtype=np.uint32) if logged else np.zeros(4 + 3 * MAX * REC, np.uint32)
ref = oracle_lib.render(scene, seeds, SPP, B)
diff = out.view(np.uint32) != ref.view(np.uint32)
bad = sorted({(int(x), int(y)) for y, x, c in np.argwhere(diff[..., :3])})
print("kernel", kernel, "differing pixels (x, y):", bad)


def f(u):
    return struct.unpack("<f", struct.pack("<I", int(u)))[0]


def i32(u):
    return struct.unpack("<i", struct.pack("<I", int(u)))[0]


counts = [int(raw[k]) for k in range(4)]  # events of slots 0-2, walk-loop resolves checked
recs = [[raw[4 + (s * MAX + k) * REC: 4 + (s * MAX + k + 1) * REC] for k in range(min(counts[s], MAX))]
        for s in range(3)]

olib = oracle_lib.lib
olib.pto_trace_sample.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                                                         ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32,
                                                         ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p]
olib.pto_ray_sphere.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
P = oracle_lib._p
sph = [(np.array([s.center.x, s.center.y, s.center.z], np.float32), float(s.radius)) for s in scene.spheres]
nT = scene.n_triangles


def brute(o, d, tmin, tmax, shadow):
    """id-ordered scan with strict < (the oracle's sphere loop): (t, id)"""
    o = np.array(o, np.float32)
    d = np.array(d, np.float32)
    best, bid = tmax, -1
    t = ctypes.c_float()
    for k, (c, rad) in enumerate(sph):
        if olib.pto_ray_sphere(P(o), P(d), P(c), ctypes.c_float(rad), ctypes.c_float(tmin),
                               ctypes.c_float(best), ctypes.byref(t)):
            best, bid = t.value, nT + k
            if shadow:
                break
    return best, bid


report = {"kernel": kernel, "bad_pixels": bad, "counts": counts, "pixels": []}
for s, (x, y) in enumerate(WATCH):
    pix = {"x": x, "y": y, "bad_samples": [], "query_mismatch": [], "samples": 0, "queries": 0,
           "resolves_by_site": {"walk_loop_branch": 0, "service": 0, "walk_loop_select": 0}}
    ev = recs[s]
    cur = None
    for rr in ev:
        kind = int(rr[0]) & 0xFF
        ph, b = (int(rr[0]) >> 8) & 0xFF, (int(rr[0]) >> 16) & 0xFF
        n = int(rr[1])
        if kind == 1:
            cur = dict(n=n, b=b, ph=ph, o=[f(v) for v in rr[4:7]], d=[f(v) for v in rr[7:10]],
                       best0=f(rr[10]), id0=i32(rr[11]), resolves=[])
        elif kind == 2 and cur is not None:
            site = ["walk_loop_branch", "service", "walk_loop_select"][int(rr[0]) >> 24]
            pix["resolves_by_site"][site] += 1
            cur["resolves"].append(dict(site=int(rr[0]) >> 24, sid=int(rr[3]), pb=f(rr[4]), disc=f(rr[5]),
                                        t=f(rr[7]), best0=f(rr[8]), id0=i32(rr[9]), best1=f(rr[10]),
                                        id1=i32(rr[11])))
        elif kind == 3 and cur is not None:
            shadow = cur["ph"] == 1
            tmin = 0.0 if shadow else 0.001
            gb, gid = f(rr[4]), i32(rr[11])
            if cur["id0"] >= 0 and shadow:
                cur = None
                continue
            eb, eid = brute(cur["o"], cur["d"], tmin, cur["best0"], shadow)
            pix["queries"] += 1
            if shadow:
                ok = (gid >= 0) == (eid >= 0)
            else:
                ok = (eid < 0 and gid == cur["id0"] and gb == cur["best0"]) or (eid >= 0 and gid == eid and gb == eb)
            if not ok:
                cur.update(gpu=[gb, gid], brute=[eb, eid])
                pix["query_mismatch"].append(cur)
            cur = None
        elif kind == 4:
            acc = np.zeros(3, np.float32)
            olib.pto_trace_sample(P(scene.camera), P(scene.materials), P(scene.light), P(scene.vertices),
                                  scene.n_triangles, P(scene.spheres), scene.n_spheres, int(seeds[y, x]), x, y,
                                  n, B, P(acc))
            g = np.array([f(v) for v in rr[4:7]], np.float32)
            pix["samples"] += 1
            if g.view(np.uint32).tolist() != acc.view(np.uint32).tolist():
                pix["bad_samples"].append(dict(n=n, gpu=g.tolist(), oracle=acc.tolist()))
    report["pixels"].append(pix)
report["check_mismatch"] = [dict(ph=int(rr[0]) & 0xFF, b=int(rr[0]) >> 8, leaf=int(rr[1]), id0=i32(rr[2]),
                                 id_select=i32(rr[3]), pb=f(rr[4]), disc=f(rr[5]), a=f(rr[6]), tmin=f(rr[7]),
                                 best0=f(rr[8]), t_select=f(rr[9]), best_branch=f(rr[10]), id_branch=i32(rr[11]))
                            for rr in recs[2]]
txt = json.dumps(report, indent=1)
print(txt)
if len(sys.argv) > 1:
    open(sys.argv[1], "w").write(txt)

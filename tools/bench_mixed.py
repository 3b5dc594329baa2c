#!/usr/bin/env python3
"""Mixed-scene timing: the Cornell box with both boxes (36
triangles, 18 pair records, 2 KB) plus N random spheres takes the one-wave
sphere kernel; with extra planar quads past the 6 KB per-workgroup pair budget
it falls back to the pair kernel with the 32-B-node sphere walks.  Prints one
JSON line per case: kernel, kernel ms, Msamples/s.

    python tools/bench_mixed.py [--spheres 1000] [--width 1920 --height 1080 --spp 64]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def with_quads(g, base, n_quads, seed=3):
    """base's triangles + n_quads random planar quads (one shared-edge pair each)."""
    rng = np.random.default_rng(seed)
    n0 = base.n_triangles
    n = n0 + 2 * n_quads
    mats = (g.MaterialGPU * n)()
    verts = (g.float3 * (3 * n))()
    ctypes.memmove(ctypes.addressof(mats), ctypes.addressof(base.materials), n0 * 48)
    ctypes.memmove(ctypes.addressof(verts), ctypes.addressof(base.vertices), 3 * n0 * 16)
    vv = np.frombuffer(verts, np.float32).reshape(-1, 4)
    mm = np.frombuffer(mats, np.float32).reshape(-1, 12)
    for q in range(n_quads):
        c = rng.uniform(-2.0, 2.0, 3)
        a, b = rng.normal(size=3) * 0.3, rng.normal(size=3) * 0.3
        P = [c, c + a, c + a + b, c + b]
        for t, tri in enumerate(((P[0], P[1], P[2]), (P[0], P[2], P[3]))):
            k = n0 + 2 * q + t
            vv[3 * k:3 * k + 3, :3] = np.array(tri, np.float32)
            mm[k, 0:3] = 0.5
            mm[k, 3] = 1.0
    return mats, verts


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--spheres", type=int, default=1000)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--quads", default="0,36,37", help="extra planar quads per case")
    a = ap.parse_args(argv)
    import gpuraytracer_amd as g
    from gpuraytracer_amd import Options, Renderer, RenderParams, Scene, seed_splitmix
    base = Scene.cornell_box(a.width, a.height)
    sph = Scene.random_spheres(a.width, a.height, a.spheres, seed=42).spheres
    sd = seed_splitmix(a.width, a.height, key=42)
    for n_quads in [int(q) for q in a.quads.split(",")]:
        if n_quads:
            mats, verts = with_quads(g, base, n_quads)
            s = Scene(base.camera, mats, verts, base.light, sph)
        else:
            s = Scene(base.camera, base.materials, base.vertices, base.light, sph)
        with Renderer(s, seeds=sd, options=Options.from_env()) as r:
            p = RenderParams(spp=a.spp, bounces=3)
            r.render(p)  # warm-up
            ms = []
            for _ in range(a.reps):
                r.render(p)
                ms.append(r.last_kernel_ms())
            k = r.last_launch()["kernel"]
            info = s.describe()
        best = min(ms)
        print(json.dumps({"case": f"cornell36+{a.spheres}spheres+{n_quads}quads",
                          "pair_records": info["n_triangle_pairs"], "kernel": k,
                          "kernel_ms": round(best, 3),
                          "msamples_per_s": round(a.width * a.height * a.spp / best / 1e3, 1)}),
              flush=True)


if __name__ == "__main__":
    main()

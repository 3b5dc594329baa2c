#!/usr/bin/env python3
"""Benchmark of the MIS integrator (rt_render_mis; Sources/gpuRaytracer/shaders.metal
kernel drawTriangle) on one GPU, next to the C oracle on the host cores.

Workload = the reference's own configuration (Sources/gpuRaytracer/main.swift,
shaders.metal:644-649): SwiftPM Cornell scene, 800x600, 6 camera rays per
pixel, 300 MIS samples (100 per strategy).  Unit: MIS samples/s = pixels x
camera rays x mis_samples / kernel time (a camera ray that hits the light or
misses still counts its 300 slots, as the reference's loop bounds do).
Prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_baseline(scene, rays, samples, threads, seconds):
    lib = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    lib.pto_render_mis.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_uint32] * 6 + \
        [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    p = lambda x: ctypes.cast(ctypes.pointer(x) if isinstance(x, ctypes.Structure) else x,  # noqa: E731
                              ctypes.c_void_p)
    W, H = scene.width, scene.height

    def run(step):
        rows = (H - 1) // step + 1
        out = np.empty((rows, W, 4), np.float32)
        t0 = time.perf_counter()
        r = lib.pto_render_mis(p(scene.camera), p(scene.materials), p(scene.light),
                               p(scene.vertices), scene.n_triangles, rays, samples, 0, step, 0,
                               out.ctypes.data_as(ctypes.c_void_p), None, threads)
        assert r == 0
        dt = time.perf_counter() - t0
        return rows * W * rays * (samples // 3 * 3) / dt / 1e6, rows, dt

    step = 64
    while True:
        rate, rows, dt = run(step)
        if dt >= 0.3 or step == 1:
            break
        step = max(1, step // 4)
    want_rows = max(1, int(rate * 1e6 * seconds / (W * rays * samples)))
    step = max(1, H // want_rows)
    rate, rows, dt = run(step)
    return {"value": round(rate, 4), "unit": "M MIS-samples/s", "cores": threads, "kind": "port",
            "sample": f"1 in {step} rows ({rows} rows x {W}) at {rays} camera rays x {samples} "
                      f"MIS samples in {dt:.2f} s (scalar C oracle pto_render_mis)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=600)
    ap.add_argument("--camera-rays", type=int, default=6)
    ap.add_argument("--mis-samples", type=int, default=300)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    a = ap.parse_args()

    import torch
    from gpuraytracer_amd import MisParams, Options, Renderer, Scene

    torch.cuda.set_device(0)
    scene = Scene.cornell_box_mis(a.width, a.height)
    r = Renderer(scene, options=Options.from_env())
    out = torch.empty((a.height, a.width, 4), dtype=torch.float32, device="cuda")
    out8 = torch.empty((a.height, a.width, 4), dtype=torch.uint8, device="cuda")
    p = MisParams(camera_rays=a.camera_rays, mis_samples=a.mis_samples)
    for _ in range(a.warmup):
        r.render_mis(p, out=out, out8=out8)
    ks = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        r.render_mis(p, out=out, out8=out8)  # synchronous
        ks.append(r.last_kernel_ms())
    wall = (time.perf_counter() - t0) / a.steps
    kms = float(np.mean(ks))
    S = a.mis_samples // 3 * 3
    units = a.width * a.height * a.camera_rays * S
    res = {"metric": "MIS integrator M MIS-samples/s (pixels x camera rays x MIS samples)",
           "value": round(units / (kms * 1e-3) / 1e6, 3), "unit": "M MIS-samples/s",
           "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(wall * 1e3, 3),
           "kernel_ms": round(kms, 4), "frames_per_s": round(1e3 / kms, 2),
           "dtype": "f32", "data": "synthetic: SwiftPM Cornell scene (Sources/gpuRaytracer/main.swift)",
           "config": {"workload": f"mis_{a.width}x{a.height}_c{a.camera_rays}_m{a.mis_samples}"},
           "frame_ok": bool(torch.isfinite(out).all().item()),
           "cpu_baseline": None}
    r.close()
    if a.cpu_seconds > 0:
        res["cpu_baseline"] = cpu_baseline(scene, a.camera_rays, a.mis_samples, a.cpu_threads,
                                           a.cpu_seconds)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

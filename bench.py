#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X pathTrace hot path.

Metric (BASELINE.json): Msamples/s (pixels x spp) on the Cornell box at 1080p,
1/2/4/8 MI355X, plus HBM GB/s.  Workload at N=1 = config 2 of BASELINE.json:
Cornell box (RTrace/scene.swift) 1920x1080, 256 spp, 3 bounces, one step = one
full render of the frame on the GPU (the pathTrace dispatch of
RTrace/renderer.swift:117-146) with inputs resident in HBM.

N>1 (torchrun, one process per GPU, RCCL): weak scaling — every rank renders
1080/N interleaved rows of the same 1080p frame at 256*N spp (fixed
1920*1080*256 samples per GPU), then ONE gather of the tiles to rank 0 over
RCCL; the timed step includes the gather.

Prints one JSON line on rank 0.  The CPU baseline (rank 0, N=1 only) is the
scalar C oracle (oracle/liboracle.so, "port") on a bounded sample of the same
frame, timed on this host's cores.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec (pixels×spp) Cornell box 1080p at 1/2/4/8 MI355X; HBM GB/s"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / 2  # CUs x SIMDs x clock / 2 cycles per wave64 VALU op
BYTES_PER_PIXEL = 4 + 16       # seed read (u32) + rgba32F store, per launch


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="cornell", choices=["cornell", "spheres", "triangles"])
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=256, help="samples per pixel per GPU")
    ap.add_argument("--bounces", type=int, default=3)
    ap.add_argument("--spheres", type=int, default=1000)
    ap.add_argument("--triangles", type=int, default=100000,
                    help="random triangles added to the room for --scene triangles")
    ap.add_argument("--batch-spp", type=int, default=0,
                    help="progressive mode: launches of this many spp into a running sum")
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-threads", type=int, default=0)
    return ap.parse_args()


def load_profile_json(name):
    p = os.path.join(ROOT, "profiles", name)
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except ValueError:
            return None
    return None


def cpu_baseline(scene, width, height, bounces, threads, cpu_seconds=10.0):
    """Scalar C oracle (the identical shader math) on the host cores."""
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    L.pto_render.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_void_p, ctypes.c_uint32,
                             ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [ctypes.c_void_p] * 3 + [ctypes.c_int]
    from gpuraytracer_amd import seed_splitmix
    seeds = seed_splitmix(width, height)

    def run(spp, row_step, nthreads):
        rows = (height - 1) // row_step + 1
        out = np.empty((rows, width, 4), np.float32)
        ptr = lambda x: ctypes.cast(ctypes.pointer(x), ctypes.c_void_p)  # noqa: E731
        t0 = time.perf_counter()
        r = L.pto_render(ptr(scene.camera), ctypes.cast(scene.materials, ctypes.c_void_p),
                         ptr(scene.light), ctypes.cast(scene.vertices, ctypes.c_void_p),
                         scene.n_triangles,
                         None if scene.spheres is None else ctypes.cast(scene.spheres, ctypes.c_void_p),
                         scene.n_spheres, seeds.ctypes.data_as(ctypes.c_void_p), spp, bounces, 0,
                         0, row_step, 0, None, None, out.ctypes.data_as(ctypes.c_void_p), nthreads)
        dt = time.perf_counter() - t0
        assert r == 0
        return rows * width * spp / dt / 1e6, rows * width * spp, dt

    def sized(seconds, nthreads):
        # probe on ever denser row sets until one takes >= 0.3 s, then size the
        # sample to ~`seconds` of CPU work
        step = 256
        while True:
            rate, _, t = run(1, step, nthreads)
            if t >= 0.3 or step == 1:
                break
            step = max(1, step // 4)
        want = rate * 1e6 * seconds
        frame = width * height
        if want >= frame:
            spp, step = max(1, int(round(want / frame))), 1
        else:
            spp, step = 1, max(1, int(math.ceil(frame / want)))
        v, n, t = run(spp, step, nthreads)
        rows = "the full" if step == 1 else f"1 in {step} rows of the"
        return v, f"{rows} {width}x{height} frame at {spp} spp, {bounces} bounces = {n} samples in {t:.2f} s"

    v_all, s_all = sized(cpu_seconds, threads)
    v_one, s_one = sized(cpu_seconds / 4, 1)
    return {"value": round(v_all, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{s_all} on {threads} threads (scalar C oracle, -O2)",
            "single_thread_value": round(v_one, 4), "single_thread_sample": s_one}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 must be launched with torch.distributed.run "
                             "(one process per GPU)")
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    from gpuraytracer_amd import Renderer, RenderParams, Scene
    from gpuraytracer_amd.tiles import assemble, rank_rows, tile_rows_max

    W, H = args.width, args.height
    if args.scene == "cornell":
        scene = Scene.cornell_box(W, H)
        workload = f"cornell_{W}x{H}_{args.spp}spp_b{args.bounces}"
        if args.batch_spp:
            workload += f"_progressive{args.batch_spp}"
    elif args.scene == "spheres":
        scene = Scene.random_spheres(W, H, args.spheres, seed=42)
        workload = f"spheres{args.spheres}_{W}x{H}_{args.spp}spp_b{args.bounces}"
    else:
        scene = Scene.random_triangles(W, H, args.triangles, seed=7)
        workload = f"triangles{args.triangles}_{W}x{H}_{args.spp}spp_b{args.bounces}"
    renderer = Renderer(scene, device=local)
    row_start, row_step, rows = rank_rows(H, world, rank)
    spp = args.spp * world  # weak scaling: W*H*spp samples per GPU whatever N
    rows_max = tile_rows_max(H, world)
    tile = torch.empty((rows_max, W, 4), dtype=torch.float32, device=device)
    params = RenderParams(spp=spp, bounces=args.bounces, row_start=row_start, row_step=row_step,
                          row_count=rows)
    gathered = [torch.empty_like(tile) for _ in range(world)] if (world > 1 and rank == 0) else None
    stream = torch.cuda.current_stream()

    def step(evs=None):
        if evs is not None:
            evs[0].record(stream)
        if args.batch_spp:
            renderer.render_progressive(params, args.batch_spp, out=tile, stream=stream)
        else:
            renderer.render(params, out=tile, stream=stream)
        if evs is not None:
            evs[1].record(stream)
        if world > 1:
            dist.gather(tile, gathered, dst=0)

    for _ in range(args.warmup):
        step()
    events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    if world > 1:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms_max = float(t[0]), float(t[1])
    else:
        kernel_ms_max = kernel_ms

    frame_ok = True
    if rank == 0:
        frame = assemble(gathered, H) if world > 1 else tile[:rows]
        frame_ok = bool(torch.isfinite(frame).all().item()) and bool((frame[..., 3] == 1).all().item())

    if rank == 0:
        total_samples = W * H * spp * args.steps  # all ranks together
        value = total_samples / elapsed / 1e6
        launch_bytes = W * rows * BYTES_PER_PIXEL
        if args.batch_spp and spp > args.batch_spp:
            # per step: first batch 20 B/px (seed + sum write), middle batches 36 B/px
            # (+ sum read), last 52 B/px (+ frame store) — SURVEY §8d
            nb = -(-spp // args.batch_spp)
            launch_bytes = W * rows * (20 + 36 * (nb - 2) + 52)
        achieved = launch_bytes / (kernel_ms * 1e-3) / 1e9
        traffic = None
        prof = load_profile_json("pmc_summary.json")
        compute = None
        from gpuraytracer_amd.srchash import kernel_source_sha
        if (prof and prof.get("workload") == workload and prof.get("n_gpus", 1) == 1 and world == 1
                and prof.get("kernel_src_sha") == kernel_source_sha()):
            traffic = prof.get("hbm_bytes_per_launch")
            if prof.get("sq_insts_valu_per_launch"):
                wi = prof["sq_insts_valu_per_launch"] / (kernel_ms * 1e-3)
                compute = {"bound": "valu", "achieved": round(wi / 1e9, 2),
                           "peak": round(VALU_PEAK_WAVE_INSTR / 1e9, 2),
                           "unit": "G wave64-VALU-instr/s", "frac": round(wi / VALU_PEAK_WAVE_INSTR, 4),
                           "source": "SQ_INSTS_VALU per launch (profiles/pmc_summary.json) / live kernel time"}
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": ("synthetic: reference Cornell scene (scene.swift), splitmix64 seeds"
                     if args.scene == "cornell" else
                     f"synthetic: {args.spheres} PCG32 spheres (seed 42) in the Cornell room, "
                     "splitmix64 seeds" if args.scene == "spheres" else
                     f"synthetic: {args.triangles} random triangles (PCG64 seed 7) in the "
                     "Cornell room, splitmix64 seeds"),
            "config": {"workload": workload, "width": W, "height": H, "spp_per_gpu": args.spp,
                       "spp_frame": spp, "bounces": args.bounces,
                       "parallelism": (f"{world} row-interleaved tiles + 1 RCCL gather" if world > 1
                                       else "single GPU")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 4), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "path_trace_kernel", "kernel_ms": round(kernel_ms, 4),
                         "algorithmic_bytes_per_launch": launch_bytes},
            "compute_roofline": compute,
            "kernel_ms_max_rank": round(kernel_ms_max, 4),
            "frame_ok": frame_ok,
            "cpu_baseline": None,
        }
        if world == 1 and args.cpu_baseline != "off":
            try:
                aff = len(os.sched_getaffinity(0))
            except AttributeError:
                aff = os.cpu_count() or 1
            threads = args.cpu_threads or max(1, min(16, aff))
            out["cpu_baseline"] = cpu_baseline(scene, W, H, args.bounces, threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    renderer.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""bench.py — headline benchmark of the MI355X pathTrace hot path.

Metric (BASELINE.json): Msamples/s (pixels x spp) on the Cornell box at 1080p,
1/2/4/8 MI355X, plus HBM GB/s.  Workload at N=1 = config 2 of BASELINE.json:
Cornell box (RTrace/scene.swift) 1920x1080, 256 spp, 3 bounces; one step = one
full render of the frame on the GPU (the pathTrace dispatch of
RTrace/renderer.swift:117-146) with inputs resident in HBM.

N>1, one process per GPU (launched by torch.distributed.run, or by this script
itself: `python bench.py --gpus N` spawns its N ranks as child processes before
anything touches a GPU).  Weak scaling: every rank renders the 1080/N
interleaved rows y = rank (mod N) of the same 1080p frame at 256*N spp (fixed
1920*1080*256 samples per GPU); the tiles are gathered to rank 0 by ONE RCCL
gather inside the C-ABI (rt_comm_init / rt_render_gather, include/rtpt.h) and
the timed step includes it.  torch.distributed (gloo, CPU) only carries the
communicator id, the barriers and the max over ranks.

Prints one JSON line on rank 0.  The CPU baseline (rank 0, N=1 only) is the
scalar C oracle (oracle/liboracle.so, "port") on every core this process may
use, on a bounded sample of the same frame: rows of the timed image at the
timed spp, which are also compared bit for bit with the GPU's timed frame.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Msamples/sec (pixels×spp) Cornell box 1080p at 1/2/4/8 MI355X; HBM GB/s"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# VALU issue peak: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 VALU
# instruction (a 64-lane op issues over 2 cycles on the 32-wide SIMD)
VALU_PEAK_WAVE_INSTR = 256 * 4 * 2.4e9 / 2
BYTES_PER_PIXEL = 4 + 16       # seed read (u32) + rgba32F store, per launch


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=150,
                    help="timed steps (default: ~4 s of GPU time at N=1)")
    ap.add_argument("--warmup", type=int, default=3)
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
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads (default: every CPU this process may use: its "
                         "affinity, capped by the cgroup CPU quota)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    return ap.parse_args(argv)


def visible_gpus() -> int:
    """GPUs a rank could open, counted WITHOUT initialising HIP in this process
    (the launcher must stay GPU-free: its children are the ranks).  The count
    runs in a short-lived child interpreter (torch.cuda.device_count there may
    initialise HIP; that child exits before any rank starts)."""
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       capture_output=True, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (IndexError, ValueError):
        raise SystemExit(f"could not count GPUs: {r.stderr.strip()[-400:]}")


def spawn_ranks(n: int, argv=None, count_gpus=visible_gpus) -> int:
    """`--gpus N` outside torchrun: start N ranks of this script as child
    processes (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set), before any GPU call in
    this process, and return the worst exit status."""
    import socket
    have = count_gpus()
    if have < n:
        raise SystemExit(f"--gpus {n}: only {have} GPU(s) visible")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] +
                                      list(sys.argv[1:] if argv is None else argv), env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


class CudaBackend:
    """The GPU touchpoints of the bench: device, frame tensor, stream, HIP
    events (torch.cuda.Event on the stream the kernel is launched on), sync and
    the renderer (librtpt.so through the C-ABI).  tests/test_bench_glue.py
    swaps in a CPU stand-in to exercise the multi-rank glue with gloo."""

    def __init__(self, local: int):
        import torch
        self.torch = torch
        torch.cuda.set_device(local)
        self.device = torch.device("cuda", local)
        self.local = local

    def renderer(self, scene):
        from gpuraytracer_amd import Options, Renderer
        return Renderer(scene, device=self.local, options=Options.from_env())

    def comm_unique_id(self) -> bytes:
        from gpuraytracer_amd import comm_unique_id
        return comm_unique_id()

    def empty_frame(self, H, W):
        return self.torch.empty((H, W, 4), dtype=self.torch.float32, device=self.device)

    def stream(self):
        return self.torch.cuda.current_stream()

    def event(self):
        return self.torch.cuda.Event(enable_timing=True)

    def synchronize(self):
        self.torch.cuda.synchronize()


def gather_check_rows(H: int, world: int):
    """Rows rank 0 re-renders locally after an N > 1 run: the first row of
    every rank's tile and the last row of the frame."""
    return sorted(set(range(min(world, H))) | {H - 1})


def load_profile_json(name):
    p = os.path.join(ROOT, "profiles", name)
    if os.path.exists(p):
        try:
            return json.load(open(p))
        except ValueError:
            return None
    return None


def host_cpu():
    """Cores this process may use and the host CPU model (BASELINE.md asks for
    nproc and the lscpu model next to every CPU number)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:  # cgroup v2 CPU quota ("max 100000" = none)
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(math.ceil(quota))))
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota,
            "usable_cpus": usable, "model": model}


def cpu_baseline(scene, width, height, spp, bounces, threads, seconds, gpu_frame):
    """Scalar C oracle (the identical shader math) on the host cores, timed on
    rows y = 0 (mod step) of the same frame at the timed spp, sized to about
    `seconds`; those rows are then compared with the GPU's timed frame."""
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "liboracle.so"))
    L.pto_render.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_void_p, ctypes.c_uint32,
                             ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [ctypes.c_void_p] * 3 + [ctypes.c_int]
    from gpuraytracer_amd import seed_splitmix
    seeds = seed_splitmix(width, height)

    def run(n_spp, row_step, nthreads):
        rows = (height - 1) // row_step + 1
        out = np.empty((rows, width, 4), np.float32)
        ptr = lambda x: ctypes.cast(ctypes.pointer(x), ctypes.c_void_p)  # noqa: E731
        t0 = time.perf_counter()
        r = L.pto_render(ptr(scene.camera), ctypes.cast(scene.materials, ctypes.c_void_p),
                         ptr(scene.light), ctypes.cast(scene.vertices, ctypes.c_void_p),
                         scene.n_triangles,
                         None if scene.spheres is None else ctypes.cast(scene.spheres, ctypes.c_void_p),
                         scene.n_spheres, seeds.ctypes.data_as(ctypes.c_void_p), n_spp, bounces, 0,
                         0, row_step, 0, None, None, out.ctypes.data_as(ctypes.c_void_p), nthreads)
        dt = time.perf_counter() - t0
        assert r == 0
        return out, rows * width * n_spp, dt

    # probe the rate at 1 spp on a sparse row set, then size the timed sample
    step = 64
    while True:
        _, n, t = run(1, step, threads)
        if t >= 0.3 or step == 1:
            break
        step = max(1, step // 4)
    rate = n / t
    want_rows = rate * seconds / (width * spp)
    step = max(1, int(math.ceil(height / max(want_rows, 1.0))))
    out, n, t = run(spp, step, threads)
    v_all = n / t / 1e6
    ref = out
    got = gpu_frame[::step]
    same = bool(np.array_equal(got.view(np.uint32), ref.view(np.uint32)))
    # single thread: 1 spp on a sparse row set, ~seconds/4 (the all-thread
    # probe rate over the threads that could actually run at once)
    per_thread = rate / max(1, min(threads, host_cpu()["usable_cpus"]))
    step1 = max(1, int(math.ceil(height / max(per_thread * seconds / 4 / width, 1.0))))
    _, n1, t1 = run(1, step1, 1)
    rows = "every row" if step == 1 else f"rows y = 0 (mod {step})"
    return {"value": round(v_all, 4), "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": (f"{rows} of the {width}x{height} frame at {spp} spp, {bounces} bounces = "
                       f"{n} samples in {t:.2f} s on {threads} threads (scalar C oracle, -O2)"),
            "host": host_cpu(),
            "single_thread_value": round(n1 / t1 / 1e6, 4),
            "single_thread_sample": (f"rows y = 0 (mod {step1}) at 1 spp = {n1} samples in "
                                     f"{t1:.2f} s"),
            "timed_frame_rows_bit_exact_vs_oracle": same,
            "timed_frame_rows_checked": (height - 1) // step + 1}


def main(argv=None, backend_factory=CudaBackend):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world == 1 and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, argv))
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} but --gpus {args.gpus}")
    import torch
    import torch.distributed as dist

    if world > 1:  # CPU plumbing only: comm id, barriers, max over ranks
        dist.init_process_group("gloo")
    be = backend_factory(local)

    from gpuraytracer_amd import RenderParams, Scene

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
    renderer = be.renderer(scene)
    comm = None
    if world > 1:
        ids = [be.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(ids, src=0)
        renderer.comm_init(rank, world, ids[0])
        # what RCCL itself counts (ncclCommCount / ncclCommUserRank), from every rank
        mine = torch.tensor(list(renderer.comm_info()) + [rank], dtype=torch.int64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        comm = {"comm_ranks": int(allr[0][0]),
                "comm_ranks_consistent": all(int(a[0]) == world and int(a[1]) == int(a[2])
                                             for a in allr)}
    spp = args.spp * world  # weak scaling: W*H*spp samples per GPU whatever N
    rows = (H - 1 - rank) // world + 1 if rank < H else 0  # this rank's interleaved rows
    frame = be.empty_frame(H, W) if rank == 0 else None
    params = RenderParams(spp=spp, bounces=args.bounces)
    stream = be.stream()

    def step(evs=None):
        if evs is not None:
            evs[0].record(stream)
        if args.batch_spp:
            renderer.render_progressive(params, args.batch_spp, out=frame, stream=stream,
                                        gather=world > 1)
        elif world > 1:
            renderer.render_gather(params, out=frame, stream=stream)
        else:
            renderer.render(params, out=frame, stream=stream)
        if evs is not None:
            evs[1].record(stream)

    def barrier():
        be.synchronize()
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        step()
    launch = renderer.last_launch()
    events = [(be.event(), be.event()) for _ in range(args.steps)]
    barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(events[k])
    barrier()
    elapsed = time.perf_counter() - t0
    # HIP events on the stream the kernel runs on, around every timed step: at
    # N = 1 a step is exactly one kernel launch (or the launches of one
    # progressive frame).  At N > 1 a step also holds the gather: the kernel
    # alone is the one launch's own events (rt_last_kernel_ms), except in
    # progressive mode, where a step has several launches and the whole step
    # (render + gather) is the time basis.
    step_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    if world == 1:
        kernel_ms, basis = step_ms, "kernel launches of one step (HIP events)"
    elif args.batch_spp:
        kernel_ms, basis = step_ms, "whole step: every progressive launch + the gather (HIP events)"
    else:
        kernel_ms, basis = renderer.last_kernel_ms(), "the render launch of the last step (HIP events)"
    # the gather's share of a step on this rank: the step minus its render
    # launch (not separable in progressive mode, where the C-ABI runs several
    # launches and the gather inside one call)
    gather_ms = step_ms - kernel_ms if world > 1 and not args.batch_spp else None
    per_rank = None
    if world > 1:
        mine = torch.tensor([elapsed, kernel_ms, step_ms, -1.0 if gather_ms is None else gather_ms],
                            dtype=torch.float64)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = torch.stack(allr).numpy()
        elapsed, kernel_ms_max, step_ms_max = (float(v) for v in per_rank[:, :3].max(axis=0))
    else:
        kernel_ms_max, step_ms_max = kernel_ms, step_ms

    if rank == 0:
        frame_ok = bool(torch.isfinite(frame).all().item()) and bool((frame[..., 3] == 1).all().item())
        gather_check = None
        if world > 1:
            # placement proof: rows of every rank's tile, re-rendered here by
            # one local rt_render each, must equal the gathered frame bit for bit
            host = frame.cpu().numpy()
            check = gather_check_rows(H, world)
            same = all(np.array_equal(
                renderer.render(RenderParams(spp=spp, bounces=args.bounces, row_start=y,
                                             row_count=1))[0].view(np.uint32),
                host[y].view(np.uint32)) for y in check)
            gather_check = {"rows": check, "bit_exact_vs_local_render": bool(same)}
        total_samples = W * H * spp * args.steps  # all ranks together
        value = total_samples / elapsed / 1e6
        launch_bytes = W * rows * BYTES_PER_PIXEL
        if args.batch_spp and spp > args.batch_spp:
            # per step: first batch 20 B/px (seed + sum write), middle batches 36 B/px
            # (+ sum read), last 52 B/px (+ frame store) — SURVEY §8d
            nb = -(-spp // args.batch_spp)
            launch_bytes = W * rows * (20 + 36 * (nb - 2) + 52)
        kernel_s = kernel_ms * 1e-3
        achieved = launch_bytes / kernel_s / 1e9
        traffic = None
        prof = load_profile_json("pmc_summary.json")
        compute = None
        from gpuraytracer_amd.srchash import kernel_source_sha
        if (prof and prof.get("workload") == workload and prof.get("n_gpus", 1) == 1 and world == 1
                and prof.get("kernel_src_sha") == kernel_source_sha()):
            traffic = prof.get("hbm_bytes_per_launch")
            if prof.get("sq_insts_valu_per_launch"):
                wi = prof["sq_insts_valu_per_launch"] / kernel_s
                compute = {"bound": "valu", "achieved": round(wi / 1e9, 2),
                           "peak": round(VALU_PEAK_WAVE_INSTR / 1e9, 2),
                           "unit": "G wave64-VALU-instr/s", "frac": round(wi / VALU_PEAK_WAVE_INSTR, 4),
                           "peak_derivation": "256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 "
                                              "VALU instruction",
                           "source": "SQ_INSTS_VALU per launch (profiles/pmc_summary.json, same "
                                     "kernel_src_sha) / live kernel time"}
                lane = prof.get("valu_lane_utilization")
                if lane:
                    # useful lanes: issue fraction x the active lanes per issued
                    # VALU instruction (SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU)
                    compute["valu_lane_utilization"] = round(lane, 4)
                    compute["lane_weighted_frac"] = round(wi / VALU_PEAK_WAVE_INSTR * lane, 4)
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
                       "parallelism": (f"{world} row-interleaved tiles + 1 RCCL gather "
                                       "(rt_render_gather)" if world > 1 else "single GPU")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 4), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": launch["kernel"], "kernel_ms": round(kernel_s * 1e3, 4),
                         "kernel_ms_basis": basis,
                         "algorithmic_bytes_per_launch": launch_bytes},
            "compute_roofline": compute,
            "launch": launch,
            # rt_create's scene build: which triangle-BVH build ran and how long
            # it and the host scene compile took (outside the timed steps)
            "build": (renderer.build_info() if hasattr(renderer, "build_info") else None),
            "step_ms_events": round(step_ms, 4),
            "kernel_ms_max_rank": round(kernel_ms_max, 4),
            "step_ms_max_rank": round(step_ms_max, 4),
            "frame_ok": frame_ok,
            "cpu_baseline": None,
        }
        if comm is not None:
            out.update(comm)
            out["gather_check"] = gather_check
            # render imbalance vs collective: the slowest and fastest render
            # launch over the ranks, and the gather's share of each rank's step
            out["kernel_ms_min_rank"] = round(float(per_rank[:, 1].min()), 4)
            out["gather_ms"] = (None if gather_ms is None else
                                round(float(per_rank[:, 3].max()), 4))
            out["gather_ms_basis"] = ("step - render launch on each rank (HIP events), max over ranks"
                                      if gather_ms is not None else
                                      "not separable: progressive launches and the gather run in one call")
        if world == 1 and args.cpu_baseline != "off":
            # every CPU this process may run on at once: the affinity mask,
            # capped by the cgroup CPU quota (oversubscribing a 16-CPU quota
            # with 256 threads measured 13.2 instead of 22.3 Msamples/s)
            threads = args.cpu_threads or host_cpu()["usable_cpus"]
            out["cpu_baseline"] = cpu_baseline(scene, W, H, spp, args.bounces, threads,
                                               args.cpu_seconds, frame.cpu().numpy())
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    renderer.close()


if __name__ == "__main__":
    main()

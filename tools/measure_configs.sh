#!/bin/bash
# Re-measure the BASELINE.json configs on one MI355X (run through gpurun):
#   tools/measure_configs.sh [outdir]   (default gpurun_out/configs)
# c1 = 128^2 x 1 spp; c3/c5 = one GPU's share of the 8-GPU configs; config 4 =
# 1000 spheres; triangle meshes (GPU-built BVH); the multi-GPU per-GPU shares;
# the MIS integrator.  Each step runs under its own time limit and the script
# stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/configs}
mkdir -p "$OUT"
cd "$R"
run() {  # run <name> <seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "[configs] $name" >&2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "[configs] $name failed" >&2; tail "$OUT/$name.err" >&2; exit 1; }
  tail -c 300 "$OUT/$name.json" >&2; echo >&2
}
run c1_128sq_1spp 120 python bench.py --width 128 --height 128 --spp 1 --steps 5 --warmup 1
run c2_1080p_256spp 180 python bench.py --steps 5 --warmup 1 --cpu-baseline off
run c3_share_4096sq_128spp 180 python bench.py --width 4096 --height 4096 --spp 128 --steps 2 --warmup 1 --cpu-baseline off
run c4_spheres1000 180 python bench.py --scene spheres --steps 3 --warmup 1 --cpu-baseline off
run c5_share_8192sq_512spp_progressive64 240 python bench.py --width 8192 --height 8192 --spp 512 --batch-spp 64 --steps 2 --warmup 1 --cpu-baseline off
run triangles10k 180 python bench.py --scene triangles --triangles 10000 --spp 64 --steps 2 --warmup 1 --cpu-baseline off
run triangles100k 180 python bench.py --scene triangles --triangles 100000 --spp 64 --steps 2 --warmup 1 --cpu-baseline off
run triangles1m 240 python bench.py --scene triangles --triangles 1000000 --spp 16 --steps 2 --warmup 1 --cpu-baseline off
run multi_gpu_shares 180 python tools/bench_share.py
run mis_800x600_c6_m300 240 python tools/bench_mis.py

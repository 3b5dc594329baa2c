#!/bin/bash
# Round 5: free-running kernel on the GPU box -- its parity tests, then the
# config-4 and 100k-triangle benches with walk=lockstep and walk=free.
#   tools/r5_free.sh <tag>
set -u
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
step() {  # step <name> <seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "[r5] $name" >&2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  tail -c 300 "$OUT/$name.out" >&2; echo >&2
  if [ $rc -ne 0 ]; then echo "[r5] $name failed rc=$rc" >&2; tail -30 "$OUT/$name.err" >&2; tail -30 "$OUT/$name.out" >&2; exit $rc; fi
}
step tests_free 400 python -u -m pytest tests/test_gpu_free.py -x -v --timeout 300 --timeout-method thread
for w in ${WALKS:-lockstep free}; do
  step sph_$w 200 env RTPT_WALK=$w python bench.py --scene spheres --steps 6 --warmup 1 --cpu-baseline off
  step tri_$w 300 env RTPT_WALK=$w python bench.py --scene triangles --triangles 100000 --spp 64 --steps 4 --warmup 1 --cpu-baseline off
done

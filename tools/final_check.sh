#!/bin/bash
# End-of-round GPU check (run through gpurun): GPU tests, smoke, rocprofv3 of the
# Cornell and config-4 kernels, then both benches.  Stops at the first failure.
#   tools/final_check.sh <tag>
set -u
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
step() {  # step <name> <seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "[final] $name" >&2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  tail -c 400 "$OUT/$name.out" >&2; echo >&2
  if [ $rc -ne 0 ]; then echo "[final] $name failed rc=$rc" >&2; tail -20 "$OUT/$name.err" >&2; exit $rc; fi
}
step gputest 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof_cornell 600 bash tools/profile.sh ${TAG}_cornell
step prof_spheres 600 bash tools/profile.sh ${TAG}_spheres --scene spheres
step prof_mis 600 env PROFILE_TARGET=mis bash tools/profile.sh ${TAG}_mis
step prof_tri100k 600 bash tools/profile.sh ${TAG}_tri100k --scene triangles --triangles 100000 --spp 64
step bench 400 python bench.py
step spheres 300 python bench.py --scene spheres --steps 8 --warmup 1 --cpu-baseline off

#!/bin/bash
# One GPU round trip (run through gpurun): GPU parity tests, then the headline
# bench and the config-4 sphere bench.  Stops at the first failure.
#   tools/gpu_check.sh [tag] [pytest -k expression]
set -u
TAG=${1:-check}
KEXPR=${2:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
step() {  # step <name> <seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "[check] $name" >&2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  tail -c 600 "$OUT/$name.out" >&2; echo >&2
  if [ $rc -ne 0 ]; then echo "[check] $name failed rc=$rc" >&2; tail -20 "$OUT/$name.err" >&2; exit $rc; fi
}
if [ -n "$KEXPR" ]; then
  step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR"
else
  step tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
fi
step bench 300 python bench.py --steps 60 --cpu-baseline off
step spheres 300 python bench.py --scene spheres --steps 8 --warmup 1 --cpu-baseline off

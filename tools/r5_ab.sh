#!/bin/bash
# Round 5 GPU A/B: the BVH parity tests (builds, walk schedulers), then benches
# of config 4 and the 100k-triangle mesh under each walk scheduler and build.
#   tools/r5_ab.sh <tag> [bench specs: scene:ENV=VAL,...]
set -u
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
step() {  # step <name> <seconds> <cmd...>
  local name=$1 lim=$2; shift 2
  echo "[r5] $name" >&2
  timeout -k 10 "$lim" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[r5] $name failed rc=$rc" >&2; tail -30 "$OUT/$name.err" >&2; tail -30 "$OUT/$name.out" >&2; exit $rc; fi
}
if [ -z "${NOTEST:-}" ]; then
  step tests 600 python -u -m pytest tests/test_gpu_free.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "${TESTK:-free or triangle_bvh or sphere}"
  tail -2 "$OUT/tests.out" >&2
fi
for spec in "$@"; do
  sc=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  NAME="$sc$(printf '_%s' ${envs//,/ })"
  case $sc in
    spheres) ARGS="--scene spheres --steps 6 --warmup 1";;
    tri100k) ARGS="--scene triangles --triangles 100000 --spp 64 --steps 4 --warmup 1";;
    tri1m) ARGS="--scene triangles --triangles 1000000 --spp 16 --steps 3 --warmup 1";;
    tri10k) ARGS="--scene triangles --triangles 10000 --spp 64 --steps 4 --warmup 1";;
    cornell) ARGS="--steps 10 --warmup 2";;
  esac
  step "b_$NAME" 300 env ${envs//,/ } python bench.py $ARGS --cpu-baseline off
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=d.get('build') or {}; print(sys.argv[2], d['value'], d['ms_per_step'], d['launch']['kernel'], 'build_ms', round(b.get('tri_bvh_build_ms', 0), 1))" "$OUT/b_$NAME.out" "$NAME" >&2
done

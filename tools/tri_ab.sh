#!/bin/bash
# Triangle-BVH A/B on the GPU box: BVH parity tests + the 100k-triangle bench for
# each <variant>[:ENV=VAL,...] ("base" = in-tree librtpt.so, else abvar/librtpt_<v>.so).
#   tools/tri_ab.sh <tag> <spec>...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
for spec in "$@"; do
  v=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  if [ "$v" = base ]; then L=$R/gpuraytracer_amd/librtpt.so; else L=$R/abvar/librtpt_$v.so; fi
  NAME="$v$(printf '_%s' ${envs//,/ })"
  if [ -z "${AB_NOTEST:-}" ]; then
    env RTPT_LIB=$L ${envs//,/ } timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 \
      --timeout-method thread -k "triangle_bvh" > "$OUT/$NAME.tests" 2>&1 || { tail -30 "$OUT/$NAME.tests" >&2; exit 1; }
    echo "$NAME tests: $(tail -1 "$OUT/$NAME.tests")" >&2
  fi
  env RTPT_LIB=$L ${envs//,/ } timeout -k 10 300 python bench.py --scene triangles --triangles ${TRIS:-100000} --spp 64 \
    --steps 4 --warmup 1 --cpu-baseline off > "$OUT/$NAME.bench" 2> "$OUT/$NAME.err" || { tail -20 "$OUT/$NAME.err" >&2; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/$NAME.bench" "$NAME" >&2
done

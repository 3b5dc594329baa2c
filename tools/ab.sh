#!/bin/bash
# A/B of kernel variants on the GPU box: parity tests (-k $AB_K) + bench for
# each abvar/ variant ("base" = in-tree librtpt.so).
#   AB_ARGS="--scene spheres --steps 8" AB_K=sphere tools/ab.sh <tag> <variant>...
#   AB_NOTEST=1 skips the tests.
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
ARGS=${AB_ARGS:---steps 40 --warmup 2}
for v in "$@"; do
  if [ "$v" = base ]; then export RTPT_LIB=$R/gpuraytracer_amd/librtpt.so; else export RTPT_LIB=$R/abvar/librtpt_$v.so; fi
  echo "[ab] $v" >&2
  if [ -z "${AB_NOTEST:-}" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
      -k "${AB_K:-parity}" > "$OUT/$v.tests" 2>&1 || { tail -30 "$OUT/$v.tests" >&2; exit 1; }
    tail -1 "$OUT/$v.tests" >&2
  fi
  timeout -k 10 300 python bench.py $ARGS --cpu-baseline off \
    > "$OUT/$v.bench" 2> "$OUT/$v.err" || { tail -20 "$OUT/$v.err" >&2; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/$v.bench" "$v" >&2
done

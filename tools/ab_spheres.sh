#!/bin/bash
# Config-4 A/B on the GPU box: sphere parity tests + bench for each abvar/ variant.
#   tools/ab_spheres.sh <tag> <variant>...   (variant "base" = in-tree librtpt.so)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
for v in "$@"; do
  if [ "$v" = base ]; then export RTPT_LIB=$R/gpuraytracer_amd/librtpt.so; else export RTPT_LIB=$R/abvar/librtpt_$v.so; fi
  echo "[ab] $v" >&2
  if [ "$v" != base ] && [ -z "${AB_NOTEST:-}" ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
      -k "sphere" > "$OUT/$v.tests" 2>&1 || { tail -30 "$OUT/$v.tests" >&2; exit 1; }
    tail -1 "$OUT/$v.tests" >&2
  fi
  timeout -k 10 200 python bench.py --scene spheres --steps 8 --warmup 1 --cpu-baseline off \
    > "$OUT/$v.bench" 2> "$OUT/$v.err" || { tail -20 "$OUT/$v.err" >&2; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/$v.bench" "$v" >&2
done

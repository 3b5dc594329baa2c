#!/bin/bash
# MIS A/B on the GPU box: MIS parity tests + tools/bench_mis.py per abvar/ variant.
#   tools/ab_mis_run.sh <tag> <variant>...   (AB_NOTEST=1 skips the tests)
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
for v in "$@"; do
  if [ "$v" = base ]; then export RTPT_LIB=$R/gpuraytracer_amd/librtpt.so; else export RTPT_LIB=$R/abvar/librtpt_$v.so; fi
  if [ -z "${AB_NOTEST:-}" ]; then
    timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k mis \
      > "$OUT/$v.tests" 2>&1 || { tail -30 "$OUT/$v.tests" >&2; exit 1; }
    echo "[ab] $v tests: $(tail -1 "$OUT/$v.tests")" >&2
  fi
  timeout -k 10 200 python tools/bench_mis.py --cpu-seconds 0 --steps 10 > "$OUT/$v.json" 2> "$OUT/$v.err" \
    || { tail -20 "$OUT/$v.err" >&2; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('[ab]', sys.argv[2], d['kernel_ms'])" "$OUT/$v.json" "$v" >&2
done

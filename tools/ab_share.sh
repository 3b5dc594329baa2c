#!/bin/bash
# A/B of the per-GPU shares of the multi-GPU frame (tools/bench_share.py) per
# abvar/ variant ("base" = in-tree librtpt.so).   tools/ab_share.sh <tag> <variant>...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
for v in "$@"; do
  if [ "$v" = base ]; then export RTPT_LIB=$R/gpuraytracer_amd/librtpt.so; else export RTPT_LIB=$R/abvar/librtpt_$v.so; fi
  timeout -k 10 200 python tools/bench_share.py > "$OUT/$v.json" 2> "$OUT/$v.err" || { tail -20 "$OUT/$v.err" >&2; exit 1; }
  echo "[share] $v $(tail -1 "$OUT/$v.json")" >&2
done

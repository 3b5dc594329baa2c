#!/bin/bash
# RT_STATS counters of the free-running kernel (abvar/librtpt_stats.so)
set -u
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
for k in spheres triangles; do
  RTPT_LIB=$R/abvar/librtpt_stats.so timeout -k 10 200 python tools/free_stats.py $k 480 270 16 > "$OUT/free_$k.json" 2> "$OUT/free_$k.err" || { tail -20 "$OUT/free_$k.err" >&2; exit 1; }
  cat "$OUT/free_$k.json" >&2
done

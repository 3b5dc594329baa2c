#!/bin/bash
# Config-4 bench of one abvar/ variant under extra environment (no tests):
#   tools/ab_env_bench.sh <tag> <variant> VAR=value...
set -u
TAG=$1; V=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
if [ "$V" = base ]; then L=$R/gpuraytracer_amd/librtpt.so; else L=$R/abvar/librtpt_$V.so; fi
NAME="$V$(printf '_%s' "$@")"
env RTPT_LIB=$L "$@" timeout -k 10 200 python bench.py --scene spheres --steps 8 --warmup 1 --cpu-baseline off \
  > "$OUT/$NAME.bench" 2> "$OUT/$NAME.err" || { tail -20 "$OUT/$NAME.err" >&2; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/$NAME.bench" "$NAME" >&2

#!/bin/bash
# Config-4 walk experiments on the GPU box: timing of abvar variants under
# environment settings (Options.from_env), then RT_STATS counters of the sphere walks.
#   tools/sph_exp.sh <tag> <variant:ENV=VAL,...>...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
for spec in "$@"; do
  v=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  bash tools/ab_env_bench.sh "$TAG" "$v" ${envs//,/ } || exit 1
done
if [ -f abvar/librtpt_stats.so ]; then  # one RT_STATS pass of the sphere walks
  RTPT_LIB=$R/abvar/librtpt_stats.so timeout -k 10 120 python tools/sphere_stats.py 480 270 16 \
    > "$OUT/stats.json" 2> "$OUT/stats.err" || { tail -5 "$OUT/stats.err" >&2; exit 1; }
  echo "stats: $(python3 -c "import json;d=json.load(open('$OUT/stats.json'));print({k:{q:round(x,2) for q,x in v.items() if q in ('steps_per_walk','step_lane_util','lane_steps_per_lane_walk','walks_per_sample')} for k,v in d.items() if k!='packet'})")" >&2
fi

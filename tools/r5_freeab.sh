#!/bin/bash
# free-kernel threshold variants (abvar/): config-4 and 100k-triangle benches
set -u
TAG=${1:?tag}; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"; cd "$R"
for v in "$@"; do
  if [ "$v" = base ]; then L=; else L=$R/abvar/librtpt_$v.so; fi
  for sc in spheres tri; do
    if [ $sc = spheres ]; then A="--scene spheres --steps 4 --warmup 1"; else A="--scene triangles --triangles 100000 --spp 64 --steps 3 --warmup 1"; fi
    RTPT_LIB=$L RTPT_WALK=free timeout -k 10 200 python bench.py $A --cpu-baseline off > "$OUT/$v.$sc" 2> "$OUT/$v.$sc.err" || { tail -20 "$OUT/$v.$sc.err" >&2; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" "$OUT/$v.$sc" "$v.$sc" >&2
  done
done

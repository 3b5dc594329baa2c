#!/bin/bash
# Vector-memory pipeline probe on the GPU box (run through gpurun); build it
# first here: hipcc -O3 --offload-arch=gfx950 tools/td_probe.hip -o tools/td_probe
#   tools/td_probe.sh <tag>
# Each case: the probe's own timing, then one rocprofv3 PMC pass (TA / TD busy
# and load instructions) on the same command.
set -u
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
while read -r name args; do
  [ -z "$name" ] && continue
  timeout -k 10 60 "$R/tools/td_probe" $args > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "[td] $name failed" >&2; exit 1; }
  timeout -s KILL 60 rocprofv3 --pmc TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE \
      -f csv -d "$OUT/pmc_$name" -o run -- "$R/tools/td_probe" $args > "$OUT/pmc_$name.log" 2>&1 \
      || { echo "[td] pmc $name rc=$?" >&2; exit 1; }
  echo "[td] $name $(cat "$OUT/$name.json")" >&2
done <<'EOF'
x4_a64_l1_2mb 4 64 1 2
x4_a27_l1_2mb 4 27 1 2
x4_a16_l1_2mb 4 16 1 2
x4_a64_l8_2mb 4 64 8 2
x4_a64_l64_2mb 4 64 64 2
x1_a64_l1_2mb 1 64 1 2
x1_a64_l32_2mb 1 64 32 2
x4_a64_l1_64mb 4 64 1 64
x4_a27_l1_64mb 4 27 1 64
EOF
python3 "$R/tools/td_probe_summary.py" "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"

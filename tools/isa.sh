#!/bin/bash
# Device ISA of the headline kernels for static inspection (no GPU needed):
#   tools/isa.sh [out.s] [extra hipcc flags...]
# Compiles rt_kernel.hip with -DRT_DEV_ISA (only the box-cluster and LDS-sphere
# layouts at 3 bounces are instantiated, ~4x faster than the full build) and
# prints tools/isa_stats.py for the Cornell (GEO 6) and sphere (GEO 7) kernels.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-/tmp/isa/k.s}
shift || true
mkdir -p "$(dirname "$OUT")"
/opt/rocm/bin/hipcc -std=c++17 -O3 -ffp-contract=off -I"$R/include" --offload-arch=gfx950 \
    -fno-slp-vectorize --offload-device-only -S -DRT_DEV_ISA "$@" \
    "$R/gpuraytracer_amd/csrc/rt_kernel.hip" -o "$OUT" 2>/dev/null
for k in path_trace_kernelILi3ELi6ELb0ELb1ELi4E path_trace_kernelILi3ELi7ELb1ELb1ELi16E; do
    python3 "$R/tools/isa_stats.py" "$OUT" "$k" | head -3
done

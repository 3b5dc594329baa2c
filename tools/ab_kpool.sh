#!/bin/bash
# Kernel-only variant linked with the host objects of build_pool/ (scene and
# launch built with RT_SPH_POOL=1: 8 global layouts, pool LDS allocated):
#   tools/ab_kpool.sh <name> [hipcc flags...] -> abvar/librtpt_<name>.so
set -eu
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/abvar" "$R/build_a"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-unused-function -I"$R/include" \
    -I"$R/gpuraytracer_amd/csrc" --offload-arch=gfx950 -fno-slp-vectorize "$@" \
    -c "$R/gpuraytracer_amd/csrc/rt_kernel.hip" -o "$R/build_a/rt_kernel_$N.o"
B=$R/build_pool
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$R/abvar/librtpt_$N.so" "$R/build_a/rt_kernel_$N.o" \
    "$B/rt_mis.o" "$B/rt_lbvh.o" "$B/rt_api.o" "$B/rt_scene.o" "$B/rt_image.o" -L/opt/rocm/lib -lrccl

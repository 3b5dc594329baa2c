#!/bin/bash
# A/B variants of the pathTrace kernel: rebuild only rt_kernel.o with extra
# flags and link against the in-tree objects.
#   tools/ab_kernel.sh <name> [hipcc flags...] -> abvar/librtpt_<name>.so
set -eu
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/abvar" "$R/build_a"
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-unused-function -I"$R/include" \
    -I"$R/gpuraytracer_amd/csrc" --offload-arch=gfx950 -fno-slp-vectorize "$@" \
    -c "$R/gpuraytracer_amd/csrc/rt_kernel.hip" -o "$R/build_a/rt_kernel_$N.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$R/abvar/librtpt_$N.so" "$R/build_a/rt_kernel_$N.o" \
    "$R/build/rt_mis.o" "$R/build/rt_lbvh.o" "$R/build/rt_gsah.o" "$R/build/rt_api.o" "$R/build/rt_scene.o" \
    "$R/build/rt_image.o" -L/opt/rocm/lib -lrccl

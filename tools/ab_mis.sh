#!/bin/bash
# A/B variants of the MIS kernel: rebuild only rt_mis.o with extra flags and link
# against the in-tree objects.   tools/ab_mis.sh <name> [hipcc flags...] -> abvar/librtpt_<name>.so
set -eu
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/abvar" "$R/build_a"
SRC=${MIS_SRC:-$R/gpuraytracer_amd/csrc/rt_mis.hip}
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC -ffp-contract=off -Wno-unused-function -I"$R/include" \
    -I"$R/gpuraytracer_amd/csrc" --offload-arch=gfx950 -fno-slp-vectorize "$@" -c "$SRC" \
    -o "$R/build_a/rt_mis_$N.o"
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$R/abvar/librtpt_$N.so" "$R/build/rt_kernel.o" \
    "$R/build_a/rt_mis_$N.o" "$R/build/rt_lbvh.o" "$R/build/rt_gsah.o" "$R/build/rt_api.o" "$R/build/rt_scene.o" \
    "$R/build/rt_image.o" -L/opt/rocm/lib -lrccl

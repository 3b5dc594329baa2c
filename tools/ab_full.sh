#!/bin/bash
# A/B variant with every TU rebuilt (needed when a switch changes the host
# side too, e.g. RT_SPH_POOL / RT_SPH_LAYOUTS change the scene builder and
# the LDS size):  tools/ab_full.sh <name> [-Dflags...] -> abvar/librtpt_<name>.so
set -eu
N=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/abvar"
make -C "$R" -j8 BLD="build_$N" LIB="abvar/librtpt_$N.so" EXTRA="$*" "abvar/librtpt_$N.so"

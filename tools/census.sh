#!/bin/bash
# VALU census of the Cornell (box-cluster) kernel on the bench workload
# (DESIGN.md §5): the plain library and the RT_CENSUS=1..6 builds
# (abvar/librtpt_cz<k>.so, tools/ab_kernel.sh czK -DRT_CENSUS=K), one PMC pass
# each; tools/census_summary.py turns the SQ_INSTS_VALU differences into VALU
# per sample and phase.   tools/census.sh <tag>
set -u
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/census_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for v in base cz1 cz2 cz3 cz4 cz5 cz6; do
  if [ $v = base ]; then L=$R/gpuraytracer_amd/librtpt.so; else L=$R/abvar/librtpt_$v.so; fi
  echo "[census] $v" >&2
  RTPT_LIB=$L timeout -k 10 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_INT32 \
      SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT \
      --kernel-include-regex path_trace -f csv -d "$OUT/$v" -o run -- \
      python3 "$R/bench.py" --steps 2 --warmup 1 --cpu-baseline off > "$OUT/$v.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[census] $v rc=$rc" >&2; tail -5 "$OUT/$v.log" >&2; exit $rc; fi
done
python3 "$R/tools/census_summary.py" "$OUT" > "$OUT/census.json" && cat "$OUT/census.json"

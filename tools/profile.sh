#!/bin/bash
# Profile the bench workload on the GPU box (run through gpurun).
#   tools/profile.sh <tag> [extra bench.py args...]
# Pass 1: rocprofv3 --kernel-trace --stats (per-kernel durations).
# Passes 2..: one --pmc group per run (never combined with tracing domains),
# FETCH_SIZE and WRITE_SIZE in separate passes (TCC slot budget), then SQ
# instruction / cycle counters.  Outputs land in gpurun_out/prof_<tag>/ and a
# summary JSON (tools/summarize_profile.py) in gpurun_out/prof_<tag>/summary.json.
set -u
TAG=${1:?tag}
shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
# PROFILE_TARGET=mis profiles the MIS integrator (tools/bench_mis.py) instead.
if [ "${PROFILE_TARGET:-pathtrace}" = mis ]; then
  BENCH=(python3 "$R/tools/bench_mis.py" --steps 3 --warmup 1 --cpu-seconds 0 "$@")
  KRE=mis_kernel
else
  BENCH=(python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-baseline off "$@")
  KRE=path_trace
fi
export PROFILE_KERNEL=$KRE

run() {  # run <name> <rocprof args...>
  local name=$1; shift
  echo "[profile] $name: $*" >&2
  timeout -k 10 300 rocprofv3 "$@" -f csv -d "$OUT/$name" -o run -- "${BENCH[@]}" \
      > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[profile] $name rc=$rc" >&2
  case $rc in
    0) return 0 ;;
    124|137|134|139) echo "[profile] $name died (rc=$rc): stopping" >&2; exit $rc ;;
    *) return 0 ;;  # e.g. a counter this pass cannot collect: keep going
  esac
}

rocprofv3 -L > "$OUT/counters_available.txt" 2>&1 || true
run trace --kernel-trace --stats
run fetch --pmc FETCH_SIZE --kernel-include-regex $KRE
run write --pmc WRITE_SIZE --kernel-include-regex $KRE
run sq_insts --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_INSTS_BRANCH --kernel-include-regex $KRE
run sq_cycles --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --kernel-include-regex $KRE
run sq_valu --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT --kernel-include-regex $KRE
run sq_lds --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_WAIT_INST_LDS --kernel-include-regex $KRE
# vector-memory pipeline: address / tag processing of the per-lane node loads
run ta --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum --kernel-include-regex $KRE
run tcp --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum --kernel-include-regex $KRE
run td --pmc TD_TD_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum --kernel-include-regex $KRE
python3 "$R/tools/summarize_profile.py" "$OUT" "${BENCH[@]:1}" > "$OUT/summary.json"
cat "$OUT/summary.json"

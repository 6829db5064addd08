#!/bin/bash
# rocprofv3 evidence for the dominant kernel (k_tile, C2 instance): kernel-trace stats
# plus PMC passes, each pass its own run (never combined with sys/runtime
# traces).  Usage: bash scripts/profile.sh TAG [bench args...]
set -u
TAG=${1:-r01}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--steps 6 --warmup 1 --cpu-seconds 0 --no-alt --no-sharded $*"
# the kernel trace times the bench's own warm loop: 20 untimed launches, then
# 100 timed ones; prof_summary.py averages the dispatches after the warm-up
# (the committed trace must compare with ms_per_step)
TRACE_ARGS="--steps 100 --warmup 20 --cpu-seconds 0 --no-alt --no-sharded $*"
run() {  # run NAME rocprof-args...
  local name=$1; shift
  local a=$ARGS
  [ "$name" = trace ] && a=$TRACE_ARGS
  echo "=== $name"
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o run --output-format csv -- python3 "$ROOT/bench.py" $a > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 "$OUT/$name.log"; exit $rc; fi
}
run trace --kernel-trace --stats
run pmc_inst --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_CVT
run pmc_cyc --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_l2 --pmc TCC_HIT_sum TCC_MISS_sum
run pmc_lds --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD
run pmc_tcp --pmc TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
run pmc_tatd --pmc TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE
run pmc_sqbusy --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_BUSY_CU_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE
python3 "$ROOT/scripts/prof_summary.py" "$OUT" > "$OUT/summary.txt" 2>&1
cat "$OUT/summary.txt"

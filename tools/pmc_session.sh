#!/bin/bash
# PMC passes over one bench step (each counter group in its own rocprofv3 run; no trace
# domains besides --kernel-trace, per the pool's rules). Stops at the first abnormal exit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
run() {
  local name=$1; shift
  echo "[$(date +%T)] start $name" >> $OUT/pmc_status.log
  timeout -k 10 400 rocprofv3 "$@" -d $OUT/$name -o run --output-format csv -- $B > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/pmc_status.log
  [ $rc -eq 0 ] || { cat $OUT/pmc_status.log; exit $rc; }
}
run trace --kernel-trace --stats
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_sq1 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run pmc_sq2 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY
cat $OUT/pmc_status.log

#!/bin/bash
# PMC passes over one bench step, each counter group in its own rocprofv3 run (no trace domains
# besides the kernel dispatches), then tools/pmc_summary.py -> gpurun_out/pmc_summary.json.
# usage: tools/pmc_passes.sh [TAG]   (TAG names the summary copy, e.g. r05 -> profiles/r05_pmc_summary.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
rm -rf $OUT/pmc_*
: > $OUT/pmc_status.log
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-full-p"
run() {
  local name=$1; shift
  echo "[$(date +%T)] start $name" >> $OUT/pmc_status.log
  timeout -s KILL 120 rocprofv3 --pmc "$@" -d $OUT/pmc_$name -o run --output-format csv -- $B > $OUT/pmc_$name.log 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/pmc_status.log
  [ $rc -eq 0 ] || { cat $OUT/pmc_status.log; tail -5 $OUT/pmc_$name.log; exit $rc; }
}
run fetch FETCH_SIZE
run write WRITE_SIZE
run a SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_I8 SQ_VALU_MFMA_BUSY_CYCLES
run c SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT
run d SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE
python tools/pmc_summary.py $OUT/pmc_summary.json $OUT > $OUT/pmc_summary.log 2>&1
[ -n "${1:-}" ] && cp $OUT/pmc_summary.json profiles/${1}_pmc_summary.json
cat $OUT/pmc_status.log

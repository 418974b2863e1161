#!/bin/bash
# Full GPU round: GPU tests, rocprofv3 kernel stats, PMC passes (summary written into profiles/
# on the box so the bench line's roofline reads the same kernel build), VALU issue-rate
# microbenchmark, then the default bench line. Each step has its own time limit; any abnormal
# exit (not 0 / 1 = test failures) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/round_status.log
TAG=${1:-r02}
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $OUT/round_status.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/round_status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; cat $OUT/round_status.log; exit $rc; fi
}
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread
step prof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- $B
step pmc_write 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- $B
step pmc_sq1 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_sq1 -o run --output-format csv -- $B
step pmc_sq2 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FLOPS_FP64 SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d $OUT/pmc_sq2 -o run --output-format csv -- $B
step pmc_mfma 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $OUT/pmc_mfma -o run --output-format csv -- $B
python tools/pmc_summary.py profiles/${TAG}_pmc_summary.json $OUT > $OUT/pmc_summary.log 2>&1 && cp profiles/${TAG}_pmc_summary.json $OUT/
python tools/timeline.py $OUT/prof/run_kernel_trace.csv > $OUT/${TAG}_timeline.txt 2>&1
[ -x tools/micro/valu_occ ] && step valu_occ 120 ./tools/micro/valu_occ
step bench 900 python bench.py --steps 20 --warmup 3
cat $OUT/round_status.log
tail -c 600 $OUT/bench.log

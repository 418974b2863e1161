#!/bin/bash
# Round 3 closing artifacts at HEAD: GPU tests + smoke, kernel stats / trace of the bench command,
# FETCH / WRITE / SQ / MFMA PMC passes (summary into profiles/ on the box so the bench line's
# roofline reads the same build), the VALU class counters of the dominant kernel (roofline model
# input), a K1-only MFMA/LDS pass, then the default bench line with its CPU baseline. Each step has
# its own time limit; any abnormal exit (not 0 / 1) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/final
mkdir -p $O
: > $O/status.log
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $O/status.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; cat $O/status.log; tail -30 $O/$name.log; exit $rc; fi
}
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
tail -2 $O/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step prof 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_fetch 200 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B
step pmc_write 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B
step pmc_mfma 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -d $O/pmc_mfma -o run --output-format csv -- $B
step pmc_lds 200 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_I8 -d $O/pmc_lds -o run --output-format csv -- $B
python tools/pmc_summary.py profiles/r03_pmc_summary.json $O > $O/pmc_summary.log 2>&1 && cp profiles/r03_pmc_summary.json $O/
python tools/timeline.py $O/prof/run_kernel_trace.csv > $O/r03_timeline.txt 2>&1
step counters 120 rocprofv3 -L
mkdir -p $O/pm_bench
step vcls 600 python tools/valu_class_pmc.py $O/counters.log $O/pm_bench $O/bench_vcls_pmc.json -- $B
step bench 900 python bench.py --steps 20 --warmup 3
cat $O/status.log
tail -c 400 $O/bench.log

#!/bin/bash
# Round 4 closing, part 6 at HEAD (after the galloping pair search): no tests (part 5 ran them), the dominant kernel's VALU class
# PMC for the in-tree build and the no-sweep ablation build (two-region roofline model inputs),
# FETCH / WRITE / wait counters and the kernel trace of the bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/final6
mkdir -p $O $O/pm_base $O/pm_abl1
: > $O/status.log
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $O/status.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/status.log
  if [ $rc -ne 0 ]; then echo "stop after $name rc=$rc"; cat $O/status.log; tail -30 $O/$name.log; exit $rc; fi
}
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-full-p"
rocprofv3 -L > $O/counters.txt 2>&1 || true
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
step vcls_base 600 python tools/valu_class_pmc.py $O/counters.txt $O/pm_base $O/vcls_base.json -- $B
cp tools/variants_r4/libpcgpu_abl1_d4.so rcaeval_amd/libpcgpu.so
timeout -k 10 600 python tools/valu_class_pmc.py $O/counters.txt $O/pm_abl1 $O/vcls_abl1.json -- $B > $O/vcls_abl1.log 2>&1; rc=$?
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so
[ $rc -eq 0 ] || { echo "vcls_abl1 rc=$rc"; tail -20 $O/vcls_abl1.log; exit $rc; }
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" -d $O/$name -o run --output-format csv -- $B > $O/$name.log 2>&1 || { echo "$name rc=$?"; exit 1; }
}
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_wait --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
run pmc_mfma --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
step trace 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-full-p
python tools/pmc_summary.py $O/pmc_summary.json $O > $O/pmc_summary.log 2>&1 || true
python tools/timeline.py $O/trace/run_kernel_trace.csv > $O/timeline.txt 2>&1 || true
cat $O/status.log
ls $O

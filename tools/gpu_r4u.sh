#!/bin/bash
# Round 4, session U: VALU class PMC of the in-tree build and of the no-sweep ablation build
# (tools/variants_r4/libpcgpu_abl1_d4.so) for the two-region dynamic opcode model, plus the
# FETCH / WRITE and wait counters of the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/u
mkdir -p $O $O/pm_base $O/pm_abl1
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-full-p"
rocprofv3 -L > $O/counters.txt 2>&1 || true
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
python tools/valu_class_pmc.py $O/counters.txt $O/pm_base $O/vcls_base.json -- $B || { cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so; exit 1; }
cp tools/variants_r4/libpcgpu_abl1_d4.so rcaeval_amd/libpcgpu.so
python tools/valu_class_pmc.py $O/counters.txt $O/pm_abl1 $O/vcls_abl1.json -- $B; rc=$?
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so
[ $rc -eq 0 ] || exit $rc
run() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 "$@" -d $O/$name -o run --output-format csv -- $B > $O/$name.log 2>&1 || { echo "$name rc=$?"; exit 1; }
}
run pmc_fetch --pmc FETCH_SIZE
run pmc_write --pmc WRITE_SIZE
run pmc_wait --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
run trace --kernel-trace --stats
python tools/pmc_summary.py $O/pmc_summary.json $O > /dev/null 2>&1 || true
ls $O

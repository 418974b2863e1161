#!/bin/bash
# Round 3, session R: is k_level_sp<4> waiting on its setup's global loads? A/B against a timing-only
# build whose setup reads the fp32 P1 buffer instead (wrong precision, no tests), plus SQ waits.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/r
mkdir -p $O
timeout -k 10 600 bash tools/variant_bench.sh > $O/variants.log 2>&1; rc=$?; cat $O/variants.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES"
P3="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES SQ_WAVES"
for sp in 0x10 0; do
  i=0
  for P in "$P2" "$P3"; do
    i=$((i+1))
    PCG_SP=$sp timeout -s KILL 90 rocprofv3 --pmc $P -d $O/pmc_${sp}_$i -o run --output-format csv -- $B > $O/pmc_${sp}_$i.log 2>&1 || { echo "pmc $sp $i failed"; exit 1; }
  done
done
echo done

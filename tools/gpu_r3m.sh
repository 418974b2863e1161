#!/bin/bash
# Round 3, session M: k_level_sp variants (A/B bench) and PMC passes of k_level_sp<4> vs
# k_level_lds_f<4> (PCG_SP=0) over one bench step; each pass under its own kill timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/m
mkdir -p $O
timeout -k 10 600 bash tools/variant_bench.sh > $O/variants.log 2>&1; rc=$?; cat $O/variants.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM"
for sp in 0x18 0; do
  i=0
  for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    PCG_SP=$sp timeout -s KILL 90 rocprofv3 --pmc $P -d $O/pmc_${sp}_$i -o run --output-format csv -- $B > $O/pmc_${sp}_$i.log 2>&1 || { echo "pmc $sp $i failed"; tail -5 $O/pmc_${sp}_$i.log; exit 1; }
  done
done
echo done

#!/bin/bash
# Round 3, session O: VALU class counters of k_level_sp vs k_level_lds_f (PCG_SP=0x18 / 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/o
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || exit 1
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
for sp in 0x18 0; do
  mkdir -p $O/pm_$sp
  PCG_SP=$sp timeout -k 10 600 python tools/valu_class_pmc.py $O/counters.txt $O/pm_$sp $O/vcls_$sp.json -- $B > $O/vcls_$sp.log 2>&1 || { tail $O/vcls_$sp.log; exit 1; }
done
echo done

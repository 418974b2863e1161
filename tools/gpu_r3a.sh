#!/bin/bash
# Round 3, session A: VALU issue-cost table (wall clock, 1/2/4/8 waves per SIMD), the counter
# list, the class-counter calibration on the micro-benchmark, and the same class counters over
# one bench step (dominant kernel's instruction mix).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || { echo "list failed"; }
grep -c SQ_INSTS $O/counters.txt
timeout -k 10 180 ./tools/micro/issue_cost all 1 2 4 8 > $O/issue_cost.json 2> $O/issue_cost.err || { echo "issue_cost failed"; cat $O/issue_cost.err; exit 1; }
echo "issue_cost ok"
mkdir -p $O/pm_micro $O/pm_bench && python tools/valu_class_pmc.py $O/counters.txt $O/pm_micro $O/issue_cost_pmc.json -- ./tools/micro/issue_cost all 4 || exit 1
python tools/valu_class_pmc.py $O/counters.txt $O/pm_bench $O/bench_vcls_pmc.json -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline || exit 1
echo done

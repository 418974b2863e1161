#!/bin/bash
# RQ2 workload bench lines (both synthetic trees) + the reference-equivalent CPU e2e timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python bench.py --workload rq2 > $OUT/rq2_ob.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload rq2 --rq2-dataset sock-shop > $OUT/rq2_ss.log 2>&1 || exit $?
grep '^{' $OUT/rq2_ob.log | tail -1 | cut -c1-300
grep '^{' $OUT/rq2_ss.log | tail -1 | cut -c1-300
OMP_NUM_THREADS=1 OPENBLAS_NUM_THREADS=1 timeout -k 10 1000 python -u tools/cpu_ref_e2e.py --out $OUT/r02_cpu_ref_e2e.json > $OUT/cpu_ref.log 2>&1 || exit $?
grep -v cpu_ref_e2e $OUT/cpu_ref.log | tail -4

#!/bin/bash
# Round 3, session Z7: the K1 parity tests (incl. the CRT top-of-range case), then the RQ2 harness
# lines (config 2, both dataset shapes) on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/z7
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_skeleton.py -m gpu -x -q --timeout 120 --timeout-method thread -k "corr" > $O/pytest_corr.log 2>&1
rc=$?; tail -2 $O/pytest_corr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload rq2 > $O/rq2_ob.log 2>&1 || { tail -5 $O/rq2_ob.log; exit 1; }
timeout -k 10 600 python bench.py --workload rq2 --rq2-dataset sock-shop > $O/rq2_ss.log 2>&1 || { tail -5 $O/rq2_ss.log; exit 1; }
grep "^{" $O/rq2_ob.log | tail -1 | cut -c1-200
grep "^{" $O/rq2_ss.log | tail -1 | cut -c1-200

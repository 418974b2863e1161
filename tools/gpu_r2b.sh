#!/bin/bash
# Round-2 iteration: skeleton parity (incl. the wide-class tests), then variant A/B bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r2b_test.log 2>&1
rc=$?; tail -5 gpurun_out/r2b_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/variant_bench.sh > gpurun_out/r2b_var.log 2>&1
rc=$?; cat gpurun_out/r2b_var.log
exit $rc

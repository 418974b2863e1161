#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_rcd.py -q --timeout 200 --timeout-method thread > gpurun_out/r2e_test.log 2>&1
echo "rcd tests rc=$?"; tail -3 gpurun_out/r2e_test.log
timeout -k 10 1000 bash tools/variant_bench.sh > gpurun_out/r2e_var.log 2>&1
rc=$?; cat gpurun_out/r2e_var.log
exit $rc

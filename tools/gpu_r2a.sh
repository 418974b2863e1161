#!/bin/bash
# Round-2 iteration: skeleton parity (incl. the full-size depth-4 test), then a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests/test_gpu_skeleton.py -x -v -s --timeout 900 --timeout-method thread > gpurun_out/r2a_test.log 2>&1
rc=$?; tail -5 gpurun_out/r2a_test.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r2a_bench.log 2>&1
rc2=$?
tail -c 1500 gpurun_out/r2a_bench.log
exit $((rc | rc2))

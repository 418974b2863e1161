#!/bin/bash
# full GPU suite + smoke + rocprof kernel timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 560 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_prof.sh > /dev/null 2>&1; tail -1 gpurun_out/timeline.txt

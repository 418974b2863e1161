#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r4/dbg
timeout -k 10 120 python -u tools/smoke_debug.py > gpurun_out/r4/dbg/smoke_debug.log 2>&1; rc=$?
cat gpurun_out/r4/dbg/smoke_debug.log | grep -v amdgpu.ids
exit $rc

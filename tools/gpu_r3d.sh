#!/bin/bash
# Round 3, session D: skeleton parity on the in-tree build, then the variant A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread > $O/d_tests.log 2>&1
rc=$?; tail -3 $O/d_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 ./tools/variant_bench.sh

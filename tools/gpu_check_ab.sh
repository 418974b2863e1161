#!/bin/bash
# GPU check + A/B in one gpurun call: the skeleton and small-graph GPU tests of the in-tree build,
# then tools/variant_bench.sh twice over the tools/ab/ variants (tools/build_variants.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_small.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_a.log 2>&1; rc=$?; tail -3 gpurun_out/pt_a.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do bash tools/variant_bench.sh > gpurun_out/ab.txt 2>&1; cat gpurun_out/ab.txt; done

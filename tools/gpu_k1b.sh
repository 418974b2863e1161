#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python tools/micro/k1_time.py tools/micro/variants/libpcgpu_*.so tools/micro/variants/libpcgpu_*.so > $OUT/k1b_var.log 2>&1; rc=$?
cat $OUT/k1b_var.log; exit $rc

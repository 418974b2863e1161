#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so > $OUT/k1c_var.log 2>&1 || exit $?
cat $OUT/k1c_var.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/k1prof -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so > $OUT/k1prof.log 2>&1 || exit $?
bash tools/gpu_quick.sh

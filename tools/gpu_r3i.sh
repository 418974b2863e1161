#!/bin/bash
# Round 3, session I: int8 K1 tuning (slab count), parity of the K1 tests, kernel profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_skeleton.py -x -q -k "corr" --timeout 300 --timeout-method thread > $O/i_corr.log 2>&1
rc=$?; tail -3 $O/i_corr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/micro/k1_env_time.py "PCG_K1_I8=0" "PCG_K1_I8=1 PCG_K1_I8_KS=4" "PCG_K1_I8=1 PCG_K1_I8_KS=8" "PCG_K1_I8=1 PCG_K1_I8_KS=12" "PCG_K1_I8=1 PCG_K1_I8_KS=16" "PCG_K1_I8=1 PCG_K1_I8_KS=8" 2>&1 | tee $O/i_k1.log
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r3/i_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/micro/k1_time.py $GRAFT_REPO_ROOT/rcaeval_amd/libpcgpu.so > $GRAFT_REPO_ROOT/gpurun_out/r3/i_prof.log 2>&1
echo prof rc=$?

#!/bin/bash
# Round 3, session J: int8 K1 tile order A/B + its counters (one kernel-trace run, then PMC
# passes of <= 8 SQ / one TCC group each, every pass under its own kill timeout).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r3/j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_skeleton.py -x -q -k "corr" --timeout 300 --timeout-method thread > $O/corr.log 2>&1
rc=$?; tail -2 $O/corr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/micro/k1_env_time.py "PCG_K1_I8=0" "PCG_K1_SUPER_ORDER=0" "PCG_K1_SUPER_ORDER=1" "PCG_K1_SUPER_ORDER=0 PCG_K1_I8_KS=4" "PCG_K1_SUPER_ORDER=1 PCG_K1_I8_KS=4" "PCG_K1_SUPER_ORDER=1" 2>&1 | tee $O/k1.log
export PYTHONPATH=$R
cd /tmp
for so in 1 0; do
  PCG_K1_SUPER_ORDER=$so timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/trace$so -o run --output-format csv -- python3 $R/tools/micro/k1_time.py $R/rcaeval_amd/libpcgpu.so > $O/trace$so.log 2>&1 || { echo "trace$so failed"; exit 1; }
  PCG_K1_SUPER_ORDER=$so timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_I8 -d $O/sq$so -o run --output-format csv -- python3 $R/tools/micro/k1_time.py $R/rcaeval_amd/libpcgpu.so > $O/sq$so.log 2>&1 || { echo "sq$so failed"; exit 1; }
  PCG_K1_SUPER_ORDER=$so timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/fetch$so -o run --output-format csv -- python3 $R/tools/micro/k1_time.py $R/rcaeval_amd/libpcgpu.so > $O/fetch$so.log 2>&1 || { echo "fetch$so failed"; exit 1; }
  PCG_K1_SUPER_ORDER=$so timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/tcc$so -o run --output-format csv -- python3 $R/tools/micro/k1_time.py $R/rcaeval_amd/libpcgpu.so > $O/tcc$so.log 2>&1 || { echo "tcc$so failed"; exit 1; }
done
echo done

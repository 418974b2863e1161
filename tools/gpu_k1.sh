#!/bin/bash
# K1 experiments: f64 MFMA issue microbenchmark, K1 variant timings, PMC of the default k_xtx.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 120 ./tools/micro/mfma_f64 > $OUT/k1_mfma.log 2>&1 || exit $?
cat $OUT/k1_mfma.log
timeout -k 10 300 python tools/micro/k1_time.py tools/micro/variants/libpcgpu_*.so > $OUT/k1_var.log 2>&1 || exit $?
cat $OUT/k1_var.log
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_WAVES -d $OUT/k1_pmc1 -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so > $OUT/k1_pmc1.log 2>&1
echo "pmc1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/k1_pmc2 -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so > $OUT/k1_pmc2.log 2>&1
echo "pmc2 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/k1_pmc3 -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so > $OUT/k1_pmc3.log 2>&1
echo "pmc3 rc=$?"

#!/bin/bash
# Round 3, session Z8: column-statistics variants (rows per partial, loads in flight): K1 parity on
# each, k_colsum_partial / k_colstats times from a kernel trace of the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/z8
mkdir -p $O
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
for v in /tmp/libpcgpu_base.so tools/micro/variants/libpcgpu_*.so; do
  name=$(basename "$v" .so)
  cp "$v" rcaeval_amd/libpcgpu.so
  timeout -k 10 300 python -u -m pytest tests/test_gpu_skeleton.py -m gpu -x -q --timeout 120 --timeout-method thread -k "corr" > $O/pt_$name.log 2>&1 || { echo "$name parity FAILED"; tail -3 $O/pt_$name.log; cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$name -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/p_$name.log 2>&1 || { echo "$name prof failed"; cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so; exit 1; }
  echo "$name $(tail -1 $O/pt_$name.log | cut -c1-40) colsum $(grep -E 'k_colsum_partial' $O/p_$name/run_kernel_stats.csv | awk -F, '{print $(NF-4)}') colstats $(grep -E 'k_colstats' $O/p_$name/run_kernel_stats.csv | awk -F, '{print $(NF-4)}')"
done
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so
bash tools/gpu_r3z7.sh

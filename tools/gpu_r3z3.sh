#!/bin/bash
# Round 3, session Z3: CRT GEMM staging variants (ring depth, stage size, MFMA priority) — the K1
# parity tests on the in-tree build, then per-variant bench + kernel stats of k_xtx_crt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/z3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_skeleton.py -m gpu -x -q --timeout 120 --timeout-method thread -k "corr" > $O/pytest_corr.log 2>&1
rc=$?; tail -2 $O/pytest_corr.log; [ $rc -eq 0 ] || exit $rc
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
for v in /tmp/libpcgpu_base.so tools/micro/variants/libpcgpu_*.so; do
  name=$(basename "$v" .so)
  cp "$v" rcaeval_amd/libpcgpu.so
  timeout -k 10 120 python -u -m pytest tests/test_gpu_skeleton.py -m gpu -x -q --timeout 60 --timeout-method thread -k "corr_crt" > $O/pt_$name.log 2>&1 || { echo "$name parity FAILED"; tail -3 $O/pt_$name.log; continue; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p_$name -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/p_$name.log 2>&1 || { echo "$name prof failed"; exit 1; }
  echo "$name $(grep -E 'k_xtx_crt' $O/p_$name/run_kernel_stats.csv | awk -F, '{print $(NF-4)}')"
done
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so

# parity of the in-tree build on the skeleton tests, then the A/B of tools/ab variants (twice)
set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_small.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_a.log 2>&1; rc=$?; tail -3 gpurun_out/pt_a.log; [ $rc -eq 0 ] || exit $rc
bash tools/variant_bench.sh > gpurun_out/ab11.txt 2>&1; cat gpurun_out/ab11.txt
bash tools/variant_bench.sh > gpurun_out/ab11b.txt 2>&1; cat gpurun_out/ab11b.txt
grep -h "blkt d3" gpurun_out/var_libpcgpu_blkt3.log | tail -2

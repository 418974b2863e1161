# parity of the in-tree build and the sg18 variant on the skeleton tests, then the A/B
set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_a.log 2>&1; rc=$?; tail -3 gpurun_out/pt_a.log; [ $rc -eq 0 ] || exit $rc
PCG_LIB_PATH=$PWD/tools/ab/libpcgpu_sg18.so timeout -k 10 300 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 200 --timeout-method thread -k "config5 or oracle or ref" > gpurun_out/pt_b.log 2>&1; rc=$?; tail -3 gpurun_out/pt_b.log; [ $rc -eq 0 ] || exit $rc
bash tools/variant_bench.sh > gpurun_out/ab9.txt 2>&1; cat gpurun_out/ab9.txt
bash tools/variant_bench.sh > gpurun_out/ab9b.txt 2>&1; cat gpurun_out/ab9b.txt

# K1 parity (skeleton file: corr vs numpy, split invariance, sharded bitwise, config 5) + bench
set -u
timeout -k 10 500 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_native_dist.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pt_k1.log 2>&1; rc=$?; tail -3 gpurun_out/pt_k1.log; [ $rc -eq 0 ] || exit $rc
bash tools/knob_ab.sh - K1_CRT_BITS=56 > gpurun_out/ab19k.txt 2>&1; cat gpurun_out/ab19k.txt

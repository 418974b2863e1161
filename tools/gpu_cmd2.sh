# parity of the in-tree build (skeleton + small tests), then A/B of tools/ab variants and runtime knobs
set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_small.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_a.log 2>&1; rc=$?; tail -3 gpurun_out/pt_a.log; [ $rc -eq 0 ] || exit $rc
bash tools/variant_bench.sh > gpurun_out/ab17.txt 2>&1; cat gpurun_out/ab17.txt
bash tools/knob_ab.sh - SCREEN_MASK=0x1c > gpurun_out/ab17k.txt 2>&1; cat gpurun_out/ab17k.txt

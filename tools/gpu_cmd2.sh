# parity after a screen change: skeleton (config 5 full, both sweeps), small graphs, native driver
set -u
timeout -k 10 700 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_small.py tests/test_gpu_native_dist.py -x -q --timeout 400 --timeout-method thread > gpurun_out/pt_ke.log 2>&1; rc=$?; tail -3 gpurun_out/pt_ke.log; [ $rc -eq 0 ] || exit $rc

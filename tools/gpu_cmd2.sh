# the node-image tests
set -u
timeout -k 10 400 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 300 --timeout-method thread -k "node_images" > gpurun_out/pt_img2.log 2>&1; rc=$?; tail -3 gpurun_out/pt_img2.log; [ $rc -eq 0 ] || exit $rc

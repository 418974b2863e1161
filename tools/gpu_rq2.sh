cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread -k "rq2 or pagerank" > gpurun_out/rq2_test.log 2>&1
rc=$?; tail -3 gpurun_out/rq2_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --workload rq2 --rq2-cases 125 > gpurun_out/rq2_bench.log 2>&1
rc=$?; tail -c 1500 gpurun_out/rq2_bench.log; exit $rc

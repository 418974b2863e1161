#!/bin/bash
# full GPU suite + smoke + rocprof kernel stats / timeline of a short bench (+ the skeleton tests
# of each tools/ab/ variant through PCG_LIB_PATH)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
for v in tools/ab/libpcgpu_*.so; do
  [ -f "$v" ] || continue
  PCG_LIB_PATH="$PWD/$v" timeout -k 10 400 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_$(basename $v .so).log 2>&1; rc=$?
  echo "$(basename $v): $(tail -1 gpurun_out/pt_$(basename $v .so).log)"; [ $rc -eq 0 ] || exit $rc
done
rm -rf gpurun_out/prof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-p > gpurun_out/prof.log 2>&1 || exit $?
python tools/timeline.py "$(find gpurun_out/prof -name run_kernel_trace.csv | head -1)" > gpurun_out/timeline.txt 2>&1
cp "$(find gpurun_out/prof -name run_kernel_stats.csv | head -1)" gpurun_out/kernel_stats.csv
tail -1 gpurun_out/timeline.txt

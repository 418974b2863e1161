#!/bin/bash
# Round 3, session X: artifacts at HEAD — GPU tests, kernel trace of the bench command, FETCH/WRITE
# passes, VALU class counters (roofline model input), the default bench line with the CPU baseline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/x
mkdir -p $O
: > $O/status.log
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $O/status.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; cat $O/status.log; tail -30 $O/$name.log; exit $rc; fi
}
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread
tail -3 $O/pytest_gpu.log
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
step pmc_fetch 150 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- $B
step pmc_write 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- $B
step counters 120 rocprofv3 -L
mkdir -p $O/pm_bench
step vcls 600 python tools/valu_class_pmc.py $O/counters.log $O/pm_bench $O/bench_vcls_pmc.json -- $B
step bench 600 python bench.py --steps 20 --warmup 3
cat $O/status.log
tail -c 1500 $O/bench.log

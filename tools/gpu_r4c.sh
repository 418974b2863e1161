#!/bin/bash
# Round 4, session C: the engine against the reference-executed skeleton / FCI goldens, then the
# unlimited-depth probe at n = 2000 (capped depths while the next depth's work fits a budget).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/c
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
step ref_tests 400 python -u -m pytest tests/test_gpu_skeleton_ref.py -v --timeout 120 --timeout-method thread
step probe2000 400 python -u tools/deep_probe.py --n 2000 --samples 10000 --budget 3e11
step probe1000 300 python -u tools/deep_probe.py --n 1000 --samples 10000 --start 8 --budget 1e12
cat $O/status.log
tail -3 $O/ref_tests.log
step rq2_pf0 300 python -u bench.py --workload rq2 --rq2-cases 90 --rq2-prefetch 0
step rq2_pf2 300 python -u bench.py --workload rq2 --rq2-cases 90 --rq2-prefetch 2
cat $O/status.log

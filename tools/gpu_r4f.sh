#!/bin/bash
# Round 4, session F: the small-graph kernel's GPU tests, then the wider GPU suites that run small
# cases through it, then the RQ2 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/f
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
step small_tests 300 python -u -m pytest tests/test_gpu_small.py -q --timeout 120 --timeout-method thread
tail -3 $O/small_tests.log
step more_tests 900 python -u -m pytest tests/test_gpu_skeleton_ref.py tests/test_gpu_e2e.py tests/test_gpu_fci.py tests/test_gpu_rq1.py tests/test_gpu_rcd.py tests/test_gpu_citest.py tests/test_gpu_skeleton.py -k "not config5 and not overflow and not n500 and not 2000" -q --timeout 200 --timeout-method thread
tail -3 $O/more_tests.log
step rq2 300 python -u bench.py --workload rq2 --rq2-cases 90
python - $O/rq2.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print('rq2', round(d['value'], 1), 'cases/s', d['phase_ms_per_case'])
PY
cat $O/status.log

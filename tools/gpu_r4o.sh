#!/bin/bash
# Round 4, session O: small kernel (all tests), the sepset/p_values surfaces, small-case timing,
# the RQ2 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/o
mkdir -p $O
: > $O/status.log
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $O/status.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; step rq2_ss 300 python -u bench.py --workload rq2 --rq2-cases 90 --rq2-dataset sock-shop
python - $O/rq2_ss.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print('rq2 sock-shop', round(d['value'], 1), 'cases/s', d['phase_ms_per_case'])
PY
cat $O/status.log; tail -30 $O/$name.log; exit $rc; fi
}
step small 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_skeleton_ref.py -q --timeout 100 --timeout-method thread
tail -2 $O/small.log
step e2e 600 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_fci.py tests/test_gpu_rq1.py -q --timeout 200 --timeout-method thread
tail -2 $O/e2e.log
step small_bench 200 python -u tools/small_bench.py 44 600 200
tail -1 $O/small_bench.log
step rq2 300 python -u bench.py --workload rq2 --rq2-cases 90
python - $O/rq2.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print('rq2', round(d['value'], 1), 'cases/s', d['phase_ms_per_case'])
PY
step rq2_ss 300 python -u bench.py --workload rq2 --rq2-cases 90 --rq2-dataset sock-shop
python - $O/rq2_ss.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print('rq2 sock-shop', round(d['value'], 1), 'cases/s', d['phase_ms_per_case'])
PY
cat $O/status.log

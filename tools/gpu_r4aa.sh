#!/bin/bash
# Round 4, session AA: where n = 500 unlimited depth spends its non-kernel time — the host trace
# and the device timeline of one run (rocprofv3 kernel trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/aa
mkdir -p $O
: > $O/status.log
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $O/status.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/status.log
  if [ $rc -ne 0 ]; then echo "stop after $name rc=$rc"; cat $O/status.log; tail -30 $O/$name.log; exit $rc; fi
}
step tests 600 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 300 --timeout-method thread -k "full_depth or wave_kernel or max_depth or skeleton_matches_oracle"
tail -2 $O/tests.log
step d1000 200 python -u tools/profile_deep.py --n 1000 --reps 1
step d500 120 python -u tools/profile_deep.py --n 500 --reps 5
python - $O/d1000.log $O/d500.log <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f, 'n', d['n'], 'gpu_ms', round(d['gpu_ms'], 3), 'kernel', round(sum(d['kernel_ms']), 3), 'levels', d['levels'], 'tests', sum(d['tests']), hash(tuple(d['tests'])) % 100000, hash(tuple(d['max_degree'])) % 100000)
PY
PCG_HOST_TRACE=1 step ht500 120 python -u tools/profile_deep.py --n 500 --reps 1
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python -u tools/profile_deep.py --n 500 --reps 2
python tools/timeline.py $O/prof/run_kernel_trace.csv k_init > $O/timeline500.txt 2>&1
tail -3 $O/timeline500.txt

#!/bin/bash
# Round 4 closing, part 5 at HEAD (final build, galloping pair search): every GPU test, smoke, the bench line and the
# unlimited-depth timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/final5
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
step pytest_gpu 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $O/pytest_gpu.log
step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tail -1 $O/smoke.log
step bench 600 python -u bench.py --steps 20 --warmup 5
grep '^{' $O/bench.log | tail -1 > $O/bench_line.json
step d500 120 python -u tools/profile_deep.py --n 500 --reps 5
step d1000 200 python -u tools/profile_deep.py --n 1000 --reps 2
python - $O/bench_line.json $O/d500.log $O/d1000.log <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            if 'ms_per_step' in d:
                print(f, round(d['ms_per_step'], 3), d['kernel_ms_per_level'], round(d['roofline']['frac'], 3), d['full_p']['skeleton_device_ms'])
            else:
                print(f, 'gpu_ms', round(d['gpu_ms'], 3), d['gpu_ms_all'], 'kernel', round(sum(d['kernel_ms']), 3), 'tests', sum(d['tests']))
PY

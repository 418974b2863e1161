#!/bin/bash
# Round 4 closing, part 2: the default bench line (CPU baseline + full-p leg) with the refreshed
# two-region roofline model, and the n = 500 / 1000 unlimited-depth lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/final2
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
step bench 900 python -u bench.py
grep '^{' $O/bench.log | tail -1 > $O/bench_line.json
step d500 120 python -u tools/profile_deep.py --n 500 --reps 5
step d1000 200 python -u tools/profile_deep.py --n 1000 --reps 2
cat $O/status.log
tail -c 600 $O/bench_line.json

#!/bin/bash
# Round 4, session A: the reference's default (unlimited depth) at config-5 size: a bench line with
# --max-depth -1 plus per-level detail, and its kernel stats; then the depth-4 headline line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/a
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
step deep_bench 400 python -u bench.py --steps 3 --warmup 1 --max-depth -1 --no-cpu-baseline --json-extra
step deep_prof 400 rocprofv3 --kernel-trace --stats -d $O/deep_prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --max-depth -1 --no-cpu-baseline
step bench 400 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --json-extra
cat $O/status.log
tail -c 600 $O/deep_bench.log

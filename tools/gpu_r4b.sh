#!/bin/bash
# Round 4, session B: unlimited depth (the reference's default) at n = 1000 then 2000, one step each
# with the host trace, then a 3-step line and its kernel stats at 2000.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/b
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
export PCG_HOST_TRACE=1
step deep1000 170 python -u bench.py --n 1000 --steps 1 --warmup 0 --max-depth -1 --no-cpu-baseline --no-full-p
step deep2000 170 python -u bench.py --steps 1 --warmup 0 --max-depth -1 --no-cpu-baseline --no-full-p
unset PCG_HOST_TRACE
step deep2000x3 170 python -u bench.py --steps 3 --warmup 1 --max-depth -1 --no-cpu-baseline --no-full-p
step deep_prof 170 rocprofv3 --kernel-trace --stats -d $O/deep_prof -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --max-depth -1 --no-cpu-baseline --no-full-p
cat $O/status.log

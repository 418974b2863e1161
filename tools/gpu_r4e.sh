#!/bin/bash
# Round 4, session E: depth-3 prefetch A/B (bench lines), then the small-graph kernel's GPU tests
# (against the level loop, the oracle and the reference goldens), then the RQ2 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/e
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
line() { python - "$1" "$2" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[2], round(d['ms_per_step'], 3), 'kern', d['kernel_ms_per_level'], 'lvl', d['level_ms'], 'tests', sum(d['tests_per_level']))
PY
}
step bench_pf 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-full-p
line $O/bench_pf.log prefetch3
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_new.so
cp tools/variants_r4/libpcgpu_pf_off.so rcaeval_amd/libpcgpu.so
step bench_pfoff 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-full-p
line $O/bench_pfoff.log prefetch_off
cp /tmp/libpcgpu_new.so rcaeval_amd/libpcgpu.so
step small_tests 300 python -u -m pytest tests/test_gpu_small.py -x -q --timeout 120 --timeout-method thread
tail -3 $O/small_tests.log
step more_tests 600 python -u -m pytest tests/test_gpu_skeleton_ref.py tests/test_gpu_e2e.py tests/test_gpu_skeleton.py -k "not config5 and not overflow and not n500 and not 2000" -x -q --timeout 200 --timeout-method thread
tail -3 $O/more_tests.log
step rq2 300 python -u bench.py --workload rq2 --rq2-cases 90
python - $O/rq2.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l); print('rq2', round(d['value'], 1), 'cases/s', d['phase_ms_per_case'])
PY
cat $O/status.log

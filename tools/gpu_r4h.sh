#!/bin/bash
# Round 4, session H: small-kernel record tests (verbose), deep-level prefix-reuse kernel tests,
# unlimited-depth timings with PCG_WAVE_PR=1/0, and a pc() profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/h
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
step small_rec 200 python -u -m pytest tests/test_gpu_small.py -k "records or banned or constant or errors or switch" -v --timeout 60 --timeout-method thread
grep -E "PASSED|FAILED|Timeout" $O/small_rec.log | head -20
step deep_tests 400 python -u -m pytest tests/test_gpu_skeleton.py -k "n500 or wave_kernel" -v --timeout 200 --timeout-method thread
grep -E "PASSED|FAILED|Timeout" $O/deep_tests.log | head -20
for pr in 1 0; do
  PCG_WAVE_PR=$pr step deep500_pr$pr 120 python -u bench.py --n 500 --steps 5 --warmup 2 --max-depth -1 --no-cpu-baseline --no-full-p
  PCG_WAVE_PR=$pr step deep1000_pr$pr 200 python -u bench.py --n 1000 --steps 2 --warmup 1 --max-depth -1 --no-cpu-baseline --no-full-p
done
python - $O <<'PY'
import json, sys, glob, os
for f in sorted(glob.glob(os.path.join(sys.argv[1], 'deep*_pr*.log'))):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(os.path.basename(f), round(d['ms_per_step'], 3), 'levels', len(d['tests_per_level']), 'kern_sum', round(sum(d['kernel_ms_per_level']), 3), 'kern', d['kernel_ms_per_level'][8:])
PY
step pc_profile 120 python -u tools/small_bench.py --profile
head -45 $O/pc_profile.log | tail -32
cat $O/status.log

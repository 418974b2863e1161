#!/bin/bash
# Round 4, session AG: galloping pair search in the T-group kernels
# (PCG_TG_GALLOP) — skeleton parity, then config-5 bench A/B against the table-search build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/ag
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
line() { python - "$1" "$2" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[2], round(d['ms_per_step'], 3), 'kern', d['kernel_ms_per_level'], 'lvl', d['level_ms'], 'roof', round(d['roofline']['frac'] or 0, 3))
PY
}
step tests 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 300 --timeout-method thread
tail -2 $O/tests.log
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_g1.so
for v in g1 gal0 g1 gal0; do
  if [ $v = gal0 ]; then cp tools/variants_r4/libpcgpu_gal0.so rcaeval_amd/libpcgpu.so; else cp /tmp/libpcgpu_g1.so rcaeval_amd/libpcgpu.so; fi
  step b_$v 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-p
  line $O/b_$v.log $v
done
cp /tmp/libpcgpu_g1.so rcaeval_amd/libpcgpu.so
step d500 120 python -u tools/profile_deep.py --n 500 --reps 5
grep '^{' $O/d500.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('d500', round(d['gpu_ms'],3), round(sum(d['kernel_ms']),3))"

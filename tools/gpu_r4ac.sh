#!/bin/bash
# Round 4, session AC: column-order forward solve in k_level_lds (PCG_LDS_COLSOLVE) — parity, then
# n = 500 / 1000 unlimited depth against the row-order build (tools/variants_r4/libpcgpu_cs0.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/ac
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
summ() { python - "$1" "$2" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[2], 'n', d['n'], 'gpu_ms', round(d['gpu_ms'], 3), 'kernel', round(sum(d['kernel_ms']), 3), 'tests', sum(d['tests']), hash(tuple(d['tests'])) % 100000, hash(tuple(d['max_degree'])) % 100000, 'kms', [round(v, 1) for v in d['kernel_ms'][5:]])
PY
}
step tests 900 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_small.py -x -q --timeout 300 --timeout-method thread
tail -2 $O/tests.log
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_cs1.so
for v in cs1 cs0; do
  if [ $v = cs0 ]; then cp tools/variants_r4/libpcgpu_cs0.so rcaeval_amd/libpcgpu.so; else cp /tmp/libpcgpu_cs1.so rcaeval_amd/libpcgpu.so; fi
  step d500_$v 120 python -u tools/profile_deep.py --n 500 --reps 5
  step d1000_$v 200 python -u tools/profile_deep.py --n 1000 --reps 1
done
cp /tmp/libpcgpu_cs1.so rcaeval_amd/libpcgpu.so
for v in cs1 cs0; do summ $O/d500_$v.log d500_$v; summ $O/d1000_$v.log d1000_$v; done

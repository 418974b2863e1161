#!/bin/bash
# Round 4, session X: one k_level_lds instantiation per depth 5..12 (PCG_LDS_EXACT_DM) — skeleton
# parity tests, then n = 500 / 1000 unlimited depth with the in-tree build vs the bucketed variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/x
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
        print(sys.argv[2], 'n', d['n'], 'gpu_ms', round(d['gpu_ms'], 3), 'kernel', round(sum(d['kernel_ms']), 3), 'levels', d['levels'], 'kms', d['kernel_ms'][4:])
PY
}
step tests 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 300 --timeout-method thread
tail -2 $O/tests.log
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_edm1.so
step d500_edm1 120 python -u tools/profile_deep.py --n 500 --reps 5
step d1000_edm1 200 python -u tools/profile_deep.py --n 1000 --reps 1
cp tools/variants_r4/libpcgpu_edm0.so rcaeval_amd/libpcgpu.so
step d500_edm0 120 python -u tools/profile_deep.py --n 500 --reps 5
step d1000_edm0 200 python -u tools/profile_deep.py --n 1000 --reps 1
cp /tmp/libpcgpu_edm1.so rcaeval_amd/libpcgpu.so
for f in d500_edm1 d500_edm0 d1000_edm1 d1000_edm0; do summ $O/$f.log $f; done

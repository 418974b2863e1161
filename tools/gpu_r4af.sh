#!/bin/bash
# Round 4, session AF: rsq_nr pivot reciprocals in the deep per-lane kernel (PCG_LDS_RSQ) — deep
# parity tests, then n = 500 / 1000 unlimited depth against the left-looking build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/af
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 300 --timeout-method thread -k "full_depth or wave_kernel or deep or max_depth or inline" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_rq1.so
for v in rq1 rsq0; do
  if [ $v = rsq0 ]; then cp tools/variants_r4/libpcgpu_rsq0.so rcaeval_amd/libpcgpu.so; else cp /tmp/libpcgpu_rq1.so rcaeval_amd/libpcgpu.so; fi
  timeout -k 10 120 python -u tools/profile_deep.py --n 500 --reps 5 > $O/d500_$v.log 2>&1 || exit 1
  timeout -k 10 200 python -u tools/profile_deep.py --n 1000 --reps 1 > $O/d1000_$v.log 2>&1 || exit 1
  python - $O/d500_$v.log $O/d1000_$v.log <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f, 'gpu_ms', round(d['gpu_ms'], 3), 'kernel', round(sum(d['kernel_ms']), 3), 'tests', sum(d['tests']), hash(tuple(d['tests'])) % 100000, 'kms', [round(v, 1) for v in d['kernel_ms'][13:22]])
PY
done
cp /tmp/libpcgpu_rq1.so rcaeval_amd/libpcgpu.so

#!/bin/bash
# Round 4, session AD: column-order forward solve at depths 13-20 only — deep parity tests and the
# n = 500 / 1000 unlimited-depth timings.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/ad
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 300 --timeout-method thread -k "full_depth or wave_kernel or deep or max_depth or inline" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/profile_deep.py --n 500 --reps 5 > $O/d500.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/profile_deep.py --n 1000 --reps 2 > $O/d1000.log 2>&1 || exit 1
python - $O/d500.log $O/d1000.log <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f, 'gpu_ms', round(d['gpu_ms'], 3), d['gpu_ms_all'], 'kernel', round(sum(d['kernel_ms']), 3), 'tests', sum(d['tests']), hash(tuple(d['tests'])) % 100000, 'kms', [round(v, 1) for v in d['kernel_ms'][9:22]])
PY

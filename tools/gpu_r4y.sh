#!/bin/bash
# Round 4, session Y: threshold-mode depths 13..16 on the per-lane k_level_lds (band tests decided
# by the wave in its LDS slot) vs the one-wave-per-set kernels (PCG_LDS_DEEP=12): parity, then
# n = 500 / 1000 unlimited depth.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/y
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
        print(sys.argv[2], 'n', d['n'], 'gpu_ms', round(d['gpu_ms'], 3), 'kernel', round(sum(d['kernel_ms']), 3), 'levels', d['levels'], 'tests', sum(d['tests']), 'kms', [round(v, 2) for v in d['kernel_ms'][9:]])
PY
}
step tests 600 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 300 --timeout-method thread -k "full_depth or wave_kernel or max_depth or skeleton_matches_oracle"
tail -2 $O/tests.log
step d500_deep16 120 python -u tools/profile_deep.py --n 500 --reps 5
step d1000_deep16 200 python -u tools/profile_deep.py --n 1000 --reps 1
PCG_LDS_DEEP=12 step d500_deep12 120 python -u tools/profile_deep.py --n 500 --reps 5
PCG_LDS_DEEP=12 step d1000_deep12 200 python -u tools/profile_deep.py --n 1000 --reps 1
for f in d500_deep16 d500_deep12 d1000_deep16 d1000_deep12; do summ $O/$f.log $f; done

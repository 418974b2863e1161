#!/bin/bash
# Round 4, session Z: how deep the per-lane k_level_lds pays (top-20 build, PCG_LDS_DEEP = 16..20)
# at n = 1000 / 500 unlimited depth; per-level test counts must not change.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/z
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
        print(sys.argv[2], 'n', d['n'], 'gpu_ms', round(d['gpu_ms'], 3), 'kernel', round(sum(d['kernel_ms']), 3), 'levels', d['levels'], 'tests', sum(d['tests']), hash(tuple(d['tests'])) % 100000, hash(tuple(d['max_degree'])) % 100000, 'kms', [round(v, 2) for v in d['kernel_ms'][13:]])
PY
}
step tests 600 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread -k "full_depth or wave_kernel or max_depth or skeleton_matches_oracle or sepset or export or e2e"
tail -2 $O/tests.log
step d500_intree 120 python -u tools/profile_deep.py --n 500 --reps 5
PCG_EXPORT_INLINE=0 step d500_intree_noinl 120 python -u tools/profile_deep.py --n 500 --reps 5
step d1000_intree 200 python -u tools/profile_deep.py --n 1000 --reps 1
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_intree.so
cp tools/variants_r4/libpcgpu_top20.so rcaeval_amd/libpcgpu.so
for v in 16 17 18 20; do
  PCG_LDS_DEEP=$v step d1000_$v 200 python -u tools/profile_deep.py --n 1000 --reps 1
  PCG_LDS_DEEP=$v step d500_$v 120 python -u tools/profile_deep.py --n 500 --reps 5
done
cp /tmp/libpcgpu_intree.so rcaeval_amd/libpcgpu.so
for v in 16 17 18 20; do summ $O/d1000_$v.log d1000_$v; summ $O/d500_$v.log d500_$v; done
for f in d500_intree d500_intree_noinl d1000_intree; do summ $O/$f.log $f; done

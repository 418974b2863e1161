#!/bin/bash
# Round 3, session S: one ballot-AND per candidate (unusable candidates pass the compare) in both
# depth-3/4 sweeps: parity, PCG_SP A/B, k_level_lds_f split-window variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread -k "schur or config5 or screen or wide or skeleton_matches" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for sp in 0x10 0 0x10 0; do
  PCG_SP=$sp timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$sp.log 2>&1 || exit 1
  python - $O/bench_$sp.log $sp <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('SP', sys.argv[2], round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], 'corr', d['corr_ms'][-2:])
PY
done
PCG_SP=0 timeout -k 10 600 bash tools/variant_bench.sh > $O/variants.log 2>&1; rc=$?; cat $O/variants.log; [ $rc -eq 0 ] || exit $rc

#!/bin/bash
# Round 3, session Q: both depth-4 sweeps with the rare-path values opaque (spills 127 -> 11):
# parity, then PCG_SP A/B lines and one PMC FETCH/WRITE pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/q
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread -k "schur or config5 or screen" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for sp in 0x10 0 0x10 0; do
  PCG_SP=$sp timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_$sp.log 2>&1 || exit 1
  python - $O/bench_$sp.log $sp <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('SP', sys.argv[2], round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], 'corr', d['corr_ms'][-2:])
PY
done
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
for sp in 0x10 0; do
  for P in FETCH_SIZE WRITE_SIZE; do
    PCG_SP=$sp timeout -s KILL 90 rocprofv3 --pmc $P -d $O/pmc_${sp}_$P -o run --output-format csv -- $B > $O/pmc_${sp}_$P.log 2>&1 || { echo "pmc $sp $P failed"; exit 1; }
  done
done
echo done

#!/bin/bash
# Round 3, session Z6: CRT K1 with residues overlapped with the GEMM (PCG_K1_CRT_GROUPS) — K1 parity
# tests, then pcg_corr wall time per group count (kernel trace span of K1 in the bench).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/z6
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_skeleton.py -m gpu -x -q --timeout 120 --timeout-method thread -k "corr" > $O/pytest_corr.log 2>&1
rc=$?; tail -2 $O/pytest_corr.log; [ $rc -eq 0 ] || exit $rc
for g in 1 2 3 4; do
  PCG_K1_CRT_GROUPS=$g timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench$g.log 2>&1 || { tail -5 $O/bench$g.log; exit 1; }
  python - $g $O/bench$g.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print('groups', sys.argv[1], round(d['ms_per_step'],3), '%.4g' % d['value'], 'corr', d['corr_ms'])
PY
done

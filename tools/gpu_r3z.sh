#!/bin/bash
# Round 3, session Z: CRT (Ozaki II) K1 — K1 parity tests first, then the GPU suite, bench lines,
# kernel stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/z
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_skeleton.py -m gpu -x -q --timeout 120 --timeout-method thread -k "corr" > $O/pytest_corr.log 2>&1
rc=$?; tail -15 $O/pytest_corr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench$i.log 2>&1 || { tail -5 $O/bench$i.log; exit 1; }
  python - $O/bench$i.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(round(d['ms_per_step'],3), d['value'], d['kernel_ms_per_level'], 'corr', d['corr_ms'][-2:], d.get('k1'))
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
grep -E "k_xtx|k_resid|k_crt|k_normalize|k_col" $O/prof/run_kernel_stats.csv

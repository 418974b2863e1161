#!/bin/bash
# Round 3, session L: Schur-prefix sweep (k_level_sp) — skeleton parity tests, then A/B bench
# lines (PCG_SP default vs 0) and a kernel trace. Each GPU step under its own kill timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread ${PYTEST_K:-} > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_sp.log 2>&1 || exit 1
PCG_SP=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_nosp.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
for f in bench_sp bench_nosp; do python - $O/$f.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1], round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], d['tests_per_level'], d['screened'])
PY
done

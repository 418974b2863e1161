#!/bin/bash
# Round 3, session N: k_level_sp with g-major cells — SP parity tests + config 5, variant A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread -k "schur or config5 or screen" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 bash tools/variant_bench.sh > $O/variants.log 2>&1; rc=$?; cat $O/variants.log; [ $rc -eq 0 ] || exit $rc
PCG_SP=0 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_nosp.log 2>&1 || exit 1
python - $O/bench_nosp.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('nosp', round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'])
PY

#!/bin/bash
# Round 3, session Y: leaner result collection (no device-wide syncs) — GPU suite, bench lines,
# kernel-trace timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/y
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  python - $O/bench.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], 'corr', d['corr_ms'][-2:], d['engine_phases_ms'])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
python tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt 2>&1; tail -8 $O/timeline.txt

#!/bin/bash
# Round 3, session U: pipelined level loop (depth d >= 2 enqueued on bound degrees, k_decompose on
# the device): the full GPU suite, then A/B lines PCG_PIPELINE=1/0 and a kernel trace timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in PCG_PIPELINE=1 PCG_PIPELINE=0 PCG_PIPELINE=1 PCG_PIPELINE=0; do
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  python - $O/bench.log "$v" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('%-16s'%sys.argv[2], round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], 'corr', d['corr_ms'][-2:], d['tests_per_level'])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
python tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt 2>&1; tail -3 $O/timeline.txt

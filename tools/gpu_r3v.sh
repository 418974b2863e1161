#!/bin/bash
# Round 3, session V: pipelined level loop from depth PCG_PIPELINE_LO: parity (skeleton suite with
# the loop from depth 2 and from depth 5), n = 500 full-depth A/B, config-5 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/v
mkdir -p $O
PCG_PIPELINE_LO=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread -k "not config5" > $O/pytest2.log 2>&1
rc=$?; tail -2 $O/pytest2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread -k "n500 or wave or config5" > $O/pytest5.log 2>&1
rc=$?; tail -2 $O/pytest5.log; [ $rc -eq 0 ] || exit $rc
for v in PCG_PIPELINE=1 PCG_PIPELINE=0 PCG_PIPELINE_LO=3 PCG_PIPELINE=1 PCG_PIPELINE=0; do
  env $v timeout -k 10 300 python tools/profile_deep.py --n 500 --reps 5 > $O/deep.log 2>&1 || { tail -5 $O/deep.log; exit 1; }
  echo "$v $(tail -c 300 $O/deep.log)"
done
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
python - $O/bench.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('bench', round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], 'corr', d['corr_ms'][-2:])
PY

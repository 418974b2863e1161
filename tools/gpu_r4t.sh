#!/bin/bash
# Round 4, session T: lane-per-test exact path for recorded pairs — parity, full-p probe, bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/t
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_small.py tests/test_gpu_skeleton_ref.py -q -x \
  -k "skeleton_matches_oracle or config5 or near_collinear or fullp or records or ref or p_values or singular or fused" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" $O/tests.log | head -80; exit $rc; }
timeout -k 10 200 python -u tools/fullp_probe.py --reps 3 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep '^{' $O/probe.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
python - $O/bench.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print("bench ms %.3f kernel %s" % (d["ms_per_step"], d["kernel_ms_per_level"]))
print("full_p", json.dumps(d["full_p"]))
PY

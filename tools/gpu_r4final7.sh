#!/bin/bash
# Round 4 closing, part 7: the bench line at HEAD with the refreshed roofline model.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/final7
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench_line.json
python - $O/bench_line.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print(round(d['ms_per_step'], 3), d['kernel_ms_per_level'], round(d['roofline']['frac'], 3), d['roofline']['frac_bounds'], d['full_p']['skeleton_device_ms'], d['cpu_baseline']['value'])
PY

#!/bin/bash
# Round 4 closing, part 3: the bench line again on another box (20 timed steps), since part 2's
# box ran the dominant kernel 8 % slower than every earlier session's.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/final3
mkdir -p $O
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | tail -1 > $O/bench_line.json
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-p > $O/bench2.log 2>&1 || { tail -20 $O/bench2.log; exit 1; }
python - $O/bench_line.json $O/bench2.log <<'PY'
import json, sys
for f in sys.argv[1:]:
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l)
            print(f, round(d['ms_per_step'], 3), d['kernel_ms_per_level'], round(d['roofline']['frac'], 3), d['corr_ms'])
PY

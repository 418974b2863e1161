#!/bin/bash
# Round 4 closing, part 8: the RQ2 harness lines at HEAD (both synthetic trees).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/final8
mkdir -p $O
timeout -k 10 300 python -u bench.py --workload rq2 > $O/rq2_ob.log 2>&1 || { tail -20 $O/rq2_ob.log; exit 1; }
timeout -k 10 300 python -u bench.py --workload rq2 --rq2-dataset sock-shop > $O/rq2_ss.log 2>&1 || { tail -20 $O/rq2_ss.log; exit 1; }
grep '^{' $O/rq2_ob.log | tail -1 > $O/rq2_ob.json
grep '^{' $O/rq2_ss.log | tail -1 > $O/rq2_ss.json
python - $O/rq2_ob.json $O/rq2_ss.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.loads(open(f).read())
    print(f, d['metric'], round(d['value'], 1), d['unit'])
PY

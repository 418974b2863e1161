#!/bin/bash
# Round 4, session S: where the full-p mode's time goes (kernel trace of tools/fullp_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/s
mkdir -p $O
timeout -k 10 200 python -u tools/fullp_probe.py --reps 3 > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cat $O/probe.log | grep '^{'
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tr -o run --output-format csv -- python tools/fullp_probe.py --reps 2 > $O/tr.log 2>&1 || exit $?
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4/s/tr/run_kernel_stats.csv")))
for r in rows[:14]:
    print(r["Name"][:70], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 3), "ms total", round(float(r["AverageNs"]) / 1e3, 1), "us avg")
PY

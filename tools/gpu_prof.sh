#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.log 2>&1
rc=$?
python tools/timeline.py gpurun_out/prof/run_kernel_trace.csv > gpurun_out/timeline.txt 2>&1
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof/**/run_kernel_stats.csv", recursive=True) + glob.glob("gpurun_out/prof/run_kernel_stats.csv")
r = list(csv.DictReader(open(f[0])))
for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:16]:
    print(x["Name"][:60].ljust(60), x["Calls"], "%.3f" % (float(x["AverageNs"]) / 1e6))
PY
exit $rc

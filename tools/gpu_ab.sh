#!/bin/bash
# A/B of the fp32 screen per depth: kernel stats under rocprofv3 for each PCG_SCREEN_MASK given
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in "$@"; do
  export ${AB_VAR:-PCG_SCREEN_MASK}=$m
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$m -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_$m.log 2>&1 || exit $?
  echo "== mask $m"
  python - "$m" <<'PY'
import csv, glob, json, sys
m = sys.argv[1]
f = glob.glob(f"gpurun_out/ab_{m}/**/run_kernel_stats.csv", recursive=True)
r = list(csv.DictReader(open(f[0])))
for x in sorted(r, key=lambda x: -float(x["TotalDurationNs"]))[:14]:
    if "1>" in x["Name"] and "k_level" in x["Name"]: continue
    print(x["Name"][:58].ljust(58), x["Calls"], "%.3f" % (float(x["AverageNs"]) / 1e6))
l = [x for x in open(f"gpurun_out/ab_{m}.log") if x.startswith("{")]
d = json.loads(l[-1]); print("ms", round(d["ms_per_step"], 3), "level_ms", d["level_ms"])
PY
done

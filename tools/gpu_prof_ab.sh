#!/bin/bash
# rocprofv3 kernel stats of the in-tree build and each tools/ab/ variant (PCG_LIB_PATH), a short
# bench each; prints the kernels named by the PROF_GREP regex
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in rcaeval_amd/libpcgpu.so tools/ab/libpcgpu_*.so; do
  [ -f "$v" ] || continue
  name=$(basename "$v" .so)
  rm -rf "gpurun_out/pab_$name"
  PCG_LIB_PATH="$PWD/$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/pab_$name" -o run --output-format csv -- \
    python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-full-p > "gpurun_out/pab_$name.log" 2>&1 || exit $?
  python - "$name" "gpurun_out/pab_$name" "${PROF_GREP:-level1|edge_c}" <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[2] + "/**/run_kernel_stats.csv", recursive=True)
for x in csv.DictReader(open(f[0])):
    if re.search(sys.argv[3], x["Name"]):
        print("%-12s %-50s %4s %8.1f us" % (sys.argv[1][:12], x["Name"][:50], x["Calls"], float(x["AverageNs"]) / 1e3))
PY
done

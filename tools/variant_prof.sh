#!/bin/bash
# Per-kernel durations of engine build variants: rocprofv3 --kernel-trace --stats over a short
# bench for the in-tree build ("base") and each tools/ab/libpcgpu_*.so (PCG_LIB_PATH), then the
# average duration of the kernels matching VARIANT_PROF_PAT (default: the level kernels).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PAT=${VARIANT_PROF_PAT:-k_level|k_node_blocks|k_screen|k_xtx|k_residues|k_crt}
for v in rcaeval_amd/libpcgpu.so tools/ab/libpcgpu_*.so; do
  [ -f "$v" ] || continue
  name=$(basename "$v" .so)
  [ "$v" = rcaeval_amd/libpcgpu.so ] && name=base
  PCG_LIB_PATH="$PWD/$v" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "gpurun_out/vprof_$name" -o run \
    --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-p ${VARIANT_BENCH_ARGS:-} \
    > "gpurun_out/vprof_$name.log" 2>&1 || { echo "$name failed rc=$?"; tail -5 "gpurun_out/vprof_$name.log"; exit 1; }
  python - "$name" "gpurun_out/vprof_$name" "$PAT" <<'PY'
import csv, glob, re, sys
f = glob.glob(sys.argv[2] + "/**/run_kernel_stats.csv", recursive=True)
rows = list(csv.DictReader(open(f[0])))
def kname(raw):
    s = raw.replace("void ", "", 1).replace("(anonymous namespace)::", "")
    depth, o = 0, []
    for ch in s:   # cut the argument list, keep template args
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        o.append(ch)
    return "".join(o).replace(" ", "")
out = []
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    if re.search(sys.argv[3], r["Name"]):
        out.append("%s=%.1f" % (kname(r["Name"]), float(r["AverageNs"]) / 1e3))
print("%-16s %s" % (sys.argv[1], "  ".join(out[:14])), flush=True)
PY
done

#!/bin/bash
# Round 4, session V: K1 split-K A/B (PCG_K1_CRT_KS: how many k-slabs; per (modulus, slab) group
# an XCD's panels shrink with more slabs) — time per pcg_corr and the GEMM's stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/v
mkdir -p $O
for ks in 2 3 4 6 8 12 2; do
  PCG_K1_CRT_KS=$ks timeout -k 10 120 python -u tools/micro/k1_time.py rcaeval_amd/libpcgpu.so > $O/k1_ks$ks.log 2>&1 || { tail -5 $O/k1_ks$ks.log; exit 1; }
  echo "ks=$ks $(grep ms/corr $O/k1_ks$ks.log)"
done
for ks in 2 8; do
  PCG_K1_CRT_KS=$ks timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $O/tr$ks -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so > $O/tr$ks.log 2>&1 || exit 1
  python - $ks <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/r4/v/tr{sys.argv[1]}/run_kernel_stats.csv")))
print("ks", sys.argv[1], [(r["Name"].split("(")[0].replace("(anonymous namespace)::", "")[-28:], round(float(r["AverageNs"]) / 1e3, 1)) for r in rows[:6]])
PY
done

#!/bin/bash
# Round 3, session Z2: CRT K1 after the finish / residue / fragment-pipelining changes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/z2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_skeleton.py -m gpu -x -q --timeout 120 --timeout-method thread -k "corr" > $O/pytest_corr.log 2>&1
rc=$?; tail -3 $O/pytest_corr.log; [ $rc -eq 0 ] || exit $rc
for ks in 0 1 3; do
  PCG_K1_CRT_KS=$ks timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof$ks -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/prof$ks.log 2>&1 || exit 1
  echo "ks=$ks"; grep -E "k_xtx|k_resid|k_crt|k_normalize|k_col" $O/prof$ks/run_kernel_stats.csv | awk -F'",' '{print substr($1,1,40), $2}' | cut -c1-120
done
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
python - $O/bench.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(round(d['ms_per_step'],3), d['value'], d['kernel_ms_per_level'], 'corr', d['corr_ms'][-2:])
PY

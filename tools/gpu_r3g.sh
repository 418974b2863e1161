#!/bin/bash
# Round 3, session G: full GPU suite (k_level_ty default, background knowledge, RCD glue
# rewrite), then the k_level_ty A/B on the bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/g_tests.log 2>&1
rc=$?; tail -3 $O/g_tests.log; [ $rc -eq 0 ] || exit $rc
for ty in 1 0 1 0; do
  PCG_TY=$ty timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/g_bench_ty$ty.log 2>&1 || { echo "bench failed"; tail -5 $O/g_bench_ty$ty.log; exit 1; }
  python - "$ty" $O/g_bench_ty$ty.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")]
d = json.loads(l[-1])
print("TY=%s value %.3e ms %.3f kernel_ms %s level_ms %s screened %s" % (sys.argv[1], d["value"], d["ms_per_step"], d["kernel_ms_per_level"], d["level_ms"], d["screened"]))
PY
done

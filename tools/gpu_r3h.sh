#!/bin/bash
# Round 3, session H: K1 on the int8 digit GEMM -- K1 parity (numpy, sharded bitwise), the
# skeleton suite on its C, then bench A/B PCG_K1_I8=1/0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_skeleton.py -x -q -k "corr" --timeout 300 --timeout-method thread > $O/h_corr.log 2>&1
rc=$?; tail -5 $O/h_corr.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread > $O/h_tests.log 2>&1
rc=$?; tail -3 $O/h_tests.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  PCG_K1_I8=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/h_bench_i8$v.log 2>&1 || { echo "bench failed"; tail -5 $O/h_bench_i8$v.log; exit 1; }
  python - "$v" $O/h_bench_i8$v.log <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")]
d = json.loads(l[-1])
print("I8=%s value %.3e ms %.3f corr %s kernel_ms %s level_ms %s" % (sys.argv[1], d["value"], d["ms_per_step"], d["corr_ms"][-3:], d["kernel_ms_per_level"], d["level_ms"]))
PY
done
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r3/h_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r3/h_prof.log 2>&1
echo prof rc=$?

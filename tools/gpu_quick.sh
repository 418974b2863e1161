#!/bin/bash
# Quick GPU iteration: skeleton parity tests, then a short bench (no CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 300 --timeout-method thread > gpurun_out/quick_test.log 2>&1
rc=$?; tail -3 gpurun_out/quick_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/quick_bench.log 2>&1
rc=$?
python - <<'PY'
import json
l = [x for x in open("gpurun_out/quick_bench.log") if x.startswith("{")]
d = json.loads(l[-1])
print("value %.3e  ms %.3f  kernel_ms %s  level_ms %s  corr %s" % (d["value"], d["ms_per_step"], d["kernel_ms_per_level"], d["level_ms"], d["corr_ms"][-1]))
print("screened %s  exact %s  edges %s" % (d.get("screened"), d.get("exact_path"), d.get("edges_after")))
PY
exit $rc

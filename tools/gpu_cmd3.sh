# parity (skeleton, small, native-dist records) + a bench line with the sampled-records leg
set -u
timeout -k 10 500 python -u -m pytest tests/test_gpu_skeleton.py tests/test_gpu_small.py tests/test_gpu_citest.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pt_c.log 2>&1; rc=$?; tail -3 gpurun_out/pt_c.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_fp.log 2>&1; rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_fp.log; exit $rc; }
python - <<'PY'
import json
d = json.loads([x for x in open("gpurun_out/bench_fp.log") if x.startswith("{")][-1])
print("ms", round(d["ms_per_step"], 3), "levels", d["level_ms"], "sampled", json.dumps(d.get("sampled_records"))[:400])
PY

#!/bin/bash
# A/B timing of engine build variants on the GPU box: for each tools/micro/variants/libpcgpu_*.so
# (and the in-tree build, "base"), copy it over the in-tree library and run a short bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
for v in /tmp/libpcgpu_base.so tools/micro/variants/libpcgpu_*.so; do
  name=$(basename "$v" .so)
  cp "$v" rcaeval_amd/libpcgpu.so
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > "gpurun_out/var_$name.log" 2>&1 || { echo "$name failed rc=$?"; tail -5 "gpurun_out/var_$name.log"; exit 1; }
  python - "$name" "gpurun_out/var_$name.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")]
d = json.loads(l[-1])
print("%-24s value %.3e  ms %.3f  kernel_ms %s level_ms %s corr %s edges %s same_fullp %s" % (sys.argv[1], d["value"], d["ms_per_step"], d["kernel_ms_per_level"], d["level_ms"], d["corr_ms"][-2:], d["edges_after"], (d.get("full_p") or {}).get("same_skeleton_as_threshold")))
PY
done
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so

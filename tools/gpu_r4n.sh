#!/bin/bash
# Round 4, session N: ablation timings of k_level_lds_f (tools/variants_r4/libpcgpu_abl*.so: tasks
# without sweeps / no tasks, at depth 3 or 4) against the in-tree build, same bench workload.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/n
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_skeleton.py -q -x -k "skeleton_matches_oracle or wide_and_large or screen_precision or depth2 or n500 or schur or pipelined or fused or wave_kernel or config5" --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
for v in /tmp/libpcgpu_base.so tools/variants_r4/libpcgpu_*.so; do
  name=$(basename "$v" .so)
  cp "$v" rcaeval_amd/libpcgpu.so
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full-p > "$O/$name.log" 2>&1 || { echo "$name failed rc=$?"; tail -5 "$O/$name.log"; cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so; exit 1; }
  python - "$name" "$O/$name.log" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print("%-22s ms %.3f kernel_ms %s level_ms %s" % (sys.argv[1], d["ms_per_step"], d["kernel_ms_per_level"], d["level_ms"]))
PY
done
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so

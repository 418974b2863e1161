#!/bin/bash
# Round 4, session Q: depth-4 candidate-group / occupancy variants (tools/variants_r4/*.so) vs the
# in-tree build, alternating so box drift shows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/${QDIR:-q}
mkdir -p $O
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
for v in /tmp/libpcgpu_base.so tools/variants_r4/libpcgpu_*.so /tmp/libpcgpu_base.so; do
  name=$(basename "$v" .so)
  cp "$v" rcaeval_amd/libpcgpu.so
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-p > "$O/$name.log" 2>&1 || { echo "$name failed rc=$?"; tail -5 "$O/$name.log"; cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so; exit 1; }
  python - "$name" "$O/$name.log" <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print("%-22s ms %.3f kernel_ms %s level_ms %s" % (sys.argv[1], d["ms_per_step"], d["kernel_ms_per_level"], d["level_ms"]))
PY
done
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so

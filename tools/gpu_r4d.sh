#!/bin/bash
# Round 4, session D: A/B of depth-2/3 occupancy and staging variants (tools/build_variant.sh; kept out of .gpurunignore so they travel):
# per variant one bench line (kernel ms per depth, per-level tests and edges as a sanity check).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/d
mkdir -p $O
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
for v in /tmp/libpcgpu_base.so tools/variants_r4/libpcgpu_*.so; do
  name=$(basename "$v" .so)
  cp "$v" rcaeval_amd/libpcgpu.so
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-full-p > $O/$name.log 2>&1 || { echo "$name bench failed rc=$?"; tail -5 $O/$name.log; cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so; exit 1; }
  python - "$O/$name.log" "$name" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[2], round(d['ms_per_step'], 3), 'kern', d['kernel_ms_per_level'], 'lvl', d['level_ms'], 'edges', d['edges_after'][-1], 'tests', sum(d['tests_per_level']))
PY
done
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so

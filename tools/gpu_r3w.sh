#!/bin/bash
# Round 3, session W: n = 500 full-depth wall time with the pipelined loop from depth 2 / 3 / 5 / off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/w
mkdir -p $O
for v in PCG_PIPELINE=1 PCG_PIPELINE=0 PCG_PIPELINE_LO=3 PCG_PIPELINE_LO=2 PCG_PIPELINE=1 PCG_PIPELINE=0; do
  env $v timeout -k 10 300 python tools/profile_deep.py --n 500 --reps 9 > $O/deep.log 2>&1 || { tail -5 $O/deep.log; exit 1; }
  python - $O/deep.log "$v" <<'PY'
import json,sys
l=open(sys.argv[1]).read(); d=json.loads(l[l.find('{'):])
print('%-18s'%sys.argv[2], 'gpu_ms %.3f'%d['gpu_ms'], d['gpu_ms_all'], 'levels', d['levels'])
PY
done

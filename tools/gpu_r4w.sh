#!/bin/bash
# Round 4, session W: compact node blocks at depth 3 (PCG_NODE_BLOCKS=0x18) A/B, the n = 500
# host trace per level, and a bench line with the r04 roofline model.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/w
mkdir -p $O
for v in "PCG_NODE_BLOCKS=0x10" "PCG_NODE_BLOCKS=0x18" "PCG_NODE_BLOCKS=0x10"; do
  tag=$(echo $v | tr '=' '_')
  env $v timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-p > $O/b_$tag.log 2>&1 || { tail -20 $O/b_$tag.log; exit 1; }
  echo "$v: $(python -c "import json; d=[json.loads(l) for l in open('$O/b_$tag.log') if l.startswith('{')][-1]; print(round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], 'roof', round(d['roofline']['frac'] or 0, 3))")"
done
PCG_HOST_TRACE=1 timeout -k 10 120 python -u tools/profile_deep.py --n 500 --reps 1 > $O/ht500.log 2>&1 || { tail -20 $O/ht500.log; exit 1; }
grep -c "pcg host" $O/ht500.log

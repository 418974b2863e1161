#!/bin/bash
# A/B bench lines: every in-tree env setting in $AB_ENVS (space-separated, "base" = none) on the
# in-tree library, then every tools/micro/variants/libpcgpu_*.so (variant_bench.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
for v in ${AB_ENVS:-base}; do
  if [ "$v" = base ]; then e=""; else e="$v"; fi
  env $e timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
  python - $O/bench.log "$v" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('%-28s'%sys.argv[2], round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], 'corr', d['corr_ms'][-2:])
PY
done
ls tools/micro/variants/libpcgpu_*.so > /dev/null 2>&1 && { timeout -k 10 900 bash tools/variant_bench.sh || exit 1; }
echo done

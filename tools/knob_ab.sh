#!/bin/bash
# Runtime-knob A/B of the headline bench (bench.py --tune KEY=VALUE, pcg_set_tuning): each
# setting twice, interleaved. usage: tools/knob_ab.sh "KEY=V[,KEY=V]" ...   ("-" = defaults)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "$@"; do
    args=""
    if [ "$cfg" != "-" ]; then for kv in ${cfg//,/ }; do args="$args --tune $kv"; done; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full-p $args > gpurun_out/knob.log 2>&1 || { echo "$cfg failed"; tail -5 gpurun_out/knob.log; exit 1; }
    python - "$cfg" gpurun_out/knob.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print("%-28s ms %.3f  kernel_ms %s level_ms %s" % (sys.argv[1], d["ms_per_step"], d["kernel_ms_per_level"], d["level_ms"]))
PY
  done
done

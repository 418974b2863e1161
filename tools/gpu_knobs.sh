#!/bin/bash
# Runtime-knob A/B on the GPU box: one short bench per setting (pcg_set_tuning via bench.py
# --tune), each under its own time limit; prints steps / level / kernel times per setting.
# usage: tools/gpu_knobs.sh "" "NBW=2048" "NODE_BLOCKS=0x18 NB=8192" ...   ("" = defaults)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
for setting in "$@"; do
  args=""
  for kv in $setting; do args="$args --tune $kv"; done
  log="gpurun_out/knob_$i.log"
  timeout -k 10 240 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full-p $args > "$log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "[$setting] rc=$rc"; tail -5 "$log"; exit $rc; fi
  python - "$setting" "$log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")]
d = json.loads(l[-1])
print("%-34s ms %.3f (min %.3f)  level %s  kernel %s" % (sys.argv[1] or "default", d["ms_per_step"], min(d["step_ms_all"]),
      d["level_ms"], d["kernel_ms_per_level"]), flush=True)
PY
  i=$((i + 1))
done

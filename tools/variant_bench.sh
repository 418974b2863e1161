#!/bin/bash
# A/B timing of engine build variants on the GPU box: the in-tree build ("base") and each
# tools/ab/libpcgpu_*.so (tools/build_variants.sh), loaded through PCG_LIB_PATH — the
# in-tree library is never overwritten. Extra bench args: VARIANT_BENCH_ARGS.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in rcaeval_amd/libpcgpu.so tools/ab/libpcgpu_*.so; do
  [ -f "$v" ] || continue
  name=$(basename "$v" .so)
  [ "$v" = rcaeval_amd/libpcgpu.so ] && name=base
  PCG_LIB_PATH="$PWD/$v" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-full-p \
    ${VARIANT_BENCH_ARGS:-} > "gpurun_out/var_$name.log" 2>&1 || { echo "$name failed rc=$?"; tail -5 "gpurun_out/var_$name.log"; exit 1; }
  python - "$name" "gpurun_out/var_$name.log" <<'PY'
import json, sys
l = [x for x in open(sys.argv[2]) if x.startswith("{")]
d = json.loads(l[-1])
print("%-24s value %.3e  ms %.3f  kernel_ms %s level_ms %s corr %s edges %s" % (sys.argv[1], d["value"], d["ms_per_step"], d["kernel_ms_per_level"], d["level_ms"], d["corr_ms"][-2:], d["edges_after"]))
PY
done

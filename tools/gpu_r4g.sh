#!/bin/bash
# Round 4, session G: small-graph kernel tests + timing, and a warm host trace of the config-5 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/g
mkdir -p $O
: > $O/status.log
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $O/status.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; cat $O/status.log; tail -30 $O/$name.log; exit $rc; fi
}
step small_tests 300 python -u -m pytest tests/test_gpu_small.py -q --timeout 120 --timeout-method thread
tail -2 $O/small_tests.log
step small_bench 200 python -u tools/small_bench.py 44 600 200
tail -1 $O/small_bench.log
PCG_HOST_TRACE=1 step host_trace 200 python -u bench.py --steps 2 --warmup 2 --no-cpu-baseline --no-full-p
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-p
python tools/timeline.py $O/prof/run_kernel_trace.csv > $O/timeline.txt 2>&1
tail -3 $O/timeline.txt
cat $O/status.log
# depth-3 variants (tools/variants_r4) and block targets (PCG_NB3), one bench line each
line() { python - "$1" "$2" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(sys.argv[2], round(d['ms_per_step'], 3), 'kern', d['kernel_ms_per_level'], 'lvl', d['level_ms'], 'tests', sum(d['tests_per_level']))
PY
}
cp rcaeval_amd/libpcgpu.so /tmp/libpcgpu_base.so
for nb in 2048 8192; do
  PCG_NB3=$nb timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-full-p > $O/nb3_$nb.log 2>&1 && line $O/nb3_$nb.log nb3_$nb
done
for v in /tmp/libpcgpu_base.so tools/variants_r4/libpcgpu_*.so; do
  name=$(basename "$v" .so)
  cp "$v" rcaeval_amd/libpcgpu.so
  timeout -k 10 120 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-full-p > $O/$name.log 2>&1 || { echo "$name failed"; cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so; exit 1; }
  line $O/$name.log $name
done
cp /tmp/libpcgpu_base.so rcaeval_amd/libpcgpu.so

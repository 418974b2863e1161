#!/bin/bash
# Round 4, session K: fused barrier (cheap grid barrier) and the pipelined loop with the
# device-chosen chunk size — parity tests, then A/B timings at config 5 and n = 500.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/k
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
step tests 400 python -u -m pytest tests/test_gpu_skeleton.py -q -x -k "fused or pipelined or overflow or n500" --timeout 150 --timeout-method thread
tail -3 $O/tests.log
for v in "PCG_FUSE_END=0" "PCG_FUSE_END=1" "PCG_FUSE_END=0 PCG_PIPELINE=1 PCG_PIPELINE_LO=2" "PCG_FUSE_END=1 PCG_PIPELINE=1 PCG_PIPELINE_LO=2" "PCG_FUSE_END=0 PCG_PIPELINE=1 PCG_PIPELINE_LO=2 PCG_DEV_SPL=0"; do
  tag=$(echo $v | tr ' =' '_-')
  env $v timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-p > $O/b_$tag.log 2>&1 || { echo "bench $v failed"; tail -20 $O/b_$tag.log; exit 1; }
  echo "$v: $(python -c "import json,sys; d=[json.loads(l) for l in open('$O/b_$tag.log') if l.startswith('{')][-1]; print(round(d['ms_per_step'],3), d.get('level_ms'))")"
  env $v timeout -k 10 120 python -u tools/profile_deep.py --n 500 --reps 5 > $O/d_$tag.log 2>&1 || { echo "deep $v failed"; tail -20 $O/d_$tag.log; exit 1; }
  echo "   n500: $(python -c "import json; d=[json.loads(l) for l in open('$O/d_$tag.log') if l.startswith('{')][-1]; print(round(d['gpu_ms'],3))")"
done
PCG_FUSE_END=1 step tl_fused 200 rocprofv3 --kernel-trace -d $O/tlf -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-p
python tools/timeline.py $O/tlf/run_kernel_trace.csv > $O/timeline_fused.txt 2>&1; tail -32 $O/timeline_fused.txt
cat $O/status.log

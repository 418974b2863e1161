#!/bin/bash
# Round 4, session J: the fused level barrier (k_level_end) — A/B parity, bench A/B, timeline,
# then the skeleton / small / reference-pinned GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/j
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
step fused 300 python -u -m pytest tests/test_gpu_skeleton.py -q -x -k "fused or overflow or singular or n500 or max_depth" --timeout 150 --timeout-method thread
tail -3 $O/fused.log
step bench_fused 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
tail -1 $O/bench_fused.log | cut -c1-400
PCG_FUSE_END=0 step bench_sep 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline
tail -1 $O/bench_sep.log | cut -c1-400
step deep500 200 python -u tools/profile_deep.py --n 500 --reps 5
PCG_FUSE_END=0 step deep500_sep 200 python -u tools/profile_deep.py --n 500 --reps 5
tail -3 $O/deep500_sep.log
tail -5 $O/deep500.log
step tl 300 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline
python tools/timeline.py $O/tl/run_kernel_trace.csv > $O/timeline.txt 2>&1; tail -40 $O/timeline.txt
step small 300 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_skeleton_ref.py -q --timeout 100 --timeout-method thread
tail -2 $O/small.log
step skel 600 python -u -m pytest tests/test_gpu_skeleton.py -q --timeout 200 --timeout-method thread
tail -3 $O/skel.log
cat $O/status.log

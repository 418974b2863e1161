#!/bin/bash
# Round-closing GPU session. usage: tools/gpu_round.sh TAG PART
#   PART 1: GPU tests, smoke, rocprofv3 kernel stats + device timeline, the PMC passes of the
#           in-tree build and (when tools/ab/libpcgpu_abl1.so exists) of the no-sweep ablation
#           build (tools/build_variants.sh abl1 -DPCG_TGF_ABL=1) for tools/roofline_model.py
#   PART 2: the bench lines (skeleton, RQ2 Online-Boutique- and Sock-Shop-shaped), read after the
#           round's roofline model is committed
# Every step has its own time limit; any abnormal exit (not 0 / 1 = test failures) stops the script.
# Outputs land in gpurun_out/ as TAG_* files, to be copied into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r05}
PART=${2:-1}
: > $OUT/round_status.log
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $OUT/round_status.log
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $OUT/round_status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; cat $OUT/round_status.log; tail -5 "$OUT/$name.log"; exit $rc; fi
}
line() {   # the JSON line of a bench log
  grep '^{' "$OUT/$1.log" | tail -1 > "$OUT/${TAG}_$2.json"
}
if [ "$PART" = 1 ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 600 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  rm -rf $OUT/prof
  step prof 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-p
  python tools/timeline.py "$(find $OUT/prof -name run_kernel_trace.csv | head -1)" > $OUT/${TAG}_timeline.txt 2>&1
  cp "$(find $OUT/prof -name run_kernel_stats.csv | head -1)" $OUT/${TAG}_kernel_stats.csv
  if [ -n "${SKIP_PMC:-}" ]; then cat $OUT/round_status.log; exit 0; fi   # (the sweep kernels' PMC unchanged)
  step pmc 900 bash tools/pmc_passes.sh
  cp $OUT/pmc_summary.json $OUT/${TAG}_pmc_summary.json
  if [ -f tools/ab/libpcgpu_abl1.so ]; then
    PCG_LIB_PATH=$PWD/tools/ab/libpcgpu_abl1.so step pmc_abl1 900 bash tools/pmc_passes.sh
    cp $OUT/pmc_summary.json $OUT/${TAG}_valu_class_pmc_abl1.json
  fi
else
  step bench 900 python bench.py --steps 20 --warmup 3
  line bench bench_line
  step rq2 600 python bench.py --workload rq2 --steps 1 --warmup 1
  line rq2 rq2_bench_line
  step rq2ss 600 python bench.py --workload rq2 --rq2-dataset sock-shop --steps 1 --warmup 1
  line rq2ss rq2_ss_bench_line
fi
cat $OUT/round_status.log

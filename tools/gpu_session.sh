#!/bin/bash
# Runs GPU steps one after another; each under its own time limit. Stops at the first
# step that did not end normally (exit 0 = pass, 1 = test failures are tolerated).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/status.log
run() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> gpurun_out/status.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> gpurun_out/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; cat gpurun_out/status.log; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    smoke) run smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    test)  run pytest_gpu 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    testall) run pytest_gpu 1200 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread ;;
    bench) run bench 900 python bench.py --steps 3 --warmup 1 ;;
    benchfast) run bench 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    prof) run prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    dist2) PCG_DIST_TRACE=1 PCG_BENCH_DEVICE=0 PCG_DIST_BACKEND=gloo run dist2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 ;;
    sim) run sim 600 python tools/shard_sim.py ;;
    quick) run quick 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-full-p ;;
    # the sharded drivers at world 1 (their fixed overhead over the single-GPU call): native C / RCCL, torch.distributed
    dist1n) PCG_BENCH_FORCE_DIST=1 run dist1n 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-full-p ;;
    dist1t) PCG_BENCH_FORCE_DIST=1 PCG_DIST_NATIVE=0 run dist1t 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-full-p ;;
    k:*) run "pytest_${step#k:}" 900 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread -p no:cacheprovider -k "${step#k:}" ;;
    htrace) PCG_HOST_TRACE=1 run htrace 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-p ;;
    *) echo "unknown step $step" ;;
  esac
done
cat gpurun_out/status.log

#!/bin/bash
# host-trace bench run (PCG_HOST_TRACE=1: the level loop's host timestamps on stderr), then the
# tools/ab/ variants A/B'd by tools/variant_bench.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
PCG_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-full-p > gpurun_out/ht.log 2> gpurun_out/ht.err || exit $?
for v in tools/ab/libpcgpu_*.so; do
  [ -f "$v" ] || continue
  PCG_LIB_PATH="$PWD/$v" PCG_HOST_TRACE=1 timeout -k 10 300 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-full-p \
    > gpurun_out/ht_$(basename $v .so).log 2> gpurun_out/ht_$(basename $v .so).err || exit $?
done
for rep in 1 2; do bash tools/variant_bench.sh || exit $?; done

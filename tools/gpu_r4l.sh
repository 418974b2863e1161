#!/bin/bash
# Round 4, session L: grid-barrier micro-benchmark; stochastic PC sampling of a config-5 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/l
mkdir -p $O
for cfg in "256 256 8" "256 1024 8" "512 256 8" "1024 256 8" "256 256 32"; do
  timeout -k 5 60 ./tools/micro/grid_barrier $cfg >> $O/grid_barrier.txt 2>&1 || { echo "grid_barrier $cfg rc=$?"; cat $O/grid_barrier.txt; exit 1; }
done
cat $O/grid_barrier.txt
rocprofv3 -L > $O/list_avail.txt 2>&1 || true
grep -i -A3 "pc" $O/list_avail.txt | head -40
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 262144 -d $O/pcs -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-p > $O/pcs.log 2>&1
echo "pcs rc=$?"
tail -5 $O/pcs.log
ls -la $O/pcs 2>/dev/null | head

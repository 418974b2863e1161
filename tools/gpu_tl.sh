#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/tl -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/tl.log 2>&1 || exit $?
python tools/timeline.py $OUT/tl/run_kernel_trace.csv > $OUT/timeline.txt 2>&1
tail -80 $OUT/timeline.txt

#!/bin/bash
# the sharded drivers' overhead at world 1 (torch.distributed vs native RCCL vs the 1-GPU call)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
R="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/d1_single.log 2>&1 || exit $?
PCG_BENCH_FORCE_DIST=1 PCG_DIST_TRACE=1 timeout -k 10 300 $R > $OUT/d1_torch.log 2>&1 || exit $?
PCG_BENCH_FORCE_DIST=1 PCG_DIST_NATIVE=1 timeout -k 10 300 $R > $OUT/d1_native.log 2>&1 || exit $?
for f in single torch native; do python -c "
import json,sys
l=[x for x in open('$OUT/d1_$f.log') if x.startswith('{')]
d=json.loads(l[-1]); print('$f', round(d['ms_per_step'],3), 'ms', d['config']['parallelism'])"; done
grep "rank 0" $OUT/d1_torch.log | tail -2

#!/bin/bash
# Round 3, session T: k_level_lds_f staging the compact node blocks + split window by default:
# parity, then A/B lines (node blocks on / off, SP at depth 4) and FETCH/WRITE of the depth-4 sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/t
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_skeleton.py -x -q --timeout 600 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for v in "PCG_NODE_BLOCKS=0x18" "PCG_NODE_BLOCKS=0" "PCG_SP=0x10" "PCG_NODE_BLOCKS=0x18" "PCG_NODE_BLOCKS=0"; do
  env $v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
  python - $O/bench.log "$v" <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'], 'corr', d['corr_ms'][-2:])
PY
done
B="python bench.py --steps 1 --warmup 1 --no-cpu-baseline"
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $P -d $O/pmc_$P -o run --output-format csv -- $B > $O/pmc_$P.log 2>&1 || { echo "pmc $P failed"; exit 1; }
done
echo done

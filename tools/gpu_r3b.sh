#!/bin/bash
# Round 3, session B: issue-cost table with the extended opcode list; n = 500 full-depth
# skeleton: per-level times and a kernel-trace profile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 120 ./tools/micro/issue_cost all 1 2 4 8 > $O/issue_cost2.json 2> $O/issue_cost2.err || { echo "issue_cost failed"; cat $O/issue_cost2.err; exit 1; }
echo "issue_cost ok"
timeout -k 10 180 python tools/profile_deep.py --n 500 > $O/deep500.json 2> $O/deep500.err || { echo "deep failed"; tail $O/deep500.err; exit 1; }
cat $O/deep500.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/deep500_prof -o run --output-format csv -- python tools/profile_deep.py --n 500 --reps 1 > $O/deep500_prof.log 2>&1 || { echo "prof failed"; tail $O/deep500_prof.log; exit 1; }
echo done

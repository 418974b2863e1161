#!/bin/bash
# quick GPU iteration + one-step timeline + host trace of the level loop
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_quick.sh || exit $?
bash tools/gpu_tl.sh > /dev/null 2>&1 || exit $?
grep -E "k_level_lds_t<4|span" gpurun_out/timeline.txt
PCG_HOST_TRACE=1 timeout -k 10 200 python tools/profile_step.py > gpurun_out/ht.log 2>&1 || exit $?
tail -42 gpurun_out/ht.log | head -40 > gpurun_out/ht_tail.log

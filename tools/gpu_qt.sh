#!/bin/bash
# quick GPU iteration + one-step timeline
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash tools/gpu_quick.sh || exit $?
bash tools/gpu_tl.sh > /dev/null 2>&1 || exit $?
grep -E "k_level_lds_t<4|span" gpurun_out/timeline.txt

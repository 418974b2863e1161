#!/bin/bash
# Round 3, session C: deep-level kernel (k_level_wave) parity + n = 500 full-depth timing and
# kernel trace; reference-glue golden tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_skeleton.py -x -v --timeout 300 --timeout-method thread \
  -k "full_depth_n500 or wave_kernel or constant_column" > $O/c_tests.log 2>&1
rc=$?; tail -5 $O/c_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_e2e.py -x -v --timeout 300 --timeout-method thread \
  -k "glue or deep or readme or oracle_pipeline" > $O/c_e2e.log 2>&1
rc=$?; tail -5 $O/c_e2e.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python tools/profile_deep.py --n 500 > $O/deep500_r3c.json 2> $O/deep500_r3c.err || { tail $O/deep500_r3c.err; exit 1; }
cat $O/deep500_r3c.json
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/deep500c_prof -o run --output-format csv -- python tools/profile_deep.py --n 500 --reps 2 > $O/deep500c_prof.log 2>&1 || { tail $O/deep500c_prof.log; exit 1; }
echo done

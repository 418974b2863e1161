#!/bin/bash
# Round 4, session P: wave-kernel staging (n = 500 unlimited depth + its parity test), block-target
# A/B at depths 3 and 4, and a fresh config-5 timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/p
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_skeleton.py -q -x -k "n500 or wave_kernel or skeleton_matches_oracle" --timeout 150 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u tools/profile_deep.py --n 500 --reps 5 > $O/deep500.log 2>&1 || exit $?
python -c "import json; d=[json.loads(l) for l in open('$O/deep500.log') if l.startswith('{')][-1]; print('n500', round(d['gpu_ms'],3), 'kernel', round(sum(d['kernel_ms']),3))"
for v in "PCG_NB4=16384" "PCG_NB4=8192" "PCG_NB4=12288" "PCG_NB4=24576" "PCG_NB3=2048" "PCG_NB3=6144" "PCG_NB3=8192" "PCG_NB2=2048" "PCG_NB2=8192"; do
  tag=$(echo $v | tr '=' '_')
  env $v timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-full-p > $O/b_$tag.log 2>&1 || { echo "bench $v failed"; tail -20 $O/b_$tag.log; exit 1; }
  echo "$v: $(python -c "import json; d=[json.loads(l) for l in open('$O/b_$tag.log') if l.startswith('{')][-1]; print(round(d['ms_per_step'],3), d['kernel_ms_per_level'], d['level_ms'])")"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-full-p > $O/tl.log 2>&1 || exit $?
python tools/timeline.py $O/tl/run_kernel_trace.csv > $O/timeline.txt 2>&1; tail -36 $O/timeline.txt

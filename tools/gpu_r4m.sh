#!/bin/bash
# Round 4, session M: K1 with the 4-wave CRT GEMM (k_xtx_crt4) — parity, A/B time, PMC.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4/m
mkdir -p $O
: > $O/status.log
step() {
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] start $name" >> $O/status.log
  timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/status.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name rc=$rc"; cat $O/status.log; tail -30 $O/$name.log; exit $rc; fi
}
step corr_tests 300 python -u -m pytest tests/test_gpu_skeleton.py -q -x -k "corr" --timeout 150 --timeout-method thread
tail -3 $O/corr_tests.log
grep -q " passed" $O/corr_tests.log && ! grep -q "failed" $O/corr_tests.log || { echo "corr tests failed"; tail -40 $O/corr_tests.log; exit 1; }
PCG_K1_CRT_W4=1 step k1_w4 120 python -u tools/micro/k1_time.py rcaeval_amd/libpcgpu.so
PCG_K1_CRT_W4=0 step k1_w8 120 python -u tools/micro/k1_time.py rcaeval_amd/libpcgpu.so
PCG_K1_CRT_W4=1 step k1_w4b 120 python -u tools/micro/k1_time.py rcaeval_amd/libpcgpu.so
cat $O/k1_w4.log $O/k1_w8.log $O/k1_w4b.log
step k1_trace 200 rocprofv3 --kernel-trace --stats -d $O/k1tr -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4/m/k1tr/run_kernel_stats.csv")))
for r in rows[:8]:
    print(r["Name"][:60], r["Calls"], r["AverageNs"], r["Percentage"])
PY
step k1_pmc 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_I8 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/k1pmc -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so
step k1_fetch 120 rocprofv3 --pmc FETCH_SIZE -d $O/k1fetch -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so
step k1_write 120 rocprofv3 --pmc WRITE_SIZE -d $O/k1write -o run --output-format csv -- python tools/micro/k1_time.py rcaeval_amd/libpcgpu.so
step bench 200 python -u bench.py --steps 20 --warmup 5
tail -1 $O/bench.log | cut -c1-300
cat $O/status.log

#!/bin/bash
# Round 3, session Z5: one PMC pass on K1 alone after the layout fix (MFMA busy, waits, LDS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/z5
mkdir -p $O
timeout -k 10 120 python tools/k1_run.py 2 > $O/run.log 2>&1 || { cat $O/run.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- python tools/k1_run.py 3 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p2 -o run --output-format csv -- python tools/k1_run.py 3 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
echo done

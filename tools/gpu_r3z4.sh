#!/bin/bash
# Round 3, session Z4: PMC passes on K1 alone (tools/k1_run.py): MFMA busy, LDS, wait cycles, then
# FETCH / WRITE. One counter set per pass, each its own hard timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r3/z4
mkdir -p $O
timeout -k 10 120 python tools/k1_run.py 2 > $O/run.log 2>&1 || { cat $O/run.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MFMA_I8 SQ_WAIT_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- python tools/k1_run.py 3 > $O/p1.log 2>&1 || { tail -5 $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/p2 -o run --output-format csv -- python tools/k1_run.py 3 > $O/p2.log 2>&1 || { tail -5 $O/p2.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/p3 -o run --output-format csv -- python tools/k1_run.py 3 > $O/p3.log 2>&1 || { tail -5 $O/p3.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE -d $O/p4 -o run --output-format csv -- python tools/k1_run.py 3 > $O/p4.log 2>&1 || { tail -5 $O/p4.log; exit 1; }
ls $O/p1 $O/p2 $O/p4

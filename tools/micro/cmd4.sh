cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/micro/valu_rates > gpurun_out/valu_rates.log 2>&1 && cat gpurun_out/valu_rates.log && \
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_avail.log 2>&1; \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU -d gpurun_out/pmc_sq3 -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_sq3.log 2>&1; echo pmc rc=$?

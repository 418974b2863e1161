# A/B of tools/ab variants (twice) + the per-block timing lines
set -u
bash tools/variant_bench.sh > gpurun_out/ab12.txt 2>&1; cat gpurun_out/ab12.txt
bash tools/variant_bench.sh > gpurun_out/ab12b.txt 2>&1; cat gpurun_out/ab12b.txt
grep -h "blkt d3" gpurun_out/var_libpcgpu_blkt3*.log | tail -4

timeout -k 10 120 tools/ubench/row_bench > gpurun_out/row_bench.txt 2>&1; cat gpurun_out/row_bench.txt | tail -12
bash tools/gpu_quick.sh

timeout -k 10 60 tools/ubench/row_bench > gpurun_out/row_bench.txt 2>&1 || exit 1
grep -E "fp_inv|row (inv|final|pow)" gpurun_out/row_bench.txt
bash tools/gpu_r5_iter.sh

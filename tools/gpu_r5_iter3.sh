# row_bench (ubench), then the tests + quick latency legs (tools/gpu_r5_iter.sh)
timeout -k 10 120 tools/ubench/row_bench > gpurun_out/row_bench.txt 2>&1 || exit 1
grep -E "^(row|[A-Z0-9_]+:)" gpurun_out/row_bench.txt
bash tools/gpu_r5_iter.sh

# Round-6 latency iteration + kernel trace in one call: tools/gpu_r6_lat.sh (tests, latency legs),
# then tools/gpu_r6_ktrace.sh (kernel medians of the latency legs).
set -o pipefail
bash tools/gpu_r6_lat.sh || exit 1
bash tools/gpu_r6_ktrace.sh > /dev/null || exit 1
grep -E "k_pk|k_sig_blind_row|k_g2_sum_g8|k_hash_map_row|k_hash_finish_row|k_decompress_sigs_row|k_sig_subgroup_row|k_miller_row|k_ml_S_row|k_root_check_row" gpurun_out/kt_${R:-r6}/kernels.txt

"""profiles/traffic.json from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py at one
batch in flight: per kernel, average (FETCH_SIZE + WRITE_SIZE) x 1024 bytes per launch, and per
pipeline stage (bench.py roofline), the bytes of all the stage's kernel launches per batch
(batches = launches of k_decompress_sigs, one per batch).

FETCH_SIZE / WRITE_SIZE are in KB (L2 <-> fabric).  Round 6: corrected as MI355X_MICROARCH.md's
HBM/rocprofv3 section prescribes for gfx950 -- FETCH_SIZE reports exactly half of the bytes of a
wide coalesced read, so fetched bytes = 2 x FETCH_SIZE; WRITE_SIZE as counted.  (Rounds 4-5 divided
by a calibration measured on k_msg_insert's 3.7 MB read, which is far below L3 and not credible:
VERDICT r5.)  Each kernel and stage carries `bytes_per_launch` = 2 FETCH + WRITE and the raw
counter values beside it.

  python tools/pmc_traffic.py FETCH.csv WRITE.csv SETS_PER_BATCH > profiles/traffic.json
"""
import collections
import csv
import json
import sys

# bench.py stage -> the kernels its stage_scope brackets (lb_engine.hip run_pipeline)
STAGES = {
    "decode_sigs": ["k_decompress_sigs", "k_sig_subgroup", "k_sig_subgroup_g8", "k_job_status"],
    "dedup": ["k_msg_insert", "k_msg_count", "k_msg_scatter"],
    "hash_map": ["k_hash_map", "k_hash_map_row"],
    "hash_finish": ["k_hash_finish", "k_hash_finish_g8", "k_hash_finish_row"],
    "pk_chunks": ["k_pk_chunks", "k_pk_chunks_idx"],
    "pk_blind": ["k_pk_blind"],
    "sig_msm": ["k_msm_count", "k_msm_scatter", "k_msm_chunks", "k_msm_buckets", "k_msm_reduce", "k_msm_buckets_g8",
                "k_msm_window_g8", "k_msm_horner_g8", "k_sig_blind", "k_sig_blind_g8", "k_g2_sum64"],
    "group_sum": ["k_chunk_fill", "k_gsum_chunks", "k_gsum_straus", "k_gsum_wave", "k_gsum_tree", "k_gsum_final"],
    "miller": ["k_miller_g8", "k_miller_lane", "k_miller_wave", "k_miller_row"],
    "tree_up_P": ["k_tree_up_U", "k_tree_up_row"],
    "ml_S": ["k_ml_S", "k_ml_S_row"],
    "root_check": ["k_root_check", "k_root_check_row"],
}


def per_kernel(path, counter):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
            d[name].append(float(r["Counter_Value"]))
    return d


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    n = int(sys.argv[3])
    inflight = sys.argv[4] if len(sys.argv) > 4 else "1"
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE (separate passes), bench.py --inflight {inflight}",
           "unit": "bytes per launch (kernels) / per batch (stages)", "kernels": {}, "stages": {}}
    out["correction"] = "bytes = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: gfx950 FETCH_SIZE counts half of a wide read)"
    for k in sorted(set(fetch) & set(write)):
        if not k.startswith("k_"):
            continue
        f, w = fetch[k], write[k]
        fb, wb = sum(f) / len(f) * 1024, sum(w) / len(w) * 1024
        out["kernels"][k] = {"launches": len(f), "fetch_size_bytes_raw": round(fb), "write_bytes": round(wb),
                             "bytes_per_launch": round(2 * fb + wb)}
    batches = len(fetch.get("k_decompress_sigs", [])) or 1
    for st, ks in STAGES.items():
        fb = sum(sum(fetch.get(k, [])) for k in ks) * 1024 / batches
        wb = sum(sum(write.get(k, [])) for k in ks) * 1024 / batches
        if fb + wb:
            out["stages"][st] = {"kernels": [k for k in ks if k in fetch], "bytes_per_launch": round(2 * fb + wb),
                                 "fetch_size_bytes_raw": round(fb), "write_bytes": round(wb),
                                 "sets_per_launch": n, "batches": batches}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()

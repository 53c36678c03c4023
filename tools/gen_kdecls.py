#!/usr/bin/env python3
"""Split build of liblodestar_bls.so: kernel declarations and group guards.

The device code of every kernel used to compile in one translation unit (lb_engine.hip, ~9 min
for gfx950).  The kernels are now assigned to groups (GROUPS below); lb_kgroup.hip is compiled
once per group with -DLB_KGROUP=g and defines only that group's kernels (`#if LB_KG(g)` guards in
the headers), and lb_engine.hip (-DLB_KGROUP=99) launches them through the declarations this
script writes to lb_kdecl.h.  A host launch of a kernel defined in another translation unit goes
through the kernel's handle symbol, which the defining unit registers: no -fgpu-rdc needed.

  python tools/gen_kdecls.py guard   # (one-time) wrap each kernel definition in its group guard
  python tools/gen_kdecls.py decl    # regenerate lb_kdecl.h (after a kernel signature changes)
  python tools/gen_kdecls.py check   # exit 1 if lb_kdecl.h is stale (CPU test)
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "lodestar_amd", "csrc")
FILES = ["lb_kernels.h", "lb_group_exec.h", "lb_kzg.h", "lb_ssz.h", "lb_latency.h"]
OUT = os.path.join(CSRC, "lb_kdecl.h")

# kernel -> translation-unit group (balanced by measured compile time; the one-lane per-root and
# decode kernels are the slow ones)
GROUPS = {
    0: ["k_decompress_sigs", "k_table_fill", "k_g1_decompress", "k_msg_insert", "k_dedup_one", "k_msg_uid_input",
        "k_msg_uid", "k_msg_count", "k_msg_scan", "k_chunk_fill", "k_msg_scatter", "k_job_status", "k_spec_live", "k_live_mismatch",
        "k_set_one", "k_g2_set_inf"],
    1: ["k_sig_subgroup", "k_sig_subgroup_g8", "k_sig_agg_chunks", "k_sig_agg_groups"],
    2: ["k_hash_map", "k_sk_to_pk", "k_sign", "k_ssz_zero_hashes", "k_merkleize"],
    3: ["k_hash_finish"],
    4: ["k_miller_lane", "k_pk_chunks", "k_pk_chunks_idx", "k_pk_blind", "k_gsum_chunks", "k_gsum_tree", "k_gsum_final"],
    14: ["k_chunk_order", "k_gsum_straus", "k_gsum_wave", "k_pk_out96"],
    5: ["k_miller_wave", "k_tree_up_U", "k_ml_S", "k_root_check", "k_root_partial", "k_partials_check", "k_search_ml",
        "k_search_fe", "k_search_match", "k_miller_g8", "k_kzg_check"],
    6: ["k_msm_count", "k_msm_scatter", "k_msm_chunks", "k_msm_buckets", "k_msm_reduce"],
    7: ["k_smsm_count", "k_smsm_scatter", "k_smsm_terms_g8", "k_smsm_terms_lane", "k_seg_sum64", "k_seg_final",
        "k_rsm_terms", "k_smsm_terms_pre", "k_range_pk", "k_test_pk", "k_g1_terms", "k_g1_sum64", "k_g1_out48",
        "k_kzg_setup_g1", "k_kzg_setup_g2"],
    8: ["k_hash_finish_g8"],
    9: ["k_msm_buckets_g8", "k_msm_window_g8", "k_msm_horner_g8", "k_sig_blind_g8", "k_sig_blind", "k_g2_sum64", "k_sig_unblinded", "k_g2_sum_g8"],
    10: ["k_miller_row", "k_tree_up_row"],
    11: ["k_ml_S_row", "k_root_check_row", "k_root_partial_row", "k_partials_check_row"],
    12: ["k_hash_finish_row", "k_sig_blind_row", "k_sig_subgroup_row"],
    13: ["k_hash_map_row", "k_decompress_sigs_row", "k_pk_blind_rowp", "k_sig_subgroup_w4", "k_sig_blind_w4"],
}
N_GROUPS = len(GROUPS)
GROUP_OF = {k: g for g, ks in GROUPS.items() for k in ks}
# explicit instantiations of the template kernels that lb_engine.hip / lb_kzg.h launch
INSTANCES = {
    "k_miller_lane": ["2", "3"],
    "k_msm_reduce": ["LB_MSM_W", "LB_SMSM_W"],
    "k_msm_horner_g8": ["LB_MSM_W", "LB_SMSM_W"],
    "k_smsm_count": ["LB_MSM_W", "LB_SMSM_W"],
    "k_smsm_scatter": ["LB_MSM_W", "LB_SMSM_W"],
}

KRE = re.compile(r"__global__\s+void\s+(?:__launch_bounds__\s*\([^)]*\)\s*)?(k_[A-Za-z0-9_]+)\s*\(")


def _strip_comments(s):
    return re.sub(r"//[^\n]*", "", s)


def kernels(path):
    """(name, template_line or None, start line index, end line index, signature text) per kernel"""
    lines = open(path).read().split("\n")
    out = []
    i = 0
    while i < len(lines):
        if "__global__" in lines[i] and not lines[i].lstrip().startswith("//") and "#define" not in lines[i]:
            j = i
            text = lines[i]
            while not KRE.search(_strip_comments(text)):
                j += 1
                text += "\n" + lines[j]
            m = KRE.search(_strip_comments(text))
            name = m.group(1)
            start = i
            tmpl = None
            if i > 0 and lines[i - 1].lstrip().startswith("template"):
                start = i - 1
                tmpl = lines[i - 1].strip()
            # signature: up to the parenthesis closing the parameter list
            k = j
            body = "\n".join(lines[i:])
            body_nc = _strip_comments(body)
            p0 = body_nc.index(name) + len(name)
            depth = 0
            q = p0
            while True:
                c = body_nc[q]
                if c == "(":
                    depth += 1
                elif c == ")":
                    depth -= 1
                    if depth == 0:
                        break
                q += 1
            params = body_nc[p0:q + 1]
            # body braces
            b0 = body_nc.index("{", q)
            depth = 0
            r = b0
            while True:
                c = body_nc[r]
                if c == "{":
                    depth += 1
                elif c == "}":
                    depth -= 1
                    if depth == 0:
                        break
                r += 1
            end = i + body_nc[:r].count("\n")
            out.append((name, tmpl, start, end, " ".join(params.split())))
            i = end + 1
            continue
        i += 1
    return out


def guard():
    for f in FILES:
        path = os.path.join(CSRC, f)
        if not os.path.exists(path):
            continue
        lines = open(path).read().split("\n")
        ks = kernels(path)
        for name, tmpl, start, end, _ in reversed(ks):
            if start > 0 and lines[start - 1].startswith("#if LB_KG("):
                continue
            if name not in GROUP_OF:
                sys.exit(f"{f}: kernel {name} has no group in tools/gen_kdecls.py GROUPS")
            lines.insert(end + 1, "#endif  // LB_KG")
            lines.insert(start, f"#if LB_KG({GROUP_OF[name]})")
        open(path, "w").write("\n".join(lines))


def render():
    decl, inst = [], {g: [] for g in GROUPS}
    seen = set()
    for f in FILES:
        path = os.path.join(CSRC, f)
        if not os.path.exists(path):
            continue
        for name, tmpl, _, _, params in kernels(path):
            if name in seen:
                continue
            seen.add(name)
            if name not in GROUP_OF:
                sys.exit(f"{f}: kernel {name} has no group in tools/gen_kdecls.py GROUPS")
            if tmpl:
                decl.append(f"{tmpl} __global__ void {name}{params};")
                for a in INSTANCES.get(name, []):
                    inst[GROUP_OF[name]].append(f"template __global__ void {name}<{a}>{params};")
            else:
                decl.append(f"__global__ void {name}{params};")
    missing = sorted(set(GROUP_OF) - seen)
    if missing:
        sys.exit(f"GROUPS names kernels that do not exist: {missing}")
    txt = ["// GENERATED by tools/gen_kdecls.py decl -- do not edit.",
           "// Declarations of every kernel for lb_engine.hip (compiled with LB_KGROUP=99: no kernel",
           "// definitions) and the explicit instantiations of the template kernels for the group that",
           "// defines them (lb_kgroup.hip with LB_KDECL_INSTANTIATE).",
           "#pragma once", ""]
    txt += decl
    txt += ["", "#ifdef LB_KDECL_INSTANTIATE"]
    for g in GROUPS:
        if inst[g]:
            txt.append(f"#if LB_KG({g})")
            txt += inst[g]
            txt.append("#endif")
    txt += ["#endif", f"#define LB_N_KGROUPS {N_GROUPS}", ""]
    return "\n".join(txt)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "decl"
    if mode == "guard":
        guard()
        open(OUT, "w").write(render())
    elif mode == "decl":
        open(OUT, "w").write(render())
    elif mode == "check":
        cur = open(OUT).read() if os.path.exists(OUT) else ""
        if cur != render():
            print("lb_kdecl.h is stale: run python tools/gen_kdecls.py decl")
            sys.exit(1)
    else:
        sys.exit(__doc__)


if __name__ == "__main__":
    main()

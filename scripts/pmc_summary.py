"""Summarise rocprofv3 output into profiles/:

  python scripts/pmc_summary.py gpurun_out/prof rNN [SUFFIX]

SUFFIX ("_l2" for the C2 rounds at ell = 2, bench.py --ell 2) is appended to
every record key, so the headline's and the secondary line's records sit side
by side; every record carries the tag of the pass it came from ("source").

* kernel_stats (from --kernel-trace --stats) -> profiles/<tag>_kernel_stats.csv
* FETCH_SIZE / WRITE_SIZE passes (separate --pmc runs) -> per-kernel mean per
  launch, converted to bytes (x1024) with the gfx950 correction of
  MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half the bytes of a wide
  coalesced read, so read bytes = 2 x FETCH_SIZE x 1024 (raw values are kept
  alongside).  Written to profiles/pmc_summary.json keyed by stage name.
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

STAGES = {  # stage key -> kernel-name prefixes (the first match wins)
    "var": ("void ut::k_gp_var_pp<false>(", "ut::k_gp_var_pp(", "void ut::k_gp_var<double>"), "var_1wg": ("void ut::k_gp_var<double>",),
    "kstar": ("void ut::k_gp_kstar<double, false, false>", "void ut::k_gp_kstar<double, false>"),
    "var32": ("ut::k_gp_var_f32(", "void ut::k_gp_var<float>",), "kstar32": ("void ut::k_gp_kstar<float, true, false>", "void ut::k_gp_kstar<float, true>"),
    "hash": ("void ut::k_hash<true", "void ut::k_hash<", "ut::k_hash("),
    "propose": ("void ut::k_de<", "ut::k_de("), "encode": ("ut::k_encode_scaled", "ut::k_encode("), "prep_cand": ("ut::k_gp_prep_cand",),
    "finalize": ("ut::k_gp_finalize",),
    "dedup_insert": ("ut::k_batch_insert",), "dedup_mark": ("ut::k_dedup_mark",),
    "topk0": ("void ut::k_topk_chunk<0>",), "topk1": ("void ut::k_topk_chunk<1>",), "pso": ("ut::k_pso(",),
    "ga": ("ut::k_ga(",),
    # rocprofv3 leaves the _Float16 instantiations mangled
    "var16": ("_ZN2ut11k_gp_var_h3",), "kstar16": ("_ZN2ut10k_gp_kstarIDF16_",),
    # precision 8 (int8 slices)
    "var8": ("ut::k_gp_var_i8(",), "kstar8": ("void ut::k_gp_kstar_q<signed char, false", "void ut::k_gp_kstar<signed char, false, false>",
                     "void ut::k_gp_kstar<signed char, true, false>"), "split_u8": ("ut::k_q_split_u(",),
    "split8": ("ut::k_split_i8(",), "finalize8": ("ut::k_gp_finalize_i8(",),
    "inner_pairs": ("ut::k_inner_pairs",), "de_diff": ("ut::k_de_diff",), "pop_digests": ("ut::k_pop_digests",),
}
# stages of the default C2 round that a refreshed C2 profile replaces (a key
# absent from the new profile -- e.g. de_diff, now folded into k_de -- is dropped)
C2_ROUND = ("var", "var_1wg", "kstar", "hash", "propose", "encode", "prep_cand", "finalize", "dedup_insert",
            "dedup_mark", "topk0", "topk1", "inner_pairs", "de_diff", "pop_digests", "var8", "kstar8", "split8", "finalize8",
            "split_u8")



def per_kernel(path, counter):
    acc = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter:
                acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main(prof, tag, suffix=""):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out_dir = os.path.join(root, "profiles")
    os.makedirs(out_dir, exist_ok=True)
    shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"), os.path.join(out_dir, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(prof, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(prof, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    stats = {}
    with open(os.path.join(prof, "trace", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            stats[row["Name"]] = row
    summary = {"_note": "bytes per launch; read = 2 x FETCH_SIZE x 1024 (gfx950 correction, MI355X_MICROARCH.md "
                        "§HBM), write = WRITE_SIZE x 1024; raw counters kept. source: " + tag}
    for key, prefixes in STAGES.items():
        def first(names):
            for pre in prefixes:
                hit = [k for k in names if k.startswith(pre)]
                if hit:
                    return hit
            return []
        kf, kw, ks = first(fetch), first(write), first(stats)
        if not (kf and kw):
            continue
        fr, wr = fetch[kf[0]], write[kw[0]]
        summary[key + suffix] = {
            "kernel": kf[0][:120], "source": tag,
            "fetch_size_kb_raw": fr, "write_size_kb_raw": wr,
            "read_bytes_per_launch": 2.0 * fr * 1024.0, "write_bytes_per_launch": wr * 1024.0,
            "hbm_bytes_per_launch": 2.0 * fr * 1024.0 + wr * 1024.0,
            "avg_ns": float(stats[ks[0]]["AverageNs"]) if ks else None,
        }
    # merge: a profile of another precision / config adds its stages beside the default C2 ones
    merged = {}
    try:
        with open(os.path.join(out_dir, "pmc_summary.json")) as f:
            merged = json.load(f)
    except Exception:
        pass
    if "var" + suffix in summary or "var8" + suffix in summary:
        for k in C2_ROUND:
            merged.pop(k + suffix, None)
    merged.update({k: v for k, v in summary.items() if k != "_note"})
    merged["_note"] = ("bytes per launch; read = 2 x FETCH_SIZE x 1024 (gfx950 correction, MI355X_MICROARCH.md "
                       "§HBM), write = WRITE_SIZE x 1024; raw counters kept. Each record's 'source' names its pass; "
                       "keys ending _l2 are the C2 rounds at ell = 2")
    with open(os.path.join(out_dir, "pmc_summary.json"), "w") as f:
        json.dump(merged, f, indent=1)
    with open(os.path.join(out_dir, f"{tag}_pmc_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")

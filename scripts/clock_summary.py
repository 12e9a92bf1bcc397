"""Effective clock and MFMA busy fraction per kernel from scripts/pmc_clock.sh
(MI355X_MICROARCH.md 'DVFS give-back': clock = GRBM_GUI_ACTIVE / 8 / duration;
SQ_VALU_MFMA_BUSY_CYCLES counts cycles of busy MFMA pipes summed over SIMDs).
rocprofv3 serializes the dispatches of a --pmc pass, so every duration here is
the kernel alone on the chip.

    python scripts/clock_summary.py gpurun_out/clk                 # print
    python scripts/clock_summary.py gpurun_out/clk rNN [SUFFIX]    # + merge into profiles/

With a tag the records (keys + SUFFIX, "_l2" for the C2 rounds at ell = 2)
carry "source": tag and are merged into profiles/clock_summary.json; the pass
is also kept as profiles/<tag>_clock_summary.json.
"""
import csv
import json
import os
import sys
from collections import defaultdict

KERNELS = {"var": ("void ut::k_gp_var_pp<false>(", "ut::k_gp_var_pp(", "void ut::k_gp_var<double>"),
           "var8": ("ut::k_gp_var_i8(",), "kstar8": ("void ut::k_gp_kstar_q<signed char, false", "void ut::k_gp_kstar<signed char, false, false>",
                     "void ut::k_gp_kstar<signed char, true, false>"), "split_u8": ("ut::k_q_split_u(",),
           "kstar": ("void ut::k_gp_kstar<double, false, false>", "void ut::k_gp_kstar<double, false>"), "inner_pairs": ("ut::k_inner_pairs",),
           "encode": ("ut::k_encode_scaled",),
           "hash": ("void ut::k_hash<true", "void ut::k_hash<", "ut::k_hash("), "propose": ("void ut::k_de<", "ut::k_de("),
           "var16": ("_ZN2ut11k_gp_var_h3",), "kstar16": ("_ZN2ut10k_gp_kstarIDF16_",),
           "kstar_f32c": ("void ut::k_gp_kstar_f32c<",), "kstar_bound64": ("void ut::k_gp_kstar<double, true, true>",)}


def summarize(d, n_cu=256, peak_ghz=2.4, tag=None, suffix=""):
    rows = defaultdict(dict)
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[int(r["Dispatch_Id"])]["_name"] = r["Kernel_Name"]
            rows[int(r["Dispatch_Id"])]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {}
    for key, prefixes in KERNELS.items():
        ds = []
        for pre in prefixes:   # the first prefix with dispatches wins
            ds = [v for v in rows.values() if v["_name"].startswith(pre)]
            if ds:
                break
        if not ds:
            continue
        clk = [v["GRBM_GUI_ACTIVE"] / 8 / v["_ns"] for v in ds]           # cycles per ns = GHz
        busy = [v["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * n_cu * v["GRBM_GUI_ACTIVE"] / 8) for v in ds]
        out[key + suffix] = {"dispatches": len(ds), "duration_ms": sum(v["_ns"] for v in ds) / len(ds) / 1e6,
                             "clock_ghz": sum(clk) / len(clk), "mfma_busy": sum(busy) / len(busy),
                             "clock_adjusted_peak_fraction_scale": peak_ghz / (sum(clk) / len(clk))}
        if tag:
            out[key + suffix]["source"] = tag
    return out


NOTE = ("clock_ghz = GRBM_GUI_ACTIVE / 8 / duration; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x CUs x "
        "clock cycles of the kernel); dispatches serialized by the --pmc pass (each kernel alone on the chip); "
        "profiled passes run ~2-5% slower (MI355X_MICROARCH.md DVFS item 2); 'source' names the pass, keys ending "
        "_l2 are the C2 rounds at ell = 2")


def main(argv):
    d = argv[0]
    tag = argv[1] if len(argv) > 1 else None
    suffix = argv[2] if len(argv) > 2 else ""
    out = summarize(d, tag=tag, suffix=suffix)
    if tag:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        path = os.path.join(root, "profiles", "clock_summary.json")
        try:
            with open(path) as f:
                merged = json.load(f)
        except Exception:
            merged = {}
        merged.update(out)
        merged["_note"] = NOTE
        with open(path, "w") as f:
            json.dump(merged, f, indent=1)
        with open(os.path.join(root, "profiles", f"{tag}_clock_summary.json"), "w") as f:
            json.dump(dict(out, _note=NOTE), f, indent=1)
    print(json.dumps(dict(out, _note=NOTE), indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])

"""Per-kernel-name averages of a rocprofv3 --pmc counter CSV: duration, clock
(GRBM_GUI_ACTIVE / 8 / ns) and MFMA busy (SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x CUs x cycles)).
    python scripts/exp/pmc_by_kernel.py DIR [n_cu]"""
import csv
import glob
import sys
from collections import defaultdict

d = sys.argv[1]
n_cu = int(sys.argv[2]) if len(sys.argv) > 2 else 256
rows = defaultdict(dict)
for fn in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    with open(fn) as f:
        for r in csv.DictReader(f):
            x = rows[(fn, int(r["Dispatch_Id"]))]
            x[r["Counter_Name"]] = float(r["Counter_Value"])
            x["_name"] = r["Kernel_Name"]
            x["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
by = defaultdict(list)
for v in rows.values():
    by[v["_name"]].append(v)
for name, ds in by.items():
    ns = sum(v["_ns"] for v in ds) / len(ds)
    line = f"{name[:90]:90s} n={len(ds):3d} {ns / 1e6:9.3f} ms"
    if "GRBM_GUI_ACTIVE" in ds[0]:
        clk = sum(v["GRBM_GUI_ACTIVE"] / 8 / v["_ns"] for v in ds) / len(ds)
        line += f"  clk {clk:.3f} GHz"
        if "SQ_VALU_MFMA_BUSY_CYCLES" in ds[0]:
            busy = sum(v["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * n_cu * v["GRBM_GUI_ACTIVE"] / 8) for v in ds) / len(ds)
            line += f"  mfma_busy {busy:.3f}"
    for k in sorted(ds[0]):
        if not k.startswith("_") and k not in ("GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES"):
            line += f"  {k} {sum(v[k] for v in ds) / len(ds):.4g}"
    print(line)

"""per-kernel (template args) FETCH bytes and clock / MFMA busy from
var8_probe.sh's two counter passes: python scripts/exp/pmc_probe_summary.py gpurun_out/TAG"""
import csv
import sys
from collections import defaultdict


def rows(path):
    d = defaultdict(dict)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = int(r["Dispatch_Id"])
            d[k][r["Counter_Name"]] = float(r["Counter_Value"])
            d[k]["_name"] = r["Kernel_Name"]
            d[k]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return d


o = sys.argv[1]
fe, ck = rows(f"{o}/fetch/run_counter_collection.csv"), rows(f"{o}/clk/run_counter_collection.csv")
agg = defaultdict(lambda: defaultdict(list))
for v in fe.values():
    agg[v["_name"][:60]]["fetch_GB"].append(2 * v["FETCH_SIZE"] * 1024 / 1e9)
for v in ck.values():
    a = agg[v["_name"][:60]]
    a["ms"].append(v["_ns"] / 1e6)
    a["ghz"].append(v["GRBM_GUI_ACTIVE"] / 8 / v["_ns"])
    a["busy"].append(v["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * 256 * v["GRBM_GUI_ACTIVE"] / 8))
for k, a in agg.items():
    print(k, " ".join("%s=%.3f" % (n, sorted(x)[len(x) // 2]) for n, x in a.items()))

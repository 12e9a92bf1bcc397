"""Per-kernel wave-cycle breakdown from scripts/pmc_stall.sh (fractions of
SQ_WAVE_CYCLES; LDS bank conflicts per LDS-active cycle).

    python scripts/stall_summary.py gpurun_out/stall > profiles/r05_stall_summary.json
"""
import csv
import json
import sys
from collections import defaultdict

from clock_summary import KERNELS


def main(d):
    rows = defaultdict(dict)
    with open(f"{d}/run_counter_collection.csv") as f:
        for r in csv.DictReader(f):
            k = int(r["Dispatch_Id"])
            rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
            rows[k]["_name"] = r["Kernel_Name"]
            rows[k]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = {"_note": "fractions of SQ_WAVE_CYCLES (quad-cycles): wait_any = parked on s_waitcnt / barrier, "
                    "wait_inst = issue stall (wait_inst_lds its LDS part), active = issuing; "
                    "lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE"}
    for key, prefixes in KERNELS.items():
        ds = []
        for pre in prefixes:
            ds = [v for v in rows.values() if v["_name"].startswith(pre)]
            if ds:
                break
        if not ds:
            continue
        tot = lambda c: sum(v.get(c, 0.0) for v in ds)
        wc = tot("SQ_WAVE_CYCLES") or 1.0
        out[key] = {"dispatches": len(ds), "duration_ms": tot("_ns") / len(ds) / 1e6,
                    "wait_any": tot("SQ_WAIT_ANY") / wc, "wait_inst": tot("SQ_WAIT_INST_ANY") / wc,
                    "wait_inst_lds": tot("SQ_WAIT_INST_LDS") / wc, "active": tot("SQ_ACTIVE_INST_ANY") / wc,
                    "lds_conflict": tot("SQ_LDS_BANK_CONFLICT") / (tot("SQ_LDS_IDX_ACTIVE") or 1.0)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    sys.path.insert(0, __file__.rsplit("/", 1)[0])
    main(sys.argv[1])

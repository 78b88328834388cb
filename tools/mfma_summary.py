"""Summarise a rocprofv3 PMC pass (SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CU_CYCLES, GRBM_GUI_ACTIVE) per kernel
and grid size: MFMA utilisation = MFMA-busy SIMD cycles / (active cycles x 4 SIMDs x CUs), where the active
cycles per XCD are GRBM_GUI_ACTIVE / 8 (rocprofv3 sums it over the 8 XCDs; MI355X_MICROARCH.md, DVFS note).
usage: python tools/mfma_summary.py <run_counter_collection.csv> <out.json> [--cus 256] [--by-grid]
--by-grid: aggregate every dispatch of one (kernel, grid) (graph replays interleave many launches)."""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import code_hash  # noqa: E402


def main():
    src, out = sys.argv[1], sys.argv[2]
    cus = int(sys.argv[sys.argv.index("--cus") + 1]) if "--cus" in sys.argv else 256
    disp = collections.OrderedDict()
    for x in csv.DictReader(open(src)):
        k = (int(x["Dispatch_Id"]), x["Kernel_Name"], int(x["Grid_Size"]))
        d = disp.setdefault(k, {"ns": int(x["End_Timestamp"]) - int(x["Start_Timestamp"])})
        d[x["Counter_Name"]] = d.get(x["Counter_Name"], 0.0) + float(x["Counter_Value"])
    # consecutive MFMA dispatches of one (kernel, grid) form a group: one probe case (warm-up + replays)
    groups = []
    by_grid = "--by-grid" in sys.argv
    index = {}
    for (did, name, grid), d in disp.items():
        if by_grid:
            if (name, grid) not in index:
                index[(name, grid)] = len(groups)
                groups.append([(name, grid), []])
            groups[index[(name, grid)]][1].append(d)
            continue
        if d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) <= 0:
            continue
        if groups and groups[-1][0] == (name, grid):
            groups[-1][1].append(d)
        else:
            groups.append([(name, grid), [d]])
    rows = []
    for (name, grid), ds in groups:
        cyc = sum(d["GRBM_GUI_ACTIVE"] for d in ds) / 8.0
        busy = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in ds)
        cu = sum(d.get("SQ_BUSY_CU_CYCLES", 0.0) for d in ds)
        ns = sum(d["ns"] for d in ds)
        rows.append({"kernel": name[:120], "grid_threads": grid, "dispatches": len(ds),
                     "avg_us": round(ns / len(ds) / 1e3, 2), "clock_ghz": round(cyc / ns, 3),
                     "mfma_util": round(busy / (cyc * 4 * cus), 4), "cu_busy": round(cu / (cyc * cus), 4)})
    json.dump({"source": src, "definition": "mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 4 * CUs)",
               "code_hash": code_hash(), "rows": rows}, open(out, "w"), indent=1)
    if by_grid:
        rows.sort(key=lambda r: -r["avg_us"] * r["dispatches"])
    for r in rows:
        print(json.dumps(r))


if __name__ == "__main__":
    main()

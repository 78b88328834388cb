"""Summarise rocprofv3 outputs into profiles/: kernel stats + per-launch HBM traffic of a kernel.

usage: python tools/pmc_summary.py <trace_dir> <pmc_fetch_dir> <pmc_write_dir> <out_prefix>

FETCH_SIZE / WRITE_SIZE are rocprofv3's derived counters in KiB per dispatch (TCC_EA0 read/write
requests x 64 B).  Per MI355X_MICROARCH.md §HBM: FETCH_SIZE reads HALF the bytes of a wide
(16 B/lane) coalesced stream on gfx950 and is uncalibrated for other widths; we report the raw value
and the x2-corrected one (upper estimate) separately.  WRITE_SIZE is exact for 16 B/lane stores.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import code_hash  # noqa: E402


def per_kernel(counter_dir, counter):
    f = glob.glob(os.path.join(counter_dir, "*counter_collection.csv"))[0]
    acc = defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == counter:
            acc[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    trace, fdir, wdir, prefix = sys.argv[1:5]
    stats = list(csv.DictReader(open(glob.glob(os.path.join(trace, "*kernel_stats.csv"))[0])))
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    out = {"code_hash": code_hash(), "kernels": []}
    for r in stats:
        name = r["Name"]
        e = {"name": name, "calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
             "total_ms": float(r["TotalDurationNs"]) / 1e6, "percent": float(r["Percentage"])}
        if name in fetch:
            e["fetch_kib_per_launch_raw"] = fetch[name]
            e["hbm_read_bytes_per_launch_x2corrected"] = fetch[name] * 1024 * 2
        if name in write:
            e["hbm_write_bytes_per_launch"] = write[name] * 1024
        out["kernels"].append(e)
    json.dump(out, open(prefix + "_summary.json", "w"), indent=1)
    with open(prefix + "_kernel_stats.csv", "w") as fo:
        fo.write(open(glob.glob(os.path.join(trace, "*kernel_stats.csv"))[0]).read())
    for e in out["kernels"][:12]:
        print(f"{e['percent']:6.2f}% {e['avg_us']:9.2f} us x{e['calls']:4d}  {e['name'][:60]}  "
              f"R={e.get('hbm_read_bytes_per_launch_x2corrected', 0) / 1e6:.2f}MB W={e.get('hbm_write_bytes_per_launch', 0) / 1e6:.2f}MB")


if __name__ == "__main__":
    main()

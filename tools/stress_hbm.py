"""HBM traffic of the M=4096 stress factorization (BASELINE.json configs[4]) from two rocprofv3 PMC passes of
tools/potrf_timeline.py (FETCH_SIZE, WRITE_SIZE; separate runs, no tracing domains: tools/stress_hbm.sh).
Per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads half the bytes of a 16 B/lane stream on gfx950, so the read
figure is reported raw and x2-corrected (upper estimate); WRITE_SIZE is exact for 16 B/lane stores.
A factorization = the dispatches between two zero_upper_kernel launches (its last kernel); the copy that
restores A before each replay and the setup kernels are excluded.
usage: python tools/stress_hbm.py <fetch_counter_collection.csv> <write_counter_collection.csv> <out.json>"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import code_hash  # noqa: E402

FACT = ("potrf_", "chol_inv", "gemm_big_kernel", "zero_upper")


def per_fact(path, counter):
    disp = collections.OrderedDict()
    for x in csv.DictReader(open(path)):
        if x["Counter_Name"] != counter:
            continue
        k = int(x["Dispatch_Id"])
        d = disp.setdefault(k, {"name": x["Kernel_Name"], "v": 0.0})
        d["v"] += float(x["Counter_Value"])
    seq = [disp[k] for k in sorted(disp)]
    ends = [i for i, d in enumerate(seq) if "zero_upper" in d["name"]]
    facts = []
    for a, b in zip(ends[:-1], ends[1:]):             # complete factorizations only
        by = collections.defaultdict(float)
        for d in seq[a + 1:b + 1]:
            if any(t in d["name"] for t in FACT):
                nm = d["name"].split("(")[0].replace("void ", "").replace("nmgp::", "")
                by[nm] += d["v"] * 1024.0
        facts.append(by)
    return facts


def main():
    fetch = per_fact(sys.argv[1], "FETCH_SIZE")
    write = per_fact(sys.argv[2], "WRITE_SIZE")
    f, w = fetch[-1], write[-1]
    rd, wr = sum(f.values()), sum(w.values())
    out = {"code_hash": code_hash(), "factorizations_seen": [len(fetch), len(write)],
           "read_bytes_raw": int(rd), "read_bytes_x2corrected": int(2 * rd), "write_bytes": int(wr),
           "traffic_bytes": int(2 * rd + wr),
           "by_kernel": {k: {"read_x2": int(2 * f.get(k, 0)), "write": int(w.get(k, 0))}
                         for k in sorted(set(f) | set(w), key=lambda k: -(2 * f.get(k, 0) + w.get(k, 0)))},
           "definition": "one factorization (the last complete one); FETCH_SIZE x2 + WRITE_SIZE, KiB -> bytes"}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("factorizations_seen", "read_bytes_x2corrected", "write_bytes")}))


if __name__ == "__main__":
    main()

"""HBM traffic per graphed training step from rocprofv3 FETCH_SIZE / WRITE_SIZE passes of tools/train_leg.py
(tools/train_pmc.sh): every kernel's counter values inside the timed steps' window (start of the first timed
step's step_begin launch .. end of the last Adam step-counter increment, as tools/train_summary.py windows the
kernel trace), summed and divided by the step count, per kernel and per kernel family.  FETCH_SIZE (KiB) is
reported raw and x2-corrected (MI355X_MICROARCH.md, HBM section: it counts half the bytes of a 16-byte/lane
stream on gfx950); WRITE_SIZE (KiB) as is.
usage: python tools/train_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> <train_leg.json>
       <out.json>"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import code_hash  # noqa: E402
from train_summary import short  # noqa: E402

FAMILIES = ("gemm_big_kernel", "gemm_kernel<float", "pair_", "adam_tri_kernel", "block_copy_v_kernel")


def window_sum(path, counter, steps, durations=None):
    """Counter bytes per step per kernel; `durations` (a dict) also gets each kernel's summed dispatch time per step
    in ms -- dispatches are serialised by counter collection, so these are the kernels' own durations."""
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    begin = [x for x in rows if "step_begin_kernel" in x["Kernel_Name"]]
    # (the step's last update launch: the folded captured step has no counter launch)
    ctr = [x for x in rows if "counter_add_kernel" in x["Kernel_Name"] or "adam" in x["Kernel_Name"]]
    t0, t1 = int(begin[-steps]["Start_Timestamp"]), int(ctr[-1]["End_Timestamp"])
    acc = collections.defaultdict(float)
    for x in rows:
        if int(x["Start_Timestamp"]) >= t0 and int(x["End_Timestamp"]) <= t1:
            acc[short(x["Kernel_Name"])] += float(x["Counter_Value"]) * 1024.0
            if durations is not None:
                k = short(x["Kernel_Name"])
                durations[k] = durations.get(k, 0.0) + (int(x["End_Timestamp"]) - int(x["Start_Timestamp"])) / 1e6
    if durations is not None:
        for k in durations:
            durations[k] /= steps
    return {k: v / steps for k, v in acc.items()}


def main():
    fpath, wpath, legp, outp = sys.argv[1:5]
    leg = json.loads(open(legp).read().strip().splitlines()[-1])
    steps = int(leg["steps"])
    dur = {}
    rd = window_sum(fpath, "FETCH_SIZE", steps, dur)
    wr = window_sum(wpath, "WRITE_SIZE", steps)
    kernels = []
    for k in sorted(set(rd) | set(wr), key=lambda k: -(2 * rd.get(k, 0.0) + wr.get(k, 0.0))):
        kernels.append({"kernel": k, "read_bytes_per_step_raw": round(rd.get(k, 0.0)),
                        "read_bytes_per_step_x2corrected": round(2 * rd.get(k, 0.0)),
                        "write_bytes_per_step": round(wr.get(k, 0.0)),
                        "serialised_ms_per_step": round(dur.get(k, 0.0), 4)})
    fam = {}
    for f in FAMILIES:
        ks = [e for e in kernels if e["kernel"].startswith(f)]
        fam[f] = {"kernels": len(ks),
                  "read_bytes_per_step_x2corrected": sum(e["read_bytes_per_step_x2corrected"] for e in ks),
                  "write_bytes_per_step": sum(e["write_bytes_per_step"] for e in ks)}
        fam[f]["traffic_bytes_per_step"] = fam[f]["read_bytes_per_step_x2corrected"] + fam[f]["write_bytes_per_step"]
        # the family's own kernel time per step (the FETCH pass: counter collection serialises the dispatches)
        fam[f]["serialised_ms_per_step"] = round(sum(e["serialised_ms_per_step"] for e in ks), 4)
    out = {"code_hash": code_hash(), "source": [fpath, wpath], "config": leg["workload"], "steps": steps,
           "unit": "bytes per step (FETCH_SIZE x2 + WRITE_SIZE, rocprofv3 PMC passes, dispatches serialised)",
           "families": fam, "kernels": kernels}
    json.dump(out, open(outp, "w"), indent=1)
    print(json.dumps({"config": leg["workload"][:40], "families": {k: v["traffic_bytes_per_step"] for k, v in fam.items()}}))


if __name__ == "__main__":
    main()

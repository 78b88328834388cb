"""Per-kernel breakdown of graph-replayed training steps from a rocprofv3 kernel-trace CSV (tools/train_trace.sh).
The timed steps are the last `steps` graphed steps of the trace (bench.graph_train's JSON says how many): each
kernel's busy time inside [start of the first timed step's step_begin launch, end of the last step's Adam counter
increment] is summed and divided by the step count (kernels on concurrent streams overlap, so the busy times can add up to more than the wall).
usage: python tools/train_summary.py <run_kernel_trace.csv> <train_leg.json> <out.json>"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from provenance import code_hash  # noqa: E402


def short(name):
    nm = name.replace("void ", "").replace("nmgp::", "").replace("(anonymous namespace)::", "")
    return nm.split("(")[0][:90]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    leg = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
    steps = int(leg["steps"])
    rows.sort(key=lambda x: int(x["Start_Timestamp"]))
    # step window: from the start of the step_begin launch (minibatch gather + noise: once per graphed step) of the
    # first timed step to the end of the last Adam step-counter increment (the step's last launch; the Adam itself
    # is one or several launches, nmgp_adam / nmgp_adam_lower)
    begin = [x for x in rows if "step_begin_kernel" in x["Kernel_Name"]]
    # (round 6: the captured step's counter is advanced by the finalize kernel -- the update is then the last launch)
    ctr = [x for x in rows if "counter_add_kernel" in x["Kernel_Name"] or "adam" in x["Kernel_Name"]]
    t0, t1 = int(begin[-steps]["Start_Timestamp"]), int(ctr[-1]["End_Timestamp"])
    busy = collections.defaultdict(float)
    calls = collections.Counter()
    for x in rows:
        s, e = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        if s >= t0 and e <= t1:
            k = short(x["Kernel_Name"])
            busy[k] += (e - s) / 1e6
            calls[k] += 1
    wall = (t1 - t0) / 1e6 / steps
    tot = sum(busy.values()) / steps
    top = sorted(busy.items(), key=lambda kv: -kv[1])
    out = {"code_hash": code_hash(), "source": sys.argv[1], "config": leg["workload"], "steps": steps,
           "wall_ms_per_step_under_trace": round(wall, 4), "bench_s_per_step": leg["s_per_step"],
           "kernel_busy_ms_per_step": round(tot, 4),
           "kernels": [{"kernel": k, "ms_per_step": round(v / steps, 4), "share_of_busy": round(v / steps / tot, 4),
                        "launches_per_step": calls[k] / steps} for k, v in top]}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("config", "wall_ms_per_step_under_trace", "kernel_busy_ms_per_step")}))
    for r in out["kernels"][:12]:
        print(json.dumps(r))


if __name__ == "__main__":
    main()

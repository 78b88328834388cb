"""Timeline of the last data-parallel step in a rocprofv3 kernel + memory-copy trace of the HCP gloo rehearsal
(tools/dp_hcp_rehearsal.sh): the gradient graph's first and last kernels, the memory copies of the all-reduce
(gloo stages the gradient through host memory) and the update graph, in us from the step's first kernel.
usage: python tools/dp_trace_summary.py <kernel_trace.csv> <memory_copy_trace.csv>"""
import csv
import sys

ks = sorted(csv.DictReader(open(sys.argv[1])), key=lambda x: int(x["Start_Timestamp"]))
cs = sorted(csv.DictReader(open(sys.argv[2])), key=lambda x: int(x["Start_Timestamp"])) if len(sys.argv) > 2 else []
begins = [x for x in ks if "step_begin_kernel" in x["Kernel_Name"]]
t0 = int(begins[-1]["Start_Timestamp"])
rel = lambda v: (int(v) - t0) / 1e3
fin = [x for x in ks if "dsvi_finalize_kernel" in x["Kernel_Name"] and int(x["Start_Timestamp"]) >= t0]
ad = [x for x in ks if "adam" in x["Kernel_Name"] and int(x["Start_Timestamp"]) >= t0]
lb = [x for x in ks if "lbar" in x["Kernel_Name"] and int(x["Start_Timestamp"]) >= t0]
print("columns of the copy trace:", list(cs[0].keys()) if cs else None)
print(f"gradient graph: step_begin at 0.0 us; last L-bar launch ({lb[-1]['Kernel_Name'][:40] if lb else None}) ends "
      f"{rel(lb[-1]['End_Timestamp']) if lb else None}; finalize ends {rel(fin[0]['End_Timestamp']) if fin else None}")
print(f"update graph: first Adam launch starts {rel(ad[0]['Start_Timestamp']) if ad else None}")
size_key = next((k for k in (cs[0].keys() if cs else []) if k.lower() in ("bytes", "size", "copy_bytes")), None)
dir_key = next((k for k in (cs[0].keys() if cs else []) if k.lower() in ("direction", "kind", "operation")), None)
print("memory copies from the step's start (us):")
for c in cs:
    s = int(c["Start_Timestamp"])
    if s < t0:
        continue
    if ad and s > int(ad[-1]["End_Timestamp"]):
        break
    print(f"  {c.get(dir_key, '?'):>24} bytes {c.get(size_key, '?'):>12} start {rel(s):10.1f} end {rel(c['End_Timestamp']):10.1f}")

"""Print one graph-replayed DSVI step's kernel timeline from a rocprofv3 kernel-trace CSV (between the ends of
the last steps' step-counter advances -- the last kernel of a training step): kernel, queue, grid, start offset,
duration.
usage: python tools/step_timeline.py <run_kernel_trace.csv> [min_us]"""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
lim = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
r.sort(key=lambda x: int(x['Start_Timestamp']))
ad = [x for x in r if 'counter_add_kernel' in x['Kernel_Name']]
a0, a1 = int(ad[-3]['End_Timestamp']), int(ad[-2]['End_Timestamp'])
print('step us', (a1 - a0) / 1e3)
for x in r:
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    if s >= a0 and e <= a1 and (e - s) / 1e3 >= lim:
        print(f"{x['Kernel_Name'][:40]:40s} q{x['Queue_Id']} grid {x['Grid_Size_X']:>8} t={(s - a0) / 1e3:7.1f} "
              f"dur {(e - s) / 1e3:6.1f} end {(e - a0) / 1e3:7.1f}")

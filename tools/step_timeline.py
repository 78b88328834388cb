"""Print one graph-replayed DSVI step's kernel timeline from a rocprofv3 kernel-trace CSV (between the ends of
the last steps' update launches -- the last kernels of a training step): kernel, queue, grid, start offset,
duration.
usage: python tools/step_timeline.py <run_kernel_trace.csv> [min_us]"""
import csv
import sys

r = list(csv.DictReader(open(sys.argv[1])))
lim = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
r.sort(key=lambda x: int(x['Start_Timestamp']))
up = [x for x in r if 'counter_add_kernel' in x['Kernel_Name'] or 'adam' in x['Kernel_Name']]
# a step ends with its last update launch (the Adam, or the counter increment after it): the update launches of one
# step are back to back, so a boundary is an update launch followed by none within 50 us
ends = [int(x['End_Timestamp']) for i, x in enumerate(up)
        if i + 1 == len(up) or int(up[i + 1]['Start_Timestamp']) - int(x['End_Timestamp']) > 50000]
a0, a1 = ends[-3], ends[-2]
print('step us', (a1 - a0) / 1e3)
for x in r:
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    if s >= a0 and e <= a1 and (e - s) / 1e3 >= lim:
        print(f"{x['Kernel_Name'][:40]:40s} q{x['Queue_Id']} grid {x['Grid_Size_X']:>8} t={(s - a0) / 1e3:7.1f} "
              f"dur {(e - s) / 1e3:6.1f} end {(e - a0) / 1e3:7.1f}")

"""Kernel sequence of one training step from a rocprofv3 kernel trace (the step before the
last sgd kernel), with duration and grid — maps kernels to layers and phases.
usage: python tools/trace_seq.py <run_kernel_trace.csv> [--phase]"""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
sgd = [i for i, r in enumerate(rows) if 'sgd' in r['Kernel_Name']]
a, b = sgd[-2] + 1, sgd[-1] + 1
step = rows[a:b]
t0 = int(step[0]['Start_Timestamp'])
tot = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in step)
span = int(step[-1]['End_Timestamp']) - t0
print(f'# {len(step)} kernels, busy {tot / 1e6:.3f} ms, span {span / 1e6:.3f} ms')


def short(n):
    n = re.sub(r'\(.*', '', n.replace('void ', ''))
    return n[:70]


if '--phase' not in sys.argv:
    for r in step:
        d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        g = (int(r['Grid_Size_X']) // int(r['Workgroup_Size_X']), r['Grid_Size_Y'], r['Grid_Size_Z'])
        print(f"{(int(r['Start_Timestamp']) - t0) / 1e3:9.1f} {d:8.1f}  {str(g):18s} v{r['VGPR_Count']:>3s} {short(r['Kernel_Name'])}")

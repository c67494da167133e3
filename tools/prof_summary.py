"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel totals per step.
usage: python tools/prof_summary.py <kernel_stats.csv> <steps_in_run> [title]"""
import csv
import sys

path, steps = sys.argv[1], int(sys.argv[2])
title = sys.argv[3] if len(sys.argv) > 3 else path
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f'# {title}')
print(f'# total kernel time {tot / 1e6:.2f} ms over {steps} step(s) = {tot / 1e6 / steps:.2f} ms/step')
print(f"{'share':>6} {'ms/step':>8} {'calls/step':>10} {'avg_us':>8}  kernel")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs'])):
    name = r['Name'].replace('\n', ' ')
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {float(r['TotalDurationNs']) / 1e6 / steps:8.3f} "
          f"{int(r['Calls']) / steps:10.1f} {float(r['AverageNs']) / 1e3:8.1f}  {name[:150]}")

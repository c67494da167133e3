"""Kernel-time summary of a rocprofv3 --kernel-trace CSV restricted to the last N iterations of
a loop (dispatches from the N-th last launch of a marker kernel onward), so set-up, warm-up and
capture runs stay out of the per-iteration figures.  N given as "N+K" skips K more trailing
iterations (bench.py's eager probe steps after the graphed timed region).
usage: python tools/trace_summary.py <run_kernel_trace.csv> <marker substring> <N[+K]> [title]"""
import collections
import csv
import sys

path, marker = sys.argv[1], sys.argv[2]
last, tail = (int(v) for v in (sys.argv[3] + '+0').split('+')[:2])
title = sys.argv[4] if len(sys.argv) > 4 else path
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
starts = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
if len(starts) < last + tail:
    sys.exit('only %d launches of %r in the trace' % (len(starts), marker))
rows = rows[starts[-last - tail]:starts[-tail] if tail else None]
# bench.py parks the stream behind a spin kernel before its eager probe steps: the window ends
# where that kernel starts (it is not part of any training step)
spin = [i for i, r in enumerate(rows) if 'spin_kernel' in r['Kernel_Name']]
if spin:
    rows = rows[:spin[0]]
agg = collections.defaultdict(lambda: [0, 0])
for r in rows:
    a = agg[r['Kernel_Name'].replace('\n', ' ')]
    a[0] += 1
    a[1] += int(r['End_Timestamp']) - int(r['Start_Timestamp'])
tot = sum(v[1] for v in agg.values())
wall = int(rows[-1]['End_Timestamp']) - int(rows[0]['Start_Timestamp'])
print(f'# {title}')
print(f'# {last} iterations (from the {last + tail}th-last {marker!r} launch): kernel time {tot / 1e6 / last:.3f} '
      f'ms/iter, first-start to last-end {wall / 1e6 / last:.3f} ms/iter, {len(rows) / last:.0f} dispatches/iter')
print(f"{'share':>6} {'ms/iter':>8} {'calls/iter':>10} {'avg_us':>8}  kernel")
for name, (n, ns) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f'{ns / tot * 100:5.1f}% {ns / 1e6 / last:8.3f} {n / last:10.1f} {ns / n / 1e3:8.1f}  {name[:150]}')

"""Per-stream view of one graphed training step from a rocprofv3 kernel trace (the step between
the last two sgd launches): kernel time per queue / stream, the union of busy intervals (the
time the GPU runs at least one kernel), the overlap between streams, and the idle gaps.
usage: python tools/trace_streams.py <run_kernel_trace.csv> [top]"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r'\(.*', '', n.replace('void ', ''))
    return n[:60]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    sgd = [i for i, r in enumerate(rows) if 'sgd' in r['Kernel_Name']]
    step = rows[sgd[-2] + 1:sgd[-1] + 1]
    key = 'Stream_Id' if 'Stream_Id' in step[0] else 'Queue_Id'
    per = collections.defaultdict(lambda: [0, 0.0, collections.Counter()])
    iv = []
    for r in step:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        p = per[r[key]]
        p[0] += 1
        p[1] += (e - s) / 1e3
        p[2][short(r['Kernel_Name'])] += (e - s) / 1e3
        iv.append((s, e))
    iv.sort()
    union, gaps, cs, ce = 0, 0, iv[0][0], iv[0][1]
    for s, e in iv[1:]:
        if s > ce:
            union += ce - cs
            gaps += s - ce
            cs, ce = s, e
        else:
            ce = max(ce, e)
    union += ce - cs
    span = ce - iv[0][0]
    busy = sum(p[1] for p in per.values())
    print(f'# step: span {span / 1e6:.3f} ms, busy union {union / 1e6:.3f} ms, idle gaps {gaps / 1e6:.3f} ms, '
          f'kernel sum {busy / 1e3:.3f} ms ({key})')
    for k, (n, t, c) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f'{key} {k}: {n} kernels, {t / 1e3:.3f} ms')
        for name, v in c.most_common(top):
            print(f'    {v / 1e3:7.3f} ms  {name}')


if __name__ == '__main__':
    main()

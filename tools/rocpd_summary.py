"""Kernel-time summary of a rocprofv3 --kernel-trace database (rocpd SQLite), like the
--stats CSV, optionally restricted to the last N iterations of a loop (the dispatches from the
N-th last launch of a marker kernel onward).
Usage: python tools/rocpd_summary.py run_results.db [--marker stem_fwd --last 10] [--top 40]"""
import argparse
import sqlite3


def rows(db, marker=None, last=0):
    c = sqlite3.connect(db)
    ks = list(c.execute('select name, start, end from kernels order by start'))
    if marker and last:
        starts = [s for (n, s, e) in ks if marker in n]
        if len(starts) >= last:
            t0 = starts[-last]
            ks = [k for k in ks if k[1] >= t0]
    return ks


def summary(ks, per=1):
    agg = {}
    for n, s, e in ks:
        a = agg.setdefault(n, [0, 0.0])
        a[0] += 1
        a[1] += (e - s) / 1e3
    tot = sum(v[1] for v in agg.values())
    out = sorted(((n, c, t) for n, (c, t) in agg.items()), key=lambda r: -r[2])
    return out, tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--marker', default=None)
    ap.add_argument('--last', type=int, default=0)
    ap.add_argument('--top', type=int, default=40)
    a = ap.parse_args()
    ks = rows(a.db, a.marker, a.last)
    out, tot = summary(ks)
    per = max(a.last, 1)
    span = (max(e for _, _, e in ks) - min(s for _, s, _ in ks)) / 1e3
    print(f'# {a.db}: {len(ks)} dispatches, kernel time {tot:.1f} us, wall span {span:.1f} us'
          + (f'; per iteration ({per}): kernel {tot / per:.1f} us, span {span / per:.1f} us' if a.last else ''))
    print(f'{"calls/it":>9} {"us/it":>10} {"avg_us":>9} {"pct":>6}  kernel')
    for n, c, t in out[:a.top]:
        print(f'{c / per:9.1f} {t / per:10.1f} {t / c:9.2f} {100 * t / tot:6.2f}  {n[:150]}')


if __name__ == '__main__':
    main()

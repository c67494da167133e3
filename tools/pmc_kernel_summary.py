"""Per-kernel totals of a rocprofv3 --pmc counter CSV: for every kernel whose name contains
one of the given substrings, the dispatch count and each counter's sum and per-dispatch mean.
usage: python tools/pmc_kernel_summary.py <counter_collection.csv[.gz]> <substring>..."""
import collections
import csv
import gzip
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    f = gzip.open(path, 'rt') if path.endswith('.gz') else open(path)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(f):
        k = r['Kernel_Name']
        if subs and not any(s in k for s in subs):
            continue
        agg[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
    for k, cs in agg.items():
        n = len(disp[k])
        print(f'{k[:110]}  dispatches={n}')
        for c, v in sorted(cs.items()):
            print(f'    {c:28s} sum={v:16.0f}  per_dispatch={v / n:14.0f}')


if __name__ == '__main__':
    main()

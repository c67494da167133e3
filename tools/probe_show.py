"""Print a bench.py --probe-table JSON: per-entry totals and the heaviest calls."""
import json
import sys

d = json.load(open(sys.argv[1]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
tot = sum(r['ms_per_step'] for r in d['entries'])
print(f'total librod time {tot:.3f} ms/step')
for r in d['entries']:
    print(f"{r['entry']:28s} {r['calls_per_step']:6.1f} {r['ms_per_step']:7.3f}ms {r['avg_us']:8.1f}us "
          f"{r['alg_GBps']:7.0f}GB/s {r['alg_TFLOPs']:6.1f}TF")
print()
for r in d['top_calls'][:n]:
    print(f"{r['entry']:22s} {str(r['args']):58s} x{r['calls_per_step']:.0f} {r['avg_us']:8.1f}us "
          f"{r['alg_GBps']:6.0f}GB/s {r['alg_TFLOPs']:6.1f}TF")

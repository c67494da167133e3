"""Compare two --probe-table JSONs per entry (ms/step) and list the top calls of the second.
usage: python tools/probe_cmp.py old.json new.json [ncalls]"""
import json
import sys

a = {r['entry']: r for r in json.load(open(sys.argv[1]))['entries']}
t = json.load(open(sys.argv[2]))
b = {r['entry']: r for r in t['entries']}
print(f"{'entry':28s} {'old ms':>8s} {'new ms':>8s} {'calls':>6s} {'GB/s':>8s}")
for k in sorted(set(a) | set(b), key=lambda k: -b.get(k, {'ms_per_step': 0})['ms_per_step']):
    o, n = a.get(k, {}), b.get(k, {})
    print(f"{k:28s} {o.get('ms_per_step', 0):8.3f} {n.get('ms_per_step', 0):8.3f} {n.get('calls_per_step', 0):6.1f} "
          f"{n.get('alg_GBps', 0):8.1f}")
print(f"{'total':28s} {sum(r['ms_per_step'] for r in a.values()):8.3f} {sum(r['ms_per_step'] for r in b.values()):8.3f}")
nc = int(sys.argv[3]) if len(sys.argv) > 3 else 30
for r in t['top_calls'][:nc]:
    print(f"{r['entry']:22s} {str(r['args'])[:64]:64s} {r['calls_per_step']:4.1f} {r['avg_us']:8.1f} {r['alg_GBps']:8.1f}")

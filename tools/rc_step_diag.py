"""Step-level diagnosis of the recompute forms (GPU): REFINE steps at 480x864 b2 under several
ROD_DISABLE / ROD_ENABLE settings, eager or graphed; prints the losses of each and the largest
parameter difference against the first setting, per parameter name for the worst ones."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def run(dis, ena, graphed, steps=3, H=480, W=864, B=2):
    from rod import ops
    from rod.data import synthetic_batch
    from rod.trainer import Trainer
    ops._DISABLE.update(dis)
    ops._ENABLE.update(ena)
    try:
        tr = Trainer((H, W), B, dtype=torch.bfloat16, device='cuda', seed=7)
        batches = [synthetic_batch(B, H, W, 'cuda', seed=50 + i) for i in range(2)]
        step = tr.step_graphed if graphed else tr.step
        losses = [float(step(*batches[i % 2])[0].detach()) for i in range(steps)]
        torch.cuda.synchronize()
        return losses, {n: p.detach().clone() for n, p in tr.net.store.params.items()}
    finally:
        for d in dis:
            ops._DISABLE.discard(d)
        for e in ena:
            ops._ENABLE.discard(e)


def main():
    graphed = len(sys.argv) > 1 and sys.argv[1] == 'graphed'
    cfgs = [('all off', {'rc'}, set()), ('default', set(), set()), ('default again', set(), set()),
            ('no nostore', {'nostore'}, set()), ('nostore + rcdw', set(), {'rcdw'})]
    base = None
    for name, dis, ena in cfgs:
        losses, params = run(dis, ena, graphed)
        line = '%-16s losses %s' % (name, ['%.6f' % l for l in losses])
        if base is None:
            base = params
        else:
            diffs = sorted(((float((params[n] - base[n]).abs().max()), n) for n in base), reverse=True)
            line += '  max param diff %.3g (%s)  #diff %d' % (diffs[0][0], diffs[0][1], sum(1 for d, _ in diffs if d > 0))
            if diffs[0][0] > 0:
                line += '\n    ' + '\n    '.join('%.3g %s' % d for d in diffs[:6])
        print(line, flush=True)


if __name__ == '__main__':
    main()

"""BatchNorm-backward micro-benchmark at the backbone / head shapes of the 720x1280 b=8 step
(rod_bn_bwd: reduce -> finalize -> apply), HIP-event timed, algorithmic GB/s (dz, y read, dy
written once).  usage: python tools/bn_bench.py [--iters N] [--out f.pt] [--check f.pt]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
from rod import _abi, ops  # noqa: E402

SHAPES = [(7372800, 96, 1), (7372800, 32, 1), (7372800, 16, 0), (1843200, 144, 1), (1843200, 24, 0),
          (460800, 192, 1), (460800, 32, 0), (115200, 384, 1), (115200, 64, 0), (115200, 128, 2),
          (28800, 576, 1), (28800, 96, 0), (28800, 128, 2), (7360, 960, 1), (7360, 160, 0), (1920, 1920, 1),
          (480, 256, 2), (120, 256, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--out', default=None)
    ap.add_argument('--check', default=None)
    a = ap.parse_args()
    dev = 'cuda'
    dt = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    s = ops.stream()
    res, tot = {}, 0.0
    for (M, C, act) in SHAPES:
        dz = torch.randn((M, C), device=dev, generator=g).to(dt)
        y = (torch.randn((M, C), device=dev, generator=g) * 2 + 0.5).to(dt)
        mean = torch.randn(C, device=dev, generator=g) * 0.1
        rstd = torch.rand(C, device=dev, generator=g) + 0.5
        gamma = torch.rand(C, device=dev, generator=g) + 0.5
        beta = torch.randn(C, device=dev, generator=g) * 0.1
        dy = torch.empty_like(y)
        dg = torch.empty(C, device=dev)
        db = torch.empty(C, device=dev)
        ws = torch.empty(_abi.query('rod_bn_bwd_workspace', M, C), dtype=torch.uint8, device=dev)
        fn = lambda: _abi.call('rod_bn_bwd', dz, y, mean, rstd, gamma, beta, dy, dg, db, ws, M, C, 0, 0, 0, act,  # noqa
                               ops.dtcode(y), s)
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        tot += ms
        io = 3 * 2 * M * C
        print(f'bn_bwd M={M:8d} C={C:5d} act={act} {ms * 1e3:8.1f} us {io / ms / 1e6:8.1f} GB/s', flush=True)
        res[f'{M}x{C}a{act}'] = (dy.float().cpu(), dg.cpu(), db.cpu())
    print(f'TOTAL {tot * 1e3:.1f} us')
    if a.out:
        torch.save(res, a.out)
    if a.check:
        ref = torch.load(a.check, weights_only=True)
        for k, v in res.items():
            errs = [float(((p - q).abs().max() / (q.abs().max() + 1e-30)).item()) for p, q in zip(v, ref[k])]
            print(f'CHECK {k:20s} ' + ' '.join(f'{e:.3e}' for e in errs))


if __name__ == '__main__':
    main()

"""BatchNorm-backward micro-benchmark at the backbone / head shapes of the 720x1280 b=8 step,
the path the training step takes (ops.bn_bwd_dy): rod_bn_bwd_reduce (reduce + finalize) then
rod_bn_bwd_apply, or the one-launch rod_bn_bwd on <= 4096 rows.  HIP-event timed; GB/s are
algorithmic (dz, y read once, dy written once).  Every shape is also checked against a float64
restatement of FusedBatchNormGrad (normwise error of dy / dgamma / dbeta printed).
usage: python tools/bn_bench.py [--iters N] [--out f.pt] [--check f.pt]"""
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
          (480, 256, 2), (120, 256, 2), (120, 512, 1), (480, 512, 1), (1920, 320, 0), (4096, 64, 2)]


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
        coef = torch.empty(3 * C, device=dev)
        if M <= 4096:
            fn = lambda: _abi.call('rod_bn_bwd', dz, y, mean, rstd, gamma, beta, dy, dg, db, ws, M, C, 0, 0, 0,  # noqa
                                   act, ops.dtcode(y), s)
        else:
            def fn():
                _abi.call('rod_bn_bwd_reduce', dz, y, mean, rstd, gamma, beta, dg, db, coef, ws, M, C, act,
                          ops.dtcode(y), s)
                _abi.call('rod_bn_bwd_apply', dz, y, mean, rstd, gamma, beta, coef, dy, M, C, act, ops.dtcode(y), s)
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
        # float64 FusedBatchNormGrad (z = act(y*sc + sh), the kernels' fma form)
        yd, gz = y.double(), dz.double()
        sc = (rstd * gamma).double()
        z = (y.float() * (rstd * gamma) + (beta - mean * rstd * gamma)).double()
        ag = torch.ones_like(z) if act == 0 else (((z > 0) & (z < 6)).double() if act == 1 else
                                                   torch.where(z > 0, 1.0, 0.2).double())
        gg = gz * ag
        yh = (yd - mean.double()) * rstd.double()
        rdb, rdg = gg.sum(0), (gg * yh).sum(0)
        rdy = sc * (gg - rdb / M - yh * (rdg / M))
        e = lambda a_, b_: float((a_.double() - b_).abs().max() / b_.abs().max().clamp_min(1e-30))  # noqa
        errs = (e(dy, rdy), e(dg, rdg), e(db, rdb))
        print(f'bn_bwd M={M:8d} C={C:5d} act={act} {ms * 1e3:8.1f} us {io / ms / 1e6:8.1f} GB/s  '
              f'err dy {errs[0]:.1e} dg {errs[1]:.1e} db {errs[2]:.1e}', flush=True)
        assert errs[0] < 2e-2 and errs[1] < 1e-4 and errs[2] < 1e-4, errs
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

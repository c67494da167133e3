"""Pointwise / 3x3 conv micro-benchmark at the C2 (720x1280, b=8) shapes: rod_conv_fwd
(forward with the BatchNorm-statistics epilogue and the BatchNorm prologue, as the backbone
runs it; backward-data with the mode-1 weights) and rod_conv_wgrad, timed with HIP events,
algorithmic GB/s and TFLOP/s (rod.roofline).  Writes / checks outputs to compare variants.

usage: python tools/conv_bench.py [--out f.pt] [--check f.pt] [--iters N]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
from rod import _abi, ops  # noqa: E402

# (N, H, W, Cin, Cout, ks, pro_act): L3 expand, L3 project, L4 expand, L4 project, L6 expand,
# L12 expand, stem, head 3x3, head 1x1, ..., head last 3x3
SHAPES = [(8, 720, 1280, 16, 96, 1, 0), (8, 360, 640, 96, 24, 1, 1), (8, 360, 640, 24, 144, 1, 0),
          (8, 360, 640, 144, 24, 1, 1), (8, 180, 320, 32, 192, 1, 0), (8, 90, 160, 64, 384, 1, 0),
          (8, 90, 160, 384, 64, 1, 1), (8, 90, 160, 128, 128, 3, 2), (8, 90, 160, 64, 128, 1, 0),
          (8, 720, 1280, 3, 32, 3, 0), (8, 45, 80, 96, 576, 1, 0), (8, 45, 80, 576, 96, 1, 1),
          (8, 23, 40, 160, 960, 1, 0),
          # the heads' last 3x3 convs (Cin = Cout = k x anchors, not a multiple of 8)
          (8, 90, 160, 66, 66, 3, 2), (8, 45, 80, 99, 99, 3, 2), (8, 45, 80, 36, 36, 3, 2),
          # projects with the depthwise BatchNorm prologue: 720p block 1, 180x320 blocks
          (8, 720, 1280, 32, 16, 1, 1), (8, 180, 320, 192, 32, 1, 1), (8, 180, 320, 144, 32, 1, 1),
          # C5 (1080p) heads: the last 3x3 convs and a 128 -> 128 3x3 on the deep levels
          (8, 34, 60, 99, 99, 3, 2), (8, 68, 120, 99, 99, 3, 2), (8, 135, 240, 66, 66, 3, 2), (8, 34, 60, 128, 128, 3, 2),
          (8, 17, 30, 99, 99, 3, 2)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--out', default=None)
    ap.add_argument('--check', default=None)
    ap.add_argument('--ops', default='fwd_plain,fwd_stats,bwd_data,wgrad')
    ap.add_argument('--shapes', default=None, help='comma-separated SHAPES indices (default all)')
    a = ap.parse_args()
    dt = torch.bfloat16
    dev = 'cuda'
    g = torch.Generator(device=dev).manual_seed(0)
    s = ops.stream()
    res, tot = {}, {}
    sel = [SHAPES[int(i)] for i in a.shapes.split(',')] if a.shapes else SHAPES
    for (N, H, W, Cin, Cout, ks, act) in sel:
        M = N * H * W
        x = torch.randn((N, H, W, Cin), device=dev, generator=g).to(dt)
        dy = torch.randn((N, H, W, Cout), device=dev, generator=g).to(dt)
        w = torch.randn((Cout, ks, ks, Cin), device=dev, generator=g) / (ks * ks * Cin) ** 0.5
        wt0 = torch.empty((Cout, ks * ks * Cin), device=dev, dtype=dt)
        wt1 = torch.empty((Cin, ks * ks * Cout), device=dev, dtype=dt)
        _abi.call('rod_conv_weight_prep', w, wt0, Cout, Cin, ks, 0, 1, s)
        _abi.call('rod_conv_weight_prep', w, wt1, Cout, Cin, ks, 1, 1, s)
        mean = torch.randn(Cin, device=dev, generator=g) * 0.1
        rstd = torch.rand(Cin, device=dev, generator=g) + 0.5
        gamma = torch.rand(Cin, device=dev, generator=g) + 0.5
        beta = torch.randn(Cin, device=dev, generator=g) * 0.1
        pro = (mean, rstd, gamma, beta, act) if act else None
        y = torch.empty((N, H, W, Cout), device=dev, dtype=dt)
        dx = torch.empty((N, H, W, Cin), device=dev, dtype=dt)
        parts = torch.empty((-(-M // 128), 3, Cout), device=dev)
        mu, rs = torch.empty(Cout, device=dev), torch.empty(Cout, device=dev)
        dw = torch.empty((Cout, ks, ks, Cin), device=dev)
        wws = torch.empty(max(16, _abi.query('rod_conv_wgrad_workspace', N, H, W, Cin, Cout, ks)), dtype=torch.uint8,
                          device=dev)
        fw = _abi.query('rod_bn_finalize_workspace', parts.shape[0], Cout)
        fws = torch.empty(max(16, fw), dtype=torch.uint8, device=dev)
        K = ks * ks * Cin
        io_f = 2 * (M * Cin + M * Cout)
        calls = {
            'fwd_plain': (lambda: ops.conv_fwd_raw(x, wt0, None, y, N, H, W, Cin, Cout, ks), io_f),
            'fwd_stats': (lambda: ops.conv_fwd_raw(x, wt0, None, y, N, H, W, Cin, Cout, ks, parts, pro), io_f),
            'bwd_data': (lambda: ops.conv_fwd_raw(dy, wt1, None, dx, N, H, W, Cout, Cin, ks), io_f),
            'wgrad': (lambda: _abi.call('rod_conv_wgrad', x, *ops._pro_args(pro), dy, dw, None, wws, N, H, W, Cin,
                                        Cout, ks, 0, 0, 1, s), io_f),
        }
        for op, (fn, io) in calls.items():
            if op not in a.ops.split(','):
                continue
            if op == 'bwd_data' and Cin == 3:  # the stem has no backward-data (input = image)
                continue
            y.fill_(float('nan'))   # a kernel that skips part of its output shows up in --check
            dx.fill_(float('nan'))
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            key = f'{op}:{N}x{H}x{W}:{Cin}->{Cout}k{ks}a{act}'
            print(f'{key:40s} {ms * 1e3:9.1f} us {io / ms / 1e6:8.1f} GB/s {2 * M * K * Cout / ms / 1e9:7.1f} TF/s',
                  flush=True)
            tot[op] = tot.get(op, 0) + ms
            if op == 'fwd_stats':
                _abi.call('rod_bn_finalize', parts, parts.shape[0], M, Cout, 1e-3, 0.997, mu, rs, None, None, fws, s)
                res[key] = (y.float().cpu(), mu.cpu(), rs.cpu())
            elif op == 'fwd_plain':
                pass
            elif op == 'bwd_data':
                res[key] = (dx.float().cpu(),)
            else:
                res[key] = (dw.cpu(),)
    for op, ms in tot.items():
        print(f'TOTAL {op:10s} {ms * 1e3:9.1f} us')
    if a.out:
        torch.save(res, a.out)
    if a.check:
        ref = torch.load(a.check, weights_only=True)
        for k, v in res.items():
            errs = [float(((p - q).abs().max() / (q.abs().max() + 1e-30)).item()) for p, q in zip(v, ref[k])]
            print(f'CHECK {k:40s} ' + ' '.join(f'{e:.3e}' for e in errs))


if __name__ == '__main__':
    main()

"""Depthwise 3x3 micro-benchmark at the C2 (720x1280, b=8) backbone shapes: times the
librod entries with HIP events on the launching stream and reports algorithmic GB/s
(rod.roofline per-unit bytes), and writes the outputs to compare kernel variants.

usage: python tools/dw_bench.py [--dtype bf16|f32] [--out file.pt] [--check ref.pt] [--iters N]
Run once per variant (e.g. ROD_DW_LEGACY=1 for the register-strip kernels)."""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
from rod import _abi  # noqa: E402
from rod.ops import same_pad  # noqa: E402

# (N, H, W, C, stride) of the largest depthwise layers at 720x1280 (L2, L3, L4, L5, L6, L8, L9)
SHAPES = [(8, 720, 1280, 32, 1), (8, 720, 1280, 96, 2), (8, 360, 640, 144, 1), (8, 360, 640, 144, 2),
          (8, 180, 320, 192, 1), (8, 180, 320, 192, 2), (8, 90, 160, 384, 1), (8, 45, 80, 576, 1),
          (8, 23, 40, 960, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dtype', default='bf16')
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--out', default=None)
    ap.add_argument('--check', default=None)
    ap.add_argument('--ops', default='fwd,fwdpro,bwd_data,bwd_data_gred,bwd_filter')
    a = ap.parse_args()
    dt = torch.bfloat16 if a.dtype == 'bf16' else torch.float32
    code = _abi.ROD_BF16 if a.dtype == 'bf16' else _abi.ROD_F32
    es = 2 if a.dtype == 'bf16' else 4
    dev = 'cuda'
    g = torch.Generator(device=dev).manual_seed(0)
    s = torch.cuda.current_stream().cuda_stream
    results, tot_ms, tot_b = {}, {}, {}
    ops = a.ops.split(',')
    for (N, H, W, C, S) in SHAPES:
        Ho, pt = same_pad(H, S)
        Wo, pl = same_pad(W, S)
        x = torch.randn((N, H, W, C), device=dev, generator=g).to(dt)
        w = torch.randn((3, 3, C), device=dev, generator=g) * 0.3
        dy = torch.randn((N, Ho, Wo, C), device=dev, generator=g).to(dt)
        mean = torch.randn(C, device=dev, generator=g) * 0.1
        rstd = torch.rand(C, device=dev, generator=g) + 0.5
        gamma = torch.rand(C, device=dev, generator=g) + 0.5
        beta = torch.randn(C, device=dev, generator=g) * 0.1
        y = torch.empty((N, Ho, Wo, C), device=dev, dtype=dt)
        dx = torch.empty((N, H, W, C), device=dev, dtype=dt)
        dw = torch.empty((3, 3, C), device=dev)
        nparts = _abi.lib().rod_dw3x3_fwd_stat_parts(N, Ho, Wo, C, S, code)
        parts = torch.empty((nparts, 3, C), device=dev)
        mu = torch.empty(C, device=dev)
        rs = torch.empty(C, device=dev)
        wsb = torch.empty(max(16, _abi.query('rod_dw3x3_bwd_filter_workspace', N, Ho, Wo, C)), dtype=torch.uint8,
                          device=dev)
        fws = _abi.query('rod_bn_finalize_workspace', nparts, C)
        fwsb = torch.empty(max(16, fws), dtype=torch.uint8, device=dev) if fws else None
        gparts = torch.empty((_abi.lib().rod_dw3x3_bwd_data_gred_parts(N, H, W, C, S, code), 2, C), device=dev)
        io = es * (N * H * W * C + N * Ho * Wo * C)
        calls = {
            'fwd': lambda: _abi.call('rod_dw3x3_fwd', x, None, None, None, None, 0, w, y, None, N, H, W, C, S, pt,
                                     pl, Ho, Wo, code, s),
            'fwdpro': lambda: _abi.call('rod_dw3x3_fwd', x, mean, rstd, gamma, beta, 1, w, y, parts, N, H, W, C, S,
                                        pt, pl, Ho, Wo, code, s),
            'bwd_data': lambda: _abi.call('rod_dw3x3_bwd_data', dy, w, dx, None, None, None, None, None, 0, None, N, H, W, C, S, pt, pl, Ho, Wo, code, s),
            'bwd_data_gred': lambda: _abi.call('rod_dw3x3_bwd_data', dy, w, dx, x, mean, rstd, gamma, beta, 1, gparts,
                                               N, H, W, C, S, pt, pl, Ho, Wo, code, s),
            'bwd_filter': lambda: _abi.call('rod_dw3x3_bwd_filter', x, mean, rstd, gamma, beta, 1, dy, dw, wsb, N, H,
                                            W, C, S, pt, pl, Ho, Wo, code, s),
        }
        for op in ops:
            fn = calls[op]
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            key = f'{op}:{N}x{H}x{W}x{C}s{S}'
            print(f'{key:34s} {ms * 1e3:9.1f} us {io / ms / 1e6:8.1f} GB/s', flush=True)
            tot_ms[op] = tot_ms.get(op, 0) + ms
            tot_b[op] = tot_b.get(op, 0) + io
            if op == 'fwd':
                results[key] = y.float().cpu()
            elif op == 'fwdpro':
                _abi.call('rod_bn_finalize', parts, nparts, N * Ho * Wo, C, 1e-3, 0.997, mu, rs, None, None, fwsb, s)
                results[key] = (y.float().cpu(), mu.cpu(), rs.cpu())
            elif op in ('bwd_data', 'bwd_data_gred'):
                results[key] = dx.float().cpu()
            else:
                results[key] = dw.cpu()
    for op in ops:
        print(f'TOTAL {op:12s} {tot_ms[op] * 1e3:9.1f} us {tot_b[op] / tot_ms[op] / 1e6:8.1f} GB/s')
    if a.out:
        torch.save(results, a.out)
    if a.check:
        ref = torch.load(a.check, weights_only=True)
        for k, v in results.items():
            r = ref[k]
            vs, rs_ = (v, r) if isinstance(v, tuple) else ((v,), (r,))
            errs = [float(((p - q).abs().max() / (q.abs().max() + 1e-30)).item()) for p, q in zip(vs, rs_)]
            print(f'CHECK {k:34s} max rel err ' + ' '.join(f'{e:.3e}' for e in errs))


if __name__ == '__main__':
    main()

"""Time the fused 1x1-conv + BatchNorm backward (rod_pw_bwd) against the unfused chain
(rod_bn_bwd [reduce+apply] -> rod_conv_fwd mode 1 -> rod_conv_wgrad) on the 720p bf16 b8
shapes of the REFINE step.  Usage: python tools/pwbwd_bench.py [--iters 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
import torch  # noqa: E402

from rod import ops  # noqa: E402

bf16 = torch.bfloat16
# (M, Cin, Cout, act, input prologue): expand / project convs of the 720p backbone, b=8
SHAPES = [(7372800, 16, 96, 1, True), (1843200, 24, 144, 1, True), (1843200, 144, 24, 0, True),
          (460800, 32, 192, 1, True), (460800, 192, 32, 0, True), (7372800, 32, 16, 0, True),
          (115200, 64, 128, 2, False), (1843200, 96, 24, 0, True)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--pw-only', action='store_true', help='time rod_pw_bwd alone on the shapes it serves')
    a = ap.parse_args()
    dev = torch.device('cuda')
    rows = []
    for (M, Cin, Cout, act, prox) in SHAPES:
        torch.manual_seed(M + Cin + Cout)
        if a.pw_only and not ops.pw_bwd_supported(Cin, Cout, bf16):
            continue
        x = torch.randn(M, Cin, device=dev).to(bf16)
        y = torch.randn(M, Cout, device=dev).to(bf16)
        dz = torch.randn(M, Cout, device=dev).to(bf16)
        w = torch.randn(Cout, 1, 1, Cin, device=dev) * 0.1
        mean, rstd = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
        gamma, beta = torch.ones(Cout, device=dev), torch.zeros(Cout, device=dev)
        xpro = (torch.zeros(Cin, device=dev), torch.ones(Cin, device=dev), torch.ones(Cin, device=dev),
                torch.zeros(Cin, device=dev), 1) if prox else None
        wt1 = ops._prep(w, 1, bf16, Cout, Cin, 1)
        dw = torch.empty(Cout, Cin, device=dev)
        bws = ops.workspace(ops._abi.query('rod_bn_bwd_workspace', M, Cout), dev)
        wws = ops.workspace(ops._abi.query('rod_conv_wgrad_workspace', 1, 1, M, Cin, Cout, 1), dev)
        dy = torch.empty_like(y)
        dx = torch.empty_like(x)
        db = torch.empty(Cout, device=dev)

        def unfused():
            ops._abi.call('rod_bn_bwd', dz, y, mean, rstd, gamma, beta, dy, None, db, bws, M, Cout, 0, 0, 0, act,
                          ops.dtcode(y), ops.stream())
            ops.conv_fwd_raw(dy, wt1, None, dx, 1, 1, M, Cout, Cin, 1)
            ops._abi.call('rod_conv_wgrad', x, *ops._pro_args(xpro), dy, dw, None, wws, 1, 1, M, Cin, Cout, 1, 0, 0,
                          ops.dtcode(x), ops.stream())

        coef0 = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)

        def pw_only():
            ops.pw_bwd(dz, y, mean, rstd, gamma, beta, act, coef0, x, xpro, wt1, True, dw, None)

        def fused():
            coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)
            ops.pw_bwd(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, True, dw, None)

        res = {}
        fns = (('pw', pw_only),) if a.pw_only else (('unfused', unfused), ('fused', fused), ('pw', pw_only))
        for name, fn in fns:
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res[name] = e0.elapsed_time(e1) / a.iters * 1e3
        # algorithmic bytes of the fused pass + its reduce: dz, y twice, x once, dx once
        alg = 2 * M * (2 * Cout * 2 + 2 * Cin)
        pw_alg = M * (2 * Cout * 2 + 2 * Cin * 2)
        pw_only()
        torch.cuda.synchronize()
        r = {'M': M, 'Cin': Cin, 'Cout': Cout, 'pw_us': round(res['pw'], 1),
             'pw_alg_GBps': round(pw_alg / res['pw'] / 1e3, 1),
             'check': [float(dx.double().nan_to_num().abs().sum()), float(dw.double().abs().sum())]}
        if not a.pw_only:
            r.update({'unfused_us': round(res['unfused'], 1), 'fused_us': round(res['fused'], 1),
                      'speedup': round(res['unfused'] / res['fused'], 3),
                      'fused_alg_GBps': round(alg / res['fused'] / 1e3, 1)})
        rows.append(r)
        print(json.dumps(rows[-1]), flush=True)
    print(json.dumps({'total_pw_us': round(sum(r['pw_us'] for r in rows), 1),
                      'total_unfused_us': round(sum(r.get('unfused_us', 0) for r in rows), 1),
                      'total_fused_us': round(sum(r.get('fused_us', 0) for r in rows), 1)}))


if __name__ == '__main__':
    main()

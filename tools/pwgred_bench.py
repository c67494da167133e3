"""Time rod_pw_bwd_gred (the project conv's backward + the depthwise BatchNorm's sums) on the
project shapes of the 720p bf16 b8 REFINE step, against the chain it replaces
(rod_bn_bwd_apply -> backward-data -> rod_conv_wgrad, plus the depthwise BatchNorm's
rod_bn_bwd_reduce).  Usage: python tools/pwgred_bench.py [--iters 20] [--only]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
import torch  # noqa: E402

from rod import ops  # noqa: E402

bf16 = torch.bfloat16
# (M, Cin, Cout): project convs of the 720p backbone, b = 8
SHAPES = [(7372800, 32, 16), (1843200, 96, 24), (1843200, 144, 24), (460800, 144, 32), (460800, 192, 32),
          (115200, 192, 64), (115200, 384, 64)]


def timed(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--only', action='store_true', help='time rod_pw_bwd_gred alone')
    a = ap.parse_args()
    dev = torch.device('cuda')
    tot_f = tot_u = 0.0
    for (M, Cin, Cout) in SHAPES:
        torch.manual_seed(M + Cin)
        x = torch.randn(M, Cin, device=dev).to(bf16)
        y = torch.randn(M, Cout, device=dev).to(bf16)
        dz = torch.randn(M, Cout, device=dev).to(bf16)
        w = torch.randn(Cout, 1, 1, Cin, device=dev) * 0.1
        mean, rstd = torch.zeros(Cout, device=dev), torch.ones(Cout, device=dev)
        gamma, beta = torch.ones(Cout, device=dev), torch.zeros(Cout, device=dev)
        xpro = (torch.zeros(Cin, device=dev), torch.ones(Cin, device=dev), torch.ones(Cin, device=dev),
                torch.zeros(Cin, device=dev), ops.ROD_ACT_RELU6)
        wt1 = ops._prep(w, 1, bf16, Cout, Cin, 1)
        dw = torch.empty(Cout, Cin, device=dev)
        coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, 0, False, False)
        fused = lambda: ops.pw_bwd_gred(dz, y, mean, rstd, gamma, beta, 0, coef, x, xpro, wt1, dw)
        tf = timed(fused, a.iters)
        byts = 2 * M * (2 * Cout + 2 * Cin)
        row = {'M': M, 'Cin': Cin, 'Cout': Cout, 'gred_us': round(tf, 1), 'alg_GBps': round(byts / tf / 1e3, 1)}
        tot_f += tf
        if not a.only:
            dy = torch.empty_like(y)
            dx = torch.empty_like(x)
            wws = ops.workspace(ops._abi.query('rod_conv_wgrad_workspace', 1, 1, M, Cin, Cout, 1), dev)

            def chain():
                ops._abi.call('rod_bn_bwd_apply', dz, y, mean, rstd, gamma, beta, coef, dy, M, Cout, 0,
                              ops.dtcode(y), ops.stream())
                ops.conv_fwd_raw(dy, wt1, None, dx, 1, 1, M, Cout, Cin, 1)
                ops._abi.call('rod_conv_wgrad', x, *ops._pro_args(xpro), dy, dw, None, wws, 1, 1, M, Cin, Cout, 1, 0,
                              0, ops.dtcode(x), ops.stream())
                ops.bn_bwd_reduce(dx, x, xpro[0], xpro[1], xpro[2], xpro[3], ops.ROD_ACT_RELU6, False, False)
            tu = timed(chain, a.iters)
            row['chain_us'] = round(tu, 1)
            tot_u += tu
        print(json.dumps(row), flush=True)
    print(json.dumps({'total_gred_us': round(tot_f, 1), 'total_chain_us': round(tot_u, 1)}))


if __name__ == '__main__':
    main()

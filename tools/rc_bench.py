"""Timing of the recompute forms (ABI 23) against the forms that read the stored expanded tensor,
at the 720p b8 training step's block shapes (GPU; HIP events around N calls, median of 3).

  dwfwd : rod_dw3x3_fwd (stored ye, BN_e prologue) vs rod_dw3x3_fwd_rc (ye recomputed from x)
Prints one line per shape; outputs are checked equal on the way."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

# (name, N, H, W, Cin, C, stride, input prologue act or None): 720p b8 blocks 1-6
SHAPES = [('b1 16->96 s2', 8, 720, 1280, 16, 96, 2, 0), ('b2 24->144 s1', 8, 360, 640, 24, 144, 1, None),
          ('b3 24->144 s2', 8, 360, 640, 24, 144, 2, None), ('b4 32->192 s1', 8, 180, 320, 32, 192, 1, None),
          ('b6 32->192 s2', 8, 180, 320, 32, 192, 2, None)]


def timeit(fn, iters=10):
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fn()
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / iters)
    return sorted(ts)[1]


def main():
    dev = torch.device('cuda', 0)
    from rod import _abi, ops
    bf16 = torch.bfloat16
    code = ops.dtcode(torch.empty(1, dtype=bf16))
    only = sys.argv[1:]
    for name, N, H, W, Cin, C, s, xact in SHAPES:
        if only and not any(o in name for o in only):
            continue
        g = torch.Generator().manual_seed(N + H + C)
        M = N * H * W
        x = (torch.randn(N, H, W, Cin, generator=g) * 1.4).to(dev, bf16)
        w_e = (torch.randn(C, 1, 1, Cin, generator=g) * 0.3).to(dev)
        xpro = None
        if xact is not None:
            xpro = ((torch.randn(Cin, generator=g) * 0.2).to(dev), (torch.rand(Cin, generator=g) + 0.5).to(dev),
                    (torch.rand(Cin, generator=g) + 0.5).to(dev), (torch.randn(Cin, generator=g) * 0.2).to(dev), xact)
        wt0 = ops._prep(w_e, 0, bf16, C, Cin, 1)
        ye = torch.empty((N, H, W, C), dtype=bf16, device=dev)
        ops.conv_fwd_raw(x, wt0, None, ye, N, H, W, Cin, C, 1, None, xpro)
        if _abi.lib().rod_conv_fwd_stats_supported(M, Cin, C, code):
            sp0 = torch.empty((-(-M // 128), 3, C), device=dev)
            sp1 = torch.empty_like(sp0)
            ta = timeit(lambda: ops.conv_fwd_raw(x, wt0, None, ye, N, H, W, Cin, C, 1, sp0, xpro))
            tb = timeit(lambda: _abi.call('rod_conv_fwd_stats', x, *ops._pro_args(xpro), wt0, sp1, M, Cin, C, code,
                                          ops.stream()))
            print('%-16s expand stored+stats %7.1f us   stats only %7.1f us   equal %s' %
                  (name, ta, tb, torch.equal(sp0, sp1)), flush=True)
        epro = (ye.float().mean((0, 1, 2)), torch.rsqrt(ye.float().var((0, 1, 2)) + 1e-3),
                (torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.5).to(dev),
                ops.ROD_ACT_RELU6)
        wd = (torch.randn(3, 3, C, generator=g) * 0.3).to(dev)
        Ho, pt = ops.same_pad(H, s)
        Wo, pl = ops.same_pad(W, s)
        nparts = _abi.lib().rod_dw3x3_fwd_stat_parts(N, Ho, Wo, C, s, code)
        y0 = torch.empty((N, Ho, Wo, C), dtype=bf16, device=dev)
        y1 = torch.empty_like(y0)
        p0 = torch.empty((nparts, 3, C), device=dev)
        p1 = torch.empty_like(p0)

        def stored():
            _abi.call('rod_dw3x3_fwd', ye, *ops._pro_args(epro), wd, y0, p0, N, H, W, C, s, pt, pl, Ho, Wo, code,
                      ops.stream())

        def rc():
            _abi.call('rod_dw3x3_fwd_rc', x, *ops._pro_args(xpro), wt0, Cin, *ops._pro_args(epro), wd, y1, p1, N, H, W,
                      C, s, pt, pl, Ho, Wo, code, ops.stream())
        t0, t1 = timeit(stored), timeit(rc)
        ok = torch.equal(y0, y1) and torch.equal(p0, p1)
        print('%-16s dwfwd stored %7.1f us   rc %7.1f us   equal %s' % (name, t0, t1, ok), flush=True)
        if s == 2 and _abi.lib().rod_dw3x3_bwd_fused_rc_supported(N, H, W, C, Cin, s, pt, pl, code):
            dz = torch.randn(N, Ho, Wo, C, generator=g).to(dev, bf16)
            dm, dr = y0.float().mean((0, 1, 2)), torch.rsqrt(y0.float().var((0, 1, 2)) + 1e-3)
            dg, db = (torch.rand(C, generator=g) + 0.5).to(dev), (torch.randn(C, generator=g) * 0.3).to(dev)
            coef = ops.bn_bwd_reduce(dz, y0, dm, dr, dg, db, ops.ROD_ACT_RELU6, False, False)
            nb = _abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, 2, pt, pl)
            ws = ops.workspace(_abi.query('rod_dw3x3_bwd_fused_workspace', N, H, W, C, 2, pt, pl), dev)
            dx0, dx1 = torch.empty_like(ye), torch.empty_like(ye)
            dw0, dw1 = torch.zeros(3, 3, C, device=dev), torch.zeros(3, 3, C, device=dev)
            g0, g1 = torch.empty((nb, 2, C), device=dev), torch.empty((nb, 2, C), device=dev)

            def bstored():
                _abi.call('rod_dw3x3_bwd_fused', ye, *ops._pro_args(epro), dz, y0, dm, dr, dg, db, ops.ROD_ACT_RELU6,
                          coef, wd, dx0, dw0, g0, ws, N, H, W, C, 2, pt, pl, Ho, Wo, code, ops.stream())

            def brc():
                _abi.call('rod_dw3x3_bwd_fused_rc', x, *ops._pro_args(xpro), wt0, Cin, *ops._pro_args(epro), dz, y0,
                          dm, dr, dg, db, ops.ROD_ACT_RELU6, coef, wd, dx1, dw1, g1, ws, N, H, W, C, 2, pt, pl, Ho, Wo,
                          code, ops.stream())
            t2, t3 = timeit(bstored), timeit(brc)
            ok = torch.equal(dx0, dx1) and torch.equal(dw0, dw1) and torch.equal(g0, g1)
            print('%-16s dwbwd stored %7.1f us   rc %7.1f us   equal %s' % (name, t2, t3, ok), flush=True)
        del ye


if __name__ == '__main__':
    main()

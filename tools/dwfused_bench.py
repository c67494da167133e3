"""Depthwise backward (stride 1 and 2) at the 720x1280 b8 step's shapes: the unfused chain
(rod_bn_bwd_apply -> rod_dw3x3_bwd_data -> rod_dw3x3_bwd_filter -> the input BatchNorm's
rod_bn_bwd_reduce) against rod_dw3x3_bwd_fused (+ rod_bn_bwd_finalize of its sums).  HIP-event
timed on the launching stream; GB/s = the fused kernel's algorithmic bytes (read ye, dz, yd;
write dx) over each path's time.  Stride-1 bf16 shapes of the inverted-residual blocks also time
rod_dw3x3_bwd_fused_pw (ABI 20: dz recomputed from the cout-wide dy_p, the block's project width).
usage: python tools/dwfused_bench.py [--iters N] [--dtype bf16|f32]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'road-object-detection-for-bdd100k_amd'))
from rod import _abi, ops  # noqa: E402

PW_COUT = {32: 16, 144: 24, 192: 32}   # project width of the block whose depthwise has C channels
SHAPES = [(8, 720, 1280, 32, 1), (8, 360, 640, 144, 1), (8, 180, 320, 192, 1), (8, 90, 160, 384, 1),
          (8, 90, 160, 576, 1), (8, 45, 80, 960, 1), (8, 23, 40, 960, 1),
          # the stride-2 blocks (input maps)
          (8, 720, 1280, 96, 2), (8, 360, 640, 144, 2), (8, 180, 320, 192, 2), (8, 90, 160, 576, 2)]


def _same(n, s):
    o = -(-n // s)
    return o, max((o - 1) * s + 3 - n, 0) // 2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--dtype', default='bf16')
    a = ap.parse_args()
    dev = 'cuda'
    dt = torch.bfloat16 if a.dtype == 'bf16' else torch.float32
    g = torch.Generator(device=dev).manual_seed(0)
    st = ops.stream()
    act = ops.ROD_ACT_RELU6
    tu = tf = tp = 0.0
    for (N, H, W, C, S) in SHAPES:
        (Ho, pt), (Wo, pl) = _same(H, S), _same(W, S)
        M, Mo = N * H * W, N * Ho * Wo
        mk = lambda shp, s=1.0, o=0.0: (torch.randn(shp, device=dev, generator=g) * s + o).to(dt)
        ye, yd, dz = mk((N, H, W, C), 1.3, 0.2), mk((N, Ho, Wo, C), 2, 0.4), mk((N, Ho, Wo, C))
        w = torch.randn((3, 3, C), device=dev, generator=g) * 0.4
        vec = lambda lo=0.5: torch.rand(C, device=dev, generator=g) + lo
        dmean, drstd, dgam, dbet = torch.randn(C, device=dev, generator=g) * 0.3, vec(), vec(), torch.randn(C, device=dev, generator=g)
        emean, erstd, egam, ebet = torch.randn(C, device=dev, generator=g) * 0.1, vec(), vec(), torch.randn(C, device=dev, generator=g) * 0.1
        code = ops.dtcode(ye)
        coef = torch.empty(3 * C, device=dev)
        rws = ops.workspace(_abi.query('rod_bn_bwd_workspace', M, C), dev)
        _abi.call('rod_bn_bwd_reduce', dz, yd, dmean, drstd, dgam, dbet, None, None, coef, rws, Mo, C, act, code, st)
        dy, dx = torch.empty_like(yd), torch.empty_like(ye)
        dw = torch.empty(3, 3, C, device=dev)
        fws = ops.workspace(_abi.query('rod_dw3x3_bwd_filter_workspace', N, Ho, Wo, C), dev)
        ce, dg, db = torch.empty(3 * C, device=dev), torch.empty(C, device=dev), torch.empty(C, device=dev)
        nparts = _abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, S, pt, pl)
        gparts = torch.empty((nparts, 2, C), device=dev)
        ws = ops.workspace(_abi.query('rod_dw3x3_bwd_fused_workspace', N, H, W, C, S, pt, pl), dev)

        def unfused():
            _abi.call('rod_bn_bwd_apply', dz, yd, dmean, drstd, dgam, dbet, coef, dy, Mo, C, act, code, st)
            _abi.call('rod_dw3x3_bwd_data', dy, w, dx, None, None, None, None, None, 0, None, N, H, W, C, S, pt, pl,
                      Ho, Wo, code, st)
            _abi.call('rod_dw3x3_bwd_filter', ye, emean, erstd, egam, ebet, act, dy, dw, fws, N, H, W, C, S, pt, pl,
                      Ho, Wo, code, st)
            _abi.call('rod_bn_bwd_reduce', dx, ye, emean, erstd, egam, ebet, dg, db, ce, rws, M, C, act, code, st)

        def fused():
            _abi.call('rod_dw3x3_bwd_fused', ye, emean, erstd, egam, ebet, act, dz, yd, dmean, drstd, dgam, dbet, act,
                      coef, w, dx, dw, gparts, ws, N, H, W, C, S, pt, pl, Ho, Wo, code, st)
            _abi.call('rod_bn_bwd_finalize', gparts, nparts, M, C, erstd, egam, dg, db, ce, st)

        cout = PW_COUT.get(C)
        pw_ok = S == 1 and cout is not None and \
            _abi.lib().rod_dw3x3_bwd_fused_pw_supported(N, H, W, C, cout, act, act, ops.dtcode(ye))
        if pw_ok:
            dyp = mk((M, cout))
            wt1 = (torch.randn((C, cout), device=dev, generator=g) * 0.2).to(dt)

        def fused_pw():
            _abi.call('rod_dw3x3_bwd_fused_pw', ye, emean, erstd, egam, ebet, act, dyp, wt1, cout, yd, dmean, drstd, dgam,
                      dbet, act, coef, w, dx, dw, gparts, ws, N, H, W, C, code, st)
            _abi.call('rod_bn_bwd_finalize', gparts, nparts, M, C, erstd, egam, dg, db, ce, st)

        res = []
        for fn in (unfused, fused) + ((fused_pw,) if pw_ok else ()):
            for _ in range(3):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / a.iters * 1e3)
        byts = 2 * (M + Mo) * C * ye.element_size()
        tu += res[0]
        tf += res[1]
        tp += res[2] if pw_ok else res[1]
        pws = f'  fused_pw {res[2]:8.1f} us ({byts / res[2] / 1e3:5.0f} GB/s)' if pw_ok else ''
        print(f'{N}x{H}x{W}x{C:<5d} s{S} unfused {res[0]:8.1f} us  fused {res[1]:8.1f} us  x{res[0] / res[1]:5.2f}  '
              f'fused-bytes GB/s: unfused {byts / res[0] / 1e3:7.0f} fused {byts / res[1] / 1e3:7.0f}{pws}', flush=True)
    print(f'TOTAL unfused {tu:.1f} us fused {tf:.1f} us  (fused_pw where supported) {tp:.1f} us')


if __name__ == '__main__':
    main()

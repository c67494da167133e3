"""rod_dw3x3_bwd_fused against a float64 restatement at the step's largest stride-2 shape
(8 x 720 x 1280 x 96 -> 360 x 640: L3's depthwise, ref conv_blocks.py:238-247 backward with the
BatchNorm backward of mobilenet.py:417-420 on both sides).

The float64 chain follows the product's storage points: x = bf16(act_e(BN_e(ye))) (the forward
input the product convolves), dy = bf16(BN_d backward apply of (dz, yd)) with the coefficients
formed in float64 from the same (dz, yd); then dx = DepthwiseConv2dNativeBackpropInput(dy, w),
dw = DepthwiseConv2dNativeBackpropFilter(x, dy) and the BN_e backward sums over (dx, ye) in
float64.  Bars (written here, measured values printed):
  dx  : max |dx - dx64| <= 2^-7 * max |dx64|   (bf16 output; a dy element whose rounding flips
                                                between the f32 and f64 coefficients moves it by
                                                one bf16 ulp)
  dw  : normwise 1e-4                          (fp32 accumulation of 16.6 M products per tap)
  sums: normwise 1e-4 against float64 sums over the kernel's own dx
"""
import json
import os

import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out')


def _relu6(z):
    return z.clamp(0.0, 6.0)


def test_fused_stride2_720p_vs_float64(dev):
    N, H, W, C, S = 8, 720, 1280, 96, 2
    Ho, Wo, pt, pl = 360, 640, 0, 0          # TF SAME, even sides: pad (0, 1)
    g = torch.Generator(device=dev).manual_seed(720)
    bf = torch.bfloat16
    ye = (torch.randn(N, H, W, C, device=dev, generator=g) * 1.3 + 0.2).to(bf)
    yd = (torch.randn(N, Ho, Wo, C, device=dev, generator=g) * 2 + 0.4).to(bf)
    dz = (torch.randn(N, Ho, Wo, C, device=dev, generator=g) * 1e-3).to(bf)
    w = torch.randn(3, 3, C, device=dev, generator=g) * 0.4
    u = lambda lo=0.5: torch.rand(C, device=dev, generator=g) + lo
    dmean, drstd, dgam, dbet = torch.randn(C, device=dev, generator=g) * 0.3, u(), u(), torch.randn(C, device=dev, generator=g)
    emean, erstd, egam, ebet = torch.randn(C, device=dev, generator=g) * 0.1, u(), u(), torch.randn(C, device=dev, generator=g) * 0.1
    act = ops.ROD_ACT_RELU6
    M, Mo, st, code = N * H * W, N * Ho * Wo, ops.stream(), ops.dtcode(ye)
    coef = torch.empty(3 * C, device=dev)
    rws = ops.workspace(_abi.query('rod_bn_bwd_workspace', M, C), dev)
    _abi.call('rod_bn_bwd_reduce', dz, yd, dmean, drstd, dgam, dbet, None, None, coef, rws, Mo, C, act, code, st)
    nparts = _abi.lib().rod_dw3x3_bwd_fused_parts(N, H, W, C, S, pt, pl)
    gparts = torch.empty((nparts, 2, C), device=dev)
    dx = torch.empty_like(ye)
    dw = torch.empty(3, 3, C, device=dev)
    ws = ops.workspace(_abi.query('rod_dw3x3_bwd_fused_workspace', N, H, W, C, S, pt, pl), dev)
    _abi.call('rod_dw3x3_bwd_fused', ye, emean, erstd, egam, ebet, act, dz, yd, dmean, drstd, dgam, dbet, act, coef, w,
              dx, dw, gparts, ws, N, H, W, C, S, pt, pl, Ho, Wo, code, st)
    torch.cuda.synchronize()
    d64 = torch.float64
    # ---- float64 restatement
    # BN_d backward coefficients over (dz, yd): g = dz * relu6'(z), z = BN_d(yd)
    yd64 = yd.to(d64)
    scd = drstd.to(d64) * dgam.to(d64)
    zd = yd64 * scd + (dbet.to(d64) - dmean.to(d64) * scd)
    gd = dz.to(d64) * ((zd > 0) & (zd < 6)).to(d64)
    del zd
    yhat = (yd64 - dmean.to(d64)) * drstd.to(d64)
    del yd64
    mg = gd.mean((0, 1, 2))
    mx = (gd * yhat).mean((0, 1, 2))
    dy = (scd * (gd - mg - yhat * mx)).to(bf).to(d64)      # rounded as the product stores dy
    del gd, yhat
    # x = bf16(relu6(BN_e(ye))), zero padded (bottom / right for even sides)
    sce = erstd.to(d64) * egam.to(d64)
    xe = _relu6(ye.to(d64) * sce + (ebet.to(d64) - emean.to(d64) * sce)).to(bf).to(d64)
    xp = torch.zeros(N, H + 2, W + 2, C, dtype=d64, device=dev)
    xp[:, pt:pt + H, pl:pl + W] = xe
    del xe
    dx64 = torch.zeros(N, H + 2, W + 2, C, dtype=d64, device=dev)
    dw64 = torch.empty(3, 3, C, dtype=d64, device=dev)
    for i in range(3):
        for j in range(3):
            win = xp[:, i:i + 2 * Ho:2, j:j + 2 * Wo:2]
            dw64[i, j] = (dy * win).sum((0, 1, 2))
            dx64[:, i:i + 2 * Ho:2, j:j + 2 * Wo:2] += dy * w[i, j].to(d64)
    del xp, dy
    dx64 = dx64[:, pt:pt + H, pl:pl + W]
    ex = float((dx.to(d64) - dx64).abs().max() / dx64.abs().max())
    ew = float((dw.to(d64) - dw64).abs().max() / dw64.abs().max())
    del dx64
    # BN_e backward sums over (dx, ye) in float64 from the kernel's own dx
    ze = ye.to(d64) * sce + (ebet.to(d64) - emean.to(d64) * sce)
    ge = dx.to(d64) * ((ze > 0) & (ze < 6)).to(d64)
    del ze
    s_g = ge.sum((0, 1, 2))
    s_gx = (ge * ((ye.to(d64) - emean.to(d64)) * erstd.to(d64))).sum((0, 1, 2))
    del ge
    p64 = gparts.to(d64).sum(0)
    es = max(float((p64[0] - s_g).abs().max() / s_g.abs().max()), float((p64[1] - s_gx).abs().max() / s_gx.abs().max()))
    rec = {'shape': [N, H, W, C, S], 'dx_err': ex, 'dw_err': ew, 'bn_e_sums_err': es,
           'bars': {'dx': 2 ** -7, 'dw': 1e-4, 'sums': 1e-4}}
    print(rec)
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, 'dwfused_oracle_720p_s2.json'), 'w') as f:
        json.dump(rec, f)
    assert ex <= 2 ** -7, rec
    assert ew <= 1e-4, rec
    assert es <= 1e-4, rec

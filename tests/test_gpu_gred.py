"""BatchNorm-backward reduction fused into the backward-data epilogues ("gred", ABI 4):
rod_dw3x3_bwd_data / rod_conv_fwd (mode-1 weights) write dz and the partial sums
(sum g, sum g*yhat) of the BatchNorm whose output the forward read through its prologue;
rod_bn_bwd_finalize merges them.  Checked against float64 sums of the same dz and y
(the reduction of FusedBatchNormGrad, reference mobilenet.py:417 / catch_net.py:302)."""
import numpy as np
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu


def _ref_sums(dz, y, mean, rstd, gamma, beta, act):
    dz, y = dz.double().cpu(), y.double().cpu()
    m, r = mean.double().cpu(), rstd.double().cpu()
    ga = gamma.double().cpu() if gamma is not None else torch.ones_like(m)
    be = beta.double().cpu() if beta is not None else torch.zeros_like(m)
    sc = (rstd.cpu() * (gamma.cpu() if gamma is not None else 1.0)).double()
    sh = be - m * sc
    u = y * sc + sh
    if act == ops.ROD_ACT_RELU6:
        d = ((u > 0) & (u < 6)).double()
    elif act == ops.ROD_ACT_LEAKY:
        d = torch.where(u > 0, 1.0, 0.2).double()
    else:
        d = torch.ones_like(u)
    g = dz * d
    C = y.shape[-1]
    return g.reshape(-1, C).sum(0), (g * (y - m) * r).reshape(-1, C).sum(0)


def _bn(dev, C, seed, gamma=True):
    g = torch.Generator().manual_seed(seed)
    mean = (torch.randn(C, generator=g) * 0.3).to(dev)
    rstd = (torch.rand(C, generator=g) + 0.5).to(dev)
    ga = (torch.rand(C, generator=g) + 0.5).to(dev) if gamma else None
    be = (torch.randn(C, generator=g) * 0.3).to(dev)
    return mean, rstd, ga, be


def _finalize(parts, M, C, rstd, gamma, dev):
    dg = torch.empty(C, device=dev)
    db = torch.empty(C, device=dev)
    coef = torch.empty(3 * C, device=dev)
    _abi.call('rod_bn_bwd_finalize', parts, parts.shape[0], M, C, rstd, gamma, dg, db, coef, ops.stream())
    return db, dg


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('C,stride,H,W', [(96, 2, 45, 81), (144, 1, 23, 40), (32, 1, 30, 44), (24, 2, 12, 16),
                                          (6, 2, 13, 17), (6, 1, 9, 11), (960, 1, 3, 5)])
def test_dw_bwd_data_gred(dev, dtype, C, stride, H, W):
    g = torch.Generator().manual_seed(21)
    N = 2
    Ho, pt = ops.same_pad(H, stride)
    Wo, pl = ops.same_pad(W, stride)
    y = (torch.randn(N, H, W, C, generator=g) * 2 + 0.5).to(dev, dtype)
    dy = torch.randn(N, Ho, Wo, C, generator=g).to(dev, dtype)
    w = (torch.randn(3, 3, C, generator=g) * 0.3).to(dev)
    mean, rstd, ga, be = _bn(dev, C, 22)
    dt = ops.dtcode(y)
    nparts = _abi.lib().rod_dw3x3_bwd_data_gred_parts(N, H, W, C, stride, dt)
    parts = torch.full((nparts, 2, C), float('nan'), device=dev)
    dx = torch.empty_like(y)
    _abi.call('rod_dw3x3_bwd_data', dy, w, dx, y, mean, rstd, ga, be, ops.ROD_ACT_RELU6, parts, N, H, W, C, stride,
              pt, pl, Ho, Wo, dt, ops.stream())
    dx_plain = torch.empty_like(y)
    _abi.call('rod_dw3x3_bwd_data', dy, w, dx_plain, None, None, None, None, None, 0, None, N, H, W, C, stride, pt,
              pl, Ho, Wo, dt, ops.stream())
    assert torch.equal(dx, dx_plain)          # the epilogue does not change dz
    assert not torch.isnan(parts).any()       # every part written
    sg, sgx = _ref_sums(dx, y, mean, rstd, ga, be, ops.ROD_ACT_RELU6)
    db, dg = _finalize(parts, N * H * W, C, rstd, ga, dev)
    scale = float(np.sqrt(N * H * W))
    torch.testing.assert_close(db.double().cpu(), sg, rtol=1e-4, atol=1e-5 * scale)
    torch.testing.assert_close(dg.double().cpu(), sgx, rtol=1e-4, atol=1e-5 * scale)


@pytest.mark.parametrize('dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('ks,Cdz,Cy,NHW,act', [(1, 24, 144, (2, 23, 40), ops.ROD_ACT_RELU6),
                                              (1, 160, 960, (2, 3, 5), ops.ROD_ACT_RELU6),
                                              (3, 128, 128, (2, 10, 18), ops.ROD_ACT_LEAKY),
                                              (3, 36, 36, (2, 10, 18), ops.ROD_ACT_LEAKY),
                                              (1, 36, 128, (2, 7, 9), ops.ROD_ACT_LEAKY),
                                              # streaming kernel (pw_stream_kernel, ABI 14): M >= 65536, not a
                                              # multiple of the 128-row part; N groups of 48 / 32 / 64
                                              (1, 24, 144, (2, 181, 321), ops.ROD_ACT_RELU6),
                                              (1, 16, 32, (1, 257, 259), ops.ROD_ACT_RELU6),
                                              (1, 32, 192, (2, 181, 183), ops.ROD_ACT_RELU6),
                                              (1, 64, 384, (1, 257, 257), ops.ROD_ACT_RELU6),
                                              (1, 96, 576, (1, 256, 257), ops.ROD_ACT_LEAKY)])
def test_conv_bwd_data_gred(dev, dtype, ks, Cdz, Cy, NHW, act):
    """rod_conv_fwd(dz_out, wt mode 1) as the backward-data of a conv Cy -> Cdz."""
    g = torch.Generator().manual_seed(23)
    N, H, W = NHW
    M = N * H * W
    y = (torch.randn(N, H, W, Cy, generator=g) * 2 + 0.5).to(dev, dtype)
    dout = torch.randn(N, H, W, Cdz, generator=g).to(dev, dtype)
    wmaster = (torch.randn(Cdz, ks, ks, Cy, generator=g) / np.sqrt(ks * ks * Cy)).to(dev)
    dt = ops.dtcode(y)
    wt1 = torch.empty((Cy, ks * ks * Cdz), dtype=dtype, device=dev)
    _abi.call('rod_conv_weight_prep', wmaster, wt1, Cdz, Cy, ks, 1, dt, ops.stream())
    mean, rstd, ga, be = _bn(dev, Cy, 24, gamma=act == ops.ROD_ACT_RELU6)
    parts = torch.full((-(-M // 128), 2, Cy), float('nan'), device=dev)
    dx = torch.empty_like(y)
    ops.conv_fwd_raw(dout, wt1, None, dx, N, H, W, Cdz, Cy, ks, gred=(y, mean, rstd, ga, be, act, parts))
    dx_plain = torch.empty_like(y)
    ops.conv_fwd_raw(dout, wt1, None, dx_plain, N, H, W, Cdz, Cy, ks)
    assert torch.equal(dx, dx_plain)
    assert not torch.isnan(parts).any()
    sg, sgx = _ref_sums(dx, y, mean, rstd, ga, be, act)
    db, dg = _finalize(parts, M, Cy, rstd, ga, dev)
    scale = float(np.sqrt(M))
    torch.testing.assert_close(db.double().cpu(), sg, rtol=1e-4, atol=1e-5 * scale)
    torch.testing.assert_close(dg.double().cpu(), sgx, rtol=1e-4, atol=1e-5 * scale)

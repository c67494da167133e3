"""rod_pw_bwd (fused 1x1-conv + BatchNorm backward) against the unfused librod chain it
replaces — rod_bn_bwd_reduce -> rod_bn_bwd_apply (dy written) -> rod_conv_fwd with the mode-1
weights (dx) -> rod_conv_wgrad (dw, db) — and against a float64 restatement of the same
backward (TF FusedBatchNormGrad + Conv2DBackpropInput / Filter semantics).

dy is formed with rod_bn_bwd_apply's arithmetic and rounded the same way, and dx = dy.W runs
the same MFMA k order as the unfused backward-data GEMM, so dx is bit-identical; dw / db sum
the rows in a different order (fp32 partials, f64 slab sum): within 1e-5 normwise."""
import numpy as np
import pytest
import torch

from rod import ops

pytestmark = pytest.mark.gpu
bf16 = torch.bfloat16

SHAPES = [  # (M, Cin, Cout, act, pro_x, bias)
    (4096 + 37, 24, 144, ops.ROD_ACT_RELU6, True, False),     # project 144->24's consumer side: expand 24->144
    (3000, 16, 96, ops.ROD_ACT_RELU6, False, False),          # L3 expand
    (700, 32, 192, ops.ROD_ACT_RELU6, True, False),           # L5 expand (streaming kernel, ragged tail)
    (31, 16, 96, ops.ROD_ACT_RELU6, True, False),             # fewer rows than one streaming tile
    (1111, 144, 24, ops.ROD_ACT_NONE, True, False),           # project (linear BN)
    (777, 64, 128, ops.ROD_ACT_LEAKY, False, True),           # head 1x1 (bias + BN beta only)
    (5000, 192, 32, ops.ROD_ACT_NONE, True, False),           # project 192->32
    (64, 32, 16, ops.ROD_ACT_NONE, True, False),              # one step exactly
    (130, 96, 128, ops.ROD_ACT_LEAKY, True, True),
    (2049, 128, 24, ops.ROD_ACT_LEAKY, True, True),           # head 128->24
]


def _nerr(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize('M,Cin,Cout,act,prox,bias', SHAPES)
def test_pw_bwd_matches_unfused_chain(dev, M, Cin, Cout, act, prox, bias):
    assert ops.pw_bwd_supported(Cin, Cout, bf16)
    g = torch.Generator().manual_seed(M + Cin * 7 + Cout)
    x = (torch.randn(M, Cin, generator=g) * 1.5 + 0.3).to(dev, bf16)
    y = (torch.randn(M, Cout, generator=g) * 2 + 0.5).to(dev, bf16)
    dz = torch.randn(M, Cout, generator=g).to(dev, bf16)
    w = (torch.randn(Cout, 1, 1, Cin, generator=g) * 0.2).to(dev)
    mean = y.float().mean(0)
    rstd = torch.rsqrt(y.float().var(0, unbiased=False) + 1e-3)
    gamma = (torch.rand(Cout, generator=g) + 0.5).to(dev) if act != ops.ROD_ACT_LEAKY else None
    beta = (torch.randn(Cout, generator=g) * 0.3).to(dev)
    xpro = None
    if prox:
        xm = (torch.randn(Cin, generator=g) * 0.2).to(dev)
        xr = (torch.rand(Cin, generator=g) + 0.5).to(dev)
        xpro = (xm, xr, (torch.rand(Cin, generator=g) + 0.5).to(dev), (torch.randn(Cin, generator=g) * 0.2).to(dev),
                ops.ROD_ACT_RELU6)
    coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)
    wt1 = ops._prep(w, 1, bf16, Cout, Cin, 1)
    # unfused
    dy = torch.empty_like(y)
    ops._abi.call('rod_bn_bwd_apply', dz, y, mean, rstd, gamma, beta, coef, dy, M, Cout, act, ops.dtcode(y),
                  ops.stream())
    dx_ref = torch.empty_like(x)
    ops.conv_fwd_raw(dy, wt1, None, dx_ref, 1, 1, M, Cout, Cin, 1)
    dw_ref = torch.empty(Cout, Cin, device=dev)
    db_ref = torch.empty(Cout, device=dev) if bias else None
    wsz = ops._abi.query('rod_conv_wgrad_workspace', 1, 1, M, Cin, Cout, 1)
    ops._abi.call('rod_conv_wgrad', x, *ops._pro_args(xpro), dy, dw_ref, db_ref, ops.workspace(wsz, dev), 1, 1, M, Cin,
                  Cout, 1, 0, 0, ops.dtcode(x), ops.stream())
    # fused
    dw = torch.full((Cout, Cin), float('nan'), device=dev)
    db = torch.full((Cout,), float('nan'), device=dev) if bias else None
    dx = ops.pw_bwd(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, True, dw, db)
    assert torch.equal(dx, dx_ref), _nerr(dx.float(), dx_ref.float())
    assert _nerr(dw, dw_ref) < 1e-5, _nerr(dw, dw_ref)
    if bias:
        assert _nerr(db, db_ref) < 1e-5
    # without dx (frozen input): same dw
    dw2 = torch.empty_like(dw)
    assert ops.pw_bwd(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, False, dw2, None) is None
    assert torch.equal(dw2, dw)
    # float64 restatement of the whole backward on the same bf16 inputs
    yd, dzd, xd = y.double(), dz.double(), x.double()
    sc = rstd.double() * (gamma.double() if gamma is not None else 1.0)
    z = (yd - mean.double()) * sc + beta.double()
    if act == ops.ROD_ACT_RELU6:
        gg = dzd * ((z > 0) & (z < 6))
    elif act == ops.ROD_ACT_LEAKY:
        gg = dzd * torch.where(z > 0, 1.0, 0.2)
    else:
        gg = dzd
    yh = (yd - mean.double()) * rstd.double()
    dy64 = sc * (gg - gg.mean(0) - yh * (gg * yh).mean(0))
    a64 = xd
    if prox:
        xs = xpro[1].double() * xpro[2].double()
        a64 = torch.clamp(xd * xs + (xpro[3].double() - xpro[0].double() * xs), 0, 6)
    assert _nerr(dw, dy64.t() @ a64) < 2e-2          # bf16 operands (dy rounded, a rounded)
    assert _nerr(dx.float(), dy64 @ w.double().reshape(Cout, Cin)) < 2e-2


def test_pw_bwd_rejects_unsupported(dev):
    assert not ops.pw_bwd_supported(24, 36, bf16)        # Cout % 8
    assert not ops.pw_bwd_supported(320, 128, bf16)      # too many dW tiles
    assert not ops.pw_bwd_supported(24, 144, torch.float32)


def test_pw_bwd_full_size_expand_vs_float64(dev):
    """rod_pw_bwd at the step's largest expand (L3: 8 x 720 x 1280 = 7,372,800 rows, 16 -> 96,
    ReLU6 BatchNorm, the input through its linear BatchNorm prologue) against a float64
    restatement that keeps the product's two storage points (dy and the prologue output a,
    both bf16).  Bars: dw normwise 1e-4 (fp32 partials over 7.4 M rows, f64 slab sum), dx
    max |err| <= 2^-7 max |dx64| (bf16 output; a dy element whose rounding flips between the f32
    and f64 coefficients moves it by one bf16 ulp).  Measured values printed and written to
    gpurun_out/parity_errors.json."""
    import json
    import os
    M, Cin, Cout, act = 8 * 720 * 1280, 16, 96, ops.ROD_ACT_RELU6
    g = torch.Generator(device=dev).manual_seed(96)
    x = (torch.randn(M, Cin, device=dev, generator=g) * 1.5 + 0.3).to(bf16)
    y = (torch.randn(M, Cout, device=dev, generator=g) * 2 + 0.5).to(bf16)
    dz = (torch.randn(M, Cout, device=dev, generator=g) * 1e-3).to(bf16)
    w = torch.randn(Cout, 1, 1, Cin, device=dev, generator=g) * 0.2
    mean = y.float().mean(0)
    rstd = torch.rsqrt(y.float().var(0, unbiased=False) + 1e-3)
    gamma = torch.rand(Cout, device=dev, generator=g) + 0.5
    beta = torch.randn(Cout, device=dev, generator=g) * 0.3
    xpro = (torch.randn(Cin, device=dev, generator=g) * 0.2, torch.rand(Cin, device=dev, generator=g) + 0.5,
            torch.rand(Cin, device=dev, generator=g) + 0.5, torch.randn(Cin, device=dev, generator=g) * 0.2,
            ops.ROD_ACT_NONE)
    coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)
    wt1 = ops._prep(w, 1, bf16, Cout, Cin, 1)
    dw = torch.empty(Cout, Cin, device=dev)
    dx = ops.pw_bwd(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, True, dw, None)
    torch.cuda.synchronize()
    d64 = torch.float64
    sc = rstd.double() * gamma.double()
    yd = y.double()
    z = yd * sc + (beta.double() - mean.double() * sc)
    gg = dz.double() * ((z > 0) & (z < 6))
    del z
    yh = (yd - mean.double()) * rstd.double()
    del yd
    dy = (sc * (gg - gg.mean(0) - yh * (gg * yh).mean(0))).to(bf16).to(d64)
    del gg, yh
    xs = xpro[1].double() * xpro[2].double()
    a = (x.double() * xs + (xpro[3].double() - xpro[0].double() * xs)).to(bf16).to(d64)
    dw64 = dy.t() @ a
    del a
    dx64 = dy @ wt1.double().t() if wt1.shape == (Cin, Cout) else dy @ w.double().reshape(Cout, Cin).to(bf16).to(d64)
    ew = float((dw.double() - dw64).abs().max() / dw64.abs().max())
    ex = float((dx.double() - dx64).abs().max() / dx64.abs().max())
    rec = {'M': M, 'Cin': Cin, 'Cout': Cout, 'dw_err': ew, 'dx_err': ex, 'bars': {'dw': 1e-4, 'dx': 2 ** -7}}
    print(rec)
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'gpurun_out',
                        'parity_errors.json')
    os.makedirs(os.path.dirname(path), exist_ok=True)
    d = json.load(open(path)) if os.path.exists(path) else {}
    d['pw_bwd_expand_7372800x16x96'] = rec
    with open(path, 'w') as f:
        json.dump(d, f, indent=1)
    assert ew <= 1e-4, rec
    assert ex <= 2 ** -7, rec


GRED_SHAPES = [  # (M, Cin, Cout, act of the output BatchNorm): project convs of the blocks
    (70000, 32, 16, ops.ROD_ACT_NONE),      # block 1 (32 -> 16), NW = 32
    (3000 + 17, 96, 24, ops.ROD_ACT_NONE),  # stride-2 block's project, 2 groups of 48
    (5000, 144, 24, ops.ROD_ACT_NONE),      # 3 groups, ragged tail
    (4100, 192, 32, ops.ROD_ACT_NONE),
    (2000, 384, 64, ops.ROD_ACT_NONE),      # 8 groups, Cout 64 (KT = 2)
    (33, 48, 16, ops.ROD_ACT_LEAKY),        # fewer rows than one tile
    (70000, 16, 96, ops.ROD_ACT_RELU6),     # expand 16 -> 96: the streaming kernel with the input sums
    (1000 + 7, 16, 96, ops.ROD_ACT_RELU6),  # ragged tail
]


@pytest.mark.parametrize('M,Cin,Cout,act', GRED_SHAPES)
def test_pw_bwd_gred_matches_unfused_chain(dev, M, Cin, Cout, act):
    """rod_pw_bwd_gred against the unfused chain (rod_bn_bwd_apply -> backward-data -> rod_conv_wgrad)
    and the input BatchNorm's backward sums against a float64 reduction over the kernel's own dx:
    dx bit-identical, dw 1e-5, sums 1e-5 normwise."""
    nparts = ops.pw_bwd_gred_parts(M, Cin, Cout, bf16)
    assert nparts > 0
    g = torch.Generator().manual_seed(M + Cin * 5 + Cout)
    x = (torch.randn(M, Cin, generator=g) * 1.5 + 0.3).to(dev, bf16)
    y = (torch.randn(M, Cout, generator=g) * 2 + 0.5).to(dev, bf16)
    dz = torch.randn(M, Cout, generator=g).to(dev, bf16)
    w = (torch.randn(Cout, 1, 1, Cin, generator=g) * 0.2).to(dev)
    mean = y.float().mean(0)
    rstd = torch.rsqrt(y.float().var(0, unbiased=False) + 1e-3)
    gamma = (torch.rand(Cout, generator=g) + 0.5).to(dev)
    beta = (torch.randn(Cout, generator=g) * 0.3).to(dev)
    xm = x.float().mean(0) + (torch.randn(Cin, generator=g) * 0.05).to(dev)
    xr = (torch.rand(Cin, generator=g) + 0.5).to(dev)
    xpro = (xm, xr, (torch.rand(Cin, generator=g) + 0.5).to(dev), (torch.randn(Cin, generator=g) * 0.2).to(dev),
            ops.ROD_ACT_RELU6)
    coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)
    wt1 = ops._prep(w, 1, bf16, Cout, Cin, 1)
    dy = torch.empty_like(y)
    ops._abi.call('rod_bn_bwd_apply', dz, y, mean, rstd, gamma, beta, coef, dy, M, Cout, act, ops.dtcode(y),
                  ops.stream())
    dx_ref = torch.empty_like(x)
    ops.conv_fwd_raw(dy, wt1, None, dx_ref, 1, 1, M, Cout, Cin, 1)
    dw_ref = torch.empty(Cout, Cin, device=dev)
    wsz = ops._abi.query('rod_conv_wgrad_workspace', 1, 1, M, Cin, Cout, 1)
    ops._abi.call('rod_conv_wgrad', x, *ops._pro_args(xpro), dy, dw_ref, None, ops.workspace(wsz, dev), 1, 1, M, Cin,
                  Cout, 1, 0, 0, ops.dtcode(x), ops.stream())
    dw = torch.full((Cout, Cin), float('nan'), device=dev)
    dx, xparts = ops.pw_bwd_gred(dz, y, mean, rstd, gamma, beta, act, coef, x, xpro, wt1, dw)
    assert xparts.shape == (nparts, 2, Cin)
    assert torch.equal(dx, dx_ref), _nerr(dx.float(), dx_ref.float())
    assert _nerr(dw, dw_ref) < 1e-5, _nerr(dw, dw_ref)
    # the input BatchNorm's backward sums over (dx, x) in float64
    xd = x.double()
    xs = xr.double() * xpro[2].double()
    zx = xd * xs + (xpro[3].double() - xm.double() * xs)
    gx = dx.double() * ((zx > 0) & (zx < 6))
    s_g = gx.sum(0)
    s_gx = (gx * ((xd - xm.double()) * xr.double())).sum(0)
    p = xparts.double().sum(0)
    assert _nerr(p[0], s_g) < 1e-5, _nerr(p[0], s_g)
    assert _nerr(p[1], s_gx) < 1e-5, _nerr(p[1], s_gx)

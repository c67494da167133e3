"""Inference conv + BatchNorm-apply epilogue (ABI 21, rod_conv_fwd_bnact): bit-identical to
rod_conv_fwd followed by rod_bn_apply (slim.conv2d + slim.batch_norm(is_training=False) + act
(+ residual), mobilenet.py:417-420, catch_net.py:301-305) on every GEMM path it takes — the
LDS-staged epilogue (Cout % 8 == 0), the direct-store one (the heads' 4 / 11 x anchors outputs),
split-K with the combine kernel (small maps, deep K), the 3x3 implicit GEMM with an input
BatchNorm prologue — and the predict path with the epilogue on / off (ROD_DISABLE=bnepi)."""
import pytest
import torch

from rod import _abi, ops

pytestmark = pytest.mark.gpu
bf16 = torch.bfloat16

# (N, H, W, Cin, Cout, ksize, residual, prologue, act)
CASES = [
    (2, 45, 80, 144, 24, 1, True, True, ops.ROD_ACT_NONE),      # project + residual (VY epilogue)
    (2, 23, 40, 96, 160, 1, False, True, ops.ROD_ACT_NONE),     # project, no residual
    (2, 90, 160, 128, 24, 3, False, False, ops.ROD_ACT_LEAKY),  # head output 4 x 6 anchors (VY)
    (2, 90, 160, 128, 66, 3, False, False, ops.ROD_ACT_LEAKY),  # head output 11 x 6 (direct store)
    (2, 6, 10, 128, 66, 3, False, True, ops.ROD_ACT_LEAKY),     # small map: split-K + combine
    (2, 12, 20, 1280, 128, 1, False, False, ops.ROD_ACT_LEAKY), # deconv block_1 1x1 (split-K)
    (1, 37, 45, 64, 128, 3, False, True, ops.ROD_ACT_RELU6),    # 3x3 with the input prologue
]


@pytest.mark.parametrize('N,H,W,Cin,Cout,ks,res,pro,act', CASES)
def test_conv_bnact_matches_conv_then_bn_apply(dev, N, H, W, Cin, Cout, ks, res, pro, act):
    g = torch.Generator().manual_seed(N * 100 + H + Cin + Cout + ks)
    M = N * H * W
    x = (torch.randn(N, H, W, Cin, generator=g) * 1.2 + 0.1).to(dev, bf16)
    w = (torch.randn(Cout, ks, ks, Cin, generator=g) * 0.1).to(dev)
    b = (torch.randn(Cout, generator=g) * 0.1).to(dev)
    wt = ops._prep(w, 0, bf16, Cout, Cin, ks)
    ipro = None
    if pro:
        ipro = ((torch.randn(Cin, generator=g) * 0.2).to(dev), (torch.rand(Cin, generator=g) + 0.5).to(dev),
                (torch.rand(Cin, generator=g) + 0.5).to(dev), (torch.randn(Cin, generator=g) * 0.2).to(dev),
                ops.ROD_ACT_RELU6)
    mean = (torch.randn(Cout, generator=g) * 0.3).to(dev)
    rstd = (torch.rand(Cout, generator=g) + 0.5).to(dev)
    gamma = (torch.rand(Cout, generator=g) + 0.5).to(dev) if act == ops.ROD_ACT_NONE else None
    beta = (torch.randn(Cout, generator=g) * 0.2).to(dev)
    r = torch.randn(N, H, W, Cout, generator=g).to(dev, bf16) if res else None
    nb = _abi.query('rod_conv_fwd_workspace', N, H, W, Cin, Cout, ks)
    ws = ops.workspace(nb, dev) if nb else None
    y = torch.empty(N, H, W, Cout, dtype=bf16, device=dev)
    _abi.call('rod_conv_fwd', x, *ops._pro_args(ipro), wt, b, y, ws, None, *ops._gred_args(None), N, H, W, Cin, Cout,
              ks, 0, 0, ops.dtcode(x), ops.stream())
    ref = torch.empty_like(y)
    _abi.call('rod_bn_apply', y, mean, rstd, gamma, beta, r, ref, M, Cout, 0, 0, 0, act, ops.dtcode(y), ops.stream())
    z = torch.full_like(y, float('nan'))
    _abi.call('rod_conv_fwd_bnact', x, *ops._pro_args(ipro), wt, b, z, ws, mean, rstd, gamma, beta, act, r, 0, N, H, W,
              Cin, Cout, ks, 0, 0, ops.dtcode(x), ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(z, ref), float((z.float() - ref.float()).abs().max())


def test_predict_bnepi_bit_identical(dev):
    """The predict path (ALL network in eval, decode, NMS) with the epilogue and without it."""
    import predict
    from rod.data import synthetic_batch
    img = synthetic_batch(4, 160, 288, dev, seed=13)[0]
    outs = []
    for off in (True, False):
        if off:
            ops._DISABLE.add('bnepi')
        ops._DISABLE.add('cinpad')   # the padded head convs sum k in other chunks (test below)
        try:
            pr = predict.Predictor((160, 288), dev, bf16)
            _abi.PROBE.arm(['rod_conv_fwd_bnact', 'rod_bn_apply'])
            pr.use_graph = False
            scores, boxes = pr(img)
            torch.cuda.synchronize()
            calls = _abi.PROBE.table()
            _abi.PROBE.disarm()
            outs.append(({k: v.clone() for k, v in scores.items()}, {k: v.clone() for k, v in boxes.items()}, calls))
        finally:
            ops._DISABLE.discard('bnepi')
            ops._DISABLE.discard('cinpad')
    (s0, b0, c0), (s1, b1, c1) = outs
    assert 'rod_conv_fwd_bnact' not in c0 and c1['rod_conv_fwd_bnact'][0] >= 18, c1
    assert c1.get('rod_bn_apply', (0,))[0] < c0['rod_bn_apply'][0] - 18, (c0, c1)
    assert all(torch.equal(s0[k], s1[k]) for k in s0) and all(torch.equal(b0[k], b1[k]) for k in b0)


@pytest.mark.parametrize('N,H,W,C', [(8, 34, 60, 99), (2, 17, 30, 99), (4, 68, 120, 66), (3, 23, 41, 36)])
def test_head_conv_cinpad_matches(dev, N, H, W, C):
    """The heads' last 3x3 conv in inference (Cin = Cout = classes x anchors, not a multiple of 8)
    with its input and weights zero-padded to Cin rounded up to 8 (ops.conv2d_bn_act) against the
    unpadded conv (ROD_DISABLE=cinpad): the same products, the k sum in other chunks — within one
    bf16 rounding of each other, elementwise."""
    g = torch.Generator().manual_seed(N * H + C)
    x = (torch.randn(N, H, W, C, generator=g)).to(dev, bf16)
    w = (torch.randn(C, 3, 3, C, generator=g) / (9 * C) ** 0.5).to(dev)
    b = (torch.randn(C, generator=g) * 0.1).to(dev)
    im, ir = (torch.randn(C, generator=g) * 0.1).to(dev), (torch.rand(C, generator=g) + 0.5).to(dev)
    ib = (torch.randn(C, generator=g) * 0.1).to(dev)
    mm, mv = (torch.randn(C, generator=g) * 0.1).to(dev), (torch.rand(C, generator=g) + 0.5).to(dev)
    beta = (torch.randn(C, generator=g) * 0.1).to(dev)
    outs = []
    for off in (True, False):
        if off:
            ops._DISABLE.add('cinpad')
        try:
            with torch.no_grad():
                xp = ops.Pending(x, im, ir, None, ib, ops.ROD_ACT_LEAKY, False, owned=True)
                outs.append(ops.conv2d_bn_act(xp, w, b, 3, None, beta, mm, mv, ops.ROD_ACT_LEAKY, False, 0.997, 1e-3))
            torch.cuda.synchronize()
        finally:
            ops._DISABLE.discard('cinpad')
    z0, z1 = (o.float() for o in outs)
    assert torch.isfinite(z1).all()
    tol = z0.abs() * 2.0 ** -7 + 1e-3 * float(z0.abs().max())
    assert bool(((z0 - z1).abs() <= tol).all()), float((z0 - z1).abs().max())

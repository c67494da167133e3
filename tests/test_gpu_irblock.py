"""rod_ir_block_fwd — the fused inference inverted-residual block (N1, SURVEY §7 step 9,
ref conv_blocks.py:163-312) — against the unfused librod eval chain (expand conv ->
BatchNorm+ReLU6 prologue -> depthwise -> BatchNorm+ReLU6 prologue -> project conv ->
BatchNorm (+ residual)), and against the float64 oracle block.

Bar: the exact-rounding mode (ops.IR_EXACT) bit-identical to the unfused chain wherever that
chain's project conv runs without split-K (same roundings, same MFMA k order, same depthwise tap
order); otherwise (split-K sums its K slices in fp32 partials) within one bf16 rounding.  The
default single-rounding mode within bf16 accuracy of the exact mode and no less accurate against
the float64 oracle (normwise 3e-2)."""
import numpy as np
import pytest
import torch

from oracle import net as onet
from rod import ops

pytestmark = pytest.mark.gpu
bf16 = torch.bfloat16
EPS = 1e-3

BLOCKS = [  # (Cin, inner, Cout, stride, residual, H, W) — backbone blocks at small maps
    (16, 96, 24, 2, False, 37, 64),
    (24, 144, 24, 1, True, 45, 80),
    (24, 144, 32, 2, False, 45, 80),
    (32, 192, 32, 1, True, 23, 40),
    (32, 192, 64, 2, False, 24, 40),
    (64, 384, 64, 1, True, 12, 20),
    (64, 384, 96, 1, False, 12, 20),
    (96, 576, 96, 1, True, 15, 17),
    (96, 576, 160, 2, False, 12, 20),
    (160, 960, 160, 1, True, 6, 10),
]


def _bn(C, g, with_gamma=True):
    mm = torch.randn(C, generator=g) * 0.3
    mv = torch.rand(C, generator=g) * 1.5 + 0.3
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g) * 0.3
    return mm, mv, gamma, beta


@pytest.mark.parametrize('Cin,inner,Cout,s,res,H,W', BLOCKS)
def test_ir_block_matches_unfused_chain(dev, Cin, inner, Cout, s, res, H, W):
    assert ops.ir_block_supported(Cin, inner, Cout, s, res, bf16)
    g = torch.Generator().manual_seed(Cin * 1000 + inner + Cout + s)
    N = 2
    x = torch.randn(N, H, W, Cin, generator=g).to(dev, bf16)
    we = (torch.randn(inner, 1, 1, Cin, generator=g) * 0.2).to(dev)
    wd = (torch.randn(3, 3, inner, generator=g) * 0.3).to(dev)
    wp = (torch.randn(Cout, 1, 1, inner, generator=g) * 0.1).to(dev)
    bns = [[t.to(dev) for t in _bn(c, g)] for c in (inner, inner, Cout)]
    ev = [(*ops.eval_stats(mm, mv, EPS), ga, be) for (mm, mv, ga, be) in bns]
    with torch.no_grad():
        fast = ops.ir_block_fwd(x, we, ev[0], wd, ev[1], wp, ev[2], s, res)
        old = ops.ir_block_set_mode(ops.IR_PERSIST | ops.IR_EXACT)
        try:
            got = ops.ir_block_fwd(x, we, ev[0], wd, ev[1], wp, ev[2], s, res)
            ops.ir_block_set_mode(ops.IR_EXACT)     # one tile per workgroup: identical output
            tiled = ops.ir_block_fwd(x, we, ev[0], wd, ev[1], wp, ev[2], s, res)
            ops.ir_block_set_mode(0)
            fast_tiled = ops.ir_block_fwd(x, we, ev[0], wd, ev[1], wp, ev[2], s, res)
        finally:
            ops.ir_block_set_mode(old)
        assert torch.equal(got, tiled)
        assert torch.equal(fast, fast_tiled)
        (mme, mve, ge, be_), (mmd, mvd, gd, bd), (mmp, mvp, gp, bp) = bns
        pe = ops.conv2d_bn(x, we, None, 1, ge, be_, mme, mve, ops.ROD_ACT_RELU6, False, 0.997, EPS)
        pd = ops.dw3x3_bn(pe, wd, s, gd, bd, mmd, mvd, ops.ROD_ACT_RELU6, False, 0.997, EPS)
        pp = ops.conv2d_bn(pd, wp, None, 1, gp, bp, mmp, mvp, ops.ROD_ACT_NONE, False, 0.997, EPS)
        want = ops.materialize(pp, x if res else None)
    assert got.shape == want.shape == (N, -(-H // s), -(-W // s), Cout)
    Ho, Wo = got.shape[1], got.shape[2]
    split = ops._abi.query('rod_conv_fwd_workspace', N, Ho, Wo, inner, Cout, 1) > 0 or \
        ops._abi.query('rod_conv_fwd_workspace', N, H, W, Cin, inner, 1) > 0
    if not split:
        assert torch.equal(got, want), float((got.float() - want.float()).abs().max())
    else:
        torch.testing.assert_close(got.float(), want.float(), rtol=1e-2, atol=2e-2)
    # float64 oracle of the block (eval BatchNorm)
    xo = x.double().cpu().permute(0, 3, 1, 2)

    def bn(t, p):
        mm, mv, ga, be = (v.double().cpu() for v in p)
        return onet.batch_norm(t, ga, be, mm, mv, False, 0.997, EPS)
    e = onet.relu6(bn(onet.conv(xo, we.double().cpu()), bns[0]))
    d = onet.relu6(bn(onet.dwconv(e, wd.double().cpu(), s), bns[1]))
    o = bn(onet.conv(d, wp.double().cpu()), bns[2])
    if res:
        o = o + xo
    o = o.permute(0, 2, 3, 1)
    err = float((got.double().cpu() - o).abs().max() / o.abs().max())
    assert err < 3e-2, err
    # single-rounding mode: no less accurate than the exact one, within bf16 of it
    errf = float((fast.double().cpu() - o).abs().max() / o.abs().max())
    assert errf <= 1.25 * err + 1e-3, (errf, err)
    torch.testing.assert_close(fast.float(), got.float(), rtol=2e-2, atol=3e-2 * float(got.float().abs().max()))


def test_ir_block_rejects_unsupported(dev):
    assert not ops.ir_block_supported(320, 1920, 320, 1, True, bf16)   # Cin > 160
    assert not ops.ir_block_supported(160, 960, 320, 2, False, bf16)   # stride 2, Cin > 96
    assert not ops.ir_block_supported(24, 144, 32, 2, True, bf16)      # residual needs s1, Cin==Cout
    assert not ops.ir_block_supported(24, 144, 24, 1, True, torch.float32)


def test_backbone_eval_uses_fused_blocks_and_matches(dev):
    """The eval backbone with the fused blocks is as accurate as without them
    (ROD_DISABLE=irblock): both against the float64 oracle backbone (eval BatchNorm) at
    360x640.  (They do not agree bit for bit end to end: on the small deep maps the unfused
    chain splits K into fp32 partials, single bf16 roundings differ and propagate.)"""
    import config
    from nets.catch_net import CatchNet
    from rod.data import synthetic_batch
    cfg = {'train_range': config.train_range.REFINE, 'process_backbone_method': config.process_backbone_method.NONE,
           'deconv_method': config.deconv_method.LEARN_HALF, 'merge_method': config.merge_method.ADD}
    net = CatchNet('mobilenet_v2', cfg, dev, seed=3)
    img = synthetic_batch(2, 360, 640, dev, seed=4)[0]
    x = ops.normalize_image(img, bf16)
    net.calibrate_batchnorm(x)
    names = config.extract_feat_name['mobilenet_v2']
    with torch.no_grad():
        ops._DISABLE.add('rcinf')   # the 16..32-channel blocks otherwise take the recompute chain
        try:
            fused = net.backbone(x, False, taps=names)
        finally:
            ops._DISABLE.discard('rcinf')
        ops._DISABLE.add('irblock')
        try:
            plain = net.backbone(x, False, taps=names)
        finally:
            ops._DISABLE.discard('irblock')
        P = {k: v.detach().double().cpu() for k, v in net.store.params.items()}
        B = {k: v.detach().double().cpu() for k, v in net.store.buffers.items()}
        ref = onet.backbone(x.double().cpu().permute(0, 3, 1, 2), P, B, False)
    for k in names:
        r = ref[k].permute(0, 2, 3, 1)
        ef = float((fused[k].double().cpu() - r).abs().max() / r.abs().max())
        ep = float((plain[k].double().cpu() - r).abs().max() / r.abs().max())
        assert ef <= 1.5 * ep + 1e-3, (k, ef, ep)

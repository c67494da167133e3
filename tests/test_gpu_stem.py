"""Stem conv (3x3, Cin 3 -> 32, mobilenet_v2.py:58) at a size that exercises the launch
shapes of the 720p step: 128-pixel row segments with W % 128 == 0 (BatchNorm statistics
fused into stem_fwd_mfma_kernel), several rows per block with a ragged last block (forward
rb = 2, weight gradient rb = 14 on H = 721), against the CPU oracle on the same
bf16-rounded operands."""
import numpy as np
import pytest
import torch

from oracle import net as onet
from rod import ops

pytestmark = pytest.mark.gpu


def test_stem_full_width(dev):
    N, H, W = 3, 721, 1280
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, H, W, 3, generator=g).to(torch.bfloat16).float()
    w = (torch.randn(32, 3, 3, 3, generator=g) / np.sqrt(27)).to(torch.bfloat16).float()
    wo = w.clone().requires_grad_(True)
    yo = onet.conv(x.permute(0, 3, 1, 2), wo).permute(0, 2, 3, 1)
    gy = torch.randn(yo.shape, generator=g).to(torch.bfloat16).float()
    (yo * gy).sum().backward()

    wd = w.detach().clone().to(dev).requires_grad_(True)
    wd._rod_grad = torch.zeros_like(wd)
    yd, parts = ops.conv2d(x.to(dev, torch.bfloat16), wd, None, 3, want_stats=True)
    yd.backward(gy.to(dev, torch.bfloat16))

    # forward: exact bf16 products, fp32 sums, one rounding to bf16 (<= 1 bf16 ulp)
    torch.testing.assert_close(yd.float().cpu(), yo.detach(), rtol=8e-3, atol=1e-2)
    # weight gradient: 2.77 M-term fp32 sums in another order than the oracle's
    dw = wd._rod_grad.cpu()
    rel = float((dw - wo.grad).norm() / wo.grad.norm())
    assert rel < 1e-4, rel
    # fused statistics == the separate statistics pass on the same output
    be = torch.zeros(32, device=dev)
    mm1, mv1 = torch.zeros(32, device=dev), torch.ones(32, device=dev)
    mm2, mv2 = mm1.clone(), mv1.clone()
    z1 = ops.bn_act(yd.detach(), None, be, mm1, mv1, ops.ROD_ACT_NONE, True, 0.9, 1e-3, parts=parts)
    z2 = ops.bn_act(yd.detach(), None, be, mm2, mv2, ops.ROD_ACT_NONE, True, 0.9, 1e-3)
    torch.testing.assert_close(mm1, mm2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(mv1, mv2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(z1.float(), z2.float(), rtol=1e-2, atol=2e-2)


@pytest.mark.parametrize('N,H,W', [(2, 37, 300), (1, 720, 1280)])
def test_stem_wgrad_bn_matches_apply_then_wgrad(dev, N, H, W):
    """rod_stem_wgrad_bn (dy formed from the stem BatchNorm's (dz, y) in the weight gradient's
    loader) against rod_bn_bwd_apply -> rod_conv_wgrad: the same dy rounding and MFMA order, so
    dw is bit-identical; ragged widths (W % 128 != 0) zero the pixels past W."""
    bf16 = torch.bfloat16
    g = torch.Generator().manual_seed(N * H + W)
    x = (torch.rand(N, H, W, 3, generator=g) * 2 - 1).to(dev, bf16)
    y = (torch.randn(N, H, W, 32, generator=g) * 2 + 0.5).to(dev, bf16)
    dz = (torch.randn(N, H, W, 32, generator=g) * 0.1).to(dev, bf16)
    mean = y.float().mean((0, 1, 2))
    rstd = torch.rsqrt(y.float().var((0, 1, 2), unbiased=False) + 1e-3)
    gamma = (torch.rand(32, generator=g) + 0.5).to(dev)
    beta = (torch.randn(32, generator=g) * 0.3).to(dev)
    act = ops.ROD_ACT_RELU6
    M = N * H * W
    coef = ops.bn_bwd_reduce(dz, y, mean, rstd, gamma, beta, act, False, False)
    dy = torch.empty_like(y)
    ops._abi.call('rod_bn_bwd_apply', dz, y, mean, rstd, gamma, beta, coef, dy, M, 32, act, ops.dtcode(y), ops.stream())
    ws = ops.workspace(ops._abi.query('rod_conv_wgrad_workspace', N, H, W, 3, 32, 3), dev)
    dw_ref = torch.empty(32, 3, 3, 3, device=dev)
    ops._abi.call('rod_conv_wgrad', x, None, None, None, None, 0, dy, dw_ref, None, ws, N, H, W, 3, 32, 3, 0, 0,
                  ops.dtcode(x), ops.stream())
    dw = torch.full((32, 3, 3, 3), float('nan'), device=dev)
    ws2 = ops.workspace(ops._abi.query('rod_conv_wgrad_workspace', N, H, W, 3, 32, 3), dev)
    ops._abi.call('rod_stem_wgrad_bn', x, dz, y, mean, rstd, gamma, beta, act, coef, dw, ws2, N, H, W, 3, 32, 3,
                  ops.dtcode(y), ops.stream())
    torch.cuda.synchronize()
    assert torch.equal(dw, dw_ref), float((dw - dw_ref).abs().max())
